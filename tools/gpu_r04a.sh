set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python tools/host_probe.py --steps 8 --warmup 6 > gpurun_out/host_probe.log 2>&1 || { echo probe fail $?; exit 1; }
head -c 3000 gpurun_out/host_probe.log
timeout -k 10 1000 bash tools/gpu_pmc_bench.sh r04a
