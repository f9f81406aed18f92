#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && stop pytest $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; [ $rc -ne 0 ] && stop bench $rc
timeout -k 10 400 python tools/bench_kernels.py > gpurun_out/kernels.jsonl 2> gpurun_out/kernels.err
rc=$?; cat gpurun_out/kernels.jsonl | cut -c1-220; [ $rc -ne 0 ] && { tail -20 gpurun_out/kernels.err; stop kernels $rc; }
cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 10 --warmup 6 > $R/gpurun_out/prof_bench.log 2>&1
rc=$?; tail -2 $R/gpurun_out/prof_bench.log; [ $rc -ne 0 ] && stop prof $rc
echo ALL_DONE
