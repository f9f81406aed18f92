#!/bin/bash
# GPU session: 1x1-conv MIOpen vs GEMM A/B; ResNet-50 bench kernel profile (steady state).
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python tools/conv1x1_bench.py > gpurun_out/conv1x1.jsonl 2> gpurun_out/conv1x1.err
rc=$?; cut -c1-260 gpurun_out/conv1x1.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/conv1x1.err; stop conv1x1 $rc; }
(cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 10 --warmup 6 > $R/gpurun_out/prof_bench.log 2>&1)
rc=$?; grep -v "^\[bench\]" gpurun_out/prof_bench.log | tail -2 | cut -c1-200; [ $rc -ne 0 ] && stop prof $rc
python tools/prof_summary.py gpurun_out/prof_bench/bench_results.db --after spin_kernel --top 45 --md gpurun_out/resnet50_steady.md > /dev/null 2>&1
head -12 gpurun_out/resnet50_steady.md
(cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gpt -o gpt -- python3 $R/bench.py --model gpt2-medium --steps 5 --warmup 3 > $R/gpurun_out/prof_gpt.log 2>&1)
rc=$?; grep -v "^\[bench\]" gpurun_out/prof_gpt.log | tail -1 | cut -c1-200; [ $rc -ne 0 ] && stop prof_gpt $rc
python tools/prof_summary.py gpurun_out/prof_gpt/gpt_results.db --after spin_kernel --top 45 --md gpurun_out/gpt2_steady.md > /dev/null 2>&1
head -12 gpurun_out/gpt2_steady.md
echo ALL_DONE
