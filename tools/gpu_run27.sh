#!/bin/bash
# 2-rank DDP rehearsal over gloo on one GPU (correctness of the multi-rank bench path), steady-state profile
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
stop() { echo "STOP: $1 rc=$2"; exit $2; }
APEX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 > gpurun_out/bench_gloo2.log 2>&1
rc=$?; grep metric gpurun_out/bench_gloo2.log | cut -c1-200; [ $rc -ne 0 ] && stop gloo2 $rc
(cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof_bench.log 2>&1)
rc=$?; [ $rc -ne 0 ] && stop prof $rc
python tools/prof_summary.py /tmp/prof_rn/rn_results.db --after spin_kernel --top 60 --md gpurun_out/resnet50_steady_r01f.md > /dev/null 2>&1
head -10 gpurun_out/resnet50_steady_r01f.md
echo ALL_DONE
