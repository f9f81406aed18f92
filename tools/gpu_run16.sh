#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
(cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_bench -o bench -- python3 $R/bench.py --steps 10 --warmup 6 > $R/gpurun_out/prof_bench.log 2>&1)
rc=$?; [ $rc -ne 0 ] && stop prof $rc
python tools/prof_summary.py /tmp/prof_bench/bench_results.db --after spin_kernel --top 60 --md gpurun_out/resnet50_steady.md > /dev/null 2>&1
echo ALL_DONE
