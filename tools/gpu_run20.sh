#!/bin/bash
# ResNet-50 O2 steady-state kernel profile (10 timed steps after the spin marker)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
(cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof_bench.log 2>&1)
rc=$?; tail -1 gpurun_out/prof_bench.log | cut -c1-150; [ $rc -ne 0 ] && { echo "STOP prof rc=$rc"; exit $rc; }
python tools/prof_summary.py /tmp/prof_rn/rn_results.db --after spin_kernel --top 60 --md gpurun_out/resnet50_steady.md > /dev/null 2>&1
head -12 gpurun_out/resnet50_steady.md
echo ALL_DONE
