#!/bin/bash
# BN fork (two-gradient backward), 32-bit pool index math: tests, bench, steady-state profile
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_groupbn.py tests/test_pooling.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_bn.log; [ $rc -ne 0 ] && stop pytest $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-150; [ $rc -ne 0 ] && stop bench $rc
(cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_rn -o rn -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof_bench.log 2>&1)
rc=$?; [ $rc -ne 0 ] && stop prof $rc
python tools/prof_summary.py /tmp/prof_rn/rn_results.db --after spin_kernel --top 60 --md gpurun_out/resnet50_steady.md > /dev/null 2>&1
head -12 gpurun_out/resnet50_steady.md
echo ALL_DONE
