#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_groupbn.py tests/test_syncbn.py tests/test_pooling.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_bn.log; [ $rc -ne 0 ] && stop pytest $rc
timeout -k 10 300 python tools/bench_kernels.py --only bn > gpurun_out/kernels_bn.jsonl 2> gpurun_out/kernels_bn.err
rc=$?; cut -c1-200 gpurun_out/kernels_bn.jsonl; [ $rc -ne 0 ] && stop kernels $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-150; [ $rc -ne 0 ] && stop bench $rc
echo ALL_DONE
