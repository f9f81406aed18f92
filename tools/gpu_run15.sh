#!/bin/bash
# full GPU tier + smoke + headline bench + transformer benches
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && stop pytest $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -ne 0 ] && stop smoke $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-200; [ $rc -ne 0 ] && stop bench $rc
timeout -k 10 400 python -u bench.py --model bert-large --steps 10 --warmup 4 > gpurun_out/bench_bert.log 2>&1
rc=$?; tail -1 gpurun_out/bench_bert.log | cut -c1-200; [ $rc -ne 0 ] && stop bench_bert $rc
echo ALL_DONE
