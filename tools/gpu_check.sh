#!/bin/bash
# One GPU-box session: gpu tests, smoke, bench, rocprof stats. Each GPU step has its own limit.
# Test failures (rc 1) do not stop the chain; crashes/timeouts (rc >= 124) do.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 400 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && stop pytest $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -ne 0 ] && stop smoke $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 8 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; [ $rc -ne 0 ] && stop bench $rc
if [ -n "$BASELINE" ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --impl torch > gpurun_out/bench_torch.log 2>&1
  rc=$?; tail -3 gpurun_out/bench_torch.log; [ $rc -ne 0 ] && stop bench_torch $rc
fi
if [ -n "$PROF" ]; then
  cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 10 --warmup 6 > $R/gpurun_out/prof_bench.log 2>&1
  rc=$?; tail -3 $R/gpurun_out/prof_bench.log; [ $rc -ne 0 ] && stop prof $rc
fi
echo ALL_DONE
