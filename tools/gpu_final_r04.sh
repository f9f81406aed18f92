#!/bin/bash
# Round-4 regression on one box: every GPU test, smoke, the driver-exact ResNet bench.
cd $GRAFT_REPO_ROOT
O=gpurun_out/final_r04
mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -12 $O/pytest_gpu.log; [ $rc -ge 2 ] && stop pytest $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -3 $O/smoke.log; [ $rc -ne 0 ] && stop smoke $rc
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log | cut -c1-300; [ $rc -ne 0 ] && stop bench $rc
if [ -n "$TRANSFORMERS" ]; then
  timeout -k 10 500 python bench.py --model gpt2-medium > $O/gpt2.log 2>&1
  rc=$?; tail -1 $O/gpt2.log | cut -c1-200; [ $rc -ne 0 ] && stop gpt2 $rc
  timeout -k 10 500 python bench.py --model bert-large > $O/bert.log 2>&1
  rc=$?; tail -1 $O/bert.log | cut -c1-200; [ $rc -ne 0 ] && stop bert $rc
fi
echo ALL_DONE
