#!/bin/bash
# full GPU tier + smoke + driver-exact bench on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05al
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu_all.log 2>&1
rc=$?; tail -8 $O/gpu_all.log | cut -c1-300; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1; tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-200
