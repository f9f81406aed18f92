#!/bin/bash
# round-6 final validation: full GPU tier, smoke, driver-exact bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06final; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu_tier.log 2>&1; rc=$?
tail -3 $O/gpu_tier.log
[ $rc -ne 0 ] && { grep -E "FAILED|ERROR" $O/gpu_tier.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
