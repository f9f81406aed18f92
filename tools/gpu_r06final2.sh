#!/bin/bash
# round-6 last-tree validation: full GPU tier, smoke, driver-exact bench x2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06final2; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu_tier.log 2>&1; rc=$?
tail -3 $O/gpu_tier.log
[ $rc -ne 0 ] && { grep -E "FAILED|ERROR" $O/gpu_tier.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { tail -5 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | cut -c1-200
done
