#!/bin/bash
# stem kernels after the ILP changes (pool fwd, bwd reduce): tests + bench; wgrad diagnostic modes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_stem.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stem_node_bench.py > $O/stem_bench.log 2>&1 || { tail -5 $O/stem_bench.log; exit 1; }
cat $O/stem_bench.log
for md in 0 1 2 4 3 7; do
  APEX_AMD_STEM_WG_MODE=$md timeout -k 10 120 python tools/stem_wgrad_probe.py >> $O/wg_modes.log 2>&1 || { tail -5 $O/wg_modes.log; exit 1; }
done
cat $O/wg_modes.log | grep kernel
