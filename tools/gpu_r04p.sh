#!/bin/bash
# branch-free prefetch (counted vmcnt waits) in the stem, conv3 backward and fused 1x1 kernels:
# tests, kernel benches, ResNet bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_stem.py tests/test_conv3_bwd.py tests/test_conv1x1_bn.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stem_node_bench.py > $O/stem_bench.log 2>&1 || { tail -5 $O/stem_bench.log; exit 1; }
cat $O/stem_bench.log
for md in 0; do
  APEX_AMD_STEM_WG_MODE=$md timeout -k 10 120 python tools/stem_wgrad_probe.py >> $O/wg_modes.log 2>&1 || { tail -5 $O/wg_modes.log; exit 1; }
done
grep kernel $O/wg_modes.log
timeout -k 10 200 python tools/conv3_bwd_bench.py > $O/c3b_bench.log 2>&1 || { tail -5 $O/c3b_bench.log; exit 1; }
cat $O/c3b_bench.log
timeout -k 10 400 python bench.py > $O/resnet.log 2>&1 || { tail -5 $O/resnet.log; exit 1; }
tail -1 $O/resnet.log | cut -c1-200
