#!/bin/bash
# A/B: every bottleneck 1x1 on the native fused kernels (stage 3/4 included) vs the per-shape routes;
# fresh 3x3 fprop tile-configuration sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05j
mkdir -p $O
bash tools/ab_bench.sh r05j_native "APEX_AMD_FUSED_BLOCK_FORCE_NATIVE=0" "APEX_AMD_FUSED_BLOCK_FORCE_NATIVE=1" 2 || exit 1
timeout -k 10 600 python -u tools/conv_cfg_sweep.py > $O/cfg_sweep.jsonl 2>&1; tail -3 $O/cfg_sweep.jsonl | cut -c1-300
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem.py > $O/stem_tests.log 2>&1
rc=$?; tail -3 $O/stem_tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/stem_node_bench.py > $O/stem_node.jsonl 2>&1; grep row $O/stem_node.jsonl
