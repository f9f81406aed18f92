#!/bin/bash
# stem wgrad (quad gather + LDS-DMA im2col): numerics, per-kernel times, diagnostic modes; the
# relaxed fp16 chain tests; one headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem.py > $O/stem_tests.log 2>&1
rc=$?; tail -15 $O/stem_tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/stem_node_bench.py > $O/stem_node.jsonl 2>&1 || { tail -5 $O/stem_node.jsonl; exit 1; }
cat $O/stem_node.jsonl
for m in 0 1 2 4 7; do
  APEX_AMD_STEM_WG_MODE=$m timeout -k 10 120 python -u tools/stem_wgrad_probe.py >> $O/stem_probe.jsonl 2>&1 || { tail -5 $O/stem_probe.jsonl; exit 1; }
done
cat $O/stem_probe.jsonl
timeout -k 10 400 python -u -m pytest -q -s --timeout 200 --timeout-method thread \
  tests/test_bottleneck_block.py::test_gpu_bottleneck_chain_fp16_arm_pins_the_tolerances \
  tests/test_bottleneck_block.py::test_gpu_bottleneck_chain_syncbn_fp16_arm > $O/fp16.log 2>&1
grep -E "passed|failed|Error|assert" $O/fp16.log | head -10
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_attention.py -k "drop" > $O/attn.log 2>&1; tail -2 $O/attn.log
timeout -k 10 400 python -u bench.py --steps 30 --warmup 10 > $O/bench.log 2>&1; tail -2 $O/bench.log
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_norm.py > $O/norm.log 2>&1; tail -3 $O/norm.log
timeout -k 10 200 python -u tools/ln_wide_bench.py > $O/ln_wide.jsonl 2>&1; cat $O/ln_wide.jsonl
