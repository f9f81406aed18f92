#!/bin/bash
# halo fprop numerics + per-shape A/B, then the round-5 GPU tests, then the halo-wgrad headline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_halo_fprop.py \
  > $O/hfp_tests.log 2>&1
rc=$?; tail -25 $O/hfp_tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/halo_fprop_bench.py > $O/hfp_bench.jsonl 2>&1 || { tail -5 $O/hfp_bench.jsonl; exit 1; }
cut -c1-160 $O/hfp_bench.jsonl
timeout -k 10 600 python -u -m pytest -q -s --timeout 200 --timeout-method thread \
  tests/test_distributed_optimizers.py::test_gpu_distributed_lamb_step_makes_no_host_sync tests/test_conv_halo_wgrad.py \
  tests/test_lt_plan_sync.py tests/test_bottleneck_block.py::test_gpu_bottleneck_chain_fp16_arm_pins_the_tolerances \
  tests/test_bottleneck_block.py::test_gpu_bottleneck_chain_syncbn_fp16_arm \
  > $O/tests.log 2>&1
grep -E "^(bf16|fp16|0 |1 )|passed|failed|Error|assert" $O/tests.log | head -30
bash tools/ab_bench.sh r05d "APEX_AMD_CONV_HFP=0" "APEX_AMD_CONV_HFP=1" 2
