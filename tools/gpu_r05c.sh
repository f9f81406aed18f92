#!/bin/bash
# same-box headline A/B of the halo wgrad, then the new round-5 GPU tests (no -x: report all)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c
mkdir -p $O
bash tools/ab_bench.sh r05c "APEX_AMD_HALO_WGRAD=0" "APEX_AMD_HALO_WGRAD=1" 2 || exit 1
timeout -k 10 600 python -u -m pytest -q -s --timeout 200 --timeout-method thread \
  tests/test_distributed_optimizers.py::test_gpu_distributed_lamb_step_makes_no_host_sync tests/test_conv_halo_wgrad.py \
  tests/test_lt_plan_sync.py tests/test_bottleneck_block.py::test_gpu_bottleneck_chain_fp16_arm_pins_the_tolerances \
  tests/test_bottleneck_block.py::test_gpu_bottleneck_chain_syncbn_fp16_arm \
  > $O/tests.log 2>&1
rc=$?; grep -E "^(bf16|fp16|0 |1 )|passed|failed|Error|assert" $O/tests.log | head -30; exit $rc
