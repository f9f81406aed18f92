#!/bin/bash
# sync-free LAMB GPU test, halo wgrad tests, then the same-box headline A/B of the halo wgrad
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_distributed_optimizers.py::test_gpu_distributed_lamb_step_makes_no_host_sync tests/test_conv_halo_wgrad.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_bench.sh r05c "APEX_AMD_HALO_WGRAD=0" "APEX_AMD_HALO_WGRAD=1" 2
