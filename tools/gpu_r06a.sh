#!/bin/bash
# round 6 first GPU call: the ADVICE-fix tests, then the headline bench + a 10-step kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_multi_tensor.py \
  tests/test_dropout_rng.py tests/test_lt_plan_sync.py tests/test_distributed_optimizers.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r05b.sh r06a || exit 1
