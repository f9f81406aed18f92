#!/bin/bash
# native global-pool gradient broadcast: tests, bench + trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aj
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_standalone_models.py \
  tests/test_stem.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r05b.sh r05aj || exit 1
