#!/bin/bash
# amp O2 input cast inside the stem's padding pass: tests, same-box A/B, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ai
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_stem.py \
  tests/test_amp.py tests/test_amp_matrix.py tests/test_standalone_models.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh r05ai_cast "APEX_AMD_STEM_INPUT_CAST=1" "APEX_AMD_STEM_INPUT_CAST=0" 2 || exit 1
bash tools/gpu_r05b.sh r05ai || exit 1
