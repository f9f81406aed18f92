#!/bin/bash
# native split-K GEMM for the short-wide dense weight gradient: tests + GPT-2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ah
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x -m gpu --timeout 150 --timeout-method thread tests/test_fused_dense.py tests/test_standalone_models.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1; do
  APEX_AMD_WIDE_WGRAD=$v timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_w$v.log 2>&1 || { tail -5 $O/gpt2_w$v.log; exit 1; }
  echo "gpt2 wide=$v $(tail -1 $O/gpt2_w$v.log | cut -c80-130)"
done
