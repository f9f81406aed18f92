#!/bin/bash
# LayerNorm backward resident blocks per CU: norm tests, same-box GPT-2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ah
mkdir -p $O
APEX_AMD_LN_BWD_BPC=4 timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_norm.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for arm in 2 4 3; do
    APEX_AMD_LN_BWD_BPC=$arm timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_${arm}_$i.log 2>&1 || exit 1
    echo "gpt2 ln_bwd_bpc=$arm round $i: $(tail -1 $O/gpt2_${arm}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/ab.txt
  done
done
