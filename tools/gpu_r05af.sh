#!/bin/bash
# one RNG-step snapshot per step: dropout / attention tests, transformer benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05af
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_dropout_rng.py \
  tests/test_attention.py tests/test_fused_dense.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && [ $rc -ne 4 ] && exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_$i.log 2>&1 || exit 1
  tail -1 $O/gpt2_$i.log | cut -c1-150
done
timeout -k 10 400 python bench.py --model bert-large > $O/bert.log 2>&1 || exit 1
tail -1 $O/bert.log | cut -c1-150
