#!/bin/bash
# round 6: GeLU pass with 4 vectors in flight — tests, route micro-bench, transformer driver-form runs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06gl
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_dense.py -m gpu -k "gelu" \
  > $O/test_fd.txt 2>&1 || { tail -30 $O/test_fd.txt; exit 1; }
tail -1 $O/test_fd.txt
timeout -k 10 300 python tools/gelu_route_bench.py > $O/gelu_routes.jsonl 2>&1 || { tail -20 $O/gelu_routes.jsonl; exit 1; }
grep fwd_ $O/gelu_routes.jsonl
timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_medium.log 2>&1 || { tail -5 $O/gpt2_medium.log; exit 1; }
tail -1 $O/gpt2_medium.log
timeout -k 10 400 python bench.py --model bert-large > $O/bert_large.log 2>&1 || { tail -5 $O/bert_large.log; exit 1; }
tail -1 $O/bert_large.log
