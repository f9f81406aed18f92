#!/bin/bash
# compile-time RED2: tests, dgrad micro-bench, bench, timeline; transformer benches (driver form)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py tests/test_bottleneck_block.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/dgrad_bnred_bench.py > $O/dg.jsonl 2>&1 || exit 1
grep '^{' $O/dg.jsonl
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-160
bash tools/gpu_r06e.sh r06aa_tl > /dev/null || exit 1
timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_medium.log 2>&1 || { tail -5 $O/gpt2_medium.log; exit 1; }
tail -1 $O/gpt2_medium.log | cut -c1-160
timeout -k 10 400 python bench.py --model bert-large > $O/bert_large.log 2>&1 || { tail -5 $O/bert_large.log; exit 1; }
tail -1 $O/bert_large.log | cut -c1-160
