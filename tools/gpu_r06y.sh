#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention.py tests/test_standalone_models.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/tap_inner_bench.py > $O/tap.jsonl 2>&1 || { tail -3 $O/tap.jsonl; exit 1; }
grep '^{' $O/tap.jsonl
timeout -k 10 300 python bench.py --model bert-large > $O/bert.log 2>&1 || { tail -3 $O/bert.log; exit 1; }
tail -1 $O/bert.log | cut -c1-160
