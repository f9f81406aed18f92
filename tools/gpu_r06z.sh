#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 300 python tools/tap_inner_bench.py > $O/tap.jsonl 2>&1 || { tail -3 $O/tap.jsonl; exit 1; }
grep '^{' $O/tap.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_igemm.py tests/test_bottleneck_block.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-160
bash tools/gpu_r06e.sh r06z_tl > /dev/null
