#!/bin/bash
# scratch-free fused 1x1 ring (DEPTH 4/5) + c3b: tests, micro-bench, census, bench, timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py tests/test_conv3_bwd.py tests/test_bottleneck_block.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/dgrad_bnred_bench.py > $O/dg.jsonl 2>&1 || { tail -3 $O/dg.jsonl; exit 1; }
cat $O/dg.jsonl
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/$O/census.log 2>&1 ) || exit 1
python3 tools/scratch_census.py $(find $O/tr -name "*kernel_trace.csv") > $O/census.md; rm -rf $O/tr; cat $O/census.md
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
bash tools/gpu_r06e.sh r06t_tl
