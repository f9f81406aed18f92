#!/bin/bash
# final-ish tree: node tests + prefetch test, bench, then per-kernel counters of the step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ac; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py tests/test_bottleneck_block.py tests/test_conv_igemm.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-160
bash tools/gpu_pmc_cmd.sh r06ac bench.py --steps 2 --warmup 2 || exit 1
