#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04al
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_stem.py tests/test_bottleneck_block.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-150
bash tools/gpu_pmc_bench.sh r04al > gpurun_out/pmc_r04al.log 2>&1 || exit 1
grep -E "stem::" gpurun_out/pmc_r04al/pmc.md | cut -c1-220
