#!/bin/bash
# stem pad pass with 8 pixels per thread per trip: stem tests, per-kernel trace, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06az; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem.py -m gpu > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/gpu_r06e.sh r06az_tl > /dev/null || exit 1
grep -E "stem::|busy" gpurun_out/r06az_tl/resnet_prof.md | cut -c1-160
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-160
