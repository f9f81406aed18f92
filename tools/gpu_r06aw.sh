#!/bin/bash
# halo wgrad split reduce with 4 partials in flight: tests, per-kernel trace, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aw; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_halo_wgrad.py tests/test_bottleneck_block.py -m gpu > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/gpu_r06e.sh r06aw_tl > /dev/null || exit 1
grep -E "reduce_kernel|busy" gpurun_out/r06aw_tl/resnet_prof.md | cut -c1-160
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-160
