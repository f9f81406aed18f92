#!/bin/bash
# round 5: halo-tile 3x3 weight gradient — numerics vs float64, then the per-shape A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a
mkdir -p $O
: timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_halo_wgrad.py > $O/tests.log 2>&1
:
timeout -k 10 300 python -u tools/halo_wgrad_bench.py --check > $O/bench.jsonl 2>&1
rc=$?; cat $O/bench.jsonl | cut -c1-200; exit $rc
