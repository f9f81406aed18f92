#!/bin/bash
# one-step dispatch timeline of the ResNet-50 bench (layer-level attribution) + BN census
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06b
mkdir -p $O
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace \
    -d $R/gpurun_out/prof_tl -o bench -- python3 $R/bench.py --steps 10 --warmup 8 \
    > $R/$O/prof.log 2>&1 ) || { tail -5 $O/prof.log; exit 1; }
db=$(find $R/gpurun_out/prof_tl -name '*results.db' | head -1)
python3 tools/prof_timeline.py "$db" --after spin_kernel --steps 10 --step 5 --md $O/timeline.md || exit 1
rm -rf $R/gpurun_out/prof_tl
APEX_AMD_BN_CENSUS=1 timeout -k 10 300 python bench.py --steps 2 --warmup 0 > $O/census.log 2>&1; tail -40 $O/census.log | cut -c1-200
