#!/bin/bash
# step timeline of the current tree (one step, dispatch order)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r06e}
O=gpurun_out/$TAG
mkdir -p $O
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace \
    -d $R/gpurun_out/prof_tl_$TAG -o bench -- python3 $R/bench.py --steps 10 --warmup 8 \
    > $R/$O/prof.log 2>&1 ) || { tail -5 $O/prof.log; exit 1; }
db=$(find $R/gpurun_out/prof_tl_$TAG -name '*results.db' | head -1)
python3 tools/prof_timeline.py "$db" --after spin_kernel --steps 10 --step 5 --md $O/timeline.md || exit 1
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 100 --md $O/resnet_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_tl_$TAG
head -12 $O/resnet_prof.md
