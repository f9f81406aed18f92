#!/bin/bash
# ResNet-50 step kernel trace on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 400 python bench.py > $O/resnet.log 2>&1 || { tail -5 $O/resnet.log; exit 1; }
tail -1 $O/resnet.log | cut -c1-200
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_resnet_r04r -o bench -- python3 $R/bench.py --steps 10 --warmup 8 \
    > $R/$O/prof_resnet.log 2>&1 ) || { tail -5 $O/prof_resnet.log; exit 1; }
db=$(find $R/gpurun_out/prof_resnet_r04r -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 70 --md $O/resnet_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_resnet_r04r
head -14 $O/resnet_prof.md
