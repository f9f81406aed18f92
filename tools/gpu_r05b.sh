#!/bin/bash
# ResNet-50 headline: driver-exact bench + a 10-step kernel trace of the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r05b}
O=gpurun_out/$TAG
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_resnet_$TAG -o bench -- python3 $R/bench.py --steps 10 --warmup 8 \
    > $R/$O/prof_resnet.log 2>&1 ) || { tail -5 $O/prof_resnet.log; exit 1; }
db=$(find $R/gpurun_out/prof_resnet_$TAG -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 100 --md $O/resnet_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_resnet_$TAG
head -12 $O/resnet_prof.md
