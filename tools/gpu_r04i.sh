#!/bin/bash
# native stem + fused conv3 backward: kernel / node tests, stem node bench, ResNet bench A/B
# (default, no native stem, no fused conv3 backward), kernel-trace profile of the ResNet step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_stem.py tests/test_conv3_bwd.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stem_node_bench.py > $O/stem_bench.log 2>&1 || { tail -5 $O/stem_bench.log; exit 1; }
cat $O/stem_bench.log
timeout -k 10 400 python bench.py > $O/resnet.log 2>&1 || { tail -5 $O/resnet.log; exit 1; }
tail -1 $O/resnet.log | cut -c1-200
APEX_AMD_NATIVE_STEM=0 timeout -k 10 400 python bench.py > $O/resnet_nostem.log 2>&1 || { tail -5 $O/resnet_nostem.log; exit 1; }
tail -1 $O/resnet_nostem.log | cut -c1-200
APEX_AMD_CONV3_BWD=0 timeout -k 10 400 python bench.py > $O/resnet_noc3b.log 2>&1 || { tail -5 $O/resnet_noc3b.log; exit 1; }
tail -1 $O/resnet_noc3b.log | cut -c1-200
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_resnet_r04i -o bench -- python3 $R/bench.py --steps 10 --warmup 8 \
    > $R/$O/prof_resnet.log 2>&1 ) || { tail -5 $O/prof_resnet.log; exit 1; }
db=$(find $R/gpurun_out/prof_resnet_r04i -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 60 --md $O/resnet_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_resnet_r04i
head -14 $O/resnet_prof.md
