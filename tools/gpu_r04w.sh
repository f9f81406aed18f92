#!/bin/bash
# coalesced aout / bits stores of the two-operand prologues: tests, ResNet defer A/B, step trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04w
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread \
  tests/test_conv1x1_bn.py tests/test_bottleneck_block.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/resnet_defer.log 2>&1 || { tail -5 $O/resnet_defer.log; exit 1; }
tail -1 $O/resnet_defer.log | cut -c1-160
APEX_AMD_DEFER_OUTPUT=0 timeout -k 10 400 python bench.py > $O/resnet_nodefer.log 2>&1 || { tail -5 $O/resnet_nodefer.log; exit 1; }
tail -1 $O/resnet_nodefer.log | cut -c1-160
timeout -k 10 400 python bench.py > $O/resnet_defer2.log 2>&1 || { tail -5 $O/resnet_defer2.log; exit 1; }
tail -1 $O/resnet_defer2.log | cut -c1-160
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_resnet_r04w -o bench -- python3 $R/bench.py --steps 10 --warmup 8 \
    > $R/$O/prof_resnet.log 2>&1 ) || { tail -5 $O/prof_resnet.log; exit 1; }
db=$(find $R/gpurun_out/prof_resnet_r04w -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 80 --md $O/resnet_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_resnet_r04w
grep -E "fused1x1|apply_kernel|apply_dual|busy" $O/resnet_prof.md | cut -c1-170
