#!/bin/bash
# split-coefficient add+ReLU prologue, native stride-2 subsample, stem reduce, MTA address patching:
# tests, then the headline A/B against the previous commit's routes where one exists
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py \
  tests/test_multi_tensor.py tests/test_stem.py tests/test_bottleneck_block.py tests/test_optimizers.py > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/stem_wgrad_probe.py > $O/stem_probe.jsonl 2>&1; grep kernel $O/stem_probe.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { tail -5 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | cut -c1-200
done
APEX_AMD_BN_CENSUS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 > $O/census.log 2>&1; grep "bn census" $O/census.log | head -40
