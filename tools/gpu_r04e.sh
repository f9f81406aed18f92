#!/bin/bash
# round-4 checkpoint: conv / node GPU tests, driver-exact bench, fprop sweep (incl. fprop3),
# kernel-trace profile of the step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04e
timeout -k 10 900 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_conv_igemm.py tests/test_bottleneck_block.py tests/test_conv1x1_bn.py > gpurun_out/r04e/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04e/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r04e/bench.log 2>&1 || { tail -5 gpurun_out/r04e/bench.log; exit 1; }
tail -1 gpurun_out/r04e/bench.log
timeout -k 10 600 python tools/conv_cfg_sweep.py > gpurun_out/r04e/sweep.jsonl 2> gpurun_out/r04e/sweep.err || { tail -5 gpurun_out/r04e/sweep.err; exit 1; }
echo SWEEP_DONE
timeout -k 10 600 bash tools/prof_ab.sh node_r04e "APEX_AMD_FUSED_BLOCK=1" node_r04e2 "APEX_AMD_FUSED_BLOCK=1" > gpurun_out/r04e/prof.log 2>&1 || { tail -5 gpurun_out/r04e/prof.log; exit 1; }
echo PROF_DONE
