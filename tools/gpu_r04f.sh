#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_conv_igemm.py tests/test_conv1x1_bn.py tests/test_bottleneck_block.py > gpurun_out/r04f/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04f/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/conv_cfg_sweep.py > gpurun_out/r04f/sweep.jsonl 2> gpurun_out/r04f/sweep.err || { tail -5 gpurun_out/r04f/sweep.err; exit 1; }
echo SWEEP_DONE
timeout -k 10 400 python bench.py > gpurun_out/r04f/bench.log 2>&1 || { tail -5 gpurun_out/r04f/bench.log; exit 1; }
tail -1 gpurun_out/r04f/bench.log
