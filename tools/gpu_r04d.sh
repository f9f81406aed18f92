#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04c
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_bottleneck_block.py tests/test_fused_dense.py -k "chain or syncbn or gelu_pass or fp32 or fused_dense_gelu" > gpurun_out/r04c/tests_blk.log 2>&1
rc=$?; tail -3 gpurun_out/r04c/tests_blk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/conv_cfg_sweep.py > gpurun_out/r04c/sweep.jsonl 2> gpurun_out/r04c/sweep.err || { tail -5 gpurun_out/r04c/sweep.err; exit 1; }
echo SWEEP_DONE
CONV_AB_ONLY_3X3=1 timeout -k 10 600 python tools/conv_bwd_ab.py --rounds 2 --iters 5 > gpurun_out/r04c/wgrad_ab.jsonl 2> gpurun_out/r04c/wgrad_ab.err || { tail -5 gpurun_out/r04c/wgrad_ab.err; exit 1; }
echo WGRAD_DONE
