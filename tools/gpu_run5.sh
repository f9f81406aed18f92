#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -m pytest tests/test_fused_dense.py tests/test_pooling.py tests/test_groupbn.py -m gpu -q -p no:cacheprovider -k "gemm256 or maxpool or resnet50" > gpurun_out/pytest_new.log 2>&1
rc=$?; tail -12 gpurun_out/pytest_new.log; [ $rc -ge 2 ] && stop pytest_new $rc
timeout -k 10 300 python tools/bench_kernels.py --only gemm > gpurun_out/kernels_gemm.jsonl 2> gpurun_out/kernels.err
rc=$?; cut -c1-250 gpurun_out/kernels_gemm.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/kernels.err; stop kernels $rc; }
timeout -k 10 300 python tools/gpu_gpt_smoke.py > gpurun_out/gpt_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/gpt_smoke.log; [ $rc -ne 0 ] && stop gpt $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; [ $rc -ne 0 ] && stop bench $rc
timeout -k 10 300 python examples/imagenet/main_amp.py --prof 30 --print-freq 10 -b 128 > gpurun_out/ex_imagenet.log 2>&1
rc=$?; tail -3 gpurun_out/ex_imagenet.log; [ $rc -ne 0 ] && stop ex_imagenet $rc
timeout -k 10 200 python examples/dcgan/main_amp.py --iters 10 > gpurun_out/ex_dcgan.log 2>&1
rc=$?; tail -2 gpurun_out/ex_dcgan.log; [ $rc -ne 0 ] && stop ex_dcgan $rc
bash tools/pyprof_gpu_check.sh > gpurun_out/pyprof_check.log 2>&1
rc=$?; tail -22 gpurun_out/pyprof_check.log; [ $rc -ne 0 ] && stop pyprof $rc
echo ALL_DONE
