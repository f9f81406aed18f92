#!/bin/bash
# GPU session: new-kernel tests first (own time limit), then the full GPU tier, then kernel benches.
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -m pytest tests/test_attention.py -m gpu -q -p no:cacheprovider > gpurun_out/pytest_attn.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_attn.log; [ $rc -ge 2 ] && stop pytest_attn $rc
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider --deselect tests/test_attention.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && stop pytest $rc
timeout -k 10 400 python tools/bench_kernels.py --only ${KERNELS:-attn,gemm} > gpurun_out/kernels.jsonl 2> gpurun_out/kernels.err
rc=$?; cut -c1-260 gpurun_out/kernels.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/kernels.err; stop kernels $rc; }
echo ALL_DONE
