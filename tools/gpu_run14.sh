#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_attention.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_t.log; [ $rc -ne 0 ] && stop pytest $rc
timeout -k 10 300 python tools/bench_kernels.py --only attn > gpurun_out/kernels_attn.jsonl 2> gpurun_out/kernels_attn.err
rc=$?; cut -c1-200 gpurun_out/kernels_attn.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/kernels_attn.err; stop kernels $rc; }
timeout -k 10 400 python -u bench.py --model gpt2-medium --steps 10 --warmup 4 > gpurun_out/bench_gpt.log 2>&1
rc=$?; tail -1 gpurun_out/bench_gpt.log | cut -c1-200; [ $rc -ne 0 ] && stop bench_gpt $rc
echo ALL_DONE
