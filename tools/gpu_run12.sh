#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_fused_dense.py tests/test_norm.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gemm.log; [ $rc -ne 0 ] && stop pytest_gemm $rc
timeout -k 10 400 python tools/bench_kernels.py --only gemm,ln > gpurun_out/kernels_gemm_ln.jsonl 2> gpurun_out/kernels_gemm.err
rc=$?; grep -E "wgrad|layer_norm_bwd" gpurun_out/kernels_gemm_ln.jsonl | cut -c1-260; [ $rc -ne 0 ] && { tail -5 gpurun_out/kernels_gemm.err; stop kernels $rc; }
timeout -k 10 400 python -u bench.py --model gpt2-medium --steps 10 --warmup 4 > gpurun_out/bench_gpt.log 2>&1
rc=$?; tail -1 gpurun_out/bench_gpt.log | cut -c1-250; [ $rc -ne 0 ] && stop bench_gpt $rc
timeout -k 10 400 python -u bench.py --model bert-large --steps 10 --warmup 4 > gpurun_out/bench_bert.log 2>&1
rc=$?; tail -1 gpurun_out/bench_bert.log | cut -c1-250; [ $rc -ne 0 ] && stop bench_bert $rc
echo ALL_DONE
