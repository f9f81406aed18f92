#!/bin/bash
# 256-tile GEMM: 8-wave (128x64 per wave) vs 4-wave (128x128 per wave) vs hipBLASLt, plus the
# GEMM numerics tests under the 4-wave config.
mkdir -p gpurun_out
APEX_AMD_GEMM256_WAVES=4 timeout -k 10 200 python -m pytest tests/test_fused_dense.py -q -x -m gpu --timeout 120 > gpurun_out/gemm_w4_tests.log 2>&1; tail -2 gpurun_out/gemm_w4_tests.log
for w in 8 4; do
  APEX_AMD_GEMM256_WAVES=$w timeout -k 10 300 python tools/bench_kernels.py --only gemm > gpurun_out/gemm_w$w.jsonl 2>&1 || exit $?
done
grep -h '"kernel"' gpurun_out/gemm_w8.jsonl | cut -c1-200
echo ---
grep -h '"kernel"' gpurun_out/gemm_w4.jsonl | cut -c1-200
