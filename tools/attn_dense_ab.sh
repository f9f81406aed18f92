#!/bin/bash
# attention forward variants (QF=2, low occupancy) + numerics under each, and the routed dense bench
mkdir -p gpurun_out
for v in "" "APEX_ATTN_FWD_QF=2" "APEX_ATTN_FWD_OCC=lo"; do
  env $v timeout -k 10 200 python -m pytest tests/test_attention.py -q -x -m gpu --timeout 120 > gpurun_out/attn_tests.log 2>&1
  rc=$?; echo "attn tests [$v] rc=$rc $(tail -1 gpurun_out/attn_tests.log)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/bench_kernels.py --only attn > gpurun_out/attn_ab.jsonl 2>&1 || exit $?
grep kernel gpurun_out/attn_ab.jsonl | grep flash_fwd | cut -c1-300
timeout -k 10 300 python tools/bench_kernels.py --only dense_route > gpurun_out/dense_route.jsonl 2>&1 || exit $?
grep kernel gpurun_out/dense_route.jsonl | cut -c1-330
STEPS="tests" TESTS="tests/test_fused_dense.py" PYTEST_FLAGS="" TESTS_TIMEOUT=300 bash tools/gpu_session.sh
