#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 200 python tools/diag_layout.py > gpurun_out/diag_layout.log 2>&1
rc=$?; cat gpurun_out/diag_layout.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && stop diag $rc
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 timeout -k 10 400 python -u bench.py > gpurun_out/bench_nowrwasm.log 2>&1
rc=$?; tail -1 gpurun_out/bench_nowrwasm.log | cut -c1-150; [ $rc -ne 0 ] && stop bench_a $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-150; [ $rc -ne 0 ] && stop bench $rc
echo ALL_DONE
