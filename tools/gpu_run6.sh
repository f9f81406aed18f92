#!/bin/bash
# GPU session: attention tests + attention A/B timing, full gpu test tier, smoke, bench (+ stock baseline).
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_attention.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; tail -6 gpurun_out/pytest_attn.log; [ $rc -ne 0 ] && stop pytest_attn $rc
timeout -k 10 300 python tools/bench_kernels.py --only attn > gpurun_out/kernels_attn.jsonl 2> gpurun_out/kernels_attn.err
rc=$?; cut -c1-300 gpurun_out/kernels_attn.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/kernels_attn.err; stop kernels $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && stop pytest $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && stop smoke $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; [ $rc -ne 0 ] && stop bench $rc
timeout -k 10 300 python tools/gpu_gpt_smoke.py > gpurun_out/gpt_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/gpt_smoke.log; [ $rc -ne 0 ] && stop gpt $rc
echo ALL_DONE
