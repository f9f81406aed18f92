#!/bin/bash
# GPU session: attention A/B timing + per-kernel profile, ResNet-50 bench, transformer benches.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_attention.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_attn.log; [ $rc -ne 0 ] && stop pytest_attn $rc
timeout -k 10 300 python tools/bench_kernels.py --only attn > gpurun_out/kernels_attn.jsonl 2> gpurun_out/kernels_attn.err
rc=$?; cut -c1-400 gpurun_out/kernels_attn.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/kernels_attn.err; stop kernels $rc; }
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_attn -o attn -- python3 $R/tools/attn_prof.py > $R/gpurun_out/prof_attn.log 2>&1)
rc=$?; tail -2 gpurun_out/prof_attn.log; [ $rc -ne 0 ] && stop prof_attn $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 8 > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; [ $rc -ne 0 ] && stop bench $rc
timeout -k 10 400 python -u bench.py --model gpt2-medium --steps 10 --warmup 4 > gpurun_out/bench_gpt.log 2>&1
rc=$?; tail -2 gpurun_out/bench_gpt.log; [ $rc -ne 0 ] && stop bench_gpt $rc
timeout -k 10 400 python -u bench.py --model bert-large --steps 10 --warmup 4 > gpurun_out/bench_bert.log 2>&1
rc=$?; tail -2 gpurun_out/bench_bert.log; [ $rc -ne 0 ] && stop bench_bert $rc
echo ALL_DONE
