#!/bin/bash
# GPU session: attention correctness + A/B timing after the branch-free PLAIN variants; GPT-2 profile.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_attention.py tests/test_standalone_models.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_attn.log; [ $rc -ne 0 ] && stop pytest_attn $rc
timeout -k 10 300 python tools/bench_kernels.py --only attn > gpurun_out/kernels_attn.jsonl 2> gpurun_out/kernels_attn.err
rc=$?; cut -c1-330 gpurun_out/kernels_attn.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/kernels_attn.err; stop kernels $rc; }
(cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_gpt -o gpt -- python3 $R/bench.py --model gpt2-medium --steps 5 --warmup 3 > $R/gpurun_out/prof_gpt.log 2>&1)
rc=$?; grep -v "^\[bench\]" gpurun_out/prof_gpt.log | tail -1 | cut -c1-200; [ $rc -ne 0 ] && stop prof_gpt $rc
python tools/prof_summary.py /tmp/prof_gpt/gpt_results.db --after spin_kernel --top 50 --md gpurun_out/gpt2_steady.md > /dev/null 2>&1
head -60 gpurun_out/gpt2_steady.md | cut -c1-200
echo ALL_DONE
