#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_attention.py tests/test_standalone_models.py tests/test_transformer_cpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_t.log; [ $rc -ne 0 ] && stop pytest $rc
timeout -k 10 400 python -u bench.py --model gpt2-medium --steps 10 --warmup 4 > gpurun_out/bench_gpt.log 2>&1
rc=$?; tail -1 gpurun_out/bench_gpt.log | cut -c1-250; [ $rc -ne 0 ] && stop bench_gpt $rc
timeout -k 10 400 python -u bench.py --model bert-large --steps 10 --warmup 4 > gpurun_out/bench_bert.log 2>&1
rc=$?; tail -1 gpurun_out/bench_bert.log | cut -c1-250; [ $rc -ne 0 ] && stop bench_bert $rc
(cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_gpt -o gpt -- python3 $R/bench.py --model gpt2-medium --steps 5 --warmup 3 > $R/gpurun_out/prof_gpt.log 2>&1)
rc=$?; [ $rc -ne 0 ] && stop prof_gpt $rc
python tools/prof_summary.py /tmp/prof_gpt/gpt_results.db --after spin_kernel --top 40 --md gpurun_out/gpt2_steady.md > /dev/null 2>&1
head -36 gpurun_out/gpt2_steady.md | cut -c1-170
echo ALL_DONE
