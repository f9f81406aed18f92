#!/bin/bash
# MHA fast path on the packed-QKV kernels: attention GPU tests, the published-config perf test
# (host enqueue cost + hipGraph replay rows); GPT-2 medium A/B of the hipBLASLt plan tuning
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_attention.py > $O/attn_tests.log 2>&1
rc=$?; tail -2 $O/attn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/perf_test_multihead_attn.py --graph --out $O/mha_published_config.jsonl > $O/mha.log 2>&1 || { tail -5 $O/mha.log; exit 1; }
cat $O/mha.log
for i in 1 2; do
  timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 4 > $O/gpt2_tune_$i.log 2>&1 || { tail -5 $O/gpt2_tune_$i.log; exit 1; }
  tail -1 $O/gpt2_tune_$i.log | cut -c1-200
  APEX_AMD_LT_TUNE=0 timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 4 > $O/gpt2_notune_$i.log 2>&1 || { tail -5 $O/gpt2_notune_$i.log; exit 1; }
  tail -1 $O/gpt2_notune_$i.log | cut -c1-200
done
timeout -k 10 400 python bench.py --model bert-large --steps 10 --warmup 4 > $O/bert.log 2>&1 || { tail -5 $O/bert.log; exit 1; }
tail -1 $O/bert.log | cut -c1-200
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_gpt2_r04j -o bench -- python3 $R/bench.py --model gpt2-medium --steps 5 --warmup 4 \
    > $R/$O/prof_gpt2.log 2>&1 ) || { tail -5 $O/prof_gpt2.log; exit 1; }
db=$(find $R/gpurun_out/prof_gpt2_r04j -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 5 --top 45 --md $O/gpt2_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_gpt2_r04j
head -14 $O/gpt2_prof.md
