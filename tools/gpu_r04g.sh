#!/bin/bash
# transformer benches on the current tree (native GeLU pass, tuned hipBLASLt plans), BGRADB A/B,
# and a kernel-trace profile of the GPT-2 medium step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04g
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_fused_dense.py tests/test_dropout_rng.py tests/test_attention.py > gpurun_out/r04g/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04g/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 4 > gpurun_out/r04g/gpt2.log 2>&1 || { tail -5 gpurun_out/r04g/gpt2.log; exit 1; }
tail -1 gpurun_out/r04g/gpt2.log
APEX_AMD_LT_BGRADB=1 timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 4 > gpurun_out/r04g/gpt2_bgradb.log 2>&1 || { tail -5 gpurun_out/r04g/gpt2_bgradb.log; exit 1; }
tail -1 gpurun_out/r04g/gpt2_bgradb.log
timeout -k 10 400 python bench.py --model bert-large --steps 10 --warmup 4 > gpurun_out/r04g/bert.log 2>&1 || { tail -5 gpurun_out/r04g/bert.log; exit 1; }
tail -1 gpurun_out/r04g/bert.log
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_gpt2_r04 -o bench -- python3 $R/bench.py --model gpt2-medium --steps 5 --warmup 4 \
    > $R/gpurun_out/r04g/prof_gpt2.log 2>&1 ) || { tail -5 gpurun_out/r04g/prof_gpt2.log; exit 1; }
db=$(find $R/gpurun_out/prof_gpt2_r04 -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 5 --top 45 --md gpurun_out/r04g/gpt2_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_gpt2_r04
head -12 gpurun_out/r04g/gpt2_prof.md
