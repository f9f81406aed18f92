#!/bin/bash
# GPT-2 medium step: repeat bench + 10-step kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ad
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_b.log 2>&1 || exit 1
tail -1 $O/gpt2_b.log | cut -c1-160
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_gpt2_r05ad -o bench -- python3 $R/bench.py --model gpt2-medium --steps 10 --warmup 8 \
    > $R/$O/prof.log 2>&1 ) || { tail -5 $O/prof.log; exit 1; }
db=$(find $R/gpurun_out/prof_gpt2_r05ad -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 60 --md $O/gpt2_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_gpt2_r05ad
head -40 $O/gpt2_prof.md | cut -c1-200
