#!/bin/bash
# GPT-2 medium steady-state per-kernel table of the final tree (10 timed steps after the mark)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ax; mkdir -p $O
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 500 rocprofv3 --kernel-trace \
    -d $R/gpurun_out/prof_gpt2 -o bench -- python3 $R/bench.py --model gpt2-medium --steps 10 --warmup 6 \
    > $R/$O/prof.log 2>&1 ) || { tail -5 $O/prof.log; exit 1; }
db=$(find $R/gpurun_out/prof_gpt2 -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 60 --md $O/gpt2_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_gpt2
head -14 $O/gpt2_prof.md
grep -E "gelu|colsum" $O/gpt2_prof.md | cut -c1-160
