#!/bin/bash
# refresh: ResNet step kernel trace, GPT-2 / BERT benches and GPT-2 kernel trace on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04z
mkdir -p $O
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_resnet_r04z -o bench -- python3 $R/bench.py --steps 10 --warmup 8 \
    > $R/$O/prof_resnet.log 2>&1 ) || { tail -5 $O/prof_resnet.log; exit 1; }
db=$(find $R/gpurun_out/prof_resnet_r04z -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 90 --md $O/resnet_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_resnet_r04z
head -12 $O/resnet_prof.md
timeout -k 10 500 python bench.py --model gpt2-medium > $O/gpt2.log 2>&1 || { tail -5 $O/gpt2.log; exit 1; }
tail -1 $O/gpt2.log | cut -c1-160
timeout -k 10 500 python bench.py --model bert-large > $O/bert.log 2>&1 || { tail -5 $O/bert.log; exit 1; }
tail -1 $O/bert.log | cut -c1-160
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_gpt2_r04z -o bench -- python3 $R/bench.py --model gpt2-medium --steps 5 --warmup 4 \
    > $R/$O/prof_gpt2.log 2>&1 ) || { tail -5 $O/prof_gpt2.log; exit 1; }
db=$(find $R/gpurun_out/prof_gpt2_r04z -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 5 --top 60 --md $O/gpt2_prof.md > /dev/null || exit 1
rm -rf $R/gpurun_out/prof_gpt2_r04z
head -30 $O/gpt2_prof.md | cut -c1-170
