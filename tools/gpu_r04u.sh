#!/bin/bash
# ResNet step: eager vs hipGraph replay, kernel trace + idle-gap attribution, host cProfile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04u
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > $O/resnet_eager.log 2>&1 || { tail -5 $O/resnet_eager.log; exit 1; }
tail -1 $O/resnet_eager.log | cut -c1-160
timeout -k 10 400 python bench.py --graph > $O/resnet_graph.log 2>&1 || { tail -5 $O/resnet_graph.log; exit 1; }
tail -1 $O/resnet_graph.log | cut -c1-160
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/prof_resnet_r04u -o bench -- python3 $R/bench.py --steps 10 --warmup 8 \
    > $R/$O/prof_resnet.log 2>&1 ) || { tail -5 $O/prof_resnet.log; exit 1; }
db=$(find $R/gpurun_out/prof_resnet_r04u -name '*results.db' | head -1)
python3 tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 80 --md $O/resnet_prof.md > /dev/null || exit 1
python3 tools/prof_gaps.py "$db" --after spin_kernel --top 30 > $O/resnet_gaps.txt || exit 1
rm -rf $R/gpurun_out/prof_resnet_r04u
head -12 $O/resnet_prof.md
head -30 $O/resnet_gaps.txt
timeout -k 10 400 python -m cProfile -o $O/bench.pstats bench.py --steps 20 --warmup 8 > $O/cprof_run.log 2>&1 || { tail -5 $O/cprof_run.log; exit 1; }
python3 -c "
import pstats
p = pstats.Stats('$O/bench.pstats')
p.sort_stats('tottime').print_stats(45)
" > $O/cprof_tottime.txt 2>&1
python3 -c "
import pstats
p = pstats.Stats('$O/bench.pstats')
p.sort_stats('cumtime').print_stats(60)
" > $O/cprof_cumtime.txt 2>&1
head -60 $O/cprof_tottime.txt | tail -50
