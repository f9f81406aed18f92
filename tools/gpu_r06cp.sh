#!/bin/bash
# kernel + memory-copy trace of the timed ResNet steps: which host->device / device copies sit in
# the step's idle gaps (the 80 us at the step start, 143 us at the forward -> backward turn)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06cp; mkdir -p $O
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace \
    --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 4 --warmup 8 > $R/$O/prof.log 2>&1 ) || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name '*.csv' | head
