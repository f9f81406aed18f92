#!/bin/bash
# step-boundary idle investigation: eager vs hipGraph replay (same box), then a HIP API + kernel
# trace of a few eager steps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/r04b/eager.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 8 --graph > gpurun_out/r04b/graph.log 2>&1 || exit 1
tail -1 gpurun_out/r04b/eager.log; tail -1 gpurun_out/r04b/graph.log
cd /tmp
APEX_BENCH_MARK=1 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04b/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 8 > $GRAFT_REPO_ROOT/gpurun_out/r04b/trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
ls -la gpurun_out/r04b/trace/*/ 2>/dev/null | head; du -sh gpurun_out/r04b
