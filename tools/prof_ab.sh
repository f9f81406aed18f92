#!/bin/bash
# Kernel-trace A/B of two bench.py configurations on one box (rocprofv3 --kernel-trace --stats,
# 10 timed steps after the APEX_BENCH_MARK spin), summarized per kernel by tools/prof_summary.py.
# Usage (on the GPU box): tools/prof_ab.sh NAME_A "ENV_A" NAME_B "ENV_B" [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
A=$1; EA=$2; B=$3; EB=$4; shift 4
mkdir -p $R/gpurun_out
for arm in "$A|$EA" "$B|$EB"; do
  name=${arm%%|*}; envs=${arm#*|}
  ( cd /tmp && export TMPDIR=/tmp APEX_BENCH_MARK=1 $envs && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      -d $R/gpurun_out/prof_$name -o bench -- python3 $R/bench.py --steps 10 --warmup 6 "$@" \
      > $R/gpurun_out/prof_$name.log 2>&1 ) || { echo "arm $name failed"; tail -5 $R/gpurun_out/prof_$name.log; exit 1; }
  db=$(find $R/gpurun_out/prof_$name -name '*results.db' | head -1)
  python3 $R/tools/prof_summary.py "$db" --after spin_kernel --top 45 --md $R/gpurun_out/prof_$name.md > /dev/null || exit 1
  python3 $R/tools/prof_gaps.py "$db" --after spin_kernel > $R/gpurun_out/prof_${name}_gaps.md || exit 1
  rm -rf $R/gpurun_out/prof_$name
  head -14 $R/gpurun_out/prof_$name.md
done
