#!/bin/bash
# register / scratch census of the transformer benches (GPT-2 medium, BERT-large)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06w; mkdir -p $O
for m in gpt2-medium bert-large; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model $m --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/$O/log_$m 2>&1 ) || { tail -3 $O/log_$m; exit 1; }
  python3 tools/scratch_census.py $(find $O/tr_$m -name "*kernel_trace.csv") --all > $O/census_$m.md; rm -rf $O/tr_$m
  echo "== $m"; awk -F'|' 'NR<=2 || $3+0>0' $O/census_$m.md
done
