#!/bin/bash
# same-box A/B/C... of the headline bench: alternating `python bench.py` runs, one env per arm
# usage: tools/ab_multi.sh TAG ROUNDS "ENV_A" "ENV_B" ["ENV_C" ...]   (an arm "-" = no extra env)
# BENCH_ARGS="--model bert-large" selects another bench.py config
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; N=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
for i in $(seq 1 $N); do
  k=0
  for E in "$@"; do
    k=$((k + 1))
    [ "$E" = "-" ] && E="APEX_AB_NOP=1"
    env $E timeout -k 10 300 python bench.py $BENCH_ARGS > $O/bench_${k}_$i.log 2>&1 || { tail -5 $O/bench_${k}_$i.log; exit 1; }
    v=$(tail -1 $O/bench_${k}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "arm$k [$E] round $i: $v" | tee -a $O/ab.txt
  done
done
