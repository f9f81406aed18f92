#!/bin/bash
# same-box A/B of the headline bench: alternating runs of `python bench.py` with env A / env B
# usage: tools/ab_bench.sh TAG "ENV_A" "ENV_B" [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; A=$2; B=$3; N=${4:-2}
O=gpurun_out/$TAG
mkdir -p $O
for i in $(seq 1 $N); do
  for arm in A B; do
    if [ $arm = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py > $O/bench_${arm}_$i.log 2>&1 || { tail -5 $O/bench_${arm}_$i.log; exit 1; }
    v=$(tail -1 $O/bench_${arm}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "$arm [$E] round $i: $v" | tee -a $O/ab.txt
  done
done
