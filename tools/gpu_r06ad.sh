#!/bin/bash
# eager vs hipGraph-replayed step, same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ad; mkdir -p $O
for i in 1 2; do
  for arm in "" "--graph"; do
    timeout -k 10 400 python bench.py $arm > $O/b_${i}_${arm:-eager}.log 2>&1 || { tail -5 $O/b_${i}_${arm:-eager}.log; exit 1; }
    echo "$i ${arm:-eager} $(tail -1 $O/b_${i}_${arm:-eager}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('timing'))")" | tee -a $O/ab.txt
  done
done
