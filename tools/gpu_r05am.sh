#!/bin/bash
# final-tree 2-rank rehearsal of the distributed bench path (gloo, both ranks on the one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05am
mkdir -p $O
APEX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 > $O/gloo2.log 2>&1 || { tail -20 $O/gloo2.log; exit 1; }
grep '"metric"' $O/gloo2.log | cut -c1-400
