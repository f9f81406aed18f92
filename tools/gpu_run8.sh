#!/bin/bash
# GPU session: hardware counters of the native kernels, then a 2-rank (gloo, shared GPU)
# rehearsal of the multi-GPU bench paths (DDP + amp O2 + fused BN; DDP transformer).
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
bash tools/gpu_pmc.sh || stop pmc $?
cd $R
APEX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --batch-size 32 > gpurun_out/bench_gloo2.log 2>&1
rc=$?; grep -v "^\[bench\]" gpurun_out/bench_gloo2.log | tail -3; [ $rc -ne 0 ] && stop gloo2 $rc
APEX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --model bert-large --steps 2 --warmup 1 --batch-size 4 > gpurun_out/bench_gloo2_bert.log 2>&1
rc=$?; tail -2 gpurun_out/bench_gloo2_bert.log; [ $rc -ne 0 ] && stop gloo2_bert $rc
echo ALL_DONE
