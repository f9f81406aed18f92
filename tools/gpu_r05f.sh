#!/bin/bash
# stem wgrad with the gather two steps ahead; wide LayerNorm backward re-route; hipBLASLt timed plans
# for the library 1x1 GEMMs (A/B); 2-rank gloo rehearsal of the distributed bench (comm timing)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem.py > $O/stem_tests.log 2>&1
rc=$?; tail -3 $O/stem_tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
for m in 0 1 2 4 7; do
  APEX_AMD_STEM_WG_MODE=$m timeout -k 10 120 python -u tools/stem_wgrad_probe.py >> $O/stem_probe.jsonl 2>&1 || { tail -5 $O/stem_probe.jsonl; exit 1; }
done
cat $O/stem_probe.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm.py > $O/norm.log 2>&1
rc=$?; tail -3 $O/norm.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/ln_wide_bench.py > $O/ln_wide.jsonl 2>&1 || { tail -5 $O/ln_wide.jsonl; exit 1; }
cat $O/ln_wide.jsonl
APEX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 2 --batch-size 64 \
  --comm-steps 3 > $O/gloo2.log 2>&1; tail -1 $O/gloo2.log | cut -c1-1500
APEX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 4 --warmup 2 --batch-size 64 \
  --comm-steps 3 --sync-bn > $O/gloo2_syncbn.log 2>&1; tail -1 $O/gloo2_syncbn.log | cut -c1-1500
bash tools/ab_bench.sh r05f_lt "APEX_AMD_RN_LT=0" "APEX_AMD_RN_LT=1" 2
