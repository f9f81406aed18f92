#!/bin/bash
# Same-box A/B: this framework vs stock PyTorch-ROCm on the headline config, plus the
# transformer benches.  Each run under its own time limit; logs under gpurun_out/ab/.
mkdir -p gpurun_out/ab
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/gpurun_out/miopen_udb
export MIOPEN_CUSTOM_CACHE_DIR=$GRAFT_REPO_ROOT/gpurun_out/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
run() { name=$1; shift; timeout -k 10 ${T:-400} python bench.py "$@" > gpurun_out/ab/$name.log 2>&1; rc=$?; tail -1 gpurun_out/ab/$name.log | cut -c1-300; return $rc; }
run resnet50_apex --steps 30 --warmup 10 && \
run resnet50_torch --impl torch --steps 30 --warmup 10 && \
run resnet50_apex_again --steps 30 --warmup 10 && \
run gpt2_medium --model gpt2-medium --steps 10 --warmup 5 && \
run bert_large --model bert-large --steps 10 --warmup 5
echo AB_DONE rc=$?
