#!/bin/bash
# which lt_gemm.mm problems fault inside hipBLASLt: tuned (top-8) vs heuristic-only, per shape
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 60 python tools/probe_lt.py "$@" 2>&1 | grep -E "^ok|Tensile|Segmentation" | head -2; echo "rc=$? args=$*"; }
APEX_AMD_LT_TUNE=0 run 200704 512 256 0 1
run 4096 512 256 0 1
# transformer wgrad problems (g^T x: m = out features, k = tokens, n = in features)
for tok in 4096 8192 16384 32768; do
  run 3072 $tok 1024 1 0
  run 1024 $tok 4096 1 0
  run 4096 $tok 1024 1 0
done
