#!/bin/bash
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 60 python tools/probe_lt.py "$@" 2>&1 | grep -E "^ok|Tensile|Segmentation" | head -2; }
run 200704 512 256 0 1
for tok in 16384 32768 65536; do run 3072 $tok 1024 1 0; run 1024 $tok 4096 1 0; done
set -o pipefail
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_fused_dense.py > gpurun_out/r04ac_tests.log 2>&1 || { tail -20 gpurun_out/r04ac_tests.log; exit 1; }
tail -1 gpurun_out/r04ac_tests.log
