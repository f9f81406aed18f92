#!/bin/bash
# A/B of the multi-tensor engine variants (tools/mta_bench.py), one process per variant.
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/mta_bench.py > gpurun_out/mta_ab.jsonl 2>&1 || exit $?
for v in ${MTA_VARIANTS:-red4}; do
  APEX_AMD_NATIVE_SO=$R/rocm-apex_amd/_variants/_C_$v.so timeout -k 10 120 python tools/mta_bench.py >> gpurun_out/mta_ab.jsonl 2>&1 || exit $?
done
cat gpurun_out/mta_ab.jsonl
