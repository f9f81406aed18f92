#!/bin/bash
# which torch copies remain in the ResNet step; counters of every native kernel of the step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05y
timeout -k 10 300 python -u tools/find_copies.py > gpurun_out/r05y/copies.txt 2>&1 || { tail -20 gpurun_out/r05y/copies.txt; exit 1; }
grep -v "^\[bench\]" gpurun_out/r05y/copies.txt | head -40
PMC_FILTER="apex_amd::|Cijk|igemm|elementwise" bash tools/gpu_pmc_cmd.sh resnet_r05y bench.py --steps 2 --warmup 2 || exit 1
