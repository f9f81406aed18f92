#!/bin/bash
# counters: memory-bound kernels (multi-tensor engine after the work-item split, LayerNorm) and
# every native kernel of the ResNet-50 step
set -o pipefail
cd $GRAFT_REPO_ROOT
PMC_FILTER="apex_amd::|at::native::vectorized_elementwise_kernel<4, at::native::AUnaryFunctor" \
  bash tools/gpu_pmc_cmd.sh membound_r05ak tools/pmc_membound.py || exit 1
PMC_FILTER="apex_amd::" bash tools/gpu_pmc_cmd.sh resnet_r05ak bench.py --steps 2 --warmup 2 || exit 1
head -30 gpurun_out/pmc_membound_r05ak/pmc.md | cut -c1-200
