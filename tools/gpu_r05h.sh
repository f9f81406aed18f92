#!/bin/bash
# fresh ResNet-50 node profile + counter passes: stem weight gradient, attention, memory-bound kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r05b.sh r05h || exit 1
PMC_FILTER="apex_amd::stem" bash tools/gpu_pmc_cmd.sh stem_r05 tools/stem_wgrad_probe.py || exit 1
PMC_FILTER="apex_amd::" bash tools/gpu_pmc_cmd.sh attn_r05 tools/pmc_attn.py || exit 1
PMC_FILTER="apex_amd::|at::native::vectorized_elementwise_kernel<4, at::native::AUnaryFunctor" \
  bash tools/gpu_pmc_cmd.sh membound_r05 tools/pmc_membound.py || exit 1
ls gpurun_out/pmc_stem_r05 gpurun_out/pmc_attn_r05 gpurun_out/pmc_membound_r05
