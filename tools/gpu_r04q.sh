#!/bin/bash
# stem weight-gradient ablation (compile-time modes: 1 no gather, 2 no MFMA, 4 no im2col loads)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04q
mkdir -p $O
for md in 0 1 2 4 7; do
  APEX_AMD_STEM_WG_MODE=$md timeout -k 10 120 python tools/stem_wgrad_probe.py >> $O/wg_modes.log 2>&1 || { tail -5 $O/wg_modes.log; exit 1; }
done
grep kernel $O/wg_modes.log
bash tools/gpu_pmc_cmd.sh stemwg_r04q tools/stem_wgrad_probe.py || exit 1
grep -i "stem::wgrad" gpurun_out/pmc_stemwg_r04q/pmc.md | cut -c1-500
