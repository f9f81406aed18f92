#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aq; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_pmc_cmd.sh attn_r06d tools/pmc_attn.py > /dev/null || exit 1
grep -E "fwd_kernel|dkdv|dq_kernel" gpurun_out/pmc_attn_r06d/pmc.md | grep "64, [12]" | cut -d"|" -f2-4
