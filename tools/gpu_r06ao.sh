#!/bin/bash
# vectorized / hoisted additive-bias loads in the attention kernels: tests, counters, BERT A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ao; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention.py tests/test_standalone_models.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_pmc_cmd.sh attn_r06b tools/pmc_attn.py > /dev/null || exit 1
grep -E "fwd_kernel|dkdv|dq_kernel" gpurun_out/pmc_attn_r06b/pmc.md | cut -d"|" -f2-4
timeout -k 10 400 python bench.py --model bert-large > $O/bert_large.log 2>&1 || { tail -5 $O/bert_large.log; exit 1; }
tail -1 $O/bert_large.log | cut -c1-160
