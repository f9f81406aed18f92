#!/bin/bash
# column-sum pass with 4 rows in flight: tests, GPT-2 trace rows, GPT-2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ay; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_dense.py -m gpu > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/gpu_r06ax.sh > /dev/null || exit 1
grep -E "colsum|busy" gpurun_out/r06ax/gpt2_prof.md | cut -c1-170
timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2.log 2>&1 || { tail -5 $O/gpt2.log; exit 1; }
tail -1 $O/gpt2.log | cut -c1-170
