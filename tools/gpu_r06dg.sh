#!/bin/bash
# round 6: native dgrad + dGeLU + bias-grad epilogue — GPU tests, route micro-bench, GPT-2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06dg
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_dense.py -m gpu \
  > $O/test_fd.txt 2>&1 || { tail -30 $O/test_fd.txt; exit 1; }
tail -2 $O/test_fd.txt
timeout -k 10 300 python tools/gelu_route_bench.py > $O/gelu_routes.jsonl 2>&1 || { tail -20 $O/gelu_routes.jsonl; exit 1; }
grep bwd_ $O/gelu_routes.jsonl
for i in 1 2; do
  for arm in A B; do
    if [ $arm = A ]; then E="APEX_AB_NOP=1"; else E="APEX_AMD_DGELU_ROUTE=pass"; fi
    env $E timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_${arm}_$i.log 2>&1 || { tail -5 $O/gpt2_${arm}_$i.log; exit 1; }
    v=$(tail -1 $O/gpt2_${arm}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "$arm [$E] round $i: $v" | tee -a $O/ab.txt
  done
done
