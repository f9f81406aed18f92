#!/bin/bash
# full GPU tier + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu_all.log 2>&1
rc=$?; tail -8 $O/gpu_all.log | cut -c1-300; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1; tail -2 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_eager_$i.log 2>&1 && tail -1 $O/bench_eager_$i.log | cut -c60-140
  timeout -k 10 300 python bench.py --graph > $O/bench_graph_$i.log 2>&1 && tail -1 $O/bench_graph_$i.log | cut -c60-140
done
