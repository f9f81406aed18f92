#!/bin/bash
# stem weight gradient (loader / math waves): tests + stem bench; PMC of the conv3 backward and
# stem kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_stem.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stem_node_bench.py > $O/stem_bench.log 2>&1 || { tail -5 $O/stem_bench.log; exit 1; }
cat $O/stem_bench.log
bash tools/gpu_pmc_cmd.sh c3b_r04l tools/conv3_bwd_bench.py || exit 1
cat gpurun_out/pmc_c3b_r04l/pmc.md | cut -c1-400
bash tools/gpu_pmc_cmd.sh stem_r04l tools/stem_node_bench.py || exit 1
grep stem gpurun_out/pmc_stem_r04l/pmc.md | cut -c1-400
