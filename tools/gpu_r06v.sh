#!/bin/bash
# 128-column default: 1x1 + node tests, bench, timeline; then the hipBLASLt tuning-cap probe
# (uncapped candidate timing at the shapes that crashed in round 4; a crash ends the script)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py tests/test_bottleneck_block.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
bash tools/gpu_r06e.sh r06v_tl > /dev/null || exit 1
for args in "3072 32768 1024 1 0" "1024 32768 4096 1 0" "4096 32768 1024 1 0" "200704 512 256 0 1" "65536 1024 1024 0 1"; do
  APEX_AMD_LT_TUNE_MAX_DIM=100000000 timeout -k 10 120 python tools/probe_lt.py $args >> $O/lt_probe.log 2>&1
  rc=$?; echo "rc=$rc args=$args" >> $O/lt_probe.log
  [ $rc -ne 0 ] && { echo "probe stopped rc=$rc at $args"; break; }
done
grep -E "^ok|^rc|Tensile" $O/lt_probe.log
