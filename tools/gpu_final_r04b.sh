#!/bin/bash
# smoke (the stem node counted), driver-exact ResNet bench, GPT-2 / BERT benches
cd $GRAFT_REPO_ROOT
O=gpurun_out/final_r04
mkdir -p $O
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log | cut -c1-250; [ $rc -ne 0 ] && stop smoke $rc
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log | cut -c1-300; [ $rc -ne 0 ] && stop bench $rc
timeout -k 10 500 python bench.py --model gpt2-medium > $O/gpt2.log 2>&1
rc=$?; tail -1 $O/gpt2.log | cut -c1-200; [ $rc -ne 0 ] && stop gpt2 $rc
timeout -k 10 500 python bench.py --model bert-large > $O/bert.log 2>&1
rc=$?; tail -1 $O/bert.log | cut -c1-200; [ $rc -ne 0 ] && stop bert $rc
echo ALL_DONE
