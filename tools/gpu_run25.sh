#!/bin/bash
# MIOpen find mode experiment: NORMAL (full find over all applicable solvers) vs default
mkdir -p gpurun_out
stop() { echo "STOP: $1 rc=$2"; exit $2; }
s=$(date +%s)
MIOPEN_FIND_MODE=NORMAL timeout -k 10 900 python -u bench.py --steps 20 --warmup 8 > gpurun_out/bench_findnormal.log 2>&1
rc=$?; e=$(date +%s); echo "wall=$((e-s))s"; tail -1 gpurun_out/bench_findnormal.log | cut -c1-200; [ $rc -ne 0 ] && stop bench $rc
s=$(date +%s)
MIOPEN_FIND_MODE=NORMAL timeout -k 10 900 python -u bench.py --steps 20 --warmup 8 > gpurun_out/bench_findnormal2.log 2>&1
rc=$?; e=$(date +%s); echo "wall2=$((e-s))s"; tail -1 gpurun_out/bench_findnormal2.log | cut -c1-200; [ $rc -ne 0 ] && stop bench2 $rc
echo ALL_DONE
