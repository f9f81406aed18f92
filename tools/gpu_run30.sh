#!/bin/bash
# stem padding A/B in one box
mkdir -p gpurun_out
stop() { echo "STOP: $1 rc=$2"; exit $2; }
for f in 0 1 0 1; do
  APEX_AMD_STEM_PAD=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 > gpurun_out/bench_stem$f.log 2>&1
  rc=$?; echo "stem_pad=$f $(tail -1 gpurun_out/bench_stem$f.log | cut -c60-120)"; [ $rc -ne 0 ] && stop bench $rc
done
echo ALL_DONE
