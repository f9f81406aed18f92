#!/bin/bash
# per-step HIP API counts: the same bench at 3 and 13 timed steps, difference / 10
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aj; mkdir -p $O
for n in 3 13; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --hip-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps $n --warmup 3 > $GRAFT_REPO_ROOT/$O/log$n 2>&1 ) || exit 1
  f=$(find $O/tr$n -name "*hip_api_stats.csv" | head -1); cp $f $O/api_stats_$n.csv; rm -rf $O/tr$n
done
python3 - <<'PY'
import csv
def load(n):
    return {r["Name"]: (int(r["Calls"]), int(r["TotalDurationNs"])) for r in csv.DictReader(open(f"gpurun_out/r06aj/api_stats_{n}.csv"))}
a, b = load(3), load(13)
for k in b:
    dc = b[k][0] - a.get(k, (0, 0))[0]
    dt = b[k][1] - a.get(k, (0, 0))[1]
    if dc: print(f"{k:40s} {dc/10:8.1f} calls/step {dt/10/1e3:9.1f} us/step")
PY
