#!/bin/bash
# Real rocprofv3 trace through the pyprof pipeline (markers -> parse -> prof).
set -e
R=$GRAFT_REPO_ROOT
cd /tmp
cat > /tmp/pyprof_demo.py <<'PY'
import sys; sys.path.insert(0, sys.argv[1])
import torch, apex.pyprof as p
p.init()
x = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16)
lin = torch.nn.Linear(1024, 4096).cuda().bfloat16()
for _ in range(3):
    y = torch.nn.functional.gelu(lin(x))
    z = torch.nn.functional.layer_norm(y, (4096,))
torch.cuda.synchronize()
print("demo ok")
PY
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --hip-trace --output-format csv -d $R/gpurun_out/pyprof_trace -o run -- python3 /tmp/pyprof_demo.py $R > $R/gpurun_out/pyprof_rocprof.log 2>&1
cd $R
find gpurun_out/pyprof_trace -name "*.csv" | head -20
python -m apex.pyprof.parse gpurun_out/pyprof_trace > gpurun_out/pyprof_parsed.txt
python -m apex.pyprof.prof gpurun_out/pyprof_parsed.txt > gpurun_out/pyprof_report.txt
head -20 gpurun_out/pyprof_report.txt
