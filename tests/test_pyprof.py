"""pyprof pipeline on a synthetic rocprofv3 CSV trace (reference apex/pyprof has no unit tests;
its examples/ scripts exercise nvtx -> parse -> prof the same way).  The GPU test runs the real
rocprofv3 in tools/gpu_* scripts."""
import os

import torch

from apex.pyprof.nvtx.nvmarker import describe
from apex.pyprof.parse import parse
from apex.pyprof.prof import annotate, render


def _write(path, header, rows):
    with open(path, "w") as f:
        f.write(",".join(header) + "\n")
        for r in rows:
            f.write(",".join(str(x) for x in r) + "\n")


def test_parse_and_prof_from_csv(tmp_path):
    lin = str({"mod": "torch.nn.functional", "op": "linear",
               "args": [describe(torch.empty(64, 128, dtype=torch.bfloat16)),
                        describe(torch.empty(256, 128, dtype=torch.bfloat16))], "traceMarker": ["t.py:1"]})
    outer = str({"mod": "Linear", "op": "forward", "args": []})
    d = str(tmp_path)
    _write(os.path.join(d, "x_kernel_trace.csv"),
           ["Kind", "Agent_Id", "Queue_Id", "Kernel_Name", "Correlation_Id", "Start_Timestamp", "End_Timestamp",
            "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Workgroup_Size_X", "Workgroup_Size_Y", "Workgroup_Size_Z"],
           [["KERNEL_DISPATCH", 1, 0, "Cijk_gemm", 7, 1000, 1400, 256, 1, 1, 256, 1, 1],
            ["KERNEL_DISPATCH", 1, 0, "elementwise", 8, 2000, 2100, 64, 1, 1, 256, 1, 1]])
    _write(os.path.join(d, "x_hip_api_trace.csv"),
           ["Domain", "Function", "Process_Id", "Thread_Id", "Correlation_Id", "Start_Timestamp", "End_Timestamp"],
           [["HIP", "hipLaunchKernel", 1, 11, 7, 500, 510], ["HIP", "hipLaunchKernel", 1, 11, 8, 900, 910]])
    _write(os.path.join(d, "x_marker_api_trace.csv"),
           ["Domain", "Function", "Process_Id", "Thread_Id", "Correlation_Id", "Start_Timestamp", "End_Timestamp"],
           [["MARKER", '"{}"'.format(outer.replace('"', '""')), 1, 11, 0, 400, 600],
            ["MARKER", '"{}"'.format(lin.replace('"', '""')), 1, 11, 0, 450, 550]])
    recs = parse(d)
    assert [r["kName"] for r in recs] == ["Cijk_gemm", "elementwise"]
    assert recs[0]["op"] == "linear" and recs[1]["marker"] is None
    r = annotate(recs[0])
    assert r["flops"] == 2 * 64 * 256 * 128 and r["kDuration"] == 400
    txt = render([r], ["idx", "op", "kernel", "sil", "flops"], csv=True)
    assert "linear" in txt and str(2 * 64 * 256 * 128) in txt


def test_nvtx_init_is_transparent():
    """init() patches torch globally, so run it in a child interpreter."""
    import subprocess
    import sys

    code = ("import torch, apex.pyprof as p; p.init(); x = torch.randn(4, 8); l = torch.nn.Linear(8, 3); "
            "y = torch.nn.functional.relu(l(x)).sum(); y.backward(); assert l.weight.grad is not None; print('ok')")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=root, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
