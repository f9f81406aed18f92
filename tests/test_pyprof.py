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


def test_backward_markers_and_layers():
    """bprop ranges carry the forward op's description and seqId; layer() nests."""
    import json
    import subprocess
    import sys

    code = r'''
import json, torch
import apex.pyprof as p
from apex.pyprof.nvtx import nvmarker as nm
log = []
nm._push = lambda text: log.append(("push", text)) or None
nm._pop = lambda h: log.append(("pop", None))
p.init()
lin = torch.nn.Linear(8, 3)
x = torch.randn(4, 8, requires_grad=True)
with p.layer("block0"):
    y = torch.nn.functional.relu(lin(x)).sum()
y.backward()
import ast
out = []
for kind, text in log:
    if kind == "push":
        if text.startswith("layer:"):
            out.append(["layer", text])
        else:
            d = ast.literal_eval(text)
            out.append([d["op"], d["mod"], d["dir"], d["seqId"]])
print(json.dumps(out))
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=root, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    ev = json.loads(r.stdout.strip().splitlines()[-1])
    fwd = {(e[0], e[1]): e[3] for e in ev if len(e) == 4 and e[2] == "fprop"}
    bwd = {(e[0], e[1]): e[3] for e in ev if len(e) == 4 and e[2] == "bprop"}
    assert ["layer", "layer:block0"] in ev
    assert ("forward", "Linear") in fwd and ("relu", "torch.nn.functional") in fwd
    for key in (("forward", "Linear"), ("relu", "torch.nn.functional"), ("sum", "Tensor")):
        assert key in bwd and bwd[key] == fwd[key], (key, fwd, bwd)


def _rec(op, args, mod="torch.nn.functional", direction="fprop", kname="k", strrepr=""):
    return {"op": op, "mod": mod, "args": args, "dir": direction, "kName": kname, "strRepr": strrepr,
            "kDuration": 1000}


def test_op_models():
    from apex.pyprof.prof import model

    T = lambda *s, dt=torch.bfloat16: describe(torch.empty(*s, dtype=dt))  # noqa: E731
    # GEMM family: bprop = 2x forward, matrix-core detection from the kernel name
    m = model(_rec("addmm", [T(256), T(64, 128), T(128, 256)], mod="torch", kname="Cijk_Alik_Bljk_MT128x128"))
    assert m.flops() == 2 * 64 * 256 * 128 + 64 * 256 and m.tc() == 1
    mb = model(_rec("matmul", [T(8, 64, 128), T(128, 32)], mod="torch", direction="bprop", kname="elementwise"))
    assert mb.flops() == 4 * 8 * 64 * 32 * 128 and mb.tc() == 0
    assert model(_rec("einsum", [describe("bik,bkj->bij"), T(2, 3, 4), T(2, 4, 5)], mod="torch")).flops() == \
        2 * 2 * 3 * 4 * 5
    lin = model(_rec("forward", [T(32, 10, 64)], mod="Linear", strrepr="in_features=64, out_features=16, bias=True"))
    assert lin.flops() == 2 * 320 * 16 * 64 + 320 * 16
    # conv: functional args and module repr agree (stride 2, pad 3, 7x7)
    x, w = T(2, 3, 224, 224), T(64, 3, 7, 7)
    f = model(_rec("conv2d", [x, w, describe(None), describe((2, 2)), describe((3, 3))]))
    mm = model(_rec("forward", [x], mod="Conv2d",
                    strrepr="3, 64, kernel_size=(7, 7), stride=(2, 2), padding=(3, 3), bias=False"))
    assert f.out == (112, 112) and mm.out == (112, 112)
    assert f.flops() == mm.flops() == 2 * 2 * 64 * 112 * 112 * 3 * 49
    # transposed conv output extent
    t = model(_rec("conv_transpose2d", [T(1, 8, 16, 16), T(8, 4, 4, 4), describe(None), describe(2), describe(1)]))
    assert t.out == (32, 32)
    # pooling / reduction / pointwise / views
    p = model(_rec("max_pool2d", [T(2, 64, 112, 112), describe(3), describe(2), describe(1)]))
    assert p.out == (56, 56)
    r = model(_rec("sum", [T(4, 5, 6), describe(1, "dim")], mod="Tensor"))
    assert r.out == (4, 6) and r.bytes() == (120 + 24) * 2
    a = model(_rec("add", [T(4, 1, 6), T(5, 1)], mod="torch"))
    assert a.flops() == 4 * 5 * 6 and a.bytes() == (24 + 5 + 120) * 2
    g = model(_rec("gelu", [T(10, 10)]))
    assert g.flops() == 9 * 100
    assert model(_rec("view", [T(10, 10), describe(100)], mod="Tensor")).bytes() == 0
    assert model(_rec("cat", [describe([torch.empty(3, 4), torch.empty(5, 4)])], mod="torch")).bytes() == \
        2 * 32 * 4
    c = model(_rec("to", [T(10, 10, dt=torch.float32), describe(torch.bfloat16)], mod="Tensor"))
    assert c.bytes() == 100 * (4 + 2)
    # multi-tensor optimizer step (lists: g, p, m, v, model copy)
    lists = describe([[torch.empty(1000, dtype=torch.bfloat16)], [torch.empty(1000)], [torch.empty(1000)],
                      [torch.empty(1000)], [torch.empty(1000, dtype=torch.bfloat16)]])
    o = model(_rec("multi_tensor_adam_capturable", [describe(65536), describe(torch.zeros(1)), lists],
                   mod="apex.amp_C"))
    assert o.bytes() == 1000 * (2 + 2 * 4 * 3 + 2)
    # normalization bprop reads x, dy and writes dx
    n = model(_rec("layer_norm", [T(8, 1024), describe((1024,)), T(1024, dt=torch.float32)], direction="bprop"))
    assert n.bytes() == 3 * 8 * 1024 * 2 + 2 * 4096


def test_prof_cli_summary(tmp_path, capsys):
    from apex.pyprof.prof import main

    recs = [_rec("linear", [describe(torch.empty(64, 128)), describe(torch.empty(256, 128))], kname="Cijk_x"),
            dict(_rec("relu", [describe(torch.empty(64, 256))]), dir="bprop")]
    f = tmp_path / "parsed.txt"
    f.write_text("\n".join(str(r) for r in recs))
    main([str(f), "-c", "idx,dir,op,tc,flops,bytes,params"])
    out = capsys.readouterr().out
    assert "linear" in out and "M=64" in out and "bprop" in out
    main([str(f), "--summary", "op"])
    out = capsys.readouterr().out
    assert "relu" in out and "TFLOP/s" in out
