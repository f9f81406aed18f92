#!/usr/bin/env python3
"""Probe: lt_gemm.mm over a shape list in a fresh process per call of this script (a hipBLASLt
candidate that faults takes the process down, so each arm runs separately).
Usage: python tools/probe_lt.py <m> <k> <n> <trans_a> <trans_b>"""
import faulthandler
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import apex  # noqa: E402,F401
from apex import _native  # noqa: E402

lt = _native.require("lt_gemm").lt_gemm
m, k, n, ta, tb = (int(v) for v in sys.argv[1:6])
dt = torch.bfloat16
a = torch.randn((k, m) if ta else (m, k), device="cuda", dtype=dt)
b = torch.randn((n, k) if tb else (k, n), device="cuda", dtype=dt)
r = lt.mm(a, b, bool(ta), bool(tb))
torch.cuda.synchronize()
print("ok", m, k, n, ta, tb, bool(r), os.environ.get("APEX_AMD_LT_TUNE"), flush=True)
