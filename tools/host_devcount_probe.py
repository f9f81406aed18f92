#!/usr/bin/env python3
"""Who calls hipGetDeviceCount in the ResNet-50 step (rocprofv3 --hip-trace: 186 calls per step)?
Wraps torch._C._cuda_getDeviceCount (the Python-reachable path, e.g. torch.cuda.is_available())
and prints the call count per step and the Python stacks of the distinct callers."""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

calls = collections.Counter()
orig = torch._C._cuda_getDeviceCount


def wrapped():
    st = traceback.extract_stack(limit=6)[:-1]
    calls["|".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in st[-4:])] += 1
    return orig()


torch._C._cuda_getDeviceCount = wrapped
sys.argv = [sys.argv[0], "--steps", "3", "--warmup", "3"]
import bench  # noqa: E402

calls.clear()
bench.main()
tot = sum(calls.values())
print(f"python-level _cuda_getDeviceCount calls over 6 steps: {tot}", flush=True)
for k, v in calls.most_common(10):
    print(v, k, flush=True)
