"""Debug launch mode (serialised launches to localise asynchronous faults).

``APEX_AMD_SYNC_LAUNCH=1`` makes every native op synchronize the device after its launches and
raise with the op's name if anything failed (csrc/include/apex_amd/dispatch.h).  The GPU test runs
a few native ops in a child process with the mode on and checks that the results match the
default (asynchronous) mode bit for bit."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
import apex
from apex.normalization import FusedLayerNorm
from apex.contrib.groupbn import BatchNorm2d_NHWC
assert apex._native.available()
torch.manual_seed(0)
ln = FusedLayerNorm(1024).cuda()
x = torch.randn(64, 1024, device="cuda", requires_grad=True)
y = ln(x)
y.sum().backward()
bn = BatchNorm2d_NHWC(64, fuse_relu=True, torch_channels_last=True).cuda()
a = torch.randn(8, 64, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
b = bn(a)
torch.save({"y": y.detach().cpu(), "gx": x.grad.cpu(), "b": b.float().cpu()}, sys.argv[2])
"""


def _run(tmp_path, name, sync):
    env = dict(os.environ)
    env.pop("APEX_AMD_SYNC_LAUNCH", None)
    if sync:
        env["APEX_AMD_SYNC_LAUNCH"] = "1"
    out = str(tmp_path / name)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, out], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    import torch

    return torch.load(out, weights_only=True)


@pytest.mark.gpu
def test_gpu_sync_launch_mode_matches_async(tmp_path):
    import torch

    a = _run(tmp_path, "async.pt", False)
    b = _run(tmp_path, "sync.pt", True)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_sync_launch_flag_documented():
    """The switch lives in the header every native TU includes (CPU-checkable)."""
    src = open(os.path.join(ROOT, "rocm-apex_amd", "csrc", "include", "apex_amd", "dispatch.h")).read()
    assert "APEX_AMD_SYNC_LAUNCH" in src and "hipDeviceSynchronize" in src
