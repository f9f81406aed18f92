"""SURVEY.md 5.2 (race detection / sanitizers), host side: the native launch planners
(csrc/include/apex_amd/launch_plan.h) built with AddressSanitizer + UBSan and swept over the
ResNet-50 / transformer shapes and adversarial edges (tools/host_checks.cpp).  GPU ASan / xnack+
runs are not available on the MI355X pool, so device-side fault finding is the APEX_AMD_SYNC_LAUNCH
debug mode instead (tests/test_debug_sync.py)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which(os.environ.get("CXX", "g++")) is None, reason="no host C++ compiler")
@pytest.mark.skipif(not os.path.isfile("/opt/rocm/include/hip/hip_runtime.h"), reason="no ROCm headers")
def test_launch_planners_under_asan_ubsan(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "host_sanitize.sh"), str(tmp_path / "host_checks")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout, r.stdout
