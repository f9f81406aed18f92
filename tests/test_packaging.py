"""Install / build-selection checks (reference setup.py:87-555 per-extension switches)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import build_native  # noqa: E402


def test_apex_is_a_real_package():
    import apex

    assert os.path.realpath(os.path.dirname(apex.__file__)) == os.path.join(ROOT, "rocm-apex_amd")
    assert apex.__name__ == "apex" and apex.amp.__name__ == "apex.amp"


def test_extension_selection_picks_sources():
    hip, cpp = build_native.sources("norm")
    names = {os.path.relpath(p, build_native.CSRC).split(os.sep)[0] for p in hip}
    assert names == {"mta", "norm"}
    binds = {os.path.basename(p) for p in cpp}
    assert "norm.cpp" in binds and "amp_C.cpp" in binds and "module.cpp" in binds
    assert "gemm.cpp" not in binds and "attn.cpp" not in binds
    hip_all, cpp_all = build_native.sources("all")
    assert len(hip_all) > len(hip) and len(cpp_all) > len(cpp)
    with pytest.raises(RuntimeError):
        build_native.selected_extensions("norm,warp_specialized_nonsense")


def test_setup_maps_reference_flags():
    out = subprocess.run([sys.executable, "-c",
                          "import sys; sys.argv=['setup.py','--fast_layer_norm','--xentropy','--name'];"
                          "import runpy; g=runpy.run_path('setup.py', run_name='not_main');"
                          "print(g['EXTENSIONS'])"],
                         cwd=ROOT, capture_output=True, text=True, timeout=120,
                         env={**os.environ, "APEX_AMD_SKIP_NATIVE": "1"})
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "norm,xentropy"
