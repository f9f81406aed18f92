"""Installable build of the framework: ``pip install --no-build-isolation .``

The importable package is ``apex`` (sources in ``rocm-apex_amd/``), plus the top-level
``amp_C`` / ``apex_C`` module names.  The native extension ``apex._C`` is compiled for gfx950 by
``tools/build_native.py`` (direct hipcc, no hipify) during ``build_py`` and shipped inside the
package.

Extension selection mirrors the reference's per-extension switches
(/root/reference/setup.py:87-555): ``APEX_AMD_EXTENSIONS=norm,gemm pip install .`` or the
reference flag names through ``--global-option`` / ``--config-settings``-free env
``APEX_AMD_SETUP_FLAGS="--fast_layer_norm --xentropy"``.  With no selection every subsystem is
built.  ``APEX_AMD_SKIP_NATIVE=1`` installs the Python package only (CPU reference ops; GPU ops
then raise)."""
import os
import sys

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))
SRC = "rocm-apex_amd"

# reference setup.py flag -> native subsystems (tools/build_native.py EXTENSIONS)
REFERENCE_FLAGS = {
    "--cpp_ext": [], "--cuda_ext": "all", "--distributed_adam": [], "--distributed_lamb": [],
    "--fast_layer_norm": ["norm"], "--xentropy": ["xentropy"], "--fast_multihead_attn": ["attn"],
    "--fmha": ["attn"], "--bnp": ["bn_nhwc"], "--fast_bottleneck": ["bn_nhwc", "conv"],
    "--peer_memory": ["contrib"], "--nccl_p2p": ["contrib"], "--transducer": ["contrib"],
    "--deprecated_fused_adam": [], "--deprecated_fused_lamb": [], "--focal_loss": ["xentropy"],
    "--index_mul_2d": [], "--fused_conv_bias_relu": ["conv"], "--cudnn_gbn": ["bn_nhwc"],
}


def _selection():
    if os.environ.get("APEX_AMD_EXTENSIONS"):
        return os.environ["APEX_AMD_EXTENSIONS"]
    flags = os.environ.get("APEX_AMD_SETUP_FLAGS", "").split()
    flags += [a for a in sys.argv if a in REFERENCE_FLAGS]
    for a in [a for a in sys.argv if a in REFERENCE_FLAGS]:
        sys.argv.remove(a)
    chosen = set()
    for f in flags:
        v = REFERENCE_FLAGS.get(f, [])
        if v == "all":
            return "all"
        chosen.update(v)
    return ",".join(sorted(chosen)) if chosen else "all"


EXTENSIONS = _selection()


class BuildWithNative(build_py):
    def run(self):
        if os.environ.get("APEX_AMD_SKIP_NATIVE", "0") != "1":
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import build_native

            build_native.build(extensions=EXTENSIONS)
        super().run()


packages = ["apex"] + ["apex." + p for p in find_packages(SRC)]
setup(
    name="apex-mi355x",
    version="0.2.0",
    description="MI355X-native (gfx950) mixed precision and distributed training utilities with the Apex API",
    package_dir={"apex": SRC},
    packages=packages,
    py_modules=["amp_C", "apex_C"],
    package_data={"apex": ["_C*.so", "csrc/include/apex_amd/*.h"]},
    include_package_data=False,
    cmdclass={"build_py": BuildWithNative},
    python_requires=">=3.9",
    install_requires=[],
    zip_safe=False,
    has_ext_modules=lambda: True,
)
