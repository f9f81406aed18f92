"""Op-level profiling for rocprofv3 (reference apex/pyprof/__init__.py).

1. ``apex.pyprof.nvtx.init()`` in the training script (ROCTX op markers with argument shapes,
   forward and backward; ``apex.pyprof.nvtx.layer(name)`` for user layer annotations),
2. ``rocprofv3 --kernel-trace --marker-trace --hip-runtime-trace --output-format csv -d out -- python3 train.py``,
3. ``python -m apex.pyprof.parse out > parsed.txt``  (kernel <-> marker correlation),
4. ``python -m apex.pyprof.prof parsed.txt``         (FLOPs / bytes / MFMA use / achieved rates per kernel).
"""
from . import nvtx, parse, prof  # noqa: F401
from .nvtx import init, layer, wrap  # noqa: F401
