"""Marker annotation (reference apex/pyprof/nvtx/__init__.py)."""
from .nvmarker import init, layer, wrap  # noqa: F401
