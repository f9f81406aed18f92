"""Marker annotation (reference apex/pyprof/nvtx/__init__.py)."""
from .nvmarker import add_wrapper as wrap  # noqa: F401
from .nvmarker import init  # noqa: F401
