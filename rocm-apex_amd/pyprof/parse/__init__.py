"""rocprofv3 trace parser (reference apex/pyprof/parse)."""
from .parse import attach_markers, decode_marker, main, parse  # noqa: F401
