"""FLOP / byte report (reference apex/pyprof/prof)."""
from .prof import annotate, main, render  # noqa: F401
