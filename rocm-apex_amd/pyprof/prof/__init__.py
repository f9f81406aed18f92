"""FLOP / byte report (reference apex/pyprof/prof)."""
from .ops import model, model_for  # noqa: F401
from .output import render, summary  # noqa: F401
from .data import Data  # noqa: F401
from .prof import annotate, foo, main  # noqa: F401
