"""Fast LayerNorm (reference apex/contrib/layer_norm/__init__.py)."""
from .layer_norm import FastLayerNorm, FastLayerNormFN  # noqa: F401
