"""MI355X-native (gfx950 / CDNA4) mixed-precision and distributed training library for
PyTorch-ROCm with the public API of Apex (reference: abhinavvishnu/rocm-apex, apex/__init__.py).

Import order mirrors the reference (apex/__init__.py:1-42): parallel (when torch.distributed is
available), amp, fp16_utils, optimizers, normalization, transformer ... plus a root logger that
prints the (tp, pp, dp) ranks of the emitting process.
"""
import logging
import warnings

import torch

__version__ = "0.1.0+gfx950"

from . import _native  # noqa: F401  (loads apex._C when built)

if torch.distributed.is_available():
    from . import parallel  # noqa: F401

from . import amp  # noqa: F401
from . import fp16_utils  # noqa: F401
from . import optimizers  # noqa: F401
from . import normalization  # noqa: F401
from . import multi_tensor_apply  # noqa: F401


class RankInfoFormatter(logging.Formatter):
    """Adds ``rank_info`` = (tensor, pipeline, data)-parallel ranks to every record."""

    def format(self, record):
        try:
            from .transformer.parallel_state import get_rank_info

            record.rank_info = get_rank_info()
        except Exception:  # pragma: no cover - before model parallel init
            record.rank_info = ""
        return super().format(record)


_library_root_logger = logging.getLogger(__name__)
if not _library_root_logger.handlers:
    _handler = logging.StreamHandler()
    _handler.setFormatter(RankInfoFormatter("%(asctime)s - PID:%(process)d - rank:%(rank_info)s - "
                                            "%(filename)s:%(lineno)d - %(levelname)s - %(message)s",
                                            "%y-%m-%d %H:%M:%S"))
    _library_root_logger.addHandler(_handler)
    _library_root_logger.propagate = False


def check_cudnn_version_and_warn(global_option: str, required_cudnn_version: int) -> bool:
    """Reference API (apex/__init__.py); MIOpen has no cuDNN version gate."""
    return True


def __getattr__(name):
    # lazy heavy subsystems
    if name in ("transformer", "contrib", "mlp", "fused_dense", "models", "ops", "utils", "RNN",
                "reparameterization", "pyprof", "testing", "amp_C"):
        import importlib

        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
