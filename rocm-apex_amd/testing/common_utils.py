"""Test helpers (reference apex/testing/common_utils.py:12-22).

``TEST_WITH_ROCM`` keeps the reference's env switch; since this framework only targets ROCm /
gfx950, ``skipIfRocm`` skips whenever the switch is on (the reference semantics), and
``skipIfNoGPU`` / ``requires_native`` are the checks our own tiers use."""
import os
import unittest
from functools import wraps

import torch

TEST_WITH_ROCM = os.getenv("APEX_TEST_WITH_ROCM", "0") == "1"
HAS_GPU = torch.cuda.is_available()


def skipIfRocm(fn):
    @wraps(fn)
    def wrapper(*args, **kwargs):
        if TEST_WITH_ROCM:
            raise unittest.SkipTest("test doesn't currently work on ROCm stack.")
        return fn(*args, **kwargs)

    return wrapper


def skipIfNoGPU(fn):
    @wraps(fn)
    def wrapper(*args, **kwargs):
        if not HAS_GPU:
            raise unittest.SkipTest("needs an MI355X (HIP) device")
        return fn(*args, **kwargs)

    return wrapper


def requires_native(submodule):
    """Skip unless the gfx950 extension exposes ``submodule`` (e.g. 'attn')."""

    def deco(fn):
        @wraps(fn)
        def wrapper(*args, **kwargs):
            from .. import _native

            if _native.submodule(submodule) is None:
                raise unittest.SkipTest("native submodule {} not built".format(submodule))
            return fn(*args, **kwargs)

        return wrapper

    return deco
