"""Test utilities (reference apex/testing)."""
from .common_utils import TEST_WITH_ROCM, requires_native, skipIfNoGPU, skipIfRocm  # noqa: F401
