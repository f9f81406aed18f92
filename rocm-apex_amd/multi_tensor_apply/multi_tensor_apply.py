"""Python front of the multi-tensor-apply engine (reference
apex/multi_tensor_apply/multi_tensor_apply.py:3-30).

``op`` is any ``amp_C`` function; the engine itself (work table cache + persistent grid) is in
``csrc/bindings/mta_host.cpp`` / ``csrc/include/apex_amd/mta.h``.
"""
from .. import _native


class MultiTensorApply(object):
    available = True  # the torch reference path makes every op available on CPU too
    warned = False

    def __init__(self, chunk_size):
        self.chunk_size = chunk_size
        MultiTensorApply.import_err = _native.import_error
        MultiTensorApply.native = _native.available()

    def check_avail(self):
        if not MultiTensorApply.available:
            raise RuntimeError("multi_tensor_applier unavailable: " + repr(MultiTensorApply.import_err))

    def __call__(self, op, noop_flag_buffer, tensor_lists, *args):
        self.check_avail()
        return op(self.chunk_size, noop_flag_buffer, tensor_lists, *args)
