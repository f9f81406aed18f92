"""Function wrappers for O1 (reference apex/amp/wrap.py).  The cast logic itself lives in
:mod:`apex.amp.amp` (a TorchFunctionMode); these helpers wrap arbitrary user callables."""
from . import utils
from .amp import _cast_call, _decorator_cast, _promote_call


def make_cast_wrapper(orig_fn, cast_fn, handle, try_caching=False):
    return _decorator_cast(cast_fn, _cast_call)(orig_fn)


def cached_cast(mod, fn, cast_fn, handle, try_caching=False, verbose=False):
    orig = utils.get_func(mod, fn)
    utils.set_func_save(handle, mod, fn, make_cast_wrapper(orig, cast_fn, handle, try_caching))


def make_promote_wrapper(orig_fn, cast_fn, handle=None):
    return _decorator_cast(None, _promote_call)(orig_fn)


def promote(mod, fn, handle, verbose=False):
    orig = utils.get_func(mod, fn)
    utils.set_func_save(handle, mod, fn, make_promote_wrapper(orig, utils.maybe_float))
