"""O1/O4 automatic casting (reference apex/amp/amp.py:17-198, apex/amp/wrap.py).

The reference monkey-patches attributes of ``torch``, ``torch.Tensor`` and
``torch.nn.functional``.  On PyTorch 2.x many calls never go through those Python attributes
(``nn.Linear`` calls the C++ binding directly, methods are bound at class creation), so here the
same cast *policy* (identical lists, registries and decorators) is enforced by one
``TorchFunctionMode`` pushed for as long as the handle is active: every torch-level call is
looked up in a {callable -> policy} table built from the lists, and its floating-point tensor
arguments are cast before dispatch.  User registrations (``register_half_function`` etc.)
still patch the named attribute, since those target user or third-party functions.
"""
import functools
import itertools

import torch
from torch.overrides import TorchFunctionMode

from . import utils
from ._amp_state import _amp_state
from .handle import AmpHandle, NoOpHandle
from .lists import functional_overrides, tensor_overrides, torch_overrides

_DECORATOR_HANDLE = None
_USER_CAST_REGISTRY = set()
_USER_PROMOTE_REGISTRY = set()
_ACTIVE_MODE = None


def _decorator_cast(cast_fn, wrap_fn):
    def wrapper(orig_fn):
        @functools.wraps(orig_fn)
        def wrapped(*args, **kwargs):
            handle = _DECORATOR_HANDLE
            if handle is None or not handle.is_active():
                return orig_fn(*args, **kwargs)
            return wrap_fn(cast_fn, orig_fn, handle, args, kwargs)

        return wrapped

    return wrapper


def _cast_call(cast_fn, orig_fn, handle, args, kwargs):
    fn = functools.partial(utils.cached_cast, cast_fn, cache=handle.cache) if handle.has_cache else cast_fn
    a, k = utils.casted_args(fn, args, kwargs)
    return orig_fn(*a, **k)


def _promote_call(cast_fn, orig_fn, handle, args, kwargs):
    types = utils.collect_fp_tensor_types(args, kwargs)
    if len(types) <= 1:
        return orig_fn(*args, **kwargs)
    if types == {torch.float16, torch.float32} or types == {torch.bfloat16, torch.float32}:
        a, k = utils.casted_args(utils.maybe_float, args, kwargs)
        return orig_fn(*a, **k)
    raise NotImplementedError("Do not know how to handle these types to promote: {}".format(types))


# --------------------------------------------------------------------------- decorators
def half_function(fn):
    return _decorator_cast(utils.maybe_half, _cast_call)(fn)


def bfloat16_function(fn):
    return _decorator_cast(utils.maybe_bfloat16, _cast_call)(fn)


def float_function(fn):
    return _decorator_cast(utils.maybe_float, _cast_call)(fn)


def promote_function(fn):
    return _decorator_cast(None, _promote_call)(fn)


# --------------------------------------------------------------------------- registries
def register_half_function(module, name):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    _USER_CAST_REGISTRY.add((module, name, utils.maybe_half))


def register_bfloat16_function(module, name):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    _USER_CAST_REGISTRY.add((module, name, utils.maybe_bfloat16))


def register_float_function(module, name):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    _USER_CAST_REGISTRY.add((module, name, utils.maybe_float))


def register_promote_function(module, name):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    _USER_PROMOTE_REGISTRY.add((module, name))


# --------------------------------------------------------------------------- policy table
_LOW, _FP32, _PROMOTE, _SEQ, _BANNED, _RNN = range(6)


def _resolve(module, names):
    out = []
    for n in names:
        f = getattr(module, n, None)
        if f is not None:
            out.append(f)
        # in-place and torch.* aliases of the same op
        f2 = getattr(module, n + "_", None)
        if f2 is not None and module is not torch.nn.functional:
            out.append(f2)
    return out


def _build_policy(patch_type, allow_banned):
    low_attr = "BFLOAT16_FUNCS" if patch_type == torch.bfloat16 else "FP16_FUNCS"
    table = {}
    for mod in (functional_overrides, torch_overrides, tensor_overrides):
        for f in _resolve(mod.MODULE, getattr(mod, low_attr)):
            table[f] = (_LOW, None)
        for f in _resolve(mod.MODULE, mod.FP32_FUNCS):
            table[f] = (_FP32, None)
        for f in _resolve(mod.MODULE, getattr(mod, "CASTS", [])):
            table[f] = (_PROMOTE, None)
        for f in _resolve(mod.MODULE, getattr(mod, "SEQUENCE_CASTS", [])):
            table[f] = (_SEQ, None)
    if not allow_banned:
        for name, msg in functional_overrides.BANNED_FUNCS:
            f = getattr(torch.nn.functional, name, None)
            if f is not None:
                table[f] = (_BANNED, msg)
            tf = getattr(torch._C._nn, name, None)
            if tf is not None:
                table[tf] = (_BANNED, msg)
    # RNN kernels: cast input + flat weights to the low type
    for n in ("lstm", "gru", "rnn_tanh", "rnn_relu", "lstm_cell", "gru_cell", "rnn_tanh_cell", "rnn_relu_cell"):
        f = getattr(torch, n, None)
        if f is not None:
            table[f] = (_RNN, None)
    return table


class _AmpCastMode(TorchFunctionMode):
    def __init__(self, handle, patch_type, table, verbose):
        super().__init__()
        self.handle = handle
        self.low = utils.maybe_bfloat16 if patch_type == torch.bfloat16 else utils.maybe_half
        self.table = table
        self.verbose = verbose

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        ent = self.table.get(func)
        if ent is None or not self.handle.is_active():
            return func(*args, **kwargs)
        kind, msg = ent
        if kind == _BANNED:
            raise NotImplementedError(msg)
        name = getattr(func, "__name__", str(func))
        if kind in (_LOW, _RNN):
            cast = utils.verbosify(self.low, name, self.verbose)
            fn = functools.partial(utils.cached_cast, cast, cache=self.handle.cache) \
                if self.handle.has_cache else cast
            a, k = utils.casted_args(fn, args, kwargs)
            return func(*a, **k)
        if kind == _FP32:
            cast = utils.verbosify(utils.maybe_float, name, self.verbose)
            a, k = utils.casted_args(cast, args, kwargs)
            return func(*a, **k)
        if kind in (_PROMOTE, _SEQ):
            tys = utils.collect_fp_tensor_types(args, kwargs)
            if len(tys) > 1 and torch.float32 in tys:
                cast = utils.verbosify(utils.maybe_float, name, self.verbose)
                a, k = utils.casted_args(cast, args, kwargs)
                return func(*a, **k)
            return func(*args, **kwargs)
        return func(*args, **kwargs)


def _install_user_registries(handle, patch_type, verbose):
    for module, name, cast_fn in _USER_CAST_REGISTRY:
        if cast_fn is utils.maybe_half and patch_type == torch.bfloat16:
            cast_fn = utils.maybe_bfloat16
        orig = getattr(module, name)
        wrapped = _decorator_cast(cast_fn, _cast_call)(orig)
        utils.set_func_save(handle, module, name, wrapped)
    for module, name in _USER_PROMOTE_REGISTRY:
        orig = getattr(module, name)
        wrapped = _decorator_cast(None, _promote_call)(orig)
        utils.set_func_save(handle, module, name, wrapped)
    _USER_CAST_REGISTRY.clear()
    _USER_PROMOTE_REGISTRY.clear()


def _uninstall():
    global _ACTIVE_MODE, _DECORATOR_HANDLE
    h = _DECORATOR_HANDLE
    if h is not None:
        for mod, fn, func in reversed(getattr(h, "_all_wrappers", [])):
            utils.set_func(mod, fn, func)
    if _ACTIVE_MODE is not None:
        try:
            _ACTIVE_MODE.__exit__(None, None, None)
        except Exception:
            pass
        _ACTIVE_MODE = None
    _DECORATOR_HANDLE = None


def init(enabled=True, loss_scale="dynamic", enable_caching=True, verbose=False, allow_banned=False,
         patch_type=torch.float16):
    """Activate O1/O4 casting; returns the handle (``handle._deactivate()`` undoes it)."""
    global _DECORATOR_HANDLE, _ACTIVE_MODE
    if not enabled:
        handle = NoOpHandle()
        _DECORATOR_HANDLE = handle
        return handle
    if _ACTIVE_MODE is not None:
        _uninstall()
    handle = AmpHandle(loss_scale, enable_caching, verbose)
    _install_user_registries(handle, patch_type, verbose)
    table = _build_policy(patch_type, allow_banned)
    mode = _AmpCastMode(handle, patch_type, table, verbose)
    mode.__enter__()
    _ACTIVE_MODE = mode
    _DECORATOR_HANDLE = handle
    _amp_state.handle = handle
    return handle
