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
# kinds: cast to the low type / to fp32, promote to the widest type (plain and sequence forms),
# banned (error on low-precision input), RNN kernels (low), and the in-place forms: match the
# self tensor's type (MATCH0), or refuse a low-precision self / any low input (ERR_ARG0 /
# ERR_ANY) because an fp32-policy op cannot run in place on a half tensor.
_LOW, _FP32, _PROMOTE, _SEQ, _BANNED, _RNN, _MATCH0, _ERR_ARG0, _ERR_ANY = range(9)
_LOW_TYPES = (torch.float16, torch.bfloat16)


def _attrs(module, names):
    return [f for f in (getattr(module, n, None) for n in names) if f is not None]


def _inplace(names):
    return [n + "_" for n in names if not n.startswith("__")]


def _build_policy(patch_type, allow_banned):
    """{callable: (kind, message)}, assembled in the same order of precedence as the reference's
    patching passes (apex/amp/amp.py:111-192): casts, promotion, in-place rules, RNNs, banned."""
    low_attr = "BFLOAT16_FUNCS" if patch_type == torch.bfloat16 else "FP16_FUNCS"
    table = {}

    def put(fns, kind, msg=None):
        for f in fns:
            table[f] = (kind, msg)

    T, tensor = torch.Tensor, tensor_overrides
    for mod in (functional_overrides, torch_overrides, tensor_overrides):
        put(_attrs(mod.MODULE, getattr(mod, low_attr)), _LOW)
        put(_attrs(mod.MODULE, mod.FP32_FUNCS), _FP32)
    for mod in (torch_overrides, tensor_overrides):
        casts = getattr(mod, "CASTS", [])
        put(_attrs(mod.MODULE, [n for n in casts if not n.startswith("__i")]), _PROMOTE)
        put(_attrs(mod.MODULE, getattr(mod, "SEQUENCE_CASTS", [])), _SEQ)
    put(_attrs(torch, _inplace(torch_overrides.FP32_FUNCS)), _ERR_ANY)
    put(_attrs(T, _inplace(tensor.FP32_FUNCS)), _ERR_ARG0)
    inplace_match = _inplace(list(getattr(tensor, low_attr)) + list(tensor.CASTS))
    inplace_match += [n for n in tensor.CASTS if n.startswith("__i")]
    put(_attrs(T, inplace_match), _MATCH0)
    for n in ("lstm", "gru", "rnn_tanh", "rnn_relu", "lstm_cell", "gru_cell", "rnn_tanh_cell", "rnn_relu_cell"):
        put(_attrs(torch, [n]), _RNN)
    for name, msg in functional_overrides.BANNED_FUNCS:
        fns = _attrs(torch.nn.functional, [name]) + _attrs(torch._C._nn, [name])
        put(fns, _FP32 if allow_banned else _BANNED, msg)
    return table


def _any_low(args, kwargs):
    return any(t in _LOW_TYPES for t in utils.collect_fp_tensor_types(args, kwargs))


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
        name = getattr(func, "__name__", str(func))
        if kind == _BANNED:
            if _any_low(args, kwargs):
                raise NotImplementedError(msg)
            return func(*args, **kwargs)
        if kind in (_ERR_ANY, _ERR_ARG0):
            bad = _any_low(args, kwargs) if kind == _ERR_ANY else (
                len(args) > 0 and utils.is_fp_tensor(args[0]) and args[0].dtype in _LOW_TYPES)
            if bad:
                raise NotImplementedError("amp: in-place {} on a {} tensor is not supported under O1 (the op runs "
                                          "in fp32)".format(name, "low-precision"))
            return func(*args, **kwargs)
        if kind == _MATCH0:
            if len(args) > 0 and utils.is_fp_tensor(args[0]):
                target = args[0].dtype
                a, k = utils.casted_args(lambda x: x.to(target) if utils.is_fp_tensor(x) else x, args[1:], kwargs)
                return func(args[0], *a, **k)
            return func(*args, **kwargs)
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


def _rnn_check_input_relaxed(orig):
    """nn.RNNBase.check_input rejects an input whose dtype differs from the weights' unless torch
    autocast is on; under O1 the RNN kernel call itself casts input and flat weights to the low
    type (the _RNN policy), so the dtype part of the check is waived while the handle is active."""

    @functools.wraps(orig)
    def check_input(self, input, batch_sizes):
        h = _DECORATOR_HANDLE
        if h is not None and h.is_active() and input.is_floating_point():
            w = self._flat_weights[0] if self._flat_weights else None
            if w is not None and w.dtype != input.dtype:
                # shape-only stand-in with the weights' dtype (an expanded 0-d tensor: no copy)
                input = torch.empty((), dtype=w.dtype, device=input.device).expand(input.shape)
        return orig(self, input, batch_sizes)

    return check_input


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
    rnn_base = torch.nn.modules.rnn.RNNBase
    utils.set_func_save(handle, rnn_base, "check_input", _rnn_check_input_relaxed(rnn_base.check_input))
    table = _build_policy(patch_type, allow_banned)
    mode = _AmpCastMode(handle, patch_type, table, verbose)
    mode.__enter__()
    _ACTIVE_MODE = mode
    _DECORATOR_HANDLE = handle
    _amp_state.handle = handle
    return handle
