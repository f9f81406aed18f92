"""What ``amp.initialize`` does to the models and optimizers once the opt-level properties are
settled (capability of reference apex/amp/_initialize.py:21-265).

Steps, in order:

1. normalise ``models`` / ``optimizers`` to lists (remembering how they were passed, since the
   return value mirrors it) and refuse what amp cannot wrap: models already inside a parallel
   wrapper, optimizers already inside a legacy FP16_Optimizer;
2. audit the incoming model: every floating parameter / buffer must be fp32 and on the GPU
   (``allow_incoming_model_not_fp32`` waives it);
3. cast the model (BN kept fp32 when ``keep_batchnorm_fp32``), wrap ``forward`` with a
   :class:`_Caster` for inputs and outputs, re-cast the optimizer state, and make every module's
   ``state_dict`` emit fp32 (:class:`O2StateDictHook`);
4. patch each optimizer for master weights / the fused amp step (``_process_optimizer``);
5. create one :class:`LossScaler` per loss, sync-free when every optimizer can take the device
   skip flag;
6. O1/O4: install the function-cast patches and keep the optimizer step outside them.
"""
import functools
import types
import warnings
from collections.abc import Iterable, Mapping

import numpy as np
import torch

from ._amp_state import _amp_state, warn_or_err
from ._process_optimizer import _process_optimizer
from .handle import disable_casts
from .scaler import LossScaler

_HALF = (torch.float16, torch.bfloat16)


class _Caster(object):
    """Casts every floating tensor found in (nested) call arguments / results to ``dtype``;
    containers keep their type, strings / arrays / non-tensors pass through."""

    def __init__(self, dtype, warn_host=False):
        self.dtype = dtype
        self.warn_host = warn_host

    def tensor(self, t):
        if isinstance(t, torch.Tensor):
            if self.warn_host and not t.is_cuda and torch.cuda.is_available():
                warnings.warn("amp: a model input is not on the GPU.")
            return t.to(self.dtype) if t.is_floating_point() else t
        return t.to(self.dtype)  # objects that only provide .to()

    def __call__(self, value):
        if isinstance(value, torch.Tensor):
            return self.tensor(value)
        if isinstance(value, (str, bytes, np.ndarray)):
            return value
        if hasattr(value, "to"):
            return self.tensor(value)
        if isinstance(value, Mapping):
            return {self(k): self(v) for k, v in value.items()}
        if isinstance(value, Iterable):
            return type(value)(self(v) for v in value)
        return value


# kept for callers of the reference-named helpers
def to_type(dtype, t):
    return _Caster(dtype, warn_host=True).tensor(t)


def applier(value, fn):
    if isinstance(fn, _Caster):
        return fn(value)
    caster = _Caster(None)
    caster.tensor = fn
    return caster(value)


def _as_list(obj, what, accept):
    """(list, passed_as_list) for a single ``accept`` instance, a list of them, or None."""
    if obj is None:
        return [], False
    if isinstance(obj, list):
        return obj, True
    if isinstance(obj, accept):
        return [obj], False
    raise TypeError("{} must be either a single {} or a list of them.".format(what, accept[0].__name__))


def check_models(models):
    from ..parallel import DistributedDataParallel as ApexDDP

    wrappers = ((torch.nn.parallel.DistributedDataParallel, "torch.nn.parallel.DistributedDataParallel"),
                (ApexDDP, "apex.parallel.DistributedDataParallel"),
                (torch.nn.parallel.DataParallel, "torch.nn.parallel.DataParallel"))
    for model in models:
        for cls, name in wrappers:
            if isinstance(model, cls):
                raise RuntimeError("amp.initialize got a model already wrapped in {}: apply parallel wrappers to "
                                   "the model(s) that amp.initialize returns, not before.".format(name))


def check_params_fp32(models):
    """Every floating parameter / buffer must arrive fp32 and on the GPU."""
    on_gpu = torch.cuda.is_available()
    for model in models:
        tensors = [("param", n, t) for n, t in model.named_parameters()]
        tensors += [("buffer", n, t) for n, t in model.named_buffers()]
        for kind, name, t in tensors:
            if not t.is_floating_point():
                continue
            low = t.dtype in _HALF if kind == "param" else t.dtype == torch.float16
            if low:
                warn_or_err("amp.initialize: {} {} is {} — pass the model in fp32; amp does any .half() / "
                            ".bfloat16() casting itself, whatever the opt_level.".format(kind, name, t.type()))
            elif on_gpu and not t.is_cuda:
                warn_or_err("amp.initialize: {} {} is {} on the host — move the model to the GPU "
                            "(model.to('cuda')) before amp.initialize.".format(kind, name, t.type()))


def check_optimizers(optimizers):
    from ..contrib.optimizers import FP16_Optimizer as FusedFP16Optimizer
    from ..fp16_utils import FP16_Optimizer as GeneralFP16Optimizer

    for optim in optimizers:
        if isinstance(optim, (GeneralFP16Optimizer, FusedFP16Optimizer)):
            raise RuntimeError("amp.initialize takes plain PyTorch or apex fused optimizers; got a {} — pass "
                               "the optimizer it wraps instead.".format(type(optim).__name__))


class O2StateDictHook(object):
    """``state_dict`` hook: half / bfloat16 entries are emitted as fp32 (O2/O3/O5 checkpoints stay
    loadable into an fp32 model)."""

    def __init__(self, fn=None):
        self.fn = fn

    def __call__(self, module, state_dict, prefix, local_metadata):
        for key, value in state_dict.items():
            if isinstance(value, torch.Tensor) and value.dtype in _HALF:
                state_dict[key] = value.float()


def _wrap_forward(model, in_caster, out_caster):
    fwd = model.forward
    # a model that declares ``_amp_casts_input = True`` takes its first positional tensor uncast
    # and casts it itself (to ``model._amp_input_dtype``) where it is first consumed: the fused
    # ResNet stem reads the fp32 batch and rounds it to the model dtype in its padding pass (the
    # same round-to-nearest-even as ``.to()``), saving the standalone cast pass
    own_cast = in_caster is not None and getattr(model, "_amp_casts_input", False)
    if own_cast:
        model._amp_input_dtype = in_caster.dtype

    @functools.wraps(fwd)
    def forward(*args, **kwargs):
        if in_caster is not None:
            if own_cast and args and isinstance(args[0], torch.Tensor) and args[0].is_cuda:
                args = (args[0],) + tuple(in_caster(args[1:]))
            else:
                args = in_caster(args)
            kwargs = in_caster(kwargs)
        return out_caster(fwd(*args, **kwargs))

    model.forward = forward


def _cast_models(models, properties, cast_model_outputs, optimizers):
    from ..fp16_utils import convert_network

    if properties.cast_model_type:
        for model in models:
            if properties.keep_batchnorm_fp32:
                convert_network(model, properties.cast_model_type)
            else:
                model.to(properties.cast_model_type)
        out = _Caster(cast_model_outputs if cast_model_outputs is not None else torch.float32)
        for model in models:
            _wrap_forward(model, _Caster(properties.cast_model_type, warn_host=True), out)
        for optimizer in optimizers:  # re-cast any existing state to the params' new dtypes
            optimizer.load_state_dict(optimizer.state_dict())
        hook = O2StateDictHook()
        for model in models:
            for module in model.modules():
                module._register_state_dict_hook(hook)
    elif cast_model_outputs is not None:
        for model in models:
            _wrap_forward(model, None, _Caster(cast_model_outputs))


def _make_loss_scalers(properties, optimizers, num_losses):
    fused = bool(optimizers) and all(getattr(o, "_amp_fused_capable", False) for o in optimizers)
    device_ok = torch.cuda.is_available() or getattr(_amp_state, "sync_free_force", False)
    _amp_state.sync_free = bool(_amp_state.sync_free_requested and fused and device_ok)
    for o in optimizers:
        o._amp_stash.fused_ok = _amp_state.sync_free
    scalers = []
    for _ in range(num_losses):
        s = LossScaler(properties.loss_scale, min_loss_scale=_amp_state.min_loss_scale,
                       max_loss_scale=_amp_state.max_loss_scale)
        s.sync_free = _amp_state.sync_free
        scalers.append(s)
    _amp_state.loss_scalers = scalers


def _step_without_casts(optimizer):
    inner = optimizer.step

    def step(self, *args, **kwargs):
        with disable_casts():
            return inner(*args, **kwargs)

    optimizer.step = types.MethodType(step, optimizer)


def _initialize(models, optimizers, properties, num_losses=1, cast_model_outputs=None):
    from ..parallel.LARC import LARC
    from .amp import init as amp_init

    if optimizers is not None and not isinstance(optimizers, (list, torch.optim.Optimizer, LARC)):
        check_optimizers([optimizers])
    opts, opts_listed = _as_list(optimizers, "optimizers", (torch.optim.Optimizer, LARC))
    check_optimizers(opts)
    mods, mods_listed = _as_list(models, "models", (torch.nn.Module,))

    check_models(mods)
    if not _amp_state.allow_incoming_model_not_fp32:
        check_params_fp32(mods)
    _cast_models(mods, properties, cast_model_outputs, opts)
    opts = [_process_optimizer(o, properties) for o in opts]
    _make_loss_scalers(properties, opts, num_losses)
    if properties.patch_torch_functions:
        amp_init(loss_scale=properties.loss_scale, patch_type=properties.patch_torch_functions_type,
                 verbose=(_amp_state.verbosity == 2))
        for o in opts:
            _step_without_casts(o)

    model_out = mods if mods_listed else mods[0]
    if opts_listed:
        return model_out, opts
    return model_out if not opts else (model_out, opts[0])
