"""Model/optimizer processing behind ``amp.initialize`` (reference apex/amp/_initialize.py:21-265)."""
import functools
import sys
import types
import warnings
from collections.abc import Iterable, Mapping

import numpy as np
import torch

from ._amp_state import _amp_state, warn_or_err
from ._process_optimizer import _process_optimizer
from .handle import disable_casts
from .scaler import LossScaler


def to_type(dtype, t):
    if isinstance(t, torch.Tensor):
        if not t.is_cuda and torch.cuda.is_available():
            warnings.warn("An input tensor was not cuda.")
        if t.is_floating_point():
            return t.to(dtype)
        return t
    return t.to(dtype)


def applier(value, fn):
    """Apply ``fn`` to every tensor (or object with ``.to``) inside nested containers."""
    if isinstance(value, torch.Tensor):
        return fn(value)
    if isinstance(value, (str, bytes)):
        return value
    if isinstance(value, np.ndarray):
        return value
    if hasattr(value, "to"):
        return fn(value)
    if isinstance(value, Mapping):
        return {applier(k, fn): applier(v, fn) for k, v in value.items()}
    if isinstance(value, Iterable):
        return type(value)(applier(v, fn) for v in value)
    return value


def check_models(models):
    from ..parallel import DistributedDataParallel as apex_DDP

    for model in models:
        parallel_type = None
        if isinstance(model, torch.nn.parallel.DistributedDataParallel):
            parallel_type = "torch.nn.parallel.DistributedDataParallel"
        if isinstance(model, apex_DDP):
            parallel_type = "apex.parallel.DistributedDataParallel"
        if isinstance(model, torch.nn.parallel.DataParallel):
            parallel_type = "torch.nn.parallel.DataParallel"
        if parallel_type is not None:
            raise RuntimeError("Incoming model is an instance of {}. ".format(parallel_type) +
                               "Parallel wrappers should only be applied to the model(s) AFTER \n"
                               "the model(s) have been returned from amp.initialize.")


def check_params_fp32(models):
    for model in models:
        for name, param in model.named_parameters():
            if param.is_floating_point():
                if param.dtype in (torch.float16, torch.bfloat16):
                    warn_or_err("Found param {} with type {}, expected torch.cuda.FloatTensor.\n"
                                "When using amp.initialize, you do not need to call .half() or .bfloat16()\n"
                                "on your model before passing it, no matter what optimization level you "
                                "choose.".format(name, param.type()))
                elif not param.is_cuda and torch.cuda.is_available():
                    warn_or_err("Found param {} with type {}, expected torch.cuda.FloatTensor.\n"
                                "When using amp.initialize, you need to provide a model with parameters\n"
                                "located on a CUDA device before passing it no matter what optimization level\n"
                                "you chose. Use model.to('cuda') to use the default device.".format(
                                    name, param.type()))
        for name, buf in model.named_buffers():
            if buf.is_floating_point():
                if buf.dtype == torch.float16:
                    warn_or_err("Found buffer {} with type {}, expected torch.cuda.FloatTensor.\n"
                                "When using amp.initialize, you do not need to call .half() on your model\n"
                                "before passing it, no matter what optimization level you choose.".format(
                                    name, buf.type()))
                elif not buf.is_cuda and torch.cuda.is_available():
                    warn_or_err("Found buffer {} with type {}, expected torch.cuda.FloatTensor.\n"
                                "When using amp.initialize, you need to provide a model with buffers\n"
                                "located on a CUDA device before passing it no matter what optimization level\n"
                                "you chose. Use model.to('cuda') to use the default device.".format(
                                    name, buf.type()))


def check_optimizers(optimizers):
    from ..contrib.optimizers import FP16_Optimizer as FP16_Optimizer_for_fused
    from ..fp16_utils import FP16_Optimizer as FP16_Optimizer_general

    for optim in optimizers:
        bad = None
        if isinstance(optim, FP16_Optimizer_general):
            bad = "apex.fp16_utils.FP16_Optimizer"
        if isinstance(optim, FP16_Optimizer_for_fused):
            bad = "apex.optimizers.FP16_Optimizer"
        if bad is not None:
            raise RuntimeError("An incoming optimizer is an instance of {}. ".format(bad) +
                               "The optimizer(s) passed to amp.initialize() must be bare \n"
                               "instances of either ordinary Pytorch optimizers, or Apex fused \n"
                               "optimizers.\n")


class O2StateDictHook(object):
    """Makes ``model.state_dict()`` emit fp32 tensors under O2/O3/O5."""

    def __init__(self, fn):
        self.fn = fn

    def __call__(self, module, state_dict, prefix, local_metadata):
        for key in state_dict:
            param = state_dict[key]
            if isinstance(param, torch.Tensor) and param.dtype in (torch.float16, torch.bfloat16):
                state_dict[key] = param.to(torch.float32)


def _initialize(models, optimizers, properties, num_losses=1, cast_model_outputs=None):
    from ..fp16_utils import convert_network
    from ..parallel.LARC import LARC
    from .amp import init as amp_init

    optimizers_was_list = False
    if isinstance(optimizers, torch.optim.Optimizer) or isinstance(optimizers, LARC):
        optimizers = [optimizers]
    elif optimizers is None:
        optimizers = []
    elif isinstance(optimizers, list):
        optimizers_was_list = True
        check_optimizers(optimizers)
    else:
        check_optimizers([optimizers])
        raise TypeError("optimizers must be either a single optimizer or a list of optimizers.")

    if isinstance(models, torch.nn.Module):
        models_was_list = False
        models = [models]
    elif isinstance(models, list):
        models_was_list = True
    else:
        raise TypeError("models must be either a single model or a list of models.")

    check_models(models)
    if not _amp_state.allow_incoming_model_not_fp32:
        check_params_fp32(models)

    if properties.cast_model_type:
        if properties.keep_batchnorm_fp32:
            for model in models:
                convert_network(model, properties.cast_model_type)
        else:
            for model in models:
                model.to(properties.cast_model_type)

        input_caster = functools.partial(to_type, properties.cast_model_type)
        output_caster = functools.partial(to_type, cast_model_outputs if cast_model_outputs is not None
                                          else torch.float32)

        for model in models:
            def patch_forward(old_fwd):
                def new_fwd(*args, **kwargs):
                    output = old_fwd(*applier(args, input_caster), **applier(kwargs, input_caster))
                    return applier(output, output_caster)
                return new_fwd

            model.forward = patch_forward(model.forward)

        for optimizer in optimizers:
            optimizer.load_state_dict(optimizer.state_dict())

        for model in models:
            for module in model.modules():
                module._register_state_dict_hook(O2StateDictHook(functools.partial(to_type, torch.float32)))

    elif cast_model_outputs is not None:
        output_caster = functools.partial(to_type, cast_model_outputs)
        for model in models:
            def patch_forward(old_fwd):
                def new_fwd(*args, **kwargs):
                    return applier(old_fwd(*args, **kwargs), output_caster)
                return new_fwd

            model.forward = patch_forward(model.forward)

    for i, optimizer in enumerate(optimizers):
        optimizers[i] = _process_optimizer(optimizer, properties)

    # sync-free scaler when every optimizer consumes a device skip flag
    all_capable = len(optimizers) > 0 and all(getattr(o, "_amp_fused_capable", False) for o in optimizers)
    _amp_state.sync_free = bool(_amp_state.sync_free_requested and all_capable and (
        torch.cuda.is_available() or getattr(_amp_state, "sync_free_force", False)))
    for o in optimizers:
        o._amp_stash.fused_ok = _amp_state.sync_free

    _amp_state.loss_scalers = []
    for _ in range(num_losses):
        s = LossScaler(properties.loss_scale, min_loss_scale=_amp_state.min_loss_scale,
                       max_loss_scale=_amp_state.max_loss_scale)
        s.sync_free = _amp_state.sync_free
        _amp_state.loss_scalers.append(s)

    if properties.patch_torch_functions:
        amp_init(loss_scale=properties.loss_scale, patch_type=properties.patch_torch_functions_type,
                 verbose=(_amp_state.verbosity == 2))
        for optimizer in optimizers:
            def patch_step(old_step):
                def new_step(self, *args, **kwargs):
                    with disable_casts():
                        return old_step(*args, **kwargs)
                return new_step

            optimizer.step = types.MethodType(patch_step(optimizer.step), optimizer)

    if optimizers_was_list:
        return (models, optimizers) if models_was_list else (models[0], optimizers)
    if models_was_list:
        return models if len(optimizers) == 0 else (models, optimizers[0])
    return models[0] if len(optimizers) == 0 else (models[0], optimizers[0])
