"""Pieces shared by the pipeline schedules (reference apex/transformer/pipeline_parallel/schedules/common.py:18-218):
``build_model`` (per-virtual-chunk model construction with pre/post-process flags, optional
DDP over the data-parallel group), ``forward_step`` and ``backward_step``."""
from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import torch

from ... import parallel_state
from ...tensor_parallel.layers import set_defaults_if_not_set_tensor_model_parallel_attributes
from ..utils import get_num_microbatches, listify_model, unwrap_model

Batch = Union[torch.Tensor, List[torch.Tensor], Tuple[torch.Tensor, ...]]
LossFunc = Callable[[torch.Tensor], torch.Tensor]
FwdStepFunc = Callable[[Batch, torch.nn.Module], Tuple[torch.Tensor, LossFunc]]


def build_model(model_provider_func: Callable[[Any, Dict[str, Any]], torch.nn.Module], wrap_with_ddp: bool = True,
                virtual_pipeline_model_parallel_size: Optional[int] = None, *args, **kwargs) -> List[torch.nn.Module]:
    """Instantiate this rank's model chunk(s): ``model_provider_func(*args, pre_process=...,
    post_process=..., **kwargs)`` once per virtual pipeline stage; returns a list."""
    if parallel_state.get_pipeline_model_parallel_world_size() > 1 and virtual_pipeline_model_parallel_size is not None:
        model = []
        for i in range(virtual_pipeline_model_parallel_size):
            parallel_state.set_virtual_pipeline_model_parallel_rank(i)
            cur_kwargs = dict(kwargs)
            cur_kwargs.update({"pre_process": parallel_state.is_pipeline_first_stage(),
                               "post_process": parallel_state.is_pipeline_last_stage()})
            model.append(model_provider_func(*args, **cur_kwargs))
    else:
        cur_kwargs = dict(kwargs)
        cur_kwargs.update({"pre_process": parallel_state.is_pipeline_first_stage(),
                           "post_process": parallel_state.is_pipeline_last_stage()})
        model = model_provider_func(*args, **cur_kwargs)
    if not isinstance(model, list):
        model = [model]
    for model_module in model:
        for param in model_module.parameters():
            set_defaults_if_not_set_tensor_model_parallel_attributes(param)
    if parallel_state.get_data_parallel_rank() == 0:
        print(" > number of parameters on (tensor, pipeline) model parallel rank ({}, {}): {}".format(
            parallel_state.get_tensor_model_parallel_rank(), parallel_state.get_pipeline_model_parallel_rank(),
            sum(sum(p.nelement() for p in m.parameters()) for m in model)), flush=True)
    if torch.cuda.is_available():
        for model_module in model:
            model_module.cuda(torch.cuda.current_device())
    if wrap_with_ddp:
        kw = {}
        if torch.cuda.is_available():
            i = torch.cuda.current_device()
            kw = dict(device_ids=[i], output_device=i)
        model = [torch.nn.parallel.distributed.DistributedDataParallel(
            m, process_group=parallel_state.get_data_parallel_group(), **kw) for m in model]
    return model


def _get_params_for_weight_decay_optimization(model):
    """(with-weight-decay, no-weight-decay) param groups: norms and biases get no decay."""
    from ....normalization.fused_layer_norm import FusedLayerNorm, FusedRMSNorm

    modules = listify_model(model)
    weight_decay_params = {"params": []}
    no_weight_decay_params = {"params": [], "weight_decay": 0.0}
    for module in modules:
        for module_ in module.modules():
            if isinstance(module_, (FusedLayerNorm, FusedRMSNorm, torch.nn.LayerNorm)):
                no_weight_decay_params["params"].extend([p for p in module_._parameters.values() if p is not None])
            else:
                weight_decay_params["params"].extend(
                    [p for n, p in module_._parameters.items() if p is not None and n != "bias"])
                no_weight_decay_params["params"].extend(
                    [p for n, p in module_._parameters.items() if p is not None and n == "bias"])
    return weight_decay_params, no_weight_decay_params


def forward_step(forward_step_func: FwdStepFunc, batch: Batch, model: torch.nn.Module,
                 input_tensor: Optional[torch.Tensor], losses_reduced: List[torch.Tensor]):
    """Run one micro-batch through this stage.  Non-first stages feed ``input_tensor`` through the
    model's ``set_input_tensor``; the last stage applies the loss function and divides by the
    number of micro-batches (gradient accumulation)."""
    unwrapped_model = unwrap_model(model)
    if hasattr(unwrapped_model, "set_input_tensor"):
        unwrapped_model.set_input_tensor(input_tensor)
    output_tensor, loss_func = forward_step_func(batch, model)
    if parallel_state.is_pipeline_last_stage():
        loss, loss_reduced = loss_func(output_tensor)
        output_tensor = loss / get_num_microbatches()
        losses_reduced.append(loss_reduced)
    return output_tensor


def backward_step(input_tensor: Optional[torch.Tensor], output_tensor: torch.Tensor,
                  output_tensor_grad: Optional[torch.Tensor], grad_scaler=None) -> Optional[torch.Tensor]:
    """Backward through this stage; returns d(loss)/d(input_tensor) (None on the first stage).
    On the last stage ``output_tensor`` is the loss (scaled by ``grad_scaler`` when given)."""
    if input_tensor is not None:
        input_tensor.retain_grad()
    if grad_scaler is not None and output_tensor_grad is None:
        output_tensor = grad_scaler.scale(output_tensor)
    torch.autograd.backward(output_tensor, grad_tensors=output_tensor_grad)
    return input_tensor.grad if input_tensor is not None else None
