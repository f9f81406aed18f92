"""Non-interleaved 1F1B pipeline schedule
(reference .../schedules/fwd_bwd_pipelining_without_interleaving.py:22-170).

Stage r runs ``pp - r - 1`` warm-up forwards, then alternates one forward / one backward
(steady state), then drains the remaining backwards (cool-down).  Paired exchanges
(send-forward + recv-backward, send-backward + recv-forward) are single batched p2p calls."""
from typing import List, Optional, Union

import torch

from ... import parallel_state
from .. import p2p_communication
from ..utils import get_kth_microbatch, get_num_microbatches, listify_model
from .common import Batch, FwdStepFunc, backward_step, forward_step


def forward_backward_pipelining_without_interleaving(forward_step_func: FwdStepFunc, batch: Batch,
                                                     model: Union[torch.nn.Module, List[torch.nn.Module]], *,
                                                     forward_only: bool,
                                                     tensor_shape: Optional[Union[List[int], torch.Size]] = None,
                                                     dtype: Optional[torch.dtype] = None, grad_scaler=None,
                                                     **kwargs):
    """Returns the per-micro-batch reduced losses on the last stage, [] elsewhere."""
    model = listify_model(model)
    if len(model) != 1:
        raise RuntimeError(f"`model` is expected be a `nn.Module`, but {type(model)}")
    model = model[0]
    num_microbatches = get_num_microbatches()
    num_warmup = min(parallel_state.get_pipeline_model_parallel_world_size()
                     - parallel_state.get_pipeline_model_parallel_rank() - 1, num_microbatches)
    num_remaining = num_microbatches - num_warmup

    input_tensors, output_tensors, losses_reduced = [], [], []
    k = 0  # next micro-batch index

    for _ in range(num_warmup):
        input_tensor = p2p_communication.recv_forward(tensor_shape=tensor_shape, dtype=dtype)
        output_tensor = forward_step(forward_step_func, get_kth_microbatch(batch, k), model, input_tensor,
                                     losses_reduced)
        k += 1
        p2p_communication.send_forward(output_tensor, tensor_shape=tensor_shape, dtype=dtype)
        if not forward_only:
            input_tensors.append(input_tensor)
            output_tensors.append(output_tensor)

    input_tensor = p2p_communication.recv_forward(tensor_shape=tensor_shape, dtype=dtype) if num_remaining > 0 else None

    for i in range(num_remaining):
        last_iteration = i == (num_remaining - 1)
        output_tensor = forward_step(forward_step_func, get_kth_microbatch(batch, k), model, input_tensor,
                                     losses_reduced)
        k += 1
        if forward_only:
            p2p_communication.send_forward(output_tensor, tensor_shape=tensor_shape, dtype=dtype)
            if not last_iteration:
                input_tensor = p2p_communication.recv_forward(tensor_shape=tensor_shape, dtype=dtype)
            continue
        output_tensor_grad = p2p_communication.send_forward_recv_backward(output_tensor, tensor_shape=tensor_shape,
                                                                          dtype=dtype)
        input_tensors.append(input_tensor)
        output_tensors.append(output_tensor)
        input_tensor = input_tensors.pop(0)
        output_tensor = output_tensors.pop(0)
        input_tensor_grad = backward_step(input_tensor, output_tensor, output_tensor_grad, grad_scaler)
        if last_iteration:
            input_tensor = None
            p2p_communication.send_backward(input_tensor_grad, tensor_shape=tensor_shape, dtype=dtype)
        else:
            input_tensor = p2p_communication.send_backward_recv_forward(input_tensor_grad, tensor_shape=tensor_shape,
                                                                        dtype=dtype)

    if not forward_only:
        for _ in range(num_warmup):
            input_tensor = input_tensors.pop(0)
            output_tensor = output_tensors.pop(0)
            output_tensor_grad = p2p_communication.recv_backward(tensor_shape=tensor_shape, dtype=dtype)
            input_tensor_grad = backward_step(input_tensor, output_tensor, output_tensor_grad, grad_scaler)
            p2p_communication.send_backward(input_tensor_grad, tensor_shape=tensor_shape, dtype=dtype)
    return losses_reduced
