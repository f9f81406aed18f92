"""Gradient accumulation without pipelining (reference .../schedules/fwd_bwd_no_pipelining.py:29-91):
all micro-batches forward+backward on one stage; gradient all-reduce (DDP) only on the last."""
import contextlib
from typing import List, Union

import torch

from ..utils import get_kth_microbatch, get_num_microbatches, listify_model
from .common import Batch, FwdStepFunc, backward_step, forward_step


def forward_backward_no_pipelining(forward_step_func: FwdStepFunc, batch: Batch,
                                   model: Union[torch.nn.Module, List[torch.nn.Module]], *, forward_only: bool,
                                   grad_scaler=None, **kwargs):
    """Returns the list of per-micro-batch reduced losses."""
    model = listify_model(model)
    if len(model) != 1:
        raise RuntimeError(f"`model` is expected be a `nn.Module`, but {type(model)}")
    model = model[0]
    no_sync = getattr(model, "no_sync", None)
    context_handler = no_sync if callable(no_sync) else contextlib.nullcontext
    losses_reduced = []
    num_micro_batches = get_num_microbatches()
    with context_handler():
        for i in range(num_micro_batches - 1):
            out = forward_step(forward_step_func, get_kth_microbatch(batch, i), model, None, losses_reduced)
            if not forward_only:
                backward_step(None, out, None, grad_scaler)
    # the last micro-batch runs outside no_sync so the data-parallel gradient reduction fires
    out = forward_step(forward_step_func, get_kth_microbatch(batch, num_micro_batches - 1), model, None,
                       losses_reduced)
    if not forward_only:
        backward_step(None, out, None, grad_scaler)
    return losses_reduced
