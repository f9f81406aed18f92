"""Point-to-point activation / gradient exchange between adjacent pipeline stages
(reference apex/transformer/pipeline_parallel/p2p_communication.py:31-404).

MI355X design choices (differences from the reference):
  * tensors travel in their compute dtype (bf16/fp16) by default — the reference always sends
    fp32 (:130-134), doubling the xGMI bytes; pass ``dtype=torch.float32`` to force it;
  * no ``torch.cuda.synchronize()`` after each exchange (reference :162): the RCCL requests are
    waited on, which orders the *stream* behind the transfer without stalling the host, so the
    next micro-batch's kernels queue while the p2p is in flight;
  * optional scatter-gather: only 1/tp of the activation crosses the pipeline link and the TP
    group rebuilds it with one all-gather (over direct xGMI links inside the node).
All sends/recvs of one call are issued as one ``batch_isend_irecv`` group.
"""
import operator
from functools import reduce
from typing import List, Optional, Tuple, Union

import torch

from .. import parallel_state
from ..utils import comm_device, gather_split_1d_tensor, split_tensor_into_1d_equal_chunks
from ._timers import _Timers

Shape = Union[List[int], torch.Size, Tuple[int, ...]]


def _run_p2pops(tensor_send_prev, tensor_send_next, tensor_recv_prev, tensor_recv_next):
    ops = []
    group = parallel_state.get_pipeline_model_parallel_group()
    if tensor_send_prev is not None:
        ops.append(torch.distributed.P2POp(torch.distributed.isend, tensor_send_prev,
                                           parallel_state.get_pipeline_model_parallel_prev_rank(), group))
    if tensor_recv_prev is not None:
        ops.append(torch.distributed.P2POp(torch.distributed.irecv, tensor_recv_prev,
                                           parallel_state.get_pipeline_model_parallel_prev_rank(), group))
    if tensor_send_next is not None:
        ops.append(torch.distributed.P2POp(torch.distributed.isend, tensor_send_next,
                                           parallel_state.get_pipeline_model_parallel_next_rank(), group))
    if tensor_recv_next is not None:
        ops.append(torch.distributed.P2POp(torch.distributed.irecv, tensor_recv_next,
                                           parallel_state.get_pipeline_model_parallel_next_rank(), group))
    if ops:
        for req in torch.distributed.batch_isend_irecv(ops):
            req.wait()


def _communicate(tensor_send_next: Optional[torch.Tensor], tensor_send_prev: Optional[torch.Tensor], recv_prev: bool,
                 recv_next: bool, tensor_shape: Optional[Shape] = None,
                 override_scatter_gather_tensors_in_pipeline: bool = False, dtype_: Optional[torch.dtype] = None, *,
                 scatter_gather_tensors_in_pipeline: bool = True, params_dtype: Optional[torch.dtype] = None,
                 fp32_residual_connection: bool = False) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Exchange with the previous / next stage; returns (recv_prev, recv_next)."""
    if tensor_shape is None:
        raise RuntimeError("`tensor_shape` must be specified. Common `tensor_shape` is "
                           "`(seq_length, micro_batch_size, hidden_size)`")
    tp = parallel_state.get_tensor_model_parallel_world_size()
    numel = reduce(operator.mul, tensor_shape, 1)
    scatter_gather = (not override_scatter_gather_tensors_in_pipeline and scatter_gather_tensors_in_pipeline
                      and tp > 1 and numel % tp == 0)
    chunk_shape = (numel // tp,) if scatter_gather else tuple(tensor_shape)
    dtype = dtype_
    if dtype is None:
        for t in (tensor_send_next, tensor_send_prev):
            if t is not None:
                dtype = t.dtype
                break
    if dtype is None:
        dtype = params_dtype if params_dtype is not None else torch.float32
    if fp32_residual_connection:
        dtype = torch.float32
    dev = comm_device()
    tensor_recv_prev = torch.empty(chunk_shape, requires_grad=True, device=dev, dtype=dtype) if recv_prev else None
    tensor_recv_next = torch.empty(chunk_shape, requires_grad=True, device=dev, dtype=dtype) if recv_next else None

    def prep(t):
        if t is None:
            return None
        t = t.detach().to(dtype)
        if scatter_gather:
            t = split_tensor_into_1d_equal_chunks(t)
        return t.contiguous()

    _run_p2pops(prep(tensor_send_prev), prep(tensor_send_next), tensor_recv_prev, tensor_recv_next)
    if scatter_gather:
        if recv_prev:
            tensor_recv_prev = gather_split_1d_tensor(tensor_recv_prev).view(tensor_shape).requires_grad_()
        if recv_next:
            tensor_recv_next = gather_split_1d_tensor(tensor_recv_next).view(tensor_shape).requires_grad_()
    return tensor_recv_prev, tensor_recv_next


def _timed(timers, name):
    class _Ctx:
        def __enter__(self):
            if timers is not None:
                timers(name).start()

        def __exit__(self, *exc):
            if timers is not None:
                timers(name).stop()

    return _Ctx()


def recv_forward(tensor_shape: Shape, override_scatter_gather_tensors_in_pipeline: bool = False, *,
                 dtype: Optional[torch.dtype] = None, timers: _Timers = None) -> torch.Tensor:
    """Receive the activation from the previous stage (forward receive)."""
    if parallel_state.is_pipeline_first_stage():
        return None
    with _timed(timers, "forward-recv"):
        input_tensor, _ = _communicate(None, None, True, False, tensor_shape,
                                       override_scatter_gather_tensors_in_pipeline, dtype)
    return input_tensor


def recv_backward(tensor_shape: Shape = None, *, dtype: Optional[torch.dtype] = None, timers: _Timers = None):
    """Receive the output gradient from the next stage (backward receive)."""
    if parallel_state.is_pipeline_last_stage():
        return None
    with _timed(timers, "backward-recv"):
        _, output_tensor_grad = _communicate(None, None, False, True, tensor_shape, dtype_=dtype)
    return output_tensor_grad


def send_forward(output_tensor: torch.Tensor, tensor_shape: Shape = None,
                 override_scatter_gather_tensors_in_pipeline: bool = False, *, dtype: Optional[torch.dtype] = None,
                 timers: _Timers = None) -> None:
    """Send the activation to the next stage (forward send)."""
    if parallel_state.is_pipeline_last_stage():
        return
    with _timed(timers, "forward-send"):
        _communicate(output_tensor, None, False, False, tensor_shape, override_scatter_gather_tensors_in_pipeline,
                     dtype)


def send_backward(input_tensor_grad: torch.Tensor, tensor_shape: Shape, *, dtype: Optional[torch.dtype] = None,
                  timers: _Timers = None) -> None:
    """Send the input gradient to the previous stage (backward send)."""
    if parallel_state.is_pipeline_first_stage():
        return
    with _timed(timers, "backward-send"):
        _communicate(None, input_tensor_grad, False, False, tensor_shape, dtype_=dtype)


def send_forward_recv_backward(output_tensor: torch.Tensor, tensor_shape: Shape, *,
                               dtype: Optional[torch.dtype] = None, timers: _Timers = None) -> torch.Tensor:
    """Batched send of the activation to the next stage + receive of its gradient."""
    if parallel_state.is_pipeline_last_stage():
        return None
    with _timed(timers, "forward-send-backward-recv"):
        _, output_tensor_grad = _communicate(output_tensor, None, False, True, tensor_shape, dtype_=dtype)
    return output_tensor_grad


def send_backward_recv_forward(input_tensor_grad: torch.Tensor, tensor_shape: Shape, *,
                               dtype: Optional[torch.dtype] = None, timers: _Timers = None) -> torch.Tensor:
    """Batched send of the input gradient to the previous stage + receive of the next activation."""
    if parallel_state.is_pipeline_first_stage():
        return None
    with _timed(timers, "backward-send-forward-recv"):
        input_tensor, _ = _communicate(None, input_tensor_grad, True, False, tensor_shape, dtype_=dtype)
    return input_tensor


def send_forward_recv_forward(output_tensor: torch.Tensor, recv_prev: bool, tensor_shape: Shape, *,
                              dtype: Optional[torch.dtype] = None, timers: _Timers = None) -> torch.Tensor:
    """Batched receive from the previous stage and send to the next (interleaved schedule)."""
    with _timed(timers, "forward-send-forward-recv"):
        input_tensor, _ = _communicate(output_tensor, None, recv_prev, False, tensor_shape, dtype_=dtype)
    return input_tensor


def send_backward_recv_backward(input_tensor_grad: torch.Tensor, recv_next: bool, tensor_shape: Shape, *,
                                dtype: Optional[torch.dtype] = None, timers: _Timers = None) -> torch.Tensor:
    """Batched receive from the next stage and send to the previous (interleaved schedule)."""
    with _timed(timers, "backward-send-backward-recv"):
        _, output_tensor_grad = _communicate(None, input_tensor_grad, False, recv_next, tensor_shape, dtype_=dtype)
    return output_tensor_grad


def send_forward_backward_recv_forward_backward(output_tensor: torch.Tensor, input_tensor_grad: torch.Tensor,
                                                recv_prev: bool, recv_next: bool, tensor_shape: Shape, *,
                                                dtype: Optional[torch.dtype] = None, timers: _Timers = None):
    """Batched send and receive with both neighbours."""
    with _timed(timers, "forward-backward-send-forward-backward-recv"):
        return _communicate(output_tensor, input_tensor_grad, recv_prev, recv_next, tensor_shape, dtype_=dtype)
