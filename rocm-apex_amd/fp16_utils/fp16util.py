"""Network precision conversion and fp32 master-parameter helpers (reference
apex/fp16_utils/fp16util.py:7-187).

Same public functions.  On the GPU the model <-> master copies are ONE multi-tensor launch over
all parameters (``amp_C.multi_tensor_scale`` with scale 1: fp32 -> fp16/bf16 rounding, or the
reverse) instead of one copy kernel per parameter; affine batch norms stay fp32 through every
conversion (MIOpen / the NHWC batch-norm kernels take fp32 statistics and affine parameters)."""
import torch
import torch.nn as nn
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

_BN = nn.modules.batchnorm._BatchNorm


def _is_affine_bn(m):
    return isinstance(m, _BN) and m.affine


class tofp16(nn.Module):
    """First layer of ``network_to_half``: casts the input to fp16."""

    def forward(self, input):
        return input.half()


def BN_convert_float(module):
    """Return ``module`` with every affine batch norm (recursively) converted back to fp32."""
    for m in module.modules():
        if _is_affine_bn(m):
            m.float()
    return module


def network_to_half(network):
    return nn.Sequential(tofp16(), BN_convert_float(network.half()))


def _cast_(t, dtype):
    if t is not None and t.is_floating_point() and t.dtype != dtype:
        t.data = t.data.to(dtype=dtype)


def convert_module(module, dtype):
    """Cast ``module``'s OWN floating parameters (and their grads) and buffers to ``dtype``."""
    for p in module.parameters(recurse=False):
        _cast_(p, dtype)
        if p is not None and p._grad is not None:
            _cast_(p._grad, dtype)
    for b in module.buffers(recurse=False):
        _cast_(b, dtype)


def convert_network(network, dtype):
    """Cast every module except affine batch norms to ``dtype``; RNN weights are re-flattened."""
    for m in network.modules():
        if _is_affine_bn(m):
            continue
        convert_module(m, dtype)
        if isinstance(m, nn.RNNBase):
            m.flatten_parameters()
    return network


class FP16Model(nn.Module):
    """``network`` converted to fp16 (batch norms fp32); inputs are cast on the way in."""

    def __init__(self, network):
        super(FP16Model, self).__init__()
        self.network = convert_network(network, dtype=torch.half)

    def forward(self, *inputs):
        return self.network(*[t.half() for t in inputs])


def backwards_debug_hook(grad):
    raise RuntimeError("master_params recieved a gradient in the backward pass!")


def prep_param_lists(model, flat_master=False):
    """(model params that need grads, their fp32 master copies).  ``flat_master`` packs all
    masters into ONE flat fp32 parameter (its grad buffer allocated up front)."""
    model_params = [p for p in model.parameters() if p.requires_grad]
    if not flat_master:
        masters = [p.detach().clone().float().requires_grad_(True) for p in model_params]
        return model_params, masters
    try:
        flat = _flatten_dense_tensors([p.data for p in model_params]).float()
    except Exception:
        print("Error in prep_param_lists:  model may contain a mixture of parameters of different types.  "
              "Use flat_master=False, or use F16_Optimizer.")
        raise
    flat = nn.Parameter(flat)
    flat.grad = torch.empty_like(flat)
    return model_params, [flat]


def _mt_copy(src, dst):
    """dst[i] <- src[i] for equal-sized lists (dtype conversion included): one multi-tensor
    launch on the GPU, per-tensor copies elsewhere."""
    if not src:
        return
    if src[0].is_cuda:
        from .. import amp_C

        pairs = [(s, d) for s, d in zip(src, dst) if s.is_contiguous() and d.is_contiguous()]
        rest = [(s, d) for s, d in zip(src, dst) if not (s.is_contiguous() and d.is_contiguous())]
        by_types = {}
        for s, d in pairs:
            by_types.setdefault((s.dtype, d.dtype), []).append((s, d))
        flag = torch.zeros(1, dtype=torch.int32, device=src[0].device)
        for group in by_types.values():
            amp_C.multi_tensor_scale(65536, flag, [[s for s, _ in group], [d for _, d in group]], 1.0)
        for s, d in rest:
            d.copy_(s)
        return
    for s, d in zip(src, dst):
        d.copy_(s)


def model_grads_to_master_grads(model_params, master_params, flat_master=False):
    """Copy model grads into the fp32 master grads (allocating them where missing)."""
    if flat_master:
        master_params[0].grad.data.copy_(_flatten_dense_tensors([p.grad.data for p in model_params]))
        return
    src, dst = [], []
    for model, master in zip(model_params, master_params):
        if model.grad is None:
            master.grad = None
            continue
        if master.grad is None:
            master.grad = torch.empty_like(master.data)
        src.append(model.grad.data)
        dst.append(master.grad.data)
    _mt_copy(src, dst)


def master_params_to_model_params(model_params, master_params, flat_master=False):
    """Copy (rounding) the fp32 masters back into the model params."""
    if flat_master:
        masters = _unflatten_dense_tensors(master_params[0].data, model_params)
        _mt_copy(list(masters), [p.data for p in model_params])
        return
    _mt_copy([m.data for m in master_params], [p.data for p in model_params])


def to_python_float(t):
    return t.item() if hasattr(t, "item") else t[0]


clip_grad_norm = torch.nn.utils.clip_grad_norm_
