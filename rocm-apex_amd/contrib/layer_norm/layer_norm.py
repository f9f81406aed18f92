"""FastLayerNorm (reference apex/contrib/layer_norm/layer_norm.py:7-58).

The reference keeps a second LayerNorm implementation specialised per hidden size (registered
launchers for 768..65536 with cooperative multi-CTA rows).  On gfx950 the general kernels of
``csrc/norm`` already pick the row width / vector count per hidden size (norm_common.h
pick_cfg: one wave64 per row up to 4K, 4-8 waves per row up to 16K+) and handle every size, so
this module is the reference API over those kernels: ``x`` may be any input dtype and
``weight`` / ``bias`` any parameter dtype, the output takes the input dtype, and the backward
returns dgamma / dbeta in the parameter dtype."""
import torch
from torch.nn import init

from ..._autocast_utils import _autocast_disabled, _cast_if_autocast_enabled
from ...ops.layer_norm import ln_bwd, ln_fwd


class FastLayerNormFN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, epsilon):
        x = x.contiguous()
        gamma = gamma.contiguous()
        beta = beta.contiguous()
        shape = (gamma.numel(),)
        y, mu, rsigma = ln_fwd(x, shape, gamma, beta, epsilon, out_dtype=x.dtype)
        ctx.save_for_backward(x, gamma, beta, mu, rsigma)
        ctx.eps = epsilon
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, mu, rsigma = ctx.saved_tensors
        dx, dgamma, dbeta = ln_bwd(dy.contiguous(), x, mu, rsigma, (gamma.numel(),), gamma, beta, ctx.eps)
        return dx, dgamma, dbeta, None


def _fast_layer_norm(x, weight, bias, epsilon):
    args = _cast_if_autocast_enabled(x, weight, bias, epsilon)
    with _autocast_disabled():
        return FastLayerNormFN.apply(*args)


class FastLayerNorm(torch.nn.Module):
    def __init__(self, hidden_size, eps=1e-5):
        super().__init__()
        self.epsilon = eps
        self.weight = torch.nn.Parameter(torch.empty(hidden_size))
        self.bias = torch.nn.Parameter(torch.empty(hidden_size))
        self.reset_parameters()

    def reset_parameters(self):
        init.ones_(self.weight)
        init.zeros_(self.bias)

    def forward(self, x):
        return _fast_layer_norm(x, self.weight, self.bias, self.epsilon)
