"""Multi-layer perceptron with fused bias + activation (reference apex/mlp/mlp.py:8-79,
csrc/mlp.cpp, csrc/mlp_cuda.cu).

Every layer is ``act(h W^T + b)`` with act in {none, relu, sigmoid} (applied after every layer,
as the reference).  GPU fp16/bf16: each layer's forward is ONE gfx950 MFMA GEMM launch with the
bias + activation epilogue; in backward each input-gradient GEMM carries the previous layer's
activation derivative as its epilogue (the reference runs separate bias/activation kernels with
cross-block semaphores, mlp_cuda.cu:528-1041), weight gradients are GEMMs and bias gradients
column sums.  Other dtypes / CPU: torch."""
import math
from copy import copy

import torch
from torch import nn

from .. import _native
from ..amp import half_function

_ACT_NAMES = {"none": 0, "relu": 1, "sigmoid": 2}


def _g():
    return _native.require("gemm").gemm


def _act(x, activation):
    if activation == 1:
        return torch.relu(x)
    if activation == 2:
        return torch.sigmoid(x)
    return x


def _dact(g, out, activation):
    if activation == 1:
        return g * (out > 0).to(g.dtype)
    if activation == 2:
        return g * out * (1 - out)
    return g


def _native_ok(args, num_layers, use_bias):
    x = args[0]
    if not _native.use_native(x) or _native.submodule("gemm") is None:
        return False
    if x.dtype not in (torch.float16, torch.bfloat16) or x.dim() != 2:
        return False
    return all(t.dtype == x.dtype and all(d % 8 == 0 for d in t.shape) for t in args[1:1 + num_layers]) and \
        x.shape[1] % 8 == 0


class MlpFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bias, activation, *args):
        num_layers = (len(args) - 1) // (2 if bias else 1)
        weights = args[1:1 + num_layers]
        biases = args[1 + num_layers:] if bias else [None] * num_layers
        native = _native_ok(args, num_layers, bias)
        outputs = []
        h = args[0]
        for w, b in zip(weights, biases):
            if native:
                g = _g()
                epi = {0: g.EPI_NONE, 1: g.EPI_RELU, 2: g.EPI_SIGMOID}[activation]
                h, _ = g.linear(h, w, b, epi, False)
            else:
                z = torch.matmul(h, w.t())
                if b is not None:
                    z = z + b
                h = _act(z, activation)
            outputs.append(h)
        ctx.save_for_backward(*args)
        ctx.outputs = outputs
        ctx.bias = bias
        ctx.activation = activation
        ctx.num_layers = num_layers
        ctx.native = native
        return outputs[-1]

    @staticmethod
    def backward(ctx, grad_o):
        args = ctx.saved_tensors
        outputs = ctx.outputs
        L, act = ctx.num_layers, ctx.activation
        x, weights = args[0], args[1:1 + L]
        dweights, dbiases = [None] * L, [None] * L
        dz = _dact(grad_o.contiguous(), outputs[-1], act)  # last layer's activation derivative
        dx = None
        for i in range(L - 1, -1, -1):
            h_prev = outputs[i - 1] if i > 0 else x
            if ctx.native:
                g = _g()
                dweights[i] = g.linear_wgrad(dz, h_prev)
                if ctx.bias:
                    dbiases[i] = g.column_sum(dz)
                if i > 0:
                    epi = {0: g.EPI_NONE, 1: g.EPI_DRELU, 2: g.EPI_DSIGMOID}[act]
                    dz = g.linear_dgrad(dz, weights[i], epi, outputs[i - 1] if act else None)
                elif ctx.needs_input_grad[2]:
                    dx = g.linear_dgrad(dz, weights[i], g.EPI_NONE, None)
            else:
                dweights[i] = dz.t().matmul(h_prev)
                if ctx.bias:
                    dbiases[i] = dz.sum(0)
                if i > 0:
                    dz = _dact(dz.matmul(weights[i]), outputs[i - 1], act)
                else:
                    dx = dz.matmul(weights[i])
        del ctx.outputs
        grads = [dx] + dweights + (dbiases if ctx.bias else [])
        return (None, None, *grads)


mlp_function = half_function(MlpFunction.apply)


class MLP(torch.nn.Module):
    """MLP(mlp_sizes, bias=True, activation='relu'): ``len(mlp_sizes) - 1`` layers."""

    def __init__(self, mlp_sizes, bias=True, activation="relu"):
        super().__init__()
        self.num_layers = len(mlp_sizes) - 1
        self.mlp_sizes = copy(mlp_sizes)
        self.bias = 1 if bias else 0
        if activation not in _ACT_NAMES:
            raise TypeError("activation must be relu or none.")
        self.activation = _ACT_NAMES[activation]
        self.weights = []
        self.biases = []
        for i in range(self.num_layers):
            w = torch.nn.Parameter(torch.empty(mlp_sizes[i + 1], mlp_sizes[i]))
            self.weights.append(w)
            setattr(self, "weight_{}".format(i), w)
            if self.bias:
                b = torch.nn.Parameter(torch.empty(mlp_sizes[i + 1]))
                self.biases.append(b)
                setattr(self, "bias_{}".format(i), b)
        self.reset_parameters()

    def reset_parameters(self):
        for weight in self.weights:
            dimsum = weight.size(0) + weight.size(1)
            nn.init.normal_(weight, 0.0, math.sqrt(2.0 / float(dimsum)))
        if self.bias:
            for bias in self.biases:
                nn.init.normal_(bias, 0.0, math.sqrt(1.0 / float(bias.size(0))))

    def _apply(self, fn, *a, **kw):
        # keep the python lists pointing at the (possibly replaced) parameters
        super()._apply(fn, *a, **kw)
        self.weights = [getattr(self, "weight_{}".format(i)) for i in range(self.num_layers)]
        if self.bias:
            self.biases = [getattr(self, "bias_{}".format(i)) for i in range(self.num_layers)]
        return self

    def forward(self, input):
        return mlp_function(self.bias, self.activation, input, *self.weights, *self.biases)

    def extra_repr(self):
        return f"MLP sizes: {self.mlp_sizes}, Bias={self.bias}, activation={self.activation}"
