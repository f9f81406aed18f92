"""Legacy contrib optimizers driven by ``apex.contrib.optimizers.FP16_Optimizer``
(reference apex/contrib/optimizers/fused_adam.py:6-206, fused_sgd.py:7-211, fused_lamb.py:6-208).

Their ``step`` receives the (loss-scaled, possibly fp16) gradients, the fp32 master params are
``group['params']`` and an optional reduced-precision copy is written out.  Each group is one
multi-tensor launch per dtype combination on the gfx950 engine (``amp_C``); the loss scale and
max-grad-norm clip are folded into a single device inverse-scale factor consumed by the kernel.
"""
import types

import torch

from ... import amp_C


def _groupify(x, n):
    if x is None:
        return [None] * n
    if isinstance(x, types.GeneratorType):
        return [list(x)]
    x = list(x)
    if x and not isinstance(x[0], (list, tuple)):
        return [x]
    return x


def _split_by(keys, *lists):
    """Partition parallel lists by a key (dtype tuple) so each multi-tensor launch is homogeneous."""
    out = {}
    for i, k in enumerate(keys):
        slot = out.setdefault(k, [[] for _ in lists])
        for j, lst in enumerate(lists):
            slot[j].append(lst[i])
    return out


class FusedAdam(torch.optim.Optimizer):
    """Adam with explicit grads / output params (reference contrib fused_adam.py).

    Update: ``p -= lr * (m_hat / (sqrt(v_hat) + eps) + wd * p)`` (``eps_inside_sqrt=False``) — the
    decoupled-decay form of the reference's ``fused_adam_cuda`` mode 1."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, eps_inside_sqrt=False,
                 weight_decay=0.0, max_grad_norm=0.0, amsgrad=False, use_mt=False, amp_scale_adjustment=1.0):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        if eps_inside_sqrt:
            raise RuntimeError("eps_inside_sqrt is not supported by the gfx950 Adam kernel")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self._amp_scale_adjustment = amp_scale_adjustment
        self._use_multi_tensor = True

    def step(self, closure=None, grads=None, output_params=None, scale=1.0, grad_norms=None):
        loss = closure() if closure is not None else None
        if hasattr(self, "_amp_stash"):
            grads = self._amp_stash.grads
            output_params = self._amp_stash.output_params
            scale = self._amp_stash.scale * self._amp_scale_adjustment
            grad_norms = self._amp_stash.grad_norms
        n = len(self.param_groups)
        grads_group = _groupify(grads, n)
        out_group = _groupify(output_params, n)
        if grad_norms is None:
            grad_norms = [None] * n
        for group, g_this, o_this, gnorm in zip(self.param_groups, grads_group, out_group, grad_norms):
            params = group["params"]
            g_this = g_this if g_this is not None else [None] * len(params)
            o_this = o_this if o_this is not None else [None] * len(params)
            combined = float(scale)
            if group["max_grad_norm"] > 0 and gnorm is not None:
                clip = ((float(gnorm) / scale) + 1e-6) / group["max_grad_norm"]
                if clip > 1:
                    combined = clip * scale
            beta1, beta2 = group["betas"]
            sel_g, sel_p, sel_m, sel_v, sel_o, keys = [], [], [], [], [], []
            for p, g, o in zip(params, g_this, o_this):
                if g is None:
                    if p.grad is None:
                        continue
                    g = p.grad
                if g.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                sel_g.append(g)
                sel_p.append(p)
                sel_m.append(st["exp_avg"])
                sel_v.append(st["exp_avg_sq"])
                sel_o.append(o)
                keys.append((g.dtype, p.dtype, o is not None and o.numel() > 0, o.dtype if o is not None else None,
                             st["step"]))
            for key, (g_l, p_l, m_l, v_l, o_l) in _split_by(keys, sel_g, sel_p, sel_m, sel_v, sel_o).items():
                dev = p_l[0].device
                noop = torch.zeros(1, dtype=torch.int32, device=dev)
                tl = [g_l, p_l, m_l, v_l] + ([o_l] if key[2] else [])
                amp_C.multi_tensor_adam_capturable(
                    65536, noop, tl, torch.tensor([float(group["lr"])], device=dev), beta1, beta2, group["eps"],
                    torch.tensor([float(key[4])], device=dev), 1, 1 if group["bias_correction"] else 0,
                    group["weight_decay"], torch.tensor([1.0 / combined], device=dev))
        return loss


class FusedSGD(torch.optim.Optimizer):
    """SGD for ``FP16_Optimizer`` (reference contrib fused_sgd.py): ``grads`` and ``output_params``
    are mandatory; fp16 model params get their copy written by the same launch."""

    def __init__(self, params, lr=0.1, momentum=0, dampening=0, weight_decay=0, nesterov=False,
                 wd_after_momentum=False, materialize_master_grads=True):
        if momentum < 0.0 or weight_decay < 0.0 or lr < 0.0:
            raise ValueError("invalid hyper-parameter")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))
        self.wd_after_momentum = wd_after_momentum

    def get_momentums(self, params):
        first_run = True
        moms = []
        for p in params:
            st = self.state[p]
            if "momentum_buffer" not in st:
                st["momentum_buffer"] = torch.zeros_like(p)
            else:
                first_run = False
            moms.append(st["momentum_buffer"])
        return moms, first_run

    def step(self, closure=None, grads=None, output_params=None, scale=1.0, grad_norms=None):
        if hasattr(self, "_amp_stash"):
            raise RuntimeError("apex.contrib.optimizers.FusedSGD should not be used with AMP.")
        loss = closure() if closure is not None else None
        if grads is None or output_params is None:
            raise RuntimeError("apex.contrib.optimizers.FusedSGD must be wrapped with "
                               "apex.contrib.optimizers.FP16_Optimizer which provides grads and output_params.")
        n = len(self.param_groups)
        for group, g_this, o_this in zip(self.param_groups, _groupify(grads, n), _groupify(output_params, n)):
            if g_this is None or o_this is None:
                raise RuntimeError("apex.contrib.optimizers.FusedSGD only works when all parameters require grad.")
            masters = group["params"]
            keys = [(g.dtype, o.dtype) for g, o in zip(g_this, o_this)]
            for (gdt, odt), (g_l, p_l, o_l) in _split_by(keys, list(g_this), list(masters), list(o_this)).items():
                moms, first = self.get_momentums(p_l)
                dev = p_l[0].device
                noop = torch.zeros(1, dtype=torch.int32, device=dev)
                tl = [g_l, p_l, moms] + ([o_l] if odt != p_l[0].dtype else [])
                amp_C.multi_tensor_sgd(65536, noop, tl, group["weight_decay"], group["momentum"],
                                       group["dampening"], group["lr"], group["nesterov"], first,
                                       self.wd_after_momentum, 1.0 / scale)
                if odt == p_l[0].dtype:
                    for o, p in zip(o_l, p_l):
                        if o.data_ptr() != p.data_ptr():
                            o.data.copy_(p.data)
        return loss


class FusedLAMB(torch.optim.Optimizer):
    """LAMB with per-dtype gradient norms blended into one global norm (reference contrib
    fused_lamb.py: fp16 / fp32 grad lists normed separately, then ``lamb`` over each dtype list)."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01,
                 amsgrad=False, adam_w_mode=True, grad_averaging=True, set_grad_none=True, max_grad_norm=1.0):
        if amsgrad:
            raise RuntimeError("FusedLAMB does not support the AMSGrad variant.")
        super().__init__(params, dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                                      weight_decay=weight_decay, grad_averaging=grad_averaging,
                                      max_grad_norm=max_grad_norm))
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.set_grad_none = set_grad_none

    def zero_grad(self, set_to_none=None):
        if self.set_grad_none if set_to_none is None else set_to_none:
            for group in self.param_groups:
                for p in group["params"]:
                    p.grad = None
        else:
            super().zero_grad(set_to_none=False)

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        by_dtype = {}
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    if p.dtype not in (torch.float32, torch.float16, torch.bfloat16):
                        raise RuntimeError("FusedLAMB only supports fp32 / fp16 / bf16 params")
                    by_dtype.setdefault(p.grad.dtype, []).append(p.grad)
        if not by_dtype:
            return loss
        dev = next(iter(by_dtype.values()))[0].device
        noop = torch.zeros(1, dtype=torch.int32, device=dev)
        sq = torch.zeros(1, dtype=torch.float32, device=dev)
        for lst in by_dtype.values():
            nrm, _ = amp_C.multi_tensor_l2norm(65536, noop, [lst], False)
            sq = sq + nrm.float().reshape(1) ** 2
        gnorm = sq.sqrt()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            group["step"] = group.get("step", 0) + 1
            lists = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedLAMB does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                slot = lists.setdefault(p.dtype, [[], [], [], []])
                for j, t in enumerate((p.grad, p, st["exp_avg"], st["exp_avg_sq"])):
                    slot[j].append(t)
            for tl in lists.values():
                amp_C.multi_tensor_lamb(65536, noop, tl, group["lr"], beta1, beta2, group["eps"], group["step"],
                                        1 if group["bias_correction"] else 0, group["weight_decay"],
                                        1 if group["grad_averaging"] else 0, self.adam_w_mode, gnorm,
                                        group["max_grad_norm"])
        return loss
