"""Legacy contrib FusedAdam (reference apex/contrib/optimizers/fused_adam.py:6-206), the optimizer behind
``apex.contrib.optimizers.FP16_Optimizer``; shared plumbing in ``_legacy_common.py``."""

import torch

from ... import amp_C
from ._legacy_common import _groupify, _split_by


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
