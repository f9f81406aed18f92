"""Legacy contrib FusedLAMB (reference apex/contrib/optimizers/fused_lamb.py:6-208), the optimizer behind
``apex.contrib.optimizers.FP16_Optimizer``; shared plumbing in ``_legacy_common.py``."""

import torch

from ... import amp_C


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
