"""FusedAdagrad (reference apex/optimizers/fused_adagrad.py:5-121)."""
import torch

from .. import amp_C


class FusedAdagrad(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-2, eps=1e-10, weight_decay=0.0, set_grad_none=True, adagrad_w_mode=False):
        defaults = dict(lr=lr, eps=eps, weight_decay=weight_decay)
        super(FusedAdagrad, self).__init__(params, defaults)
        self.adagrad_w_mode = 1 if adagrad_w_mode else 0
        self.set_grad_none = set_grad_none
        self._dummy_overflow_buf = None

    def zero_grad(self, set_to_none=None):
        if self.set_grad_none if set_to_none is None else set_to_none:
            for group in self.param_groups:
                for p in group["params"]:
                    p.grad = None
        else:
            super(FusedAdagrad, self).zero_grad(set_to_none=False)

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            buckets = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdagrad does not support sparse gradients")
                state = self.state[p]
                if len(state) == 0:
                    state["sum"] = torch.zeros_like(p)
                if p.dtype not in (torch.float16, torch.bfloat16, torch.float32):
                    raise RuntimeError("FusedAdagrad only support fp16, bfloat16 and fp32.")
                b = buckets.setdefault(p.dtype, ([], [], []))
                b[0].append(p.grad)
                b[1].append(p)
                b[2].append(state["sum"])
            for gs, ps, hs in buckets.values():
                dev = ps[0].device
                if self._dummy_overflow_buf is None or self._dummy_overflow_buf.device != dev:
                    self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int32, device=dev)
                amp_C.multi_tensor_adagrad(65536, self._dummy_overflow_buf, [gs, ps, hs], group["lr"], group["eps"],
                                           self.adagrad_w_mode, group["weight_decay"])
        return loss
