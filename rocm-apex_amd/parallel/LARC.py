"""LARC optimizer wrapper (reference apex/parallel/LARC.py:5-107): layer-wise adaptive rate
scaling with 'clip' (min with the global lr) or 'scale' mode; weight decay is absorbed into the
adaptive rate and removed from the inner optimizer for the step."""
import torch
from torch.optim import Optimizer


class LARC(object):
    def __init__(self, optimizer, trust_coefficient=0.02, clip=True, eps=1e-8):
        self.optim = optimizer
        self.trust_coefficient = trust_coefficient
        self.eps = eps
        self.clip = clip

    def __getstate__(self):
        return self.optim.__getstate__()

    def __setstate__(self, state):
        self.optim.__setstate__(state)

    @property
    def state(self):
        return self.optim.state

    def __repr__(self):
        return self.optim.__repr__()

    @property
    def param_groups(self):
        return self.optim.param_groups

    @param_groups.setter
    def param_groups(self, value):
        self.optim.param_groups = value

    def state_dict(self):
        return self.optim.state_dict()

    def load_state_dict(self, state_dict):
        self.optim.load_state_dict(state_dict)

    def zero_grad(self):
        self.optim.zero_grad()

    def add_param_group(self, param_group):
        self.optim.add_param_group(param_group)

    def step(self):
        with torch.no_grad():
            weight_decays = []
            for group in self.optim.param_groups:
                wd = group["weight_decay"] if "weight_decay" in group else 0
                weight_decays.append(wd)
                group["weight_decay"] = 0
                for p in group["params"]:
                    if p.grad is None:
                        continue
                    param_norm = torch.norm(p.data)
                    grad_norm = torch.norm(p.grad.data)
                    # adaptive lr computed on device (no host sync)
                    adaptive_lr = self.trust_coefficient * param_norm / (grad_norm + param_norm * wd + self.eps)
                    if self.clip:
                        adaptive_lr = torch.minimum(adaptive_lr / group["lr"], torch.ones_like(adaptive_lr))
                    ok = (param_norm != 0) & (grad_norm != 0)
                    adaptive_lr = torch.where(ok, adaptive_lr, torch.ones_like(adaptive_lr))
                    p.grad.data.add_(p.data * wd * ok.to(p.dtype))
                    p.grad.data.mul_(adaptive_lr.to(p.grad.dtype))
        self.optim.step()
        for i, group in enumerate(self.optim.param_groups):
            group["weight_decay"] = weight_decays[i]
