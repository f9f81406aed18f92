"""LARC: layer-wise adaptive rate control around any optimizer (reference
apex/parallel/LARC.py:5-107).

Per parameter tensor p with gradient g (and the group's weight decay wd, which LARC absorbs —
the wrapped optimizer steps with wd = 0):

    ratio = trust_coefficient * ||p|| / (||g|| + wd * ||p|| + eps)
    clip mode:  ratio = min(ratio / lr, 1)
    g <- (g + wd * p) * ratio          (ratio = 1 where ||p|| or ||g|| is zero)

MI355X form: all tensor norms of a dtype group come from ONE multi-tensor L2-norm launch per
list (params, grads; ``amp_C.multi_tensor_l2norm`` per-tensor mode) and the update of every
gradient is two foreach kernels with the ratios kept on the device — no per-parameter norm
launches and no host synchronization.  Everything else (state, param_groups, state_dict, ...)
is the wrapped optimizer's, by delegation."""
import torch

from .. import amp_C


class LARC(object):
    def __init__(self, optimizer, trust_coefficient=0.02, clip=True, eps=1e-8):
        self.optim = optimizer
        self.trust_coefficient = trust_coefficient
        self.clip = clip
        self.eps = eps

    # ---- everything not LARC-specific is the wrapped optimizer's ----
    def __getattr__(self, name):
        if name == "optim":
            raise AttributeError(name)
        return getattr(self.optim, name)

    def __getstate__(self):
        return self.optim.__getstate__()

    def __setstate__(self, state):
        self.optim.__setstate__(state)

    def __repr__(self):
        return self.optim.__repr__()

    @property
    def param_groups(self):
        return self.optim.param_groups

    @param_groups.setter
    def param_groups(self, value):
        self.optim.param_groups = value

    @property
    def state(self):
        return self.optim.state

    # ---- the adaptive step ----
    @staticmethod
    def _norms(tensors):
        if tensors[0].is_cuda:
            flag = torch.zeros(1, dtype=torch.int32, device=tensors[0].device)
            _, per = amp_C.multi_tensor_l2norm(65536, flag, [tensors], True)
            return per.float()
        return torch.stack([t.float().norm() for t in tensors])

    def _scale_group(self, group, wd):
        params = [p for p in group["params"] if p.grad is not None]
        if not params:
            return
        by_dtype = {}
        for p in params:
            by_dtype.setdefault((p.dtype, p.grad.dtype, p.device), []).append(p)
        for ps in by_dtype.values():
            grads = [p.grad.data for p in ps]
            pn = self._norms([p.data for p in ps])
            gn = self._norms(grads)
            ratio = self.trust_coefficient * pn / (gn + pn * wd + self.eps)
            if self.clip:
                ratio = torch.clamp(ratio / group["lr"], max=1.0)
            live = (pn != 0) & (gn != 0)
            ratio = torch.where(live, ratio, torch.ones_like(ratio)).to(grads[0].dtype)
            if wd != 0:
                wdv = (live.to(grads[0].dtype) * wd).unbind(0)
                torch._foreach_add_(grads, torch._foreach_mul([p.data for p in ps], list(wdv)))
            torch._foreach_mul_(grads, list(ratio.unbind(0)))

    def step(self, closure=None):
        saved = []
        with torch.no_grad():
            for group in self.optim.param_groups:
                wd = group.get("weight_decay", 0)
                saved.append(wd)
                group["weight_decay"] = 0
                self._scale_group(group, wd)
        try:
            return self.optim.step(closure) if closure is not None else self.optim.step()
        finally:
            for group, wd in zip(self.optim.param_groups, saved):
                group["weight_decay"] = wd
