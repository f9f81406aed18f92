"""FusedLAMB (reference apex/optimizers/fused_lamb.py:4-215).

Global grad norm over all grads (one l2norm launch per grad dtype + a tiny combine), then per
group: one fused stage-1 launch (moments, update written into the grad buffer, AND per-tensor
||p|| / ||update|| in the same pass) and one stage-2 launch (trust-ratio apply).  The reference
needs >= 10 launches for the same step."""
import torch

from .. import amp_C
from ._common import AmpFusedMixin, amp_ctx, bucket, collect, device_step, lr_tensor


class FusedLAMB(AmpFusedMixin, torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01,
                 amsgrad=False, adam_w_mode=True, grad_averaging=True, set_grad_none=True, max_grad_norm=1.0,
                 use_nvlamb=False, materialize_master_grads=True):
        if amsgrad:
            raise RuntimeError("FusedLAMB does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        grad_averaging=grad_averaging, max_grad_norm=max_grad_norm)
        super(FusedLAMB, self).__init__(params, defaults)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.set_grad_none = set_grad_none
        self.use_nvlamb = use_nvlamb
        self.materialize_master_grads = materialize_master_grads
        self._dummy_overflow_buf = None

    def zero_grad(self, set_to_none=None):
        if self.set_grad_none if set_to_none is None else set_to_none:
            for group in self.param_groups:
                for p in group["params"]:
                    p.grad = None
        else:
            super(FusedLAMB, self).zero_grad(set_to_none=False)

    def _noop(self, device):
        if self._dummy_overflow_buf is None or self._dummy_overflow_buf.device != device:
            self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int32, device=device)
        return self._dummy_overflow_buf

    def _state(self, p):
        state = self.state[p]
        if len(state) == 0:
            state["exp_avg"] = torch.zeros_like(p)
            state["exp_avg_sq"] = torch.zeros_like(p)
        return state

    def _global_grad_norm(self, all_items, device, inv=None):
        noop = self._noop(device)
        norms = []
        for _, its in bucket(all_items, lambda it: it[0].dtype).items():
            norms.append(amp_C.multi_tensor_l2norm(65536, noop, [[it[0] for it in its]], False)[0])
        if not norms:
            return torch.zeros(1, device=device)
        gn = norms[0] if len(norms) == 1 else torch.stack([n.reshape(()) for n in norms]).norm().reshape(1)
        if inv is not None:
            gn = gn * inv
        return gn

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        st = amp_ctx(self)
        per_group = [list(collect(self, g, st)) for g in self.param_groups]
        all_items = [it for its in per_group for it in its]
        if not all_items:
            return loss
        device = all_items[0][1].device
        inv = st.inv_scale if (st is not None and st.fused_pending) else None
        global_grad_norm = self._global_grad_norm(all_items, device, inv)
        max_grad_norm = self.defaults["max_grad_norm"]
        for group, items in zip(self.param_groups, per_group):
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            grad_averaging = 1 if group["grad_averaging"] else 0
            group["step"] = group.get("step", 0) + 1
            if not items:
                continue
            if st is None:
                for _, its in bucket(items, lambda it: (it[0].dtype, it[1].dtype)).items():
                    ps = [it[1] for it in its]
                    ss = [self._state(p) for p in ps]
                    amp_C.multi_tensor_lamb(65536, self._noop(device),
                                            [[it[0] for it in its], ps, [s["exp_avg"] for s in ss],
                                             [s["exp_avg_sq"] for s in ss]],
                                            group["lr"], beta1, beta2, group["eps"], group["step"], bias_correction,
                                            group["weight_decay"], grad_averaging, self.adam_w_mode,
                                            global_grad_norm, max_grad_norm, self.use_nvlamb)
                continue
            step_t = device_step(group, st, device)
            lr_t = lr_tensor(group, device)
            mgn = torch.full((1,), float(max_grad_norm), device=device)
            inv_t = inv if inv is not None else torch.ones(1, device=device)
            key = lambda it: (it[0].dtype, it[1].dtype, None if it[2] is None else it[2].dtype)  # noqa: E731
            for (_, _, ot), its in bucket(items, key).items():
                ps = [it[1] for it in its]
                ss = [self._state(p) for p in ps]
                lists = [[it[0] for it in its], ps, [s["exp_avg"] for s in ss], [s["exp_avg_sq"] for s in ss]]
                if ot is not None:
                    lists.append([it[2] for it in its])
                amp_C.multi_tensor_lamb_mp(65536, self._noop(device), lists, lr_t, beta1, beta2, group["eps"],
                                           step_t, bias_correction, group["weight_decay"], grad_averaging,
                                           self.adam_w_mode, global_grad_norm, mgn, self.use_nvlamb,
                                           st.skip_flag, inv_t)
            if any(it[2] is not None for it in items):
                st.model_written_by_step = True
        return loss
