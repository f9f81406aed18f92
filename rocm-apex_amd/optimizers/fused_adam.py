"""FusedAdam (reference apex/optimizers/fused_adam.py:4-173).

Drop-in for ``torch.optim.Adam`` (``adam_w_mode=False``) / ``AdamW`` (default).  One
multi-tensor launch per dtype combination per param group (plain regime), or the sync-free
fused-amp kernel that reads model grads, applies the inverse loss scale, updates the fp32
master/moments and writes the low-precision model weights in a single HBM pass
(see :mod:`apex.optimizers._common`)."""
import torch

from .. import amp_C
from ._common import AmpFusedMixin, amp_ctx, bucket, collect, device_step, lr_tensor


class FusedAdam(AmpFusedMixin, torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, adam_w_mode=True,
                 weight_decay=0.0, amsgrad=False, set_grad_none=True, capturable=False,
                 materialize_master_grads=True):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay)
        super(FusedAdam, self).__init__(params, defaults)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.set_grad_none = set_grad_none
        self.capturable = capturable
        self.materialize_master_grads = materialize_master_grads
        self._dummy_overflow_buf = None

    def zero_grad(self, set_to_none=None):
        if self.set_grad_none if set_to_none is None else set_to_none:
            for group in self.param_groups:
                for p in group["params"]:
                    p.grad = None
        else:
            super(FusedAdam, self).zero_grad(set_to_none=False)

    def _noop(self, device):
        if self._dummy_overflow_buf is None or self._dummy_overflow_buf.device != device:
            self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int32, device=device)
        return self._dummy_overflow_buf

    def _state(self, p):
        state = self.state[p]
        if len(state) == 0:
            state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return state

    def step(self, closure=None, grads=None, output_params=None, scale=None, grad_norms=None):
        if any(p is not None for p in [grads, output_params, scale, grad_norms]):
            raise RuntimeError("FusedAdam has been updated.  Simply initialize it identically to torch.optim.Adam, "
                               "and call step() with no arguments.")
        loss = closure() if closure is not None else None
        st = amp_ctx(self)
        for group in self.param_groups:
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            group["step"] = group.get("step", 0) + 1
            items = list(collect(self, group, st))
            if not items:
                continue
            device = items[0][1].device
            if st is None and not self.capturable:
                # reference regime: one launch per param dtype (grads share it)
                for _, its in bucket(items, lambda it: (it[0].dtype, it[1].dtype)).items():
                    gs = [it[0] for it in its]
                    ps = [it[1] for it in its]
                    ss = [self._state(p) for p in ps]
                    amp_C.multi_tensor_adam(65536, self._noop(device),
                                            [gs, ps, [s["exp_avg"] for s in ss], [s["exp_avg_sq"] for s in ss]],
                                            group["lr"], beta1, beta2, group["eps"], group["step"],
                                            self.adam_w_mode, bias_correction, group["weight_decay"])
                continue
            # sync-free / capturable regime
            skip = st.skip_flag if st is not None else self._noop(device)
            inv = st.inv_scale if (st is not None and st.fused_pending) else None
            if st is not None:
                step_t = device_step(group, st, device)
            else:
                step_t = group.get("_step_t")
                if step_t is None or step_t.device != device:
                    # seeded from the host count (a resumed optimizer continues its bias
                    # correction); group['step'] was already bumped for this call
                    step_t = group["_step_t"] = torch.full((1,), float(group["step"] - 1), dtype=torch.float32,
                                                           device=device)
                step_t.add_(1.0)
            lr_t = lr_tensor(group, device)
            key = lambda it: (it[0].dtype, it[1].dtype, None if it[2] is None else it[2].dtype)  # noqa: E731
            for (gt, pt, ot), its in bucket(items, key).items():
                gs = [it[0] for it in its]
                ps = [it[1] for it in its]
                ss = [self._state(p) for p in ps]
                lists = [gs, ps, [s["exp_avg"] for s in ss], [s["exp_avg_sq"] for s in ss]]
                if ot is not None:
                    lists.append([it[2] for it in its])
                amp_C.multi_tensor_adam_capturable(65536, skip, lists, lr_t, beta1, beta2, group["eps"], step_t,
                                                   self.adam_w_mode, bias_correction, group["weight_decay"], inv)
            if st is not None and any(it[2] is not None for it in items):
                st.model_written_by_step = True
        return loss
