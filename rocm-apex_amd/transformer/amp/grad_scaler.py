"""Model-parallel-aware GradScaler (reference apex/transformer/amp/grad_scaler.py:8-106).

``torch.amp.GradScaler`` whose inf/NaN verdict is MAX-reduced over the model-parallel group,
so every TP/PP rank skips (or takes) the same step.  Unlike the reference, the step decision
does not ``.item()`` each per-device flag on the host: the flags are summed on the device and
one all-reduce + one host read decides the step."""
from collections import defaultdict

import torch

from .. import parallel_state


def _model_parallel_group_or_none():
    try:
        return parallel_state.get_model_parallel_group()
    except AssertionError:
        return None


class GradScaler(torch.amp.GradScaler):
    def __init__(self, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True, device="cuda"):
        super().__init__(device, init_scale=init_scale, growth_factor=growth_factor, backoff_factor=backoff_factor,
                         growth_interval=growth_interval, enabled=enabled)

    def _reduce(self, t):
        group = _model_parallel_group_or_none()
        if group is not None and torch.distributed.is_initialized():
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
        return t

    def _maybe_opt_step(self, optimizer, optimizer_state, *args, **kwargs):
        flags = list(optimizer_state["found_inf_per_device"].values())
        found_inf = torch.stack([f.to(flags[0].device).float().reshape(()) for f in flags]).sum().reshape(1)
        self._reduce(found_inf)
        if found_inf.item() == 0:
            return optimizer.step(*args, **kwargs)
        return None

    def update(self, new_scale=None):
        if not self._enabled:
            return
        _scale, _growth_tracker = self._check_scale_growth_tracker("update")
        if new_scale is not None:
            if isinstance(new_scale, float):
                self._scale.fill_(new_scale)
            else:
                reason = "new_scale should be a float or a 1-element torch.cuda.FloatTensor with requires_grad=False."
                assert new_scale.numel() == 1 and new_scale.requires_grad is False, reason
                self._scale.copy_(new_scale)
        else:
            found_infs = [found_inf.to(device=_scale.device, non_blocking=True)
                          for state in self._per_optimizer_states.values()
                          for found_inf in state["found_inf_per_device"].values()]
            assert len(found_infs) > 0, "No inf checks were recorded prior to update."
            found_inf_combined = torch.stack([f.reshape(()) for f in found_infs]).sum().reshape(1)
            self._reduce(found_inf_combined)
            torch._amp_update_scale_(_scale, _growth_tracker, found_inf_combined, self._growth_factor,
                                     self._backoff_factor, self._growth_interval)
        from torch.amp.grad_scaler import _refresh_per_optimizer_state

        self._per_optimizer_states = defaultdict(_refresh_per_optimizer_state)
