"""DistributedFusedAdamV2: the reversible-step variant (reference
apex/contrib/optimizers/distributed_fused_adam_v2.py:7-615)."""
from ... import amp_C
from .distributed_fused_adam import DistributedFusedAdam


class DistributedFusedAdamV2(DistributedFusedAdam):
    """Reference v2 (reversible step, distributed_fused_adam_v2.py + the
    ``maybe_adam_undo`` kernel, apex/contrib/csrc/optimizers/fused_adam_cuda_kernel.cu:657).

    ``revert_step()`` rolls the last step back in place with the inverse-Adam kernel
    (``amp_C.multi_tensor_adam_undo``): it reuses the reduced gradient shard that is still in the
    reduce-scatter staging buffer, so no copy of the master / moment shards is ever kept.  Valid
    until the next backward starts reducing (checked); a skipped step reverts to a no-op."""

    def __init__(self, *args, revertible=True, **kwargs):
        super().__init__(*args, **kwargs)
        self._revertible = revertible
        self._stepped_generation = None

    def revert_step(self):
        flat = self._flat
        if not self._revertible or self._stepped_generation is None:
            raise RuntimeError("revert_step needs revertible=True and a previous step")
        if flat.generation != self._stepped_generation:
            raise RuntimeError("revert_step: gradients of a later backward already replaced the step's "
                               "reduced gradients")
        g0 = self.param_groups[0]
        beta1, beta2 = g0["betas"]
        amp_C.multi_tensor_adam_undo(65536, self._skip, self._adam_lists(flat.grad_shard_views()), self._lr_t,
                                     beta1, beta2, g0["eps"], self._step_t, self.adam_w_mode,
                                     1 if g0["bias_correction"] else 0, g0["weight_decay"], self._inv)
        self._step_t.sub_(1 - self._skip.float())
        for g in self.param_groups:
            g["step"] = max(0, g.get("step", 1) - 1)
        self._stepped_generation = None
        flat.all_gather_params(self._ag_dtype)
