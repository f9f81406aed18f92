"""FusedSGD (reference apex/optimizers/fused_sgd.py:6-227).

Momentum SGD over ``multi_tensor_sgd``.  Under amp with master weights the kernel writes the
low-precision model weights itself (depth-4 launch), as in the reference; in the sync-free amp
regime it additionally skips on the device overflow flag and (``materialize_master_grads=False``)
reads the loss-scaled model grads directly."""
import torch
from torch.optim.optimizer import required

from .. import amp_C
from ._common import AmpFusedMixin, amp_ctx, bucket, collect, lr_tensor


class FusedSGD(AmpFusedMixin, torch.optim.Optimizer):
    def __init__(self, params, lr=required, momentum=0, dampening=0, weight_decay=0, nesterov=False,
                 wd_after_momentum=False, materialize_master_grads=True, set_grad_none=False):
        if lr is not required and lr < 0.0:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if momentum < 0.0:
            raise ValueError("Invalid momentum value: {}".format(momentum))
        if weight_decay < 0.0:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay, nesterov=nesterov)
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super(FusedSGD, self).__init__(params, defaults)
        self.wd_after_momentum = wd_after_momentum
        self.materialize_master_grads = materialize_master_grads
        self.most_recent_scale = 1.0
        self.scale_set_by_backward = False
        self.set_grad_none = set_grad_none
        dev = self.param_groups[0]["params"][0].device
        self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int32, device=dev)

    def __setstate__(self, state):
        super(FusedSGD, self).__setstate__(state)
        for group in self.param_groups:
            group.setdefault("nesterov", False)

    def zero_grad(self, set_to_none=None):
        if self.set_grad_none if set_to_none is None else set_to_none:
            for group in self.param_groups:
                for p in group["params"]:
                    p.grad = None
        else:
            super(FusedSGD, self).zero_grad(set_to_none=False)

    def get_momentums(self, params):
        momentums = []
        first_run = True
        for p in params:
            param_state = self.state[p]
            if "momentum_buffer" not in param_state:
                first_run = True
                param_state["momentum_buffer"] = torch.zeros_like(p)
            else:
                first_run = False
            momentums.append(param_state["momentum_buffer"])
        return momentums, first_run

    def _noop(self, device):
        if self._dummy_overflow_buf.device != device:
            self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int32, device=device)
        return self._dummy_overflow_buf

    def _launch(self, launch_set, group, first_run, scale):
        if len(launch_set[0]) == 0:
            return
        amp_C.multi_tensor_sgd(65536, self._noop(launch_set[0][0].device), launch_set, group["weight_decay"],
                               group["momentum"], group["dampening"], group["lr"], group["nesterov"], first_run,
                               self.wd_after_momentum, scale)

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        st = amp_ctx(self)
        if st is not None:
            self._step_sync_free(st)
            return loss
        explicit_master_params = hasattr(self, "_amp_stash") and hasattr(self._amp_stash, "fp32_from_fp16_groups")
        for gid, group in enumerate(self.param_groups):
            first_runs = [True, True]
            if explicit_master_params:
                stash = self._amp_stash
                fp32_params = [p for p in stash.fp32_from_fp32_groups[gid] if p.grad is not None]
                fp32_grads = [p.grad for p in fp32_params]
                fp32_moms, first_runs[1] = self.get_momentums(fp32_params)
                masters = stash.fp32_from_fp16_groups[gid]
                models = stash.fp16_groups[gid]
                if self.materialize_master_grads:
                    sel = [i for i, p in enumerate(masters) if p.grad is not None]
                    grads16 = [masters[i].grad for i in sel]
                else:
                    sel = [i for i, p in enumerate(models) if p.grad is not None]
                    grads16 = [models[i].grad for i in sel]
                m_params = [masters[i] for i in sel]
                moms16, first_runs[0] = self.get_momentums(m_params)
                fp16_set = [grads16, m_params, moms16, [models[i] for i in sel]]
                launch_sets = [fp16_set, [fp32_grads, fp32_params, fp32_moms]]
            else:
                launch_sets = []
                for dt in (torch.float16, torch.bfloat16, torch.float32):
                    ps = [p for p in group["params"] if p.dtype == dt and p.grad is not None]
                    moms, fr = self.get_momentums(ps)
                    launch_sets.append([[p.grad for p in ps], ps, moms])
                    first_runs.append(fr)
                first_runs = first_runs[2:]
            for launch_set, first_run in zip(launch_sets, first_runs):
                assert len(launch_set[0]) == len(launch_set[1]) == len(launch_set[2])
                self._launch(launch_set, group, first_run, 1.0 / self.most_recent_scale)
        self.most_recent_scale = 1.0
        self.scale_set_by_backward = False
        return loss

    def _step_sync_free(self, st):
        inv = st.inv_scale if st.fused_pending else None
        wrote = False
        for group in self.param_groups:
            items = list(collect(self, group, st))
            if not items:
                continue
            device = items[0][1].device
            lr_t = lr_tensor(group, device)
            key = lambda it: (it[0].dtype, it[1].dtype, None if it[2] is None else it[2].dtype)  # noqa: E731
            for (_, _, ot), its in bucket(items, key).items():
                ps = [it[1] for it in its]
                moms, first_run = self.get_momentums(ps)
                lists = [[it[0] for it in its], ps, moms]
                if ot is not None:
                    lists.append([it[2] for it in its])
                    wrote = True
                amp_C.multi_tensor_sgd_capturable(65536, st.skip_flag, lists, group["weight_decay"],
                                                  group["momentum"], group["dampening"], lr_t, group["nesterov"],
                                                  first_run, self.wd_after_momentum, inv)
        if wrote:
            st.model_written_by_step = True
        self.most_recent_scale = 1.0
        self.scale_set_by_backward = False
