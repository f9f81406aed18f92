"""Legacy ``handle.wrap_optimizer`` API: a wrapped optimizer with one dynamic loss scaler per loss
(capability of reference apex/amp/opt.py:9-103).

Design on the device ``LossScaler`` (``apex.amp.scaler``):

* every loss owns a scaler; on a GPU it runs sync-free (scale, overflow flag and skip decision
  stay in device memory), so ``scale_loss`` never reads anything back to the host;
* the gradients a loss produced are unscaled in place by one multi-tensor launch (which also sets
  that loss's overflow flag), and with several losses they are summed into persistent fp32
  accumulators on the device instead of being cloned aside and added back;
* ``step()`` does the single host read of the step — the OR of the losses' skip flags — then
  either skips (reporting the overflow) or runs the wrapped optimizer on the summed gradients.
"""
import contextlib

import torch

from ._amp_state import maybe_print
from .scaler import LossScaler


class OptimWrapper(object):
    def __init__(self, optimizer, amp_handle, num_loss):
        self._optimizer = optimizer
        self._amp_handle = amp_handle
        self._num_loss = int(num_loss)
        self._loss_idx = 0
        self._scalers = [LossScaler("dynamic") for _ in range(self._num_loss)]
        self._host_skip = [False] * self._num_loss  # CPU scalers decide on the host
        self._acc = {}  # id(param) -> fp32 gradient sum over the losses of this step

    def _params(self):
        return [p for group in self._optimizer.param_groups for p in group["params"]]

    def _cur_loss_scaler(self):
        if not 0 <= self._loss_idx < self._num_loss:
            raise RuntimeError("scale_loss called more times than num_loss={} before step()".format(self._num_loss))
        return self._scalers[self._loss_idx]

    @contextlib.contextmanager
    def scale_loss(self, loss):
        if not self._amp_handle.is_active():
            yield loss
            return
        scaler = self._cur_loss_scaler()
        scaler.sync_free = loss.is_cuda
        params = self._params()
        if self._loss_idx > 0:
            for p in params:  # earlier losses' gradients already sit in the accumulators
                p.grad = None
        if loss.is_cuda:
            scaler._ensure(loss.device)
        yield scaler.scale_loss_value(loss)
        grads = [p.grad for p in params if p.grad is not None]
        scaler.clear_overflow_state()
        if grads:
            scaler.unscale(grads, grads, None, models_are_masters=True)
        skip = scaler.update_scale()
        self._host_skip[self._loss_idx] = bool(skip)
        if self._num_loss > 1:
            for p in params:
                if p.grad is None:
                    continue
                acc = self._acc.get(id(p))
                if acc is None:
                    self._acc[id(p)] = p.grad.detach().float().clone()
                else:
                    acc.add_(p.grad.detach())
        self._loss_idx += 1

    def _skip_this_step(self, n):
        flags = [s.skip_flag for s in self._scalers[:n] if s.sync_free and s.skip_flag is not None]
        skip = any(self._host_skip[:n])
        if flags:
            skip = skip or bool(torch.stack([f.reshape(()) for f in flags]).any())  # one host read
        return skip

    def step(self, closure=None):
        if not self._amp_handle.is_active():
            return self._optimizer.step(closure=closure)
        if closure is not None:
            raise NotImplementedError("The `closure` argument is unsupported by the amp optimizer wrapper.")
        n, self._loss_idx = self._loss_idx, 0
        params = self._params()
        for p in params:
            self._amp_handle.remove_cache(p)
        if self._acc:
            for p in params:
                acc = self._acc.get(id(p))
                if acc is not None:
                    p.grad = acc.to(p.dtype) if p.dtype != torch.float32 else acc
            self._acc = {}
        skip = self._skip_this_step(n)
        self._host_skip = [False] * self._num_loss
        if skip:
            maybe_print("Gradient overflow, skipping update")
            return None
        return self._optimizer.step()

    # everything else (param_groups, state, state_dict, add_param_group, ...) is the wrapped
    # optimizer's own
    def __getattr__(self, attr):
        return getattr(self._optimizer, attr)

    def zero_grad(self, set_to_none=True):
        self._acc = {}
        return self._optimizer.zero_grad(set_to_none=set_to_none)


def _delegate(name):
    def method(self, *args, **kwargs):
        return getattr(self._optimizer, name)(*args, **kwargs)

    method.__name__ = name
    return method


for _name in ("__getstate__", "__setstate__", "__repr__", "state_dict", "load_state_dict", "add_param_group"):
    setattr(OptimWrapper, _name, _delegate(_name))
