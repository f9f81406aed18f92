"""Standalone loss scalers of the legacy ``fp16_utils`` API (``LossScaler`` = static,
``DynamicLossScaler``); capability of reference apex/fp16_utils/loss_scaler.py:10-186.

Design: the scale policy (what happens to the scale on overflow / after a clean window) is a small
state machine driven by a count of clean steps since the last overflow, and overflow detection is
ONE device-side reduction per device over every gradient (``isfinite`` folded into a single flag)
followed by one host read — not a host round trip per tensor.  The amp runtime does not use
these classes (it has the sync-free device scaler in ``apex.amp.scaler``); they exist for code
written against ``apex.fp16_utils``."""
import torch


def to_python_float(t):
    return t.item() if hasattr(t, "item") else t[0]


def _any_non_finite(tensors):
    """True when any element of ``tensors`` is inf/NaN: one flag per device, one host read each."""
    flags = {}
    for t in tensors:
        bad = torch.logical_not(torch.isfinite(t)).any()
        prev = flags.get(t.device)
        flags[t.device] = bad if prev is None else torch.logical_or(prev, bad)
    return any(bool(f) for f in flags.values())


class _ScaleApplier(object):
    """Shared surface: the current scale and the two ways of applying it."""

    cur_scale = 1.0

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        s = self.loss_scale
        return tuple(None if g is None else g * s for g in grad_in)

    def backward(self, loss, retain_graph=False):
        (loss * self.loss_scale).backward(retain_graph=retain_graph)


class LossScaler(_ScaleApplier):
    """Fixed scale; never reports an overflow."""

    def __init__(self, scale=1):
        self.cur_scale = scale

    def has_overflow(self, params):
        return False

    @staticmethod
    def _has_inf_or_nan(x):
        return False

    def update_scale(self, overflow):
        return None


class DynamicLossScaler(_ScaleApplier):
    """Scale that backs off by ``scale_factor`` on an overflow (never below 1) and grows by the same
    factor after every ``scale_window`` consecutive overflow-free steps."""

    def __init__(self, init_scale=2 ** 32, scale_factor=2.0, scale_window=1000):
        self.cur_scale = init_scale
        self.scale_factor = scale_factor
        self.scale_window = scale_window
        self.cur_iter = 0
        self._clean = 0  # overflow-free steps since the last overflow (or the start)

    @property
    def last_overflow_iter(self):
        """Iteration of the most recent overflow (-1 before the first)."""
        return self.cur_iter - self._clean - 1

    @last_overflow_iter.setter
    def last_overflow_iter(self, it):
        self._clean = self.cur_iter - int(it) - 1

    def has_overflow(self, params):
        return _any_non_finite([p.grad.detach() for p in params if p.grad is not None])

    @staticmethod
    def _has_inf_or_nan(x):
        return _any_non_finite([x])

    def update_scale(self, overflow):
        if overflow:
            self.cur_scale = max(self.cur_scale / self.scale_factor, 1)
            self._clean = 0
        else:
            self._clean += 1
            if self._clean % self.scale_window == 0:
                self.cur_scale *= self.scale_factor
        self.cur_iter += 1
