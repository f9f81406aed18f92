"""``amp.scale_loss`` / ``amp.disable_casts`` and the legacy handle objects
(reference apex/amp/handle.py:16-281)."""
import contextlib

import torch

from ._amp_state import _amp_state, maybe_print
from .opt import OptimWrapper
from .scaler import LossScaler


def _as_list(optimizers):
    if isinstance(optimizers, (list, tuple)):
        return list(optimizers)
    return [optimizers]


def _patch_skip_step(opt, loss_scaler, loss_id):
    """On overflow (sync mode) the next ``optimizer.step()`` becomes a no-op that restores the
    real step afterwards (reference apex/amp/handle.py:129-154)."""
    opt_step = opt.step

    def skip_step(closure=None):
        if closure is not None:
            raise RuntimeError("Currently, Amp does not support closure use with optimizers.")
        maybe_print(("Gradient overflow.  Skipping step, loss scaler "
                     "{} reducing loss scale to {}").format(loss_id, loss_scaler.loss_scale()))
        if hasattr(opt._amp_stash, "all_fp32_from_fp16_params"):
            for param in opt._amp_stash.all_fp32_from_fp16_params:
                param.grad = None
        if hasattr(opt, "most_recent_scale"):
            opt.most_recent_scale = 1.0
            opt.scale_set_by_backward = False
        opt.step = opt_step
        opt._amp_stash.already_patched = False

    opt.step = skip_step
    opt._amp_stash.already_patched = True


def _passthrough(scaler):
    """Nothing to scale or unscale: no master weights and a static scale of 1."""
    props = _amp_state.opt_properties
    return (not props.master_weights) and (not scaler.dynamic) and scaler.loss_scale() == 1.0


def _finish_backward(optimizers, scaler, loss_id, delay_overflow_check):
    """Unscale into the master grads, update the scale and arm the skip (device flag in
    sync-free mode, patched ``step`` otherwise)."""
    scaler.clear_overflow_state()
    for opt in optimizers:
        opt._post_amp_backward(scaler)
        opt._amp_stash.params_have_scaled_gradients = False
    if scaler.sync_free:
        scaler.detach_waiting_holders()
    skip = scaler.update_scale() if not delay_overflow_check else False
    if scaler.sync_free:
        for opt in optimizers:
            st = opt._amp_stash
            # several backward passes may feed one step (several losses / scalers): the step
            # must skip if any of them overflowed, so the device flags are OR-ed until it runs
            if st.skip_flag is None or st.exits_since_step == 0:
                st.skip_flag = scaler.skip_flag
            else:
                st.skip_flag = torch.maximum(st.skip_flag, scaler.skip_flag)
            st.exits_since_step += 1
            st.inv_scale = scaler.inv_scale_used
            scaler.add_holder(st)
        return
    if skip:
        for opt in (o for o in optimizers if not o._amp_stash.already_patched):
            _patch_skip_step(opt, scaler, loss_id)


@contextlib.contextmanager
def scale_loss(loss, optimizers, loss_id=0, model=None, delay_unscale=False, delay_overflow_check=False):
    """Yields ``loss.float() * loss_scale``; on exit (unless ``delay_unscale``) checks the grads
    for inf/NaN, unscales them into the master grads and updates the loss scale.

    ``model`` is accepted for API compatibility and unused (as in the reference)."""
    props = getattr(_amp_state, "opt_properties", None)
    if props is None:
        raise RuntimeError("Invoked 'with amp.scale_loss`, but internal Amp state has not been initialized.  "
                           "model, optimizer = amp.initialize(model, optimizer, opt_level=...) must be called "
                           "before `with amp.scale_loss`.")
    if not props.enabled:
        yield loss
        return
    opts = _as_list(optimizers)
    scaler = _amp_state.loss_scalers[loss_id]
    try:
        if _passthrough(scaler):
            yield loss.float()
            return
        if not delay_unscale:
            for opt in (o for o in opts if not o._amp_stash.params_have_scaled_gradients):
                opt._prepare_amp_backward()
        if loss.is_cuda:
            scaler._ensure(loss.device)
        yield scaler.scale_loss_value(loss)
        if delay_unscale:
            for opt in opts:
                opt._amp_stash.params_have_scaled_gradients = True
        else:
            _finish_backward(opts, scaler, loss_id, delay_overflow_check)
    finally:
        if props.patch_torch_functions:
            _amp_state.handle._clear_cache()


@contextlib.contextmanager
def disable_casts():
    """Temporarily disables O1/O4 casting (reference apex/amp/handle.py:163-167)."""
    h = getattr(_amp_state, "handle", None)
    prev = h._is_active if h is not None else None
    if h is not None:
        h._is_active = False
    try:
        yield
    finally:
        if h is not None:
            h._is_active = prev


class NoOpHandle(object):
    """Legacy handle when amp is disabled: casts inactive, loss passed through unscaled."""

    has_cache = False
    verbose = False

    def is_active(self):
        return False

    @contextlib.contextmanager
    def _disable_casts(self):
        yield

    def wrap_optimizer(self, optimizer, num_loss=1):
        return OptimWrapper(optimizer, self, num_loss)

    @contextlib.contextmanager
    def scale_loss(self, loss, optimizer):
        yield loss

    def _clear_cache(self):
        pass

    def _deactivate(self):
        pass


class AmpHandle(NoOpHandle):
    """Legacy handle (reference apex/amp/handle.py:170-251): owns the O1 weight-cast cache, the
    default loss scaler and the list of patched functions (uninstalled by ``_deactivate``)."""

    def __init__(self, loss_scale="dynamic", enable_caching=True, verbose=False):
        self._enable_caching = enable_caching
        self._verbose = verbose
        self._cache = {}
        self._default_scaler = LossScaler(loss_scale)
        self._is_active = True
        self._all_wrappers = []

    has_cache = property(lambda self: self._enable_caching)
    cache = property(lambda self: self._cache)
    verbose = property(lambda self: self._verbose)

    def is_active(self):
        return self._is_active

    @contextlib.contextmanager
    def _disable_casts(self):
        prev, self._is_active = self._is_active, False
        try:
            yield
        finally:
            self._is_active = prev

    def wrap_optimizer(self, optimizer, num_loss=1):
        self._default_scaler = None  # scaling moves to the per-loss scalers of the wrapper
        return OptimWrapper(optimizer, self, num_loss)

    @contextlib.contextmanager
    def scale_loss(self, loss, optimizer):
        raise RuntimeError("The old Amp API is no longer supported.  Please move to the new API: "
                           "amp.initialize() + amp.scale_loss().")
        yield  # pragma: no cover

    def _clear_cache(self):
        self._cache.clear()

    def _save_func(self, mod, fn, func):
        self._all_wrappers.append((mod, fn, func))

    def _deactivate(self):
        from . import amp as _amp

        _amp._uninstall()
        self._all_wrappers = []

    def remove_cache(self, param):
        if self._enable_caching:
            self._cache.pop(param, None)
