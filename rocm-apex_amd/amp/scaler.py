"""Dynamic / static loss scaler (reference apex/amp/scaler.py:42-226).

Two execution modes with identical observable semantics (``loss_scale()``, ``_unskipped``,
the overflow message, halving on overflow, doubling after ``scale_window`` clean steps,
min/max clamps, ``amp.state_dict()`` format):

* **sync mode** (reference behaviour): ``update_scale`` reads the overflow flag with one D2H
  copy per step and returns ``should_skip`` to the caller.
* **sync-free mode** (MI355X design, default when every optimizer can consume a device skip
  flag): the scale lives in a device tensor, ``update_scale`` is one 1-thread kernel that
  writes the skip flag, the inverse scale used by this step's gradients and the next scale.
  Fused optimizers skip on the flag inside their kernels.  The host mirror is refreshed lazily
  (``loss_scale()``, ``state_dict()``), which is also when skipped steps are reported.
"""
import torch

from .. import amp_C
from ._amp_state import _amp_state, maybe_print


def scale_check_overflow_python(model_grad, master_grad, scale, check_overflow=False):
    if check_overflow:
        s = float(model_grad.float().sum())
        if s in (float("inf"), -float("inf")) or s != s:
            return True
    if master_grad is not model_grad:
        master_grad.copy_(model_grad)
    if scale != 1.0:
        master_grad.mul_(scale)
    return False


def axpby_check_overflow_python(model_grad, stashed_grad, master_grad, a, b, check_overflow=False):
    if check_overflow:
        s = float(model_grad.float().sum())
        if s in (float("inf"), -float("inf")) or s != s:
            return True
    assert stashed_grad.dtype == master_grad.dtype
    master_grad.data = a * model_grad.data.to(master_grad.dtype) + b * stashed_grad.data
    return False


class LossScaler(object):
    warned_no_fused_kernel = False
    warned_unscaling_non_fp32_grad = False
    has_fused_kernel = True

    def __init__(self, loss_scale, init_scale=2.0 ** 16, scale_factor=2.0, scale_window=2000,
                 min_loss_scale=None, max_loss_scale=2.0 ** 24):
        if loss_scale == "dynamic":
            self.dynamic = True
            self._loss_scale = min(max_loss_scale, init_scale)
        else:
            self.dynamic = False
            self._loss_scale = float(loss_scale)
        self._max_loss_scale = max_loss_scale
        self._min_loss_scale = min_loss_scale
        self._scale_seq_len = scale_window
        self._scale_factor = scale_factor
        self._unskipped = 0
        self._has_overflow = False
        self._device = None
        self._overflow_buf = None
        self._skip_flag = None
        self._state = None        # float32[4]: scale, inv_scale_used, unskipped, skipped_total
        self._device_ahead = False
        self._seen_skips = 0
        self._inv_view = None
        self._holders = []        # optimizer stashes whose pending step reads our flag / inverse scale
        self.sync_free = False

    # ------------------------------------------------------------------ device buffers
    def _ensure(self, device):
        device = torch.device(device)
        if self._overflow_buf is None or self._overflow_buf.device != device:
            self._device = device
            self._overflow_buf = torch.zeros(1, dtype=torch.int32, device=device)
            self._skip_flag = torch.zeros(1, dtype=torch.int32, device=device)
            self._state = torch.tensor([self._loss_scale, 1.0 / self._loss_scale, float(self._unskipped), 0.0],
                                       dtype=torch.float32, device=device)
            self._inv_view = self._state[1:2]
            self._seen_skips = 0
        return self._overflow_buf

    @property
    def overflow_buf(self):
        return self._overflow_buf

    @property
    def skip_flag(self):
        """Device int32[1]: 1 when this step must be skipped (sync-free mode)."""
        return self._skip_flag

    @property
    def inv_scale_used(self):
        """Device float32[1]: 1/scale that the current gradients carry (sync-free mode)."""
        return self._inv_view

    def add_holder(self, stash):
        if not any(h is stash for h in self._holders):
            self._holders.append(stash)

    def detach_waiting_holders(self):
        """Before ``update_scale`` rewrites the flag / inverse scale in place: optimizers that
        still wait for their step (another loss fed them through this scaler) get private
        copies.  The single-loss loop never gets here with a waiting holder, so it copies
        nothing."""
        waiting = [h for h in self._holders if h.exits_since_step > 0]
        for h in waiting:
            if h.skip_flag is self._skip_flag:
                h.skip_flag = self._skip_flag.clone()
            if h.inv_scale is self._inv_view:
                h.inv_scale = self._inv_view.clone()
        self._holders = waiting

    def scale_tensor(self):
        return self._state[0:1]

    # ------------------------------------------------------------------ host view
    def _sync_from_device(self):
        if self._device_ahead and self._state is not None:
            st = self._state.tolist()
            self._loss_scale = st[0]
            self._unskipped = int(st[2])
            skipped = int(st[3])
            if skipped > self._seen_skips:
                maybe_print("Gradient overflow.  Skipped {} step(s) since last report, loss scaler now "
                            "{}".format(skipped - self._seen_skips, self._loss_scale))
                self._seen_skips = skipped
            self._device_ahead = False

    def _push_to_device(self):
        if self._state is not None:
            self._state[0] = self._loss_scale
            self._state[2] = float(self._unskipped)

    def loss_scale(self):
        self._sync_from_device()
        return self._loss_scale

    def scale_loss_value(self, loss):
        """loss.float() * scale without a host sync in sync-free mode."""
        if self.sync_free and self._state is not None and loss.is_cuda:
            return loss.float() * self._state[0]
        return loss.float() * self.loss_scale()

    # ------------------------------------------------------------------ unscale
    def unscale_python(self, model_grads, master_grads, scale):
        for model, master in zip(model_grads, master_grads):
            if model is not None:
                if not LossScaler.warned_unscaling_non_fp32_grad and master.dtype != torch.float32:
                    maybe_print("Attempting to unscale a grad with type {} ".format(master.type()) +
                                "Unscaling non-fp32 grads may indicate an error. "
                                "When using Amp, you don't need to call .half() on your model.")
                    LossScaler.warned_unscaling_non_fp32_grad = True
                self._has_overflow = scale_check_overflow_python(model, master, 1.0 / scale, self.dynamic)
                if self._has_overflow and self.dynamic:
                    break

    def unscale(self, model_grads, master_grads, unused_scale, models_are_masters=False, scale_override=None):
        if self._has_overflow:
            return
        if not model_grads:
            return
        self._ensure(model_grads[0].device)
        if self.sync_free and scale_override is None and model_grads[0].is_cuda:
            # inverse of the current device scale, computed on device
            inv = torch.reciprocal(self._state[0:1])
            amp_C.multi_tensor_scale_t(65536, self._overflow_buf, [model_grads, master_grads], inv)
            return
        scale = self._loss_scale if scale_override is None else scale_override
        if scale == 1.0 and models_are_masters and not self.dynamic:
            return
        amp_C.multi_tensor_scale(65536, self._overflow_buf, [model_grads, master_grads], 1.0 / scale)

    def check_overflow(self, grads):
        """Sync-free overflow probe without materializing unscaled copies."""
        if not grads:
            return
        self._ensure(grads[0].device)
        by_dtype = {}
        for g in grads:
            by_dtype.setdefault(g.dtype, []).append(g)
        for gs in by_dtype.values():
            amp_C.multi_tensor_check_finite(65536, self._overflow_buf, [gs])

    def unscale_with_stashed_python(self, model_grads, stashed_master_grads, master_grads, a, b):
        for model, stashed, master in zip(model_grads, stashed_master_grads, master_grads):
            if model is None and stashed is None:
                continue
            self._has_overflow = axpby_check_overflow_python(model, stashed, master, a, b, self.dynamic)
            if self._has_overflow and self.dynamic:
                break

    def unscale_with_stashed(self, model_grads, stashed_master_grads, master_grads, scale_override=None):
        if self._has_overflow or not model_grads:
            return
        self._ensure(model_grads[0].device)
        grads_have_scale, stashed_have_scale, out_scale = self.loss_scale(), 1.0, 1.0
        if scale_override is not None:
            grads_have_scale, stashed_have_scale, out_scale = scale_override
        amp_C.multi_tensor_axpby(65536, self._overflow_buf, [model_grads, stashed_master_grads, master_grads],
                                 out_scale / grads_have_scale, out_scale / stashed_have_scale, 0)

    def clear_overflow_state(self):
        self._has_overflow = False
        if self._overflow_buf is not None:
            self._overflow_buf.zero_()

    # ------------------------------------------------------------------ update
    def update_scale(self):
        """Reference semantics; returns should_skip (always False in sync-free mode, where the
        skip decision stays on the device)."""
        if self.sync_free and self._state is not None:
            amp_C.amp_update_scale_(self._overflow_buf, self._skip_flag, self._state, self._scale_factor,
                                    1.0 / self._scale_factor, self._scale_seq_len,
                                    float(self._min_loss_scale or 0.0), float(self._max_loss_scale),
                                    self.dynamic)
            self._device_ahead = True
            return False
        if self.dynamic and not self._has_overflow and self._overflow_buf is not None:
            self._has_overflow = bool(self._overflow_buf.item())
        if self._has_overflow and self.dynamic:
            should_skip = True
            if self._min_loss_scale:
                self._loss_scale = max(self._min_loss_scale, self._loss_scale / self._scale_factor)
            else:
                self._loss_scale = self._loss_scale / self._scale_factor
            self._unskipped = 0
        else:
            should_skip = False
            self._unskipped += 1
        if self._unskipped == self._scale_seq_len and self.dynamic:
            self._loss_scale = min(self._max_loss_scale, self._loss_scale * self._scale_factor)
            self._unskipped = 0
        return should_skip

    # ------------------------------------------------------------------ checkpoint support
    def state(self):
        self._sync_from_device()
        return {"loss_scale": self._loss_scale, "unskipped": self._unskipped}

    def load(self, loss_scale, unskipped):
        self._sync_from_device()
        self._loss_scale = loss_scale
        self._unskipped = unskipped
        self._push_to_device()
