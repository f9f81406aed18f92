"""Optimizer patching for amp (reference apex/amp/_process_optimizer.py:14-489).

Reference behaviour is kept: with master weights, fp16/bf16 params are replaced in the param
groups by fp32 masters, grads are unscaled into fp32 master grads after backward, and the
masters are copied back into the model after ``step()``.

Data parallel: gradients of parameters owned by ``apex.parallel.DistributedDataParallel`` are
views into its persistent all-reduce buckets.  Where the single-GPU fused path drops grads (sets
them to None, letting autograd hand over fresh buffers), DDP-owned grads are instead zeroed in
place, one memset per bucket (``parallel.distributed.zero_bucketed_grads``), so backward keeps
accumulating into the buckets and nothing is copied per parameter.

MI355X fast path ("fused amp"): when the optimizer is one of this package's fused optimizers
constructed with ``materialize_master_grads=False`` and the loss scaler runs sync-free, no fp32
master grads are materialized at all.  After backward only a read-only overflow probe runs
(2 B/param for bf16 grads); the optimizer kernel then reads the *model* grads, applies the
device inverse scale in fp32 registers, updates the fp32 master/state and writes the bf16/fp16
model weights in the same pass, skipping on the device skip flag.  That is one HBM pass instead
of unscale-copy + update + master->model copy.
"""
import types

import torch

from .. import amp_C
from ..fp16_utils import master_params_to_model_params
from ._amp_state import maybe_print

_LOW = (torch.float16, torch.bfloat16)


class AmpOptimizerState(object):
    def __init__(self):
        pass


def _is_fused_amp(opt):
    return bool(getattr(opt, "_amp_fused_capable", False)) and not getattr(opt, "materialize_master_grads", True)


def _ddp():
    from ..parallel import distributed

    return distributed


def _reset_grads(params, to_none):
    """Reset model grads after a step / on zero_grad: DDP-owned ones are zeroed in their buckets
    (views kept), the rest set to None (``to_none``) or zeroed in place."""
    owned = _ddp().zero_bucketed_grads(params)
    for param in params:
        if id(param) in owned or param.grad is None:
            continue
        if to_none:
            param.grad = None
        else:
            if param.grad.grad_fn is not None:
                param.grad.detach_()
            else:
                param.grad.requires_grad_(False)
            param.grad.zero_()


def _master_params_to_model_params(self):
    stash = self._amp_stash
    if len(stash.all_fp16_params) > 0:
        dev = stash.all_fp16_params[0].device
        buf = stash.dummy_overflow_buf if stash.dummy_overflow_buf.device == dev else torch.zeros(
            1, dtype=torch.int32, device=dev)
        amp_C.multi_tensor_scale(65536, buf, [stash.all_fp32_from_fp16_params, stash.all_fp16_params], 1.0)


def lazy_init_with_master_weights(self):
    stash = self._amp_stash
    stash.fp16_groups = []
    stash.fp32_from_fp16_groups = []
    stash.fp32_from_fp32_groups = []
    for param_group in self.param_groups:
        fp16_this, fp32_this, fp32_from_fp16_this = [], [], []
        for i, param in enumerate(param_group["params"]):
            if not param.requires_grad:
                continue
            if param.dtype in _LOW:
                fp16_this.append(param)
                master = param.detach().clone().float()
                master.requires_grad = True
                param_group["params"][i] = master
                fp32_from_fp16_this.append(master)
                if param in self.state:
                    self.state[master] = self.state.pop(param)
            elif param.dtype == torch.float32:
                fp32_this.append(param)
                param_group["params"][i] = param
            else:
                raise TypeError("Optimizer's parameters must be float32, float16 or bfloat16. "
                                "Received {}".format(param.type()))
        stash.fp16_groups.append(fp16_this)
        stash.fp32_from_fp16_groups.append(fp32_from_fp16_this)
        stash.fp32_from_fp32_groups.append(fp32_this)

    stash.all_fp16_params = [p for g in stash.fp16_groups for p in g]
    stash.all_fp32_from_fp16_params = [p for g in stash.fp32_from_fp16_groups for p in g]
    stash.all_fp32_from_fp32_params = [p for g in stash.fp32_from_fp32_groups for p in g]
    stash.all_fp16_grad_stash = [None for _ in stash.all_fp16_params]
    stash.all_fp32_from_fp32_grad_stash = [None for _ in stash.all_fp32_from_fp32_params]
    # model param -> master param, used by the fused optimizers to write both in one pass
    stash.master_of = {id(m): p for m, p in zip(stash.all_fp16_params, stash.all_fp32_from_fp16_params)}
    stash.model_of = {id(p): m for m, p in zip(stash.all_fp16_params, stash.all_fp32_from_fp16_params)}
    for param in stash.all_fp32_from_fp16_params:
        param.grad = None
    for param in stash.all_fp32_from_fp32_params:
        param.grad = None
    # recast preexisting per-param state tensors
    self.load_state_dict(self.state_dict())


def _host_scale(scaler):
    """The host copy of the loss scale when it is authoritative without a device read: always
    for a static scaler; for a sync-free dynamic scaler the device value is read only when a
    caller really needs the number (accumulated grads), never on the common path — a device
    read would serialise the step and break hipGraph capture."""
    if not scaler.dynamic:
        return scaler._loss_scale
    return None if scaler.sync_free else scaler.loss_scale()


# accumulate fresh fp32 grads onto stashed ones with the device loss scale (sync-free); False =
# read the scale on the host as the reference does (A/B, tests)
_STASH_DEVICE_SCALE = True


def post_backward_models_are_masters(scaler, params, stashed_grads, scale_override=None):
    host = _host_scale(scaler)
    grads_have_scale, stashed_have_scale, out_scale = host, 1.0, 1.0
    if host == 1.0 and not scaler.dynamic:
        for i in range(len(stashed_grads)):
            stashed_grads[i] = None
        return
    if scale_override is not None:
        grads_have_scale, stashed_have_scale, out_scale = scale_override
    needing, needing_with_stash, stashed = [], [], []
    for param, stashed_grad in zip(params, stashed_grads):
        if param.grad is None and stashed_grad is not None:
            param.grad = stashed_grad
        elif param.grad is not None and stashed_grad is None:
            needing.append(param.grad)
        elif param.grad is not None and stashed_grad is not None:
            needing_with_stash.append(param.grad)
            stashed.append(stashed_grad)
    if needing_with_stash and grads_have_scale is None:
        if _STASH_DEVICE_SCALE and scale_override is None and scaler.sync_free and needing_with_stash[0].is_cuda:
            # sync-free accumulation onto the stash (e.g. zero_grad left zeroed fp32 grads): the
            # fresh grads unscaled by the DEVICE scale (overflow-checked), then the stash added —
            # the reference's axpby(1 / scale, 1) without reading the scale on the host
            scaler.unscale(needing_with_stash, needing_with_stash, None, models_are_masters=True)
            torch._foreach_add_(needing_with_stash, stashed)
            needing_with_stash, stashed = [], []
        else:
            grads_have_scale = scaler.loss_scale()  # accumulation across losses needs the number
    if needing:
        scaler.unscale(needing, needing, None, models_are_masters=True,
                       scale_override=None if scale_override is None else grads_have_scale / out_scale)
    if needing_with_stash:
        scaler.unscale_with_stashed(needing_with_stash, stashed, needing_with_stash,
                                    scale_override=(grads_have_scale, stashed_have_scale, out_scale))
    for i in range(len(stashed_grads)):
        stashed_grads[i] = None


def prepare_backward_with_master_weights(self):
    stash = self._amp_stash
    self._amp_lazy_init()
    stash.exit_mode = "ref"
    if _is_fused_amp(self) and stash.fused_ok and not any(
            p.grad is not None for p in stash.all_fp32_from_fp16_params):
        # fused exit: keep existing (still scaled) grads aside; fresh grads land in .grad.  A
        # DDP bucket view known to be zero stays attached (backward accumulates into the bucket);
        # a non-zero one is stashed as a copy, since the bucket is about to be overwritten
        stash.exit_mode = "fused"
        zero_views = _ddp().zeroed_bucket_params(stash.all_fp16_params + stash.all_fp32_from_fp32_params)
        for params, stashed in ((stash.all_fp16_params, stash.all_fp16_grad_stash),
                                (stash.all_fp32_from_fp32_params, stash.all_fp32_from_fp32_grad_stash)):
            for i, param in enumerate(params):
                g = param.grad
                if g is None or id(param) in zero_views:
                    stashed[i] = None
                    continue
                stashed[i] = g.clone() if getattr(param, "_apex_ddp_owner", None) is not None else g
                param.grad = None
        return
    for param in stash.all_fp16_params:
        param.grad = None
    for i, param in enumerate(stash.all_fp32_from_fp32_params):
        stash.all_fp32_from_fp32_grad_stash[i] = param.grad
        param.grad = None


def _post_backward_fused(self, scaler):
    """Fused fast path.  When grads are accumulated across scale_loss exits (stash present) the
    two contributions are combined into fp32 master grads, each with the inverse scale it was
    produced under, and the following step uses the materialized masters."""
    stash = self._amp_stash
    has_stash = any(g is not None for g in stash.all_fp16_grad_stash) or any(
        g is not None for g in stash.all_fp32_from_fp32_grad_stash)
    if not has_stash:
        grads = [p.grad for p in stash.all_fp16_params if p.grad is not None]
        grads += [p.grad for p in stash.all_fp32_from_fp32_params if p.grad is not None]
        scaler.check_overflow(grads)
        stash.fused_pending = True
        return
    inv_now = torch.reciprocal(scaler.scale_tensor())
    inv_prev = scaler.inv_scale_used.clone()  # written by the previous exit's update_scale
    pairs = list(zip(stash.all_fp16_params, stash.all_fp32_from_fp16_params, stash.all_fp16_grad_stash))
    pairs += [(p, p, s) for p, s in zip(stash.all_fp32_from_fp32_params, stash.all_fp32_from_fp32_grad_stash)]
    probe = []
    for model, master, old in pairs:
        g = model.grad
        if g is None and old is None:
            continue
        acc = torch.zeros_like(master, dtype=torch.float32)
        if g is not None:
            acc.add_(g.float() * inv_now)
        if old is not None:
            acc.add_(old.float() * inv_prev)
        probe.append(acc)
        if model is not master:
            model.grad = None
        master.grad = acc
    scaler.check_overflow(probe)
    for i in range(len(stash.all_fp16_grad_stash)):
        stash.all_fp16_grad_stash[i] = None
    for i in range(len(stash.all_fp32_from_fp32_grad_stash)):
        stash.all_fp32_from_fp32_grad_stash[i] = None
    stash.fused_pending = False


def post_backward_with_master_weights(self, scaler):
    stash = self._amp_stash
    self._amp_lazy_init()
    if getattr(stash, "exit_mode", "ref") == "fused":
        if scaler.sync_free:
            return _post_backward_fused(self, scaler)
        # fused exit requested but the scaler runs in sync mode: restore stashed grads and
        # materialize master grads like the reference
        for i, param in enumerate(stash.all_fp16_params):
            stash.all_fp16_grad_stash[i] = None
    fp16_needing, new_fp32, fp16_with_stash, preexisting = [], [], [], []
    for fp16_param, fp32_param in zip(stash.all_fp16_params, stash.all_fp32_from_fp16_params):
        if fp16_param.grad is None and fp32_param.grad is not None:
            continue
        elif fp16_param.grad is not None and fp32_param.grad is None:
            fp32_param.grad = torch.empty_like(fp32_param)
            fp16_needing.append(fp16_param.grad)
            new_fp32.append(fp32_param.grad)
        elif fp16_param.grad is not None and fp32_param.grad is not None:
            fp16_with_stash.append(fp16_param.grad)
            preexisting.append(fp32_param.grad)
    if fp16_needing:
        scaler.unscale(fp16_needing, new_fp32, _host_scale(scaler), models_are_masters=False)
    if fp16_with_stash:
        scaler.unscale_with_stashed(fp16_with_stash, preexisting, preexisting)
    post_backward_models_are_masters(scaler, stash.all_fp32_from_fp32_params, stash.all_fp32_from_fp32_grad_stash)
    stash.fused_pending = False


def lazy_init_no_master_weights(self):
    stash = self._amp_stash
    stash.all_fp16_params = []
    stash.all_fp32_params = []
    for param_group in self.param_groups:
        for param in param_group["params"]:
            if param.dtype in _LOW:
                stash.all_fp16_params.append(param)
            elif param.dtype == torch.float32:
                stash.all_fp32_params.append(param)
            else:
                raise TypeError("Optimizer's parameters must be float32, float16 or bfloat16. "
                                "Received {}".format(param.type()))
    stash.all_fp16_grad_stash = [None for _ in stash.all_fp16_params]
    stash.all_fp32_grad_stash = [None for _ in stash.all_fp32_params]


def prepare_backward_no_master_weights(self):
    stash = self._amp_stash
    self._amp_lazy_init()
    for i, param in enumerate(stash.all_fp16_params):
        stash.all_fp16_grad_stash[i] = param.grad
        param.grad = None
    for i, param in enumerate(stash.all_fp32_params):
        stash.all_fp32_grad_stash[i] = param.grad
        param.grad = None


def post_backward_no_master_weights(self, scaler):
    stash = self._amp_stash
    self._amp_lazy_init()
    for params, stashed in ((stash.all_fp16_params, stash.all_fp16_grad_stash),
                            (stash.all_fp32_params, stash.all_fp32_grad_stash)):
        post_backward_models_are_masters(scaler, params, stashed)


# ---- FusedSGD variants (reference apex/amp/_process_optimizer.py:258-310) -------------------
def prepare_backward_with_master_weights_FusedSGD(self):
    if self.materialize_master_grads:
        prepare_backward_with_master_weights(self)
    else:
        stash = self._amp_stash
        self._amp_lazy_init()
        for i, param in enumerate(stash.all_fp16_params):
            stash.all_fp16_grad_stash[i] = param.grad
            param.grad = None
        for i, param in enumerate(stash.all_fp32_from_fp32_params):
            stash.all_fp32_from_fp32_grad_stash[i] = param.grad
            param.grad = None


def post_backward_with_master_weights_FusedSGD(self, scaler):
    if self.materialize_master_grads:
        post_backward_with_master_weights(self, scaler)
        return
    stash = self._amp_stash
    self._amp_lazy_init()
    grads_have_scale = scaler.loss_scale()
    stashed_have_scale = self.most_recent_scale
    out_scale = grads_have_scale
    if self.scale_set_by_backward:
        out_scale = min(grads_have_scale, self.most_recent_scale)
    for params, stashed in ((stash.all_fp16_params, stash.all_fp16_grad_stash),
                            (stash.all_fp32_from_fp32_params, stash.all_fp32_from_fp32_grad_stash)):
        post_backward_models_are_masters(scaler, params, stashed, (grads_have_scale, stashed_have_scale, out_scale))
    self.most_recent_scale = out_scale
    self.scale_set_by_backward = True


def _amp_lazy_init(self):
    stash = self._amp_stash
    if not stash.lazy_init_called:
        self._lazy_init_maybe_master_weights()
        stash.lazy_init_called = True


def _process_optimizer(optimizer, properties):
    if hasattr(optimizer, "_amp_stash"):
        raise RuntimeError("A given optimizer should only be passed through amp.initialize once.")
    optimizer._amp_stash = AmpOptimizerState()
    stash = optimizer._amp_stash
    stash.lazy_init_called = False
    stash.already_patched = False
    stash.params_have_scaled_gradients = False
    stash.fused_pending = False
    stash.fused_ok = True
    stash.skip_flag = None
    stash.inv_scale = None
    stash.master_weights = bool(properties.master_weights)

    for name in ("_lazy_init_maybe_master_weights", "_master_params_to_model_params", "_prepare_amp_backward",
                 "_post_amp_backward", "_amp_lazy_init"):
        if hasattr(optimizer, name):
            raise RuntimeError("Incoming optimizer already has {} defined.".format(name))

    dev = None
    for g in optimizer.param_groups:
        for p in g["params"]:
            dev = p.device
            break
        if dev is not None:
            break
    stash.dummy_overflow_buf = torch.zeros(1, dtype=torch.int32, device=dev if dev is not None else "cpu")

    from ..optimizers import FusedSGD

    is_fused_sgd = isinstance(optimizer, FusedSGD) and not _is_fused_amp(optimizer)

    if properties.master_weights:
        optimizer._lazy_init_maybe_master_weights = types.MethodType(lazy_init_with_master_weights, optimizer)
        optimizer._master_params_to_model_params = types.MethodType(_master_params_to_model_params, optimizer)

        old_step = optimizer.step

        def new_step(self, closure=None):
            if closure is not None:
                raise RuntimeError("Currently, Amp does not support closure use with optimizers.")
            retval = old_step()
            st = self._amp_stash
            if not (isinstance(self, FusedSGD) or getattr(st, "model_written_by_step", False)):
                self._master_params_to_model_params()
            st.model_written_by_step = False
            for param in st.all_fp32_from_fp16_params:
                param.grad = None
            if st.fused_pending:
                # model grads were consumed directly by the fused kernel
                _reset_grads(st.all_fp16_params + st.all_fp32_from_fp32_params, True)
                st.fused_pending = False
            return retval

        optimizer.step = types.MethodType(new_step, optimizer)

        def new_zero_grad(self, set_to_none=None):
            st = self._amp_stash
            self._amp_lazy_init()
            to_none = _is_fused_amp(self) if set_to_none is None else set_to_none
            _reset_grads(st.all_fp16_params + st.all_fp32_from_fp32_params, to_none)
            for param in st.all_fp32_from_fp16_params:
                param.grad = None

        optimizer.zero_grad = types.MethodType(new_zero_grad, optimizer)

        if is_fused_sgd:
            optimizer._prepare_amp_backward = types.MethodType(prepare_backward_with_master_weights_FusedSGD,
                                                               optimizer)
            optimizer._post_amp_backward = types.MethodType(post_backward_with_master_weights_FusedSGD, optimizer)
        else:
            optimizer._prepare_amp_backward = types.MethodType(prepare_backward_with_master_weights, optimizer)
            optimizer._post_amp_backward = types.MethodType(post_backward_with_master_weights, optimizer)
    else:
        optimizer._lazy_init_maybe_master_weights = types.MethodType(lazy_init_no_master_weights, optimizer)
        optimizer._prepare_amp_backward = types.MethodType(prepare_backward_no_master_weights, optimizer)
        optimizer._post_amp_backward = types.MethodType(post_backward_no_master_weights, optimizer)

    optimizer._amp_lazy_init = types.MethodType(_amp_lazy_init, optimizer)

    # sync-free skip flags of the scale_loss exits feeding one step are OR-ed (handle.py);
    # the step closes that window
    stash.exits_since_step = 0
    step_before_count = optimizer.step

    def counted_step(self, *args, **kwargs):
        try:
            return step_before_count(*args, **kwargs)
        finally:
            self._amp_stash.exits_since_step = 0

    optimizer.step = types.MethodType(counted_step, optimizer)

    old_add_param_group = optimizer.add_param_group

    def new_add_param_group(self, new_group):
        st = self._amp_stash
        if not st.lazy_init_called:
            self._lazy_init_maybe_master_weights()
            st.lazy_init_called = True
        assert isinstance(new_group, dict), "param group must be a dict"
        new_params = new_group["params"]
        if isinstance(new_params, torch.Tensor):
            new_group["params"] = [new_params]
        elif isinstance(new_params, set):
            raise TypeError("optimizer parameters need to be organized in ordered collections, but "
                            "the ordering of tensors in sets will change between runs. Please use a list instead.")
        else:
            new_group["params"] = list(new_params)
        if properties.master_weights:
            fp16_this, fp32_this, fp32_from_fp16_this = [], [], []
            for i, param in enumerate(new_group["params"]):
                if not param.requires_grad:
                    continue
                if param.dtype in _LOW:
                    fp16_this.append(param)
                    master = param.detach().clone().float()
                    master.requires_grad = True
                    new_group["params"][i] = master
                    fp32_from_fp16_this.append(master)
                elif param.dtype == torch.float32:
                    fp32_this.append(param)
                else:
                    raise TypeError("Optimizer's parameters must be float32, float16 or bfloat16. "
                                    "Received {}".format(param.type()))
            st.fp16_groups.append(fp16_this)
            st.fp32_from_fp16_groups.append(fp32_from_fp16_this)
            st.fp32_from_fp32_groups.append(fp32_this)
            st.all_fp16_params += fp16_this
            st.all_fp32_from_fp16_params += fp32_from_fp16_this
            st.all_fp32_from_fp32_params += fp32_this
            st.all_fp16_grad_stash += [None for _ in fp16_this]
            st.all_fp32_from_fp32_grad_stash += [None for _ in fp32_this]
            for m, p in zip(fp16_this, fp32_from_fp16_this):
                st.master_of[id(m)] = p
                st.model_of[id(p)] = m
        else:
            for param in new_group["params"]:
                if param.dtype in _LOW:
                    st.all_fp16_params.append(param)
                    st.all_fp16_grad_stash.append(None)
                elif param.dtype == torch.float32:
                    st.all_fp32_params.append(param)
                    st.all_fp32_grad_stash.append(None)
                else:
                    raise TypeError("Optimizer's parameters must be float32, float16 or bfloat16. "
                                    "Received {}".format(param.type()))
        old_add_param_group(new_group)

    optimizer.add_param_group = types.MethodType(new_add_param_group, optimizer)
    return optimizer
