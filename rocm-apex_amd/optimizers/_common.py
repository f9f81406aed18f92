"""Shared plumbing for the fused optimizers.

Every fused optimizer here can run in two amp regimes:

* plain / reference regime: params are whatever sits in ``param_groups`` (fp32 masters under
  O2/O5), grads are ``p.grad``, one multi-tensor launch per dtype group (reference behaviour);
* sync-free amp regime (``optimizer._amp_stash.skip_flag`` set by ``amp.scale_loss``): the
  kernels receive the device skip flag and skip the whole update on overflow, the step count
  lives on the device, and — when the optimizer owns master weights for low-precision model
  params — the kernel also writes the bf16/fp16 model copy (one pass, no separate
  master->model copy).  With ``materialize_master_grads=False`` the grads are the *model* grads
  (still loss-scaled) and the inverse scale is applied in-kernel.
"""
import torch

_LOW = (torch.float16, torch.bfloat16)


def amp_ctx(opt):
    st = getattr(opt, "_amp_stash", None)
    if st is None or getattr(st, "skip_flag", None) is None:
        return None
    return st


def collect(opt, group, st):
    """Yield (grad, param, model_out_or_None) for params of ``group`` that have a gradient."""
    fused = st is not None and getattr(st, "fused_pending", False)
    model_of = getattr(st, "model_of", None) if st is not None else None
    for p in group["params"]:
        model = model_of.get(id(p)) if model_of else None
        if fused:
            g = model.grad if model is not None else p.grad
        else:
            g = p.grad
        if g is None:
            continue
        if g.is_sparse:
            raise RuntimeError("{} does not support sparse gradients".format(type(opt).__name__))
        yield g, p, model


def bucket(items, keyfn):
    out = {}
    for it in items:
        out.setdefault(keyfn(it), []).append(it)
    return out


def device_step(group, st, device):
    """Device-resident step counter: incremented only when the step is not skipped."""
    t = group.get("_step_t")
    if t is None or t.device != device:
        # the caller has already bumped the host counter for this call; the device counter
        # starts from the last *completed* step and is the authority from here on
        t = torch.full((1,), float(group.get("step", 1) - 1), dtype=torch.float32, device=device)
        group["_step_t"] = t
    # step += 1 - skip  (stays on device)
    t.add_(1.0 - st.skip_flag.to(torch.float32))
    return t


def lr_tensor(group, device):
    lr = group["lr"]
    if isinstance(lr, torch.Tensor):
        return lr.to(device=device, dtype=torch.float32).reshape(1)
    t = group.get("_lr_t")
    if t is None or t.device != device:
        t = torch.empty(1, dtype=torch.float32, device=device)
        group["_lr_t"] = t
    if group.get("_lr_t_val") != lr:
        t.fill_(float(lr))
        group["_lr_t_val"] = lr
    return t


def sync_steps_for_state_dict(opt):
    for group in opt.param_groups:
        t = group.get("_step_t")
        if t is not None:
            group["step"] = int(round(float(t.item())))


class AmpFusedMixin(object):
    """Marks an optimizer as able to consume the sync-free amp skip flag."""

    _amp_fused_capable = True

    def state_dict(self):
        sync_steps_for_state_dict(self)
        sd = super().state_dict()
        for g in sd["param_groups"]:
            for k in [k for k in g if k.startswith("_")]:
                del g[k]
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for group in self.param_groups:
            group.pop("_step_t", None)
            group.pop("_lr_t", None)
            group.pop("_lr_t_val", None)
