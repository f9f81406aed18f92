"""Plain-PyTorch (fp32 math) reference implementations of the multi-tensor ops.

They define the numerics the HIP kernels in ``csrc/mta/mta_ops.hip`` are tested against, and
they are the CPU path of :mod:`apex.amp_C`.  Semantics follow the reference's
``csrc/multi_tensor_*.cu`` (file:line cited per op).
"""
import math

import torch


def _f(t):
    return t.float()


def _finite(t) -> bool:
    return bool(torch.isfinite(t).all())


def _set(noop):
    noop.fill_(1)


def multi_tensor_scale(chunk_size, noop, tl, scale):
    """reference csrc/multi_tensor_scale_kernel.cu:30-111"""
    for x, y in zip(tl[0], tl[1]):
        xf = _f(x)
        if not _finite(xf):
            _set(noop)
        y.copy_(xf * float(scale))


def multi_tensor_scale_t(chunk_size, noop, tl, scale):
    return multi_tensor_scale(chunk_size, noop, tl, float(scale.reshape(-1)[0]))


def multi_tensor_axpby(chunk_size, noop, tl, a, b, arg_to_check):
    """reference csrc/multi_tensor_axpby_kernel.cu:28-126"""
    for x, y, o in zip(tl[0], tl[1], tl[2]):
        xf, yf = _f(x), _f(y)
        if arg_to_check == -1 and not (_finite(xf) and _finite(yf)):
            _set(noop)
        elif arg_to_check == 0 and not _finite(xf):
            _set(noop)
        elif arg_to_check == 1 and not _finite(yf):
            _set(noop)
        o.copy_(a * xf + b * yf)


def multi_tensor_check_finite(chunk_size, noop, tl):
    for x in tl[0]:
        if not _finite(_f(x)):
            _set(noop)
            return


def _norms(tl0, per_tensor, maxnorm=False):
    sq = []
    for x in tl0:
        xf = _f(x)
        sq.append(xf.abs().max() if (maxnorm and xf.numel()) else (xf.new_zeros(()) if maxnorm else (xf * xf).sum()))
    dev = tl0[0].device if len(tl0) else "cpu"
    if maxnorm:
        per = torch.stack(sq) if sq else torch.zeros(0, device=dev)
        total = per.max().reshape(1) if len(sq) else torch.zeros(1, device=dev)
    else:
        per_sq = torch.stack(sq) if sq else torch.zeros(0, device=dev)
        total = per_sq.sum().sqrt().reshape(1)
        per = per_sq.sqrt()
    return total, (per if per_tensor else torch.zeros(0, device=dev))


def multi_tensor_l2norm(chunk_size, noop, tl, per_tensor=False):
    """reference csrc/multi_tensor_l2norm_kernel.cu:301-368"""
    total, per = _norms(tl[0], per_tensor)
    if not _finite(total):
        _set(noop)
    return total, per


def multi_tensor_l2norm_mp(chunk_size, noop, tl, per_tensor=False):
    """reference csrc/multi_tensor_l2norm_kernel_mp.cu: a no-op when noop is set — before the
    call, or by a non-finite value found during it (the step is skipped; norms read as 0)."""
    dev = tl[0][0].device
    skipped = (torch.zeros(1, device=dev), torch.zeros(len(tl[0]) if per_tensor else 0, device=dev))
    if int(noop.reshape(-1)[0]) != 0:
        return skipped
    total, per = multi_tensor_l2norm(chunk_size, noop, tl, per_tensor)
    return skipped if int(noop.reshape(-1)[0]) != 0 else (total, per)


def multi_tensor_maxnorm(chunk_size, noop, tl, per_tensor=False):
    total, per = _norms(tl[0], per_tensor, maxnorm=True)
    for x in tl[0]:
        if not _finite(_f(x)):
            _set(noop)
    return total, per


def multi_tensor_l2norm_scale(chunk_size, noop, tl, scale, per_tensor=False):
    """reference csrc/multi_tensor_l2norm_scale_kernel.cu:29-134 (norm of the unscaled input)"""
    total, per = _norms(tl[0], per_tensor)
    if not _finite(total):
        _set(noop)
    for x, y in zip(tl[0], tl[1]):
        y.copy_(_f(x) * scale)
    return total, per


def multi_tensor_norm_out(chunk_size, noop, tl, out, alpha, beta, norm_type):
    """reference csrc/multi_tensor_l2norm_kernel.cu:371-456 (cleanup_v2 blend)"""
    for i, x in enumerate(tl[0]):
        xf = _f(x)
        if norm_type == 0:
            out[i] = alpha * out[i] + beta * (xf.abs().max() if xf.numel() else 0.0)
        else:
            out[i] = math.sqrt(alpha * float(out[i]) ** 2 + beta * float((xf * xf).sum()))


def _adam_elem(g, p, m, v, lr, beta1, beta2, eps, bc1, bc2, mode, wd):
    if mode == 0:
        g = g + wd * p
        m = beta1 * m + (1 - beta1) * g
        v = beta2 * v + (1 - beta2) * g * g
        denom = (v / bc2).sqrt() + eps
        p = p - lr * ((m / bc1) / denom)
    else:
        m = beta1 * m + (1 - beta1) * g
        v = beta2 * v + (1 - beta2) * g * g
        denom = (v / bc2).sqrt() + eps
        p = p - lr * (((m / bc1) / denom) + wd * p)
    return p, m, v


def multi_tensor_adam(chunk_size, noop, tl, lr, beta1, beta2, eps, step, mode, bias_correction, weight_decay):
    """reference csrc/multi_tensor_adam.cu:24-171"""
    bc1 = 1 - beta1 ** step if bias_correction else 1.0
    bc2 = 1 - beta2 ** step if bias_correction else 1.0
    outs = tl[4] if len(tl) == 5 else [None] * len(tl[0])
    for g, p, m, v, o in zip(tl[0], tl[1], tl[2], tl[3], outs):
        pn, mn, vn = _adam_elem(_f(g), _f(p), _f(m), _f(v), lr, beta1, beta2, eps, bc1, bc2, mode, weight_decay)
        p.copy_(pn)
        m.copy_(mn)
        v.copy_(vn)
        if o is not None:
            o.copy_(pn)


def multi_tensor_adam_capturable(chunk_size, noop, tl, lr, beta1, beta2, eps, step, mode, bias_correction,
                                 weight_decay, inv_scale=None):
    if int(noop.reshape(-1)[0]) != 0:
        return
    st = float(step.reshape(-1)[0])
    lrv = float(lr.reshape(-1)[0])
    inv = float(inv_scale.reshape(-1)[0]) if inv_scale is not None else 1.0
    bc1 = 1 - beta1 ** st if bias_correction else 1.0
    bc2 = 1 - beta2 ** st if bias_correction else 1.0
    outs = tl[4] if len(tl) == 5 else [None] * len(tl[0])
    for g, p, m, v, o in zip(tl[0], tl[1], tl[2], tl[3], outs):
        pn, mn, vn = _adam_elem(_f(g) * inv, _f(p), _f(m), _f(v), lrv, beta1, beta2, eps, bc1, bc2, mode,
                                weight_decay)
        p.copy_(pn)
        m.copy_(mn)
        v.copy_(vn)
        if o is not None:
            o.copy_(pn)


def multi_tensor_adam_undo(chunk_size, noop, tl, lr, beta1, beta2, eps, step, mode, bias_correction,
                           weight_decay, inv_scale=None):
    """Inverse of one fp32-master Adam step (lists g, p, m, v[, model copy]); the HIP op is
    csrc/mta/mta_ops.hip AdamUndoOp (capability of the reference's maybe_adam_undo)."""
    if int(noop.reshape(-1)[0]) != 0:
        return
    st = float(step.reshape(-1)[0])
    lrv = float(lr.reshape(-1)[0])
    inv = float(inv_scale.reshape(-1)[0]) if inv_scale is not None else 1.0
    bc1 = 1 - beta1 ** st if bias_correction else 1.0
    bc2 = 1 - beta2 ** st if bias_correction else 1.0
    outs = tl[4] if len(tl) == 5 else [None] * len(tl[0])
    for g, p, m, v, o in zip(tl[0], tl[1], tl[2], tl[3], outs):
        gf, pf, mf, vf = _f(g) * inv, _f(p), _f(m), _f(v)
        upd = (mf / bc1) / ((vf / bc2).sqrt() + eps)
        if mode == 0:
            p0 = pf + lrv * upd
            gf = gf + weight_decay * p0
        else:
            p0 = (pf + lrv * upd) / (1.0 - lrv * weight_decay)
        p.copy_(p0)
        m.copy_((mf - (1 - beta1) * gf) / beta1)
        v.copy_(((vf - (1 - beta2) * gf * gf) / beta2).clamp_min(0.0))
        if o is not None:
            o.copy_(p0)


def _sgd(tl, wd, momentum, dampening, lr, nesterov, first_run, wd_after_momentum, scale):
    outs = tl[3] if len(tl) == 4 else [None] * len(tl[0])
    for g, w, mom, o in zip(tl[0], tl[1], tl[2], outs):
        gf = _f(g) * scale
        wf = _f(w)
        mf = _f(mom)
        if wd != 0 and not wd_after_momentum:
            gf = gf + wd * wf
        if momentum != 0:
            mf = gf.clone() if first_run else mf * momentum + (1 - dampening) * gf
            gf = gf + momentum * mf if nesterov else mf
        if wd != 0 and wd_after_momentum:
            gf = gf + wd * wf
        wn = wf + (-lr * gf)
        w.copy_(wn)
        mom.copy_(mf)
        if o is not None:
            o.copy_(wn)


def multi_tensor_sgd(chunk_size, noop, tl, wd, momentum, dampening, lr, nesterov, first_run, wd_after_momentum,
                     scale):
    """reference csrc/multi_tensor_sgd_kernel.cu:29-139 (skips when noop is set, :46)"""
    if int(noop.reshape(-1)[0]) != 0:
        return
    _sgd(tl, wd, momentum, dampening, lr, nesterov, first_run, wd_after_momentum, scale)


def multi_tensor_sgd_capturable(chunk_size, noop, tl, wd, momentum, dampening, lr, nesterov, first_run,
                                wd_after_momentum, scale=None):
    if int(noop.reshape(-1)[0]) != 0:
        return
    _sgd(tl, wd, momentum, dampening, float(lr.reshape(-1)[0]), nesterov, first_run, wd_after_momentum,
         float(scale.reshape(-1)[0]) if scale is not None else 1.0)


def multi_tensor_adagrad(chunk_size, noop, tl, lr, eps, mode, weight_decay):
    """reference csrc/multi_tensor_adagrad.cu:24-84"""
    for g, p, h in zip(tl[0], tl[1], tl[2]):
        gf, pf, hf = _f(g), _f(p), _f(h)
        if mode == 0:
            gf = gf + weight_decay * pf
            hf = hf + gf * gf
            pf = pf - lr * (gf / (hf.sqrt() + eps))
        else:
            hf = hf + gf * gf
            pf = pf - lr * (gf / (hf.sqrt() + eps) + weight_decay * pf)
        p.copy_(pf)
        h.copy_(hf)


def multi_tensor_novograd(chunk_size, noop, tl, grad_norms, lr, beta1, beta2, eps, step, bias_correction,
                          weight_decay, grad_averaging, mode, norm_type):
    """reference csrc/multi_tensor_novograd.cu:33-188"""
    multi_tensor_norm_out(chunk_size, noop, [tl[0]], grad_norms, beta2, 1.0 - beta2, norm_type)
    bc1 = 1 - beta1 ** step if bias_correction else 1.0
    bc2 = math.sqrt(1 - beta2 ** step) if bias_correction else 1.0
    beta3 = 1 - beta1 if grad_averaging == 1 else 1.0
    for i, (g, p, m) in enumerate(zip(tl[0], tl[1], tl[2])):
        gn = float(grad_norms[i])
        gf, pf, mf = _f(g), _f(p), _f(m)
        if mode == 0:
            denom = gn / bc2 + eps
            gf = gf / denom + weight_decay * pf
            mf = beta1 * mf + beta3 * gf
            pf = pf - lr * (mf / bc1)
        else:
            mf = beta1 * mf + beta3 * gf
            denom = gn / bc2 + eps
            pf = pf - lr * ((mf / bc1) / denom + weight_decay * pf)
        p.copy_(pf)
        m.copy_(mf)


def _lamb(tl, lr, beta1, beta2, eps, bc1, bc2, weight_decay, grad_averaging, mode, gnorm, max_grad_norm,
          use_nvlamb, inv=1.0):
    beta3 = 1 - beta1 if grad_averaging == 1 else 1.0
    clip = gnorm / max_grad_norm if (max_grad_norm > 0 and gnorm > max_grad_norm) else 1.0
    outs = tl[4] if len(tl) == 5 else [None] * len(tl[0])
    for g, p, m, v, o in zip(tl[0], tl[1], tl[2], tl[3], outs):
        gf, pf, mf, vf = _f(g) * inv, _f(p), _f(m), _f(v)
        sg = gf / clip
        pd = pf if weight_decay != 0 else torch.zeros_like(pf)
        if mode == 0:
            sg = sg + weight_decay * pd
            mf = mf * beta1 + beta3 * sg
            vf = vf * beta2 + (1 - beta2) * sg * sg
            upd = (mf / bc1) / ((vf / bc2).sqrt() + eps)
        else:
            mf = mf * beta1 + beta3 * sg
            vf = vf * beta2 + (1 - beta2) * sg * sg
            upd = ((mf / bc1) / ((vf / bc2).sqrt() + eps)) + weight_decay * pd
        ratio = lr
        if use_nvlamb or weight_decay != 0:
            pn, un = float(pf.norm()), float(upd.norm())
            ratio = lr * (pn / un) if (pn != 0 and un != 0) else lr
        pn_ = pf - ratio * upd
        g.copy_(upd)
        p.copy_(pn_)
        m.copy_(mf)
        v.copy_(vf)
        if o is not None:
            o.copy_(pn_)


def multi_tensor_lamb(chunk_size, noop, tl, lr, beta1, beta2, epsilon, step, bias_correction, weight_decay,
                      grad_averaging, mode, global_grad_norm, max_grad_norm, use_nvlamb_python=None):
    """reference csrc/multi_tensor_lamb.cu:41-413"""
    bc1 = 1 - beta1 ** step if bias_correction else 1.0
    bc2 = 1 - beta2 ** step if bias_correction else 1.0
    _lamb(tl, lr, beta1, beta2, epsilon, bc1, bc2, weight_decay, grad_averaging, mode,
          float(global_grad_norm.reshape(-1)[0]), max_grad_norm, bool(use_nvlamb_python))


def multi_tensor_lamb_mp(chunk_size, noop, tl, lr, beta1, beta2, epsilon, step, bias_correction, weight_decay,
                         grad_averaging, mode, global_grad_norm, max_grad_norm, use_nvlamb_python, found_inf,
                         inv_scale):
    """reference csrc/multi_tensor_lamb_mp.cu:367-496"""
    if float(found_inf.reshape(-1)[0]) != 0:
        return
    st = float(step.reshape(-1)[0])
    bc1 = 1 - beta1 ** st if bias_correction else 1.0
    bc2 = 1 - beta2 ** st if bias_correction else 1.0
    _lamb(tl, float(lr.reshape(-1)[0]), beta1, beta2, epsilon, bc1, bc2, weight_decay, grad_averaging, mode,
          float(global_grad_norm.reshape(-1)[0]), float(max_grad_norm.reshape(-1)[0]), bool(use_nvlamb_python),
          inv=float(inv_scale.reshape(-1)[0]))


def multi_tensor_lamb_stage1_cuda(chunk_size, noop, tl, per_tensor_decay, step, beta1, beta2, epsilon,
                                  global_grad_norm, max_global_grad_norm, beta3=None):
    """reference csrc/multi_tensor_lamb_stage_1.cu:17-151 (lists g, p, m, v, update); ``beta3``
    (default 1 - beta1) is the gradient weight in the first moment (1 for grad_averaging=False)"""
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    b3 = (1 - beta1) if beta3 is None else beta3
    gn = float(global_grad_norm.reshape(-1)[0])
    clip = gn / max_global_grad_norm if gn > max_global_grad_norm else 1.0
    for i, (g, p, m, v, u) in enumerate(zip(*tl)):
        sg = _f(g) / clip
        mf = _f(m) * beta1 + b3 * sg
        vf = _f(v) * beta2 + (1 - beta2) * sg * sg
        u.copy_((mf / bc1) / ((vf / bc2).sqrt() + epsilon) + float(per_tensor_decay[i]) * _f(p))
        m.copy_(mf)
        v.copy_(vf)


def multi_tensor_lamb_stage2_cuda(chunk_size, noop, tl, per_tensor_param_norm, per_tensor_update_norm, lr,
                                  weight_decay, use_nvlamb_python=None):
    """reference csrc/multi_tensor_lamb_stage_2.cu:20-125 (lists p, update[, model-dtype copy])"""
    outs = tl[2] if len(tl) == 3 else [None] * len(tl[0])
    for i, (p, u, o) in enumerate(zip(tl[0], tl[1], outs)):
        ratio = lr
        if use_nvlamb_python or weight_decay != 0:
            pn, un = float(per_tensor_param_norm[i]), float(per_tensor_update_norm[i])
            ratio = lr * (pn / un) if (pn != 0 and un != 0) else lr
        p.copy_(_f(p) - ratio * _f(u))
        if o is not None:
            o.copy_(p)


def multi_tensor_lamb_stage1_capturable(chunk_size, skip, tl, per_tensor_decay, step, bias_correction, beta1, beta2,
                                        epsilon, global_grad_norm, max_global_grad_norm, beta3):
    """Skip-gated stage 1 with the bias corrections from the device step count (no-op while
    ``skip`` is set)."""
    if int(skip.reshape(-1)[0]) != 0:
        return
    st = float(step.reshape(-1)[0])
    bc1 = (1 - beta1 ** st) if bias_correction else 1.0
    bc2 = (1 - beta2 ** st) if bias_correction else 1.0
    gn = float(global_grad_norm.reshape(-1)[0])
    clip = gn / max_global_grad_norm if gn > max_global_grad_norm else 1.0
    for i, (g, p, m, v, u) in enumerate(zip(*tl)):
        sg = _f(g) / clip
        mf = _f(m) * beta1 + beta3 * sg
        vf = _f(v) * beta2 + (1 - beta2) * sg * sg
        u.copy_((mf / bc1) / ((vf / bc2).sqrt() + epsilon) + float(per_tensor_decay[i]) * _f(p))
        m.copy_(mf)
        v.copy_(vf)


def multi_tensor_lamb_stage2_capturable(chunk_size, skip, tl, per_tensor_param_norm, per_tensor_update_norm, lr,
                                        weight_decay, use_nvlamb):
    """Skip-gated stage 2 with a device learning rate."""
    if int(skip.reshape(-1)[0]) != 0:
        return
    multi_tensor_lamb_stage2_cuda(chunk_size, skip, tl, per_tensor_param_norm, per_tensor_update_norm,
                                  float(lr.reshape(-1)[0]), weight_decay, use_nvlamb)


def multi_tensor_cast(chunk_size, noop, tl):
    for x, y in zip(tl[0], tl[1]):
        y.copy_(x)


def amp_update_scale_(overflow, skip_flag, state, growth_factor, backoff_factor, growth_interval, min_scale,
                      max_scale, dynamic):
    scale = float(state[0])
    state[1] = 1.0 / scale
    ovf = int(overflow.reshape(-1)[0]) != 0
    skip = bool(dynamic and ovf)
    skip_flag.fill_(int(skip))
    if not dynamic:
        state[2] += 1
        return
    unsk = float(state[2])
    if skip:
        scale = scale * backoff_factor
        if min_scale > 0:
            scale = max(min_scale, scale)
        unsk = 0.0
        state[3] += 1
    else:
        unsk += 1
    if int(unsk) == growth_interval:
        scale = min(max_scale, scale * growth_factor)
        unsk = 0.0
    state[0] = scale
    state[2] = unsk


def mta_cache_clear():
    pass


def mta_cache_size():
    return 0
