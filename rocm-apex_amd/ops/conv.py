"""1x1 stride-1 convolution routed per operation to the fastest engine for its shape.

On a channels_last activation a 1x1 stride-1 convolution IS a GEMM over the dense NHWC view:
``y[M, Cout] = x[M, Cin] W[Cout, Cin]^T`` with M = N*H*W, and its backward is the dgrad
``dx = dy W`` and the weight gradient ``dW = dy^T x`` (K = M, split-K in the native kernel).
``Conv1x1NHWC`` is a drop-in ``nn.Conv2d(cin, cout, 1, bias=False)`` (same parameter and
state_dict) whose forward, data gradient and weight gradient each go to MIOpen, to hipBLASLt
(``torch.matmul`` on the NHWC views) or to the native split-K MFMA GEMM (``csrc/gemm/gemm_mfma.hip``),
from the per-op A/B of every ResNet-50 1x1 shape at bs 256 (``profiles/conv_routes_ab_r03.jsonl``,
``tools/conv_bwd_ab.py``; 1 x MI355X, one process, interleaved):

* forward: hipBLASLt 1.1-4x MIOpen almost everywhere (e.g. 28x28 128->512: 64 vs 109 us,
  14x14 256->1024: 49 vs 84 us); MIOpen keeps the 56x56 -> 64-channel ones (58 / 127 us vs
  84 / 151), native the 7x7 512->2048 (46 vs 54 / 68 us);
* data gradient: hipBLASLt 1.1-2.4x MIOpen except where dx has 64 channels (56x56);
* weight gradient: native split-K at 14x14 / 7x7 and for 512->256 at 28x28 (1.2-1.5x MIOpen),
  MIOpen elsewhere (hipBLASLt's plain K = N*H*W GEMM is 2-10x slower there).

Everything else (CPU, autocast, other layouts / dtypes, odd channel counts) is plain
``nn.Conv2d``.  ``APEX_AMD_CONV1X1=0`` disables the routing (A/B switch).

Reference capability: the fused 1x1 convolutions of apex/contrib/bottleneck (cudnn-frontend
graphs, ``apex/contrib/csrc/bottleneck/bottleneck.cpp``) — here the GEMM is our own MFMA kernel.
"""
import functools
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native

_ENABLED = os.environ.get("APEX_AMD_CONV1X1", "1") != "0"
_STEM_PAD = os.environ.get("APEX_AMD_STEM_PAD", "1") != "0"

MIOPEN, LIB, NATIVE = "miopen", "lib", "native"
_ROUTES_R02 = os.environ.get("APEX_AMD_CONV1X1_ROUTES", "") == "r02"


def route(m, cin, cout):
    """(forward, dgrad, wgrad) engines for a 1x1 stride-1 conv with M = N*H*W rows, each one of
    ``"miopen"`` / ``"lib"`` (hipBLASLt) / ``"native"`` (profiles/conv_routes_ab_r03.jsonl)."""
    if _ROUTES_R02:  # the round-2 policy (A/B): MIOpen forward except the Cin >= 1024 reductions
        fwd = LIB if (cin >= 1024 and m <= 65536) else MIOPEN
        bwd = NATIVE if (m <= 65536 or (cin >= 512 and cout >= 256 and m <= 262144)) else MIOPEN
        return fwd, bwd, bwd
    if m >= 524288 and cout <= 64:
        fwd = MIOPEN
    elif m <= 16384 and cin <= 512:
        fwd = NATIVE
    else:
        fwd = LIB
    dgrad = MIOPEN if cin <= 64 else LIB
    wgrad = NATIVE if (m <= 65536 or (cin >= 512 and cout >= 256 and m <= 262144)) else MIOPEN
    return fwd, dgrad, wgrad


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, routes):
        fwd, dgrad, wgrad = routes
        n, c, h, wd = x.shape
        cout = w.size(0)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, c)  # zero-copy: x is channels_last contiguous
        w2 = w.view(cout, c)
        if fwd == LIB:
            y = torch.matmul(x2, w2.t()).view(n, h, wd, cout).permute(0, 3, 1, 2)
        elif fwd == NATIVE:
            g = _native.require("conv1x1").gemm
            y = g.linear(x2, w2, None, g.EPI_NONE, False)[0].view(n, h, wd, cout).permute(0, 3, 1, 2)
        else:
            y = F.conv2d(x, w)
        ctx.save_for_backward(x, w)
        ctx.routes = routes
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        _, dgrad, wgrad = ctx.routes
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        n, c, h, wd = x.shape
        cout = w.size(0)
        gy = gy.contiguous(memory_format=torch.channels_last)
        mi_x, mi_w = need_x and dgrad == MIOPEN, need_w and wgrad == MIOPEN
        dx = dw = None
        if mi_x or mi_w:
            dx, dw, _ = torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                            [mi_x, mi_w, False])
        gy2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)  # a view: gy is channels_last contiguous
        if need_x and dgrad != MIOPEN:
            if dgrad == LIB:
                dx2 = torch.matmul(gy2, w.view(cout, c))
            else:
                g = _native.require("conv1x1").gemm
                dx2 = g.linear_dgrad(gy2, w.view(cout, c), g.EPI_NONE, None)
            dx = dx2.view(n, h, wd, c).permute(0, 3, 1, 2)
        if need_w and wgrad != MIOPEN:
            g = _native.require("conv1x1").gemm
            dw = g.linear_wgrad(gy2, x.permute(0, 2, 3, 1).reshape(-1, c)).view_as(w)
        return dx, dw, None


class Conv1x1NHWC(nn.Conv2d):
    """``nn.Conv2d(in_channels, out_channels, 1, stride, bias=False)`` with per-shape native routing."""

    def __init__(self, in_channels, out_channels, stride=1):
        super().__init__(in_channels, out_channels, kernel_size=1, stride=stride, bias=False)

    def _native_ok(self, x):
        w = self.weight
        return (_ENABLED and self.stride == (1, 1) and x.is_cuda and x.dim() == 4 and x.dtype == w.dtype
                and x.dtype in (torch.bfloat16, torch.float16) and self.in_channels % 64 == 0
                and self.out_channels % 64 == 0 and x.is_contiguous(memory_format=torch.channels_last)
                and not torch.is_autocast_enabled("cuda") and _native.available())

    def forward(self, x):
        if self._native_ok(x):
            n, _, h, wd = x.shape
            routes = route(n * h * wd, self.in_channels, self.out_channels)
            if routes != (MIOPEN, MIOPEN, MIOPEN):
                return _Conv1x1Fn.apply(x, self.weight, routes)
        return super().forward(x)


# ------------------------------------------------------------------------------------------------
# Implicit-GEMM convolutions (csrc/conv/conv_igemm.hip): 3x3 stride 1/2 and strided 1x1, NHWC.
# ------------------------------------------------------------------------------------------------
_TAP_ENABLED = os.environ.get("APEX_AMD_CONV_IGEMM", "1") != "0"
# the stride-2 3x3 data gradient at <= 128 channels (ResNet-50 stage 2's first block) on the native
# per-phase tap kernels instead of MIOpen (A/B knob)
_S2_DGRAD_128 = os.environ.get("APEX_AMD_S2_DGRAD_128", "0") == "1"
# the halo-tile 3x3 weight gradient (csrc/conv/conv3x3_wgrad.hip); 0 = the r04 routes (A/B)
_HALO_WGRAD = os.environ.get("APEX_AMD_HALO_WGRAD", "1") != "0"
# its stride-2 form (even-sized inputs: ResNet-50's three downsampling 3x3s) instead of MIOpen's
# igemm_wrw; 0 = MIOpen (A/B)
_HALO_WGRAD_S2 = os.environ.get("APEX_AMD_HALO_WGRAD_S2", "1") != "0"


def _conv_ext():
    return _native.require("conv").conv


def _nhwc(t):
    """[N, H, W, C] zero-copy view of an NCHW-shaped channels_last tensor."""
    return t.permute(0, 2, 3, 1)


def _fwd_taps(k, pad):
    return [(r - pad, s - pad) for r in range(k) for s in range(k)]


def _w_krc(w):
    """[K, taps, C] view of a channels_last [K, C, R, S] weight (copy only if not channels_last)."""
    k, c, r, s = w.shape
    return w.permute(0, 2, 3, 1).reshape(k, r * s, c)


def _dgrad_phases(k, stride, pad, h, w):
    """Per output phase (ph, pw) of the data gradient: (oh, ow, [(r, s, dh, dw)]).  dX[h] collects
    dY[p] * W[r] over h = stride*p + r - pad; for h = stride*a + ph the contributing r satisfy
    (ph + pad - r) % stride == 0 and read dY[a + (ph + pad - r) // stride]."""
    out = []
    for ph in range(stride):
        for pw in range(stride):
            taps = [(r, s_, (ph + pad - r) // stride, (pw + pad - s_) // stride)
                    for r in range(k) for s_ in range(k)
                    if (ph + pad - r) % stride == 0 and (pw + pad - s_) % stride == 0]
            oh, ow = (h - ph + stride - 1) // stride, (w - pw + stride - 1) // stride
            out.append((ph, pw, oh, ow, taps))
    return out


def conv_tap_forward(x, w, stride, pad, stats_shift=None, pcoef=None):
    """NHWC conv through the native tap kernel: x [N,C,H,W] channels_last, w [K,C,R,S].
    ``stats_shift`` (fp32 [K], e.g. the consuming BN's running mean): also return the BN
    statistics partials [2, tiles, K] of the output from the kernel's epilogue, ``(y, part)``.
    ``pcoef`` (fp32 [2C]): convolve relu(x * pcoef[:C] + pcoef[C:]) instead of x — the producing
    batch norm + ReLU applied on the halo-tile kernel's staged input (padding stays zero; 3x3
    stride 1, K % 128 == 0 only: ``hfp_supported``)."""
    n, c, h, wd = x.shape
    kout, _, k, _ = w.shape
    oh, ow = (h + 2 * pad - k) // stride + 1, (wd + 2 * pad - k) // stride + 1
    y = torch.empty((n, kout, oh, ow), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    taps = _fwd_taps(k, pad)
    ext = _conv_ext()
    part = ext.tap_fprop(_nhwc(x), _w_krc(w).contiguous(), _nhwc(y), oh, ow, stride, stride, 1, 1, 0, 0,
                         [t[0] for t in taps], [t[1] for t in taps], stats_shift=stats_shift, pcoef=pcoef)
    return y if stats_shift is None else (y, part)


# ------------------------------------------------------------------------------------------------
# conv -> per-channel scale/bias (frozen BN) -> (+ residual) -> ReLU in ONE kernel: the fprop
# epilogue applies the chain to the fp32 accumulator before the bf16/fp16 store.  Capability of
# the reference's cudnn-frontend conv+scale+bias+ReLU graphs
# (apex/contrib/csrc/bottleneck/bottleneck.cpp:1-120, run_conv_scale_bias_add_activation).
# ------------------------------------------------------------------------------------------------
def conv_bn_act_supported(x, w, residual=None):
    """True when ``conv_bn_act`` runs the native fused kernel for these operands."""
    k = w.shape[2] if w.dim() == 4 else 0
    return (x.is_cuda and x.dim() == 4 and w.dim() == 4 and x.dtype == w.dtype
            and x.dtype in (torch.bfloat16, torch.float16) and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0
            and w.shape[2] == w.shape[3] and k in (1, 3)
            and x.is_contiguous(memory_format=torch.channels_last)
            and (residual is None or residual.dtype == x.dtype) and _native.available())


def _conv_bn_act_reference(x, w, scale, bias, residual, relu, stride, padding):
    """fp32-accumulated torch composition of the fused op (CPU / unsupported-shape path)."""
    y = F.conv2d(x, w, None, stride, padding)
    y = y * scale.to(y.dtype).view(1, -1, 1, 1) + bias.to(y.dtype).view(1, -1, 1, 1)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class _ConvBnActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, scale, bias, residual, relu, stride, padding):
        n, c, h, wd = x.shape
        kout, _, k, _ = w.shape
        ph, pw = padding
        oh, ow = (h + 2 * ph - k) // stride + 1, (wd + 2 * pw - k) // stride + 1
        y = torch.empty((n, kout, oh, ow), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        taps = [(r - ph, s_ - pw) for r in range(k) for s_ in range(k)]
        res = None
        if residual is not None:
            res = _nhwc(residual.contiguous(memory_format=torch.channels_last))
        _conv_ext().tap_fprop(_nhwc(x), _w_krc(w).contiguous(), _nhwc(y), oh, ow, stride, stride, 1, 1, 0, 0,
                              [t[0] for t in taps], [t[1] for t in taps], scale.float().contiguous(),
                              bias.float().contiguous(), res, bool(relu))
        ctx.save_for_backward(x, w, scale, y if relu else None)
        ctx.conf = (relu, stride, padding, residual is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, scale, y = ctx.saved_tensors
        relu, stride, padding, has_res = ctx.conf
        gy = gy.contiguous(memory_format=torch.channels_last)
        if relu:
            gy = torch.where(y > 0, gy, torch.zeros((), dtype=gy.dtype, device=gy.device))
        g_res = gy if has_res and ctx.needs_input_grad[4] else None
        g = gy * scale.to(gy.dtype).view(1, -1, 1, 1)
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = dw = None
        if need_x or need_w:
            dx, dw, _ = torch.ops.aten.convolution_backward(g, x, w, None, [stride, stride], list(padding), [1, 1],
                                                            False, [0, 0], 1, [need_x, need_w, False])
        return dx, dw, None, None, g_res, None, None, None


def conv_bn_act(x, w, scale, bias, residual=None, relu=True, stride=1, padding=0):
    """``act(conv2d(x, w) * scale + bias [+ residual])`` with per-output-channel fp32 ``scale`` /
    ``bias`` (a frozen BatchNorm), no conv bias, groups = dilation = 1, square 1x1 / 3x3 kernels.

    On a channels_last bf16/fp16 GPU activation with C, K multiples of 64 the whole chain is one
    native implicit-GEMM launch (the scale / bias / residual / ReLU run on the fp32 accumulator);
    the backward masks with the saved output and runs the MIOpen data / weight gradients of the
    scaled gradient.  ``scale`` and ``bias`` receive no gradient (frozen statistics).  Elsewhere
    (CPU, fp32, odd channel counts) it is the equivalent torch composition."""
    from .._autocast_utils import _autocast_disabled, _cast_if_autocast_enabled

    padding = (padding, padding) if isinstance(padding, int) else tuple(padding)
    x, w, residual = _cast_if_autocast_enabled(x, w, residual)
    with _autocast_disabled():
        if conv_bn_act_supported(x, w, residual):
            return _ConvBnActFn.apply(x, w.contiguous(memory_format=torch.channels_last), scale.detach(),
                                      bias.detach(), residual, relu, stride, padding)
        return _conv_bn_act_reference(x, w, scale.detach(), bias.detach(), residual, relu, stride, padding)


# APEX_AMD_TAP_PREFETCH=1: build the data-gradient weight images on a side stream during the
# forward (opt-in: the concurrent launches slowed the step 1.6 %, same box,
# profiles/r06/ab_tap_prefetch_nc256_r06ab.txt; default: in line, in front of each dgrad)
_TAP_PREFETCH = os.environ.get("APEX_AMD_TAP_PREFETCH", "0") == "1"
_SIDE = {}


def _side_stream(dev):
    st = _SIDE.get(dev)
    if st is None:
        st = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return st


def tap_images_async(w, x_shape, stride, pad):
    """The data-gradient weight images of every phase of ``conv_tap_dgrad(.., w, x_shape, stride,
    pad)``, built on a side stream during the forward (the weight is final for the step there):
    the ~5 us transposition launches then overlap the forward's kernels instead of sitting in
    front of each dgrad.  Returns an opaque handle for ``conv_tap_dgrad(pre=...)``, or None
    (disabled, capturing, not CUDA, or a weight the native transposition does not take)."""
    if not (_TAP_PREFETCH and w.is_cuda) or torch.cuda.is_current_stream_capturing():
        return None
    ext = _conv_ext()
    n, c, h, wd = x_shape
    kout, _, k, _ = w.shape
    if not (hasattr(ext, "tap_weights") and w.is_contiguous(memory_format=torch.channels_last)
            and kout % 8 == 0 and c % 8 == 0):
        return None
    cur = torch.cuda.current_stream(w.device)
    side = _side_stream(w.device)
    side.wait_stream(cur)
    imgs = []
    with torch.cuda.stream(side):
        for _, _, oh, ow, taps in _dgrad_phases(k, stride, pad, h, wd):
            if taps and oh > 0 and ow > 0:
                imgs.append(ext.tap_weights(w, [r * w.shape[3] + s_ for r, s_, _, _ in taps]))
    ev = torch.cuda.Event()
    ev.record(side)
    return imgs, ev, w._version


def conv_tap_dgrad(gy, w, x_shape, stride, pad, mask=None, red=None, pre=None):
    """Data gradient through the native tap kernel.  ``mask`` (optional, the layer input's producer
    ReLU output, same shape as dx): dx *= (mask > 0) in the kernel's epilogue — the previous
    stage's dReLU fused into this dconv.  ``red = (x, coef, mean)`` (stride 1): dx is the gradient
    of relu(bn(x)) with forward coefficients ``coef`` [2C] and batch mean ``mean``; the epilogue
    masks it with that ReLU (recomputed) and returns ``(dx, part)``, part = [2, tiles, C] partials
    of sum(dx) and sum(dx * (x - mean)) — the BN's backward reduction, no pass over dx."""
    n, c, h, wd = x_shape
    kout, _, k, _ = w.shape
    ext = _conv_ext()
    phases = _dgrad_phases(k, stride, pad, h, wd)
    covered = all(p[4] for p in phases)
    alloc = torch.empty if covered else torch.zeros  # phases no tap reaches get zero gradient
    dx = alloc((n, h, wd, c), dtype=gy.dtype, device=gy.device).permute(0, 3, 1, 2)
    wk = w.permute(1, 2, 3, 0)  # [C, R, S, K] view
    native_w = (hasattr(ext, "tap_weights") and w.is_contiguous(memory_format=torch.channels_last)
                and kout % 8 == 0 and c % 8 == 0)
    if red is not None and len(phases) != 1:
        raise ValueError("conv_tap_dgrad: the BN reduction epilogue takes a single-phase (stride 1) dgrad")
    part = None
    imgs = None
    if pre is not None and native_w and pre[2] == w._version:  # images from tap_images_async
        imgs, ev, _ = pre
        cur = torch.cuda.current_stream(gy.device)
        cur.wait_event(ev)
        for t in imgs:
            t.record_stream(cur)
        imgs = list(imgs)
    for ph, pw, oh, ow, taps in phases:
        if not taps or oh <= 0 or ow <= 0:
            continue
        if imgs:
            wt = imgs.pop(0)
        elif native_w:  # [C, taps, K] in one tiled transpose launch (layout.hip conv_tap_weights)
            wt = ext.tap_weights(w, [r * w.shape[3] + s_ for r, s_, _, _ in taps])
        elif len(taps) == k * k:  # every tap in (r, s) row-major order: one permute-copy, no stack
            wt = wk.reshape(c, k * k, kout).contiguous()  # [C, taps, K]
        else:
            wt = torch.stack([wk[:, r, s_, :] for r, s_, _, _ in taps], 1).contiguous()
        if red is not None:
            rx, rcoef, rmean = red
            part = ext.tap_fprop(_nhwc(gy), wt, _nhwc(dx), oh, ow, 1, 1, stride, stride, ph, pw,
                                 [t[2] for t in taps], [t[3] for t in taps], red_x=_nhwc(rx), red_coef=rcoef,
                                 red_mean=rmean)
            continue
        ext.tap_fprop(_nhwc(gy), wt, _nhwc(dx), oh, ow, 1, 1, stride, stride, ph, pw,
                      [t[2] for t in taps], [t[3] for t in taps], mask=None if mask is None else _nhwc(mask))
    return dx if red is None else (dx, part)


def conv_tap_wgrad(gy, x, w_shape, stride, pad, out_dtype, xcoef=None):
    """``xcoef`` (fp32 [2C]): the weight gradient of a conv whose input was relu(x * xcoef[:C] +
    xcoef[C:]) — the producing BN + ReLU recomputed on the halo-tile kernel's staged input (3x3
    stride 1 where ``halo_wgrad_supported``).  3x3 pad-1 weight gradients of stride 1, and of stride
    2 over an even-sized input, run on the halo-tile kernel where it takes the shape."""
    kout, c, k, _ = w_shape
    dw = torch.empty((kout, k, k, c), dtype=out_dtype, device=gy.device)
    taps = _fwd_taps(k, pad)
    _conv_ext().wgrad(_nhwc(x), _nhwc(gy), dw.view(kout, k * k, c), stride, stride, [t[0] for t in taps],
                      [t[1] for t in taps], xcoef)
    return dw.permute(0, 3, 1, 2)  # [K, C, R, S] in channels_last memory


@functools.lru_cache(maxsize=None)
def _halo_wgrad(cin, cout, h, w, stride=1):
    """``h``, ``w``: the conv's INPUT size."""
    if not _HALO_WGRAD or (stride == 2 and not _HALO_WGRAD_S2):
        return False
    ext = _native.submodule("conv")
    if ext is None or not hasattr(ext, "halo_wgrad_supported"):
        return False
    return bool(ext.halo_wgrad_supported(1, h, w, cin, cout, stride))


@functools.lru_cache(maxsize=None)
def tap_route(cin, cout, k, stride, h, w=None):
    """(fwd, dgrad, wgrad) through the native kernels for this shape, from the per-shape A/B
    against MIOpen on MI355X (ResNet-50 bs 256 bf16; r04: profiles/conv_cfg_sweep_r04.jsonl,
    profiles/wgrad3x3_variants_r04.jsonl — r02: conv_cfg_sweep_r02.jsonl):
      * 3x3 forward: native everywhere (fprop2 tiles: 0.64-1.0x MIOpen's time, e.g. 7x7x512 67.7
        vs 102.8 us; 56x56x128 stride 2 ties at 95.8 vs 95.6);
      * 3x3 data gradient: native except the stride-2 one at <= 128 channels (per-phase launches,
        173.9 vs 171.0 us);
      * 1x1 stride 2 (downsample): data gradient native (0.70-0.91x MIOpen);
      * 3x3 weight gradient, stride 1: the halo-tile kernel (conv3x3_wgrad.hip) wherever it takes
        the shape; r04 routes otherwise (wgrad2 128 x 64 only at 28x28x128: 136 vs 149 us, MIOpen
        5-12 % ahead at the other shapes);
      * 3x3 weight gradient, stride 2 (even-sized input): the halo-tile kernel's stride-2 form
        (round 6), else MIOpen."""
    if not _TAP_ENABLED:
        return False, False, False
    if k == 3:
        wg = ((stride == 1 and (_halo_wgrad(cin, cout, h, h if w is None else w)
                                or (cin == 128 and cout == 128 and h == 28)))
              or (stride == 2 and _halo_wgrad(cin, cout, h, h if w is None else w, 2)))
        return True, not (stride == 2 and cout <= 128) or _S2_DGRAD_128, wg
    if k == 1 and stride == 2:
        return False, True, False
    return False, False, False


class _ConvTapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, route):
        fwd, dg, wg = route
        y = conv_tap_forward(x, w, stride, pad) if fwd else F.conv2d(x, w, None, stride, pad)
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, pad, dg, wg)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, pad, dg, wg = ctx.conf
        gy = gy.contiguous(memory_format=torch.channels_last)
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = dw = None
        if (need_x and not dg) or (need_w and not wg):
            dx_m, dw_m, _ = torch.ops.aten.convolution_backward(
                gy, x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
                [need_x and not dg, need_w and not wg, False])
            dx, dw = dx_m, dw_m
        if need_x and dg:
            dx = conv_tap_dgrad(gy, w, x.shape, stride, pad)
        if need_w and wg:
            dw = conv_tap_wgrad(gy, x, w.shape, stride, pad, w.dtype)
        return dx, dw, None, None, None


class Conv2dNHWC(nn.Conv2d):
    """``nn.Conv2d(cin, cout, k, stride, padding=k // 2, bias=False)`` whose forward / data
    gradient / weight gradient run on the gfx950 implicit-GEMM kernels (``tap_route`` per shape)
    for channels_last bf16/fp16 activations; same parameter and state_dict as nn.Conv2d, plain
    nn.Conv2d everywhere else (CPU, fp32, autocast, odd channel counts)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1):
        super().__init__(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                         padding=kernel_size // 2, bias=False)

    def _native_ok(self, x):
        w = self.weight
        return (x.is_cuda and x.dim() == 4 and x.dtype == w.dtype and x.dtype in (torch.bfloat16, torch.float16)
                and self.in_channels % 64 == 0 and self.out_channels % 64 == 0 and self.groups == 1
                and self.dilation == (1, 1) and self.stride[0] == self.stride[1]
                and x.is_contiguous(memory_format=torch.channels_last)
                and w.is_contiguous(memory_format=torch.channels_last)
                and not torch.is_autocast_enabled("cuda") and _native.available())

    def forward(self, x):
        if self._native_ok(x):
            route = tap_route(self.in_channels, self.out_channels, self.kernel_size[0], self.stride[0], x.shape[2],
                              x.shape[3])
            if any(route):
                return _ConvTapFn.apply(x, self.weight, self.stride[0], self.padding[0], route)
        return super().forward(x)


class ChannelPadConv2d(nn.Conv2d):
    """``nn.Conv2d`` whose input channels are zero-padded to ``pad_to`` on the GPU path.

    The ResNet stem (7x7/2, 3 -> 64) is MIOpen's slowest convolution per FLOP on gfx950 because
    3 input channels break its NHWC vector loads; with a 4th zero channel (and a zero weight slice)
    the same convolution's forward + weight gradient runs 0.64 ms instead of 0.83 ms at bs 256
    (``tools/stem_bench.py``).  The padded copy of the input costs one 100 MB write.  Parameters
    and state_dict are those of the unpadded ``nn.Conv2d``; the weight gradient flows back through
    the concatenation to the real slice only.  Used only when the input needs no gradient
    (images), so the padding never sits on a backward path.  ``APEX_AMD_STEM_PAD=0`` disables it."""

    def __init__(self, *args, pad_to=4, **kw):
        super().__init__(*args, **kw)
        self.pad_to = pad_to

    def forward(self, x):
        c = self.in_channels
        if (_STEM_PAD and x.is_cuda and x.dim() == 4 and self.groups == 1 and c < self.pad_to and not x.requires_grad
                and x.is_contiguous(memory_format=torch.channels_last)):
            n, _, h, w = x.shape
            xp = torch.empty((n, self.pad_to, h, w), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
            xp[:, :c].copy_(x)
            xp[:, c:].zero_()
            wt = self.weight
            wp = torch.cat([wt, wt.new_zeros((wt.size(0), self.pad_to - c) + tuple(wt.shape[2:]))], dim=1)
            wp = wp.contiguous(memory_format=torch.channels_last)
            return F.conv2d(xp, wp, self.bias, self.stride, self.padding, self.dilation, 1)
        return super().forward(x)
