"""Fused dense layers (reference apex/fused_dense/fused_dense.py:5-85).

``FusedDense``           y = x W^T + b                      (GEMM + bias epilogue)
``FusedDenseGeluDense``  y = gelu(x W1^T + b1) W2^T + b2    (GEMM + bias + GeLU-with-aux epilogue,
                                                             then GEMM + bias)
Backward: dgrad GEMMs (the first one with the GeLU-derivative epilogue), wgrad GEMMs and
column-sum bias gradients — every piece is a gfx950 kernel (``csrc/gemm/gemm_mfma.hip``); the
reference's ROCm build leaves d_bias uninitialised and makes the GeLU variants no-ops
(csrc/fused_dense.cpp:64-68, csrc/fused_dense_cuda.cu:1361-1495).

Runs the native path for fp16/bf16 GPU tensors with K, N multiples of 8; otherwise (CPU, fp32,
odd sizes) the same math in torch.  GeLU is the tanh approximation (the cuBLASLt GELU epilogue
the reference targets).

Routing (static, identical on every rank and every run; ``APEX_AMD_DENSE_ROUTE``):

* ``lt`` (default): hipBLASLt with the fused epilogues of ``csrc/bindings/lt_epilogue.cpp`` —
  forward GEMM+bias / GEMM+bias+GeLU writing the pre-activation aux in ONE launch, backward
  dGeLU+bias-grad and weight-grad+bias-grad epilogues (the reference's cuBLASLt
  GELU_AUX_BIAS / DGELU_BGRAD / BGRADB, csrc/fused_dense_cuda.cu:220,471,843,977).  At the
  GPT-2 / BERT MLP shapes hipBLASLt's main loop is ahead of the native MFMA kernel
  (profiles/gemm8p_shapes_ab_r02.jsonl), so the epilogue fusion rides on the faster GEMM.  Kernel
  coverage differs by dtype (profiles/lt_probe_r03.jsonl, ROCm 7.2 on gfx950): fp16 has every
  epilogue; bf16 has BIAS and BGRADB but no GELU_AUX_BIAS, and its DGELU kernels give wrong
  results (disabled in lt_epilogue.cpp), so bf16 runs GEMM+bias then one GeLU pass forward, and
  backward the native MFMA dgrad GEMM with dGeLU and the bias-gradient column sums in its
  epilogue (``_DGELU_ROUTE``; 197 vs 201 us library dgrad + pass at the GPT-2 MLP shape,
  profiles/r06/gelu_routes_r06ar.jsonl) + the library wgrad.  BGRADB is opt-in (see ``_lt_bgradb``);  A shape the library has no kernel for at all falls back to the torch ops;
* ``native``: every GEMM on the gfx950 MFMA kernels (``csrc/gemm/gemm_mfma.hip``) with their
  own fused epilogues;
* ``library``: plain torch ops (addmm + GeLU + sum) — the A/B baseline;
* ``auto``: opt-in per-shape timing of native vs lt on the live tensors (first call of each shape;
  the decision may differ between ranks, so it is never the default).
``route_table()`` lists the decisions taken so far."""
import os

import torch
from torch import nn

from .. import _native
from ..amp import half_function


def _g():
    return _native.require("gemm").gemm


def _fd():
    return _native.require("fused_dense_cuda").fused_dense_cuda


def fused_linear_available(x, weight, bias=None):
    if not _native.use_native(x) or _native.submodule("gemm") is None:
        return False
    if x.dtype not in (torch.float16, torch.bfloat16) or weight.dtype != x.dtype:
        return False
    if bias is not None and bias.dtype != x.dtype:
        return False
    k = x.shape[-1]
    n = weight.shape[0]
    return k % 8 == 0 and n % 8 == 0 and x.numel() > 0


def linear_bias_forward(x, weight, bias):
    shape = x.shape[:-1] + (weight.shape[0],)
    return _fd().linear_bias_forward(x, weight, bias).view(shape)


def _gelu_tanh(x):
    return torch.nn.functional.gelu(x, approximate="tanh")


def _gelu_pass(z):
    """tanh-GeLU of a GPU pre-activation: the native vector kernel (exp + rcp form, one 16-byte
    load / store per 8 elements) where it applies, else torch's GeLU."""
    if (_native.use_native(z) and _native.submodule("gemm") is not None and z.dtype in (torch.float16, torch.bfloat16)
            and z.is_contiguous() and z.numel() % 8 == 0):
        return _g().gelu(z)
    return _gelu_tanh(z)


_ROUTES = {}
# FusedDenseGeluDense backward where hipBLASLt has no usable DGELU kernel (bf16 on gfx950): the
# native MFMA dgrad GEMM with dGeLU AND the bias-gradient column sums in its epilogue (the
# reference's DGELU_BGRAD, csrc/fused_dense_cuda.cu:977) — "native" (default) — or the library
# dgrad + one dGeLU / column-sum pass over its output ("pass", A/B)
_DGELU_ROUTE = os.environ.get("APEX_AMD_DGELU_ROUTE", "native")


def route_mode():
    return os.environ.get("APEX_AMD_DENSE_ROUTE", "lt")


def _lt(*tensors):
    """hipBLASLt epilogue GEMMs, or None when the route is not lt, the extension lacks them, or
    the operands are not all CUDA fp16 / all CUDA bf16 (the wrapper's kernels take those only:
    fp32 and mixed-dtype calls run the torch ops instead)."""
    if route_mode() not in ("lt", "auto"):
        return None
    ts = [t for t in tensors if t is not None]
    if not ts or ts[0].dtype not in (torch.float16, torch.bfloat16):
        return None
    if any(not t.is_cuda or t.dtype != ts[0].dtype for t in ts):
        return None
    return _native.submodule("lt_gemm")


_LT_SYNCED = {}


def sync_lt_plans(group=None, src=0):
    """Make every rank of ``group`` use group-rank ``src``'s hipBLASLt algorithm picks.

    The library route times its top candidates per problem in each process (lt_epilogue.cpp
    lt_run), so two tensor-parallel ranks could run different kernels for the same GEMM and
    produce bitwise-different partial sums.  This broadcasts ``src``'s (problem, pick) table and
    applies it (the screened candidate lists are identical on every rank: same library, same
    problem).  Returns the number of picks applied here.  Reference counterpart: cuBLASLt's
    single heuristic answer (csrc/fused_dense_cuda.cu:298-299, requestedAlgoCount = 1)."""
    import torch.distributed as dist

    lt = _native.submodule("lt_gemm")
    if lt is None or not hasattr(lt, "plan_choices") or not (dist.is_available() and dist.is_initialized()):
        return 0
    if dist.get_world_size(group) <= 1:
        return 0
    obj = [lt.plan_choices() if dist.get_rank(group) == src else None]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(group, src) if group is not None else src, group=group)
    dev = torch.cuda.current_device() if torch.cuda.is_available() else 0
    return sum(1 for key in obj[0] if lt.set_plan_choice(list(key), dev))


def maybe_sync_lt_plans(group, problem):
    """sync_lt_plans(group) the first time this process runs ``problem`` (a hashable key of the
    GEMM: op, shape, dtype) for ``group``; returns True when it synced, so the caller re-runs the
    GEMM on the agreed pick.

    The decision depends only on the tensor-parallel call sequence, which every rank of the group
    runs identically (same problems, same order), so all ranks enter the collective together.  A
    process-wide counter of planned problems would not do: library GEMMs outside the TP layers
    (the ResNet 1x1s, non-TP fused_dense) plan problems on some ranks only and would leave the
    other ranks outside the broadcast."""
    import torch.distributed as dist

    lt = _native.submodule("lt_gemm")
    if lt is None or not hasattr(lt, "plan_choices") or not (dist.is_available() and dist.is_initialized()):
        return False
    if dist.get_world_size(group) <= 1:
        return False
    seen = _LT_SYNCED.setdefault(id(group), set())
    if problem in seen:
        return False
    seen.add(problem)
    sync_lt_plans(group)
    return True


def route_table():
    """{(op, M, N, K, dtype): 'native' | 'library'} decided so far in this process."""
    return {k: ("native" if v else "library") for k, v in _ROUTES.items()}


def _time_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def _use_native(key, native_fn, library_fn):
    """Static route, or (APEX_AMD_DENSE_ROUTE=auto only) a measured per-shape choice."""
    mode = route_mode()
    if mode != "auto":
        _ROUTES.setdefault(key, mode == "native")
        return mode == "native"
    hit = _ROUTES.get(key)
    if hit is not None:
        return hit
    if torch.cuda.is_current_stream_capturing():
        return True
    with torch.no_grad():
        t_native, t_lib = _time_ms(native_fn), _time_ms(library_fn)
    _ROUTES[key] = t_native <= t_lib
    return _ROUTES[key]


def _lib_dense_fwd(x, w, b):
    x2 = x.reshape(-1, x.shape[-1])
    lt = _lt(x2, w, b)
    if lt is not None and x2.is_contiguous():
        r = lt.linear(x2, w.contiguous(), b, lt.EPI_BIAS if b is not None else lt.EPI_NONE)
        if r:
            return r[0].view(x.shape[:-1] + (w.shape[0],))
    out = torch.addmm(b, x2, w.t()) if b is not None else x2.matmul(w.t())
    return out.view(x.shape[:-1] + (w.shape[0],))


def native_wgrad_ok(g2, x2):
    """The native split-K wgrad beats hipBLASLt's ``g.t() @ x`` when the N x K output is small
    (<= 1M elements: too few output tiles for hipBLASLt to fill 256 CUs) and K = M is deep
    (profiles/wgrad_shapes_ab_r03.jsonl: 1024 x 1024 at 8k / 16k tokens 1.06-1.64x); at
    3072-4096 x 1024 the two tie or hipBLASLt leads."""
    if not (g2.is_cuda and _native.use_native(g2) and _native.submodule("gemm") is not None):
        return False
    if g2.dtype not in (torch.float16, torch.bfloat16) or x2.dtype != g2.dtype or g2.dim() != 2 or x2.dim() != 2:
        return False
    m, n = g2.shape
    k = x2.shape[1]
    return (n * k <= (1 << 20) and m >= 4096 and n % 64 == 0 and k % 64 == 0 and g2.is_contiguous()
            and x2.is_contiguous())


def _native_wide_wgrad(g2, x2):
    if os.environ.get("APEX_AMD_WIDE_WGRAD", "1") == "0":
        return False
    if not (g2.is_cuda and _native.use_native(g2) and _native.submodule("gemm") is not None):
        return False
    if g2.dtype not in (torch.float16, torch.bfloat16) or x2.dtype != g2.dtype or g2.dim() != 2 or x2.dim() != 2:
        return False
    m, n = g2.shape
    k = x2.shape[1]
    return n <= 1024 and k >= 4096 and m >= 8192 and n % 256 == 0 and k % 256 == 0 and m % 64 == 0


def wgrad_gemm(g2, x2):
    """dW[N, K] = g2[M, N]^T x2[M, K] for the dense layers: the native split-K kernel for small
    outputs (``native_wgrad_ok``), else hipBLASLt through the wrapper's per-shape top-8 timing
    (``lt_gemm.mm``: 149 vs 176 us for torch.matmul's first-heuristic kernel at the GPT-2 QKV
    shape 16384 x 3072 x 1024, ties elsewhere; profiles/gemm_routes_r04t.jsonl) up to 16384 tokens,
    else torch.matmul."""
    if native_wgrad_ok(g2, x2):
        return _g().linear_wgrad(g2, x2)
    if _native_wide_wgrad(g2, x2):
        # short-wide weight (<= 1024 rows, >= 4096 columns, e.g. the MLP's 4h -> h projection):
        # the native split-K GEMM leads hipBLASLt (153 vs 164 us at 16384 tokens,
        # profiles/gemm_routes_r04t.jsonl)
        m, n = g2.shape
        return _g().matmul(g2, False, x2, False, n, x2.shape[1], m, 0, None, None, False)[0]
    lt = _lt(g2, x2)
    # only where the timed plans were validated (<= 16384 tokens, every dim <= 16384): at 65536
    # tokens hipBLASLt's own first answer for this layout faults (tools/gpu_r04ab.sh probes)
    if (lt is not None and hasattr(lt, "mm") and g2.dim() == 2 and x2.dim() == 2
            and max(g2.size(0), g2.size(1), x2.size(1)) <= 16384):
        r = lt.mm(g2.contiguous(), x2.contiguous(), True, False)
        if r:
            return r[0]
    return g2.t().matmul(x2)


def _lt_bgradb():
    # hipBLASLt's heuristic answers BGRADB at the transformer shapes with a 32x32-tile kernel that
    # runs ~10x slower than the plain wgrad GEMM (1.1 ms vs ~0.1 ms at 16384 tokens,
    # profiles/gpt2_medium_steady_r03a.md), so the bias-grad epilogue is opt-in
    return os.environ.get("APEX_AMD_LT_BGRADB", "0") == "1"


def _lib_wgrad(g2, x2, has_bias):
    """(dW, db): matmul + column sum, or (APEX_AMD_LT_BGRADB=1) one hipBLASLt launch with the BGRADB
    epilogue."""
    lt = _lt(g2, x2)
    if lt is not None and has_bias and _lt_bgradb():
        r = lt.wgrad_bgrad(g2.contiguous(), x2.contiguous(), has_bias)
        if r:
            return r[0], (r[1] if has_bias else None)
    return wgrad_gemm(g2, x2), (_native.column_sum(g2, g2.dtype) if has_bias else None)


def _lib_dense_bwd(x, w, gy, has_bias):
    g2 = gy.reshape(-1, gy.shape[-1])
    x2 = x.reshape(-1, x.shape[-1])
    dw, db = _lib_wgrad(g2, x2, has_bias)
    return g2.matmul(w).view(x.shape), dw, db


def _shape_key(op, x, w):
    return (op, x.numel() // x.shape[-1], w.shape[0], w.shape[1], str(x.dtype))


class FusedDenseFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, bias):
        ctx.save_for_backward(input, weight)
        ctx.native = fused_linear_available(input, weight, bias)
        ctx.has_bias = bias is not None
        if ctx.native and _use_native(_shape_key("dense_fwd", input, weight) + (bias is not None,),
                                      lambda: linear_bias_forward(input, weight, bias),
                                      lambda: _lib_dense_fwd(input, weight, bias)):
            return linear_bias_forward(input, weight, bias)
        if input.is_cuda:
            return _lib_dense_fwd(input, weight, bias)
        out = torch.matmul(input, weight.t())
        return out + bias if bias is not None else out

    @staticmethod
    def backward(ctx, grad_output):
        input, weight = ctx.saved_tensors
        gy = grad_output.contiguous()
        if ctx.native and _use_native(_shape_key("dense_bwd", input, weight) + (ctx.has_bias,),
                                      lambda: _fd().linear_bias_backward(input, weight, gy),
                                      lambda: _lib_dense_bwd(input, weight, gy, ctx.has_bias)):
            dx, dw, db = _fd().linear_bias_backward(input, weight, gy)
            return dx.view(input.shape), dw, (db if ctx.has_bias else None)
        return _lib_dense_bwd(input, weight, gy, ctx.has_bias)


class DenseNoBiasFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight):
        return FusedDenseFunc.forward(ctx, input, weight, None)

    @staticmethod
    def backward(ctx, grad_output):
        dx, dw, _ = FusedDenseFunc.backward(ctx, grad_output)
        return dx, dw


def _lib_gelu_dense_fwd(x, w1, b1, w2, b2):
    x2 = x.reshape(-1, x.shape[-1])
    lt = _lt(x2, w1, b1, w2, b2)
    if lt is not None and x2.is_contiguous():
        w1c, w2c = w1.contiguous(), w2.contiguous()
        r1 = lt.linear(x2, w1c, b1, lt.EPI_GELU_AUX_BIAS)
        if r1:
            out1, gelu_in = r1
        else:
            # no GELU_AUX_BIAS kernel (gfx950 bf16): GEMM + bias epilogue writes the
            # pre-activation, one elementwise GeLU pass
            r1 = lt.linear(x2, w1c, b1, lt.EPI_BIAS)
            gelu_in = r1[0] if r1 else torch.addmm(b1, x2, w1.t())
            out1 = _gelu_pass(gelu_in)
        r2 = lt.linear(out1, w2c, b2, lt.EPI_BIAS)
        out2 = r2[0] if r2 else torch.addmm(b2, out1, w2.t())
        return out1, out2.view(x.shape[:-1] + (w2.shape[0],)), gelu_in
    gelu_in = torch.addmm(b1, x2, w1.t())
    out1 = _gelu_tanh(gelu_in)
    out2 = torch.addmm(b2, out1, w2.t())
    return out1, out2.view(x.shape[:-1] + (w2.shape[0],)), gelu_in


class FusedDenseGeluDenseFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight1, bias1, weight2, bias2):
        ctx.native = (fused_linear_available(input, weight1, bias1) and weight2.dtype == input.dtype
                      and bias2.dtype == input.dtype and weight2.shape[0] % 8 == 0 and weight2.shape[1] % 8 == 0)
        key = _shape_key("gelu_dense_fwd", input, weight1) + (weight2.shape[0],)
        if ctx.native and _use_native(key,
                                      lambda: _fd().linear_gelu_linear_forward(input, weight1, bias1, weight2, bias2),
                                      lambda: _lib_gelu_dense_fwd(input, weight1, bias1, weight2, bias2)):
            out1, out2, gelu_in = _fd().linear_gelu_linear_forward(input, weight1, bias1, weight2, bias2)
            out2 = out2.view(input.shape[:-1] + (weight2.shape[0],))
        elif input.is_cuda:
            out1, out2, gelu_in = _lib_gelu_dense_fwd(input, weight1, bias1, weight2, bias2)
        else:
            gelu_in = torch.matmul(input, weight1.t()) + bias1
            out1 = _gelu_tanh(gelu_in)
            out2 = torch.matmul(out1, weight2.t()) + bias2
        ctx.save_for_backward(input, weight1, weight2, gelu_in, out1)
        return out2

    @staticmethod
    def backward(ctx, grad_output):
        input, weight1, weight2, gelu_in, output1 = ctx.saved_tensors
        gy = grad_output.contiguous()
        key = _shape_key("gelu_dense_bwd", input, weight1) + (weight2.shape[0],)
        if ctx.native and _use_native(key,
                                      lambda: _fd().linear_gelu_linear_backward(input, gelu_in, output1, weight1,
                                                                                weight2, gy),
                                      lambda: FusedDenseGeluDenseFunc._lib_backward(input, weight1, weight2,
                                                                                    gelu_in, output1, gy)):
            dx, dw1, db1, dw2, db2 = _fd().linear_gelu_linear_backward(input, gelu_in, output1, weight1, weight2, gy)
            return dx.view(input.shape), dw1, db1, dw2, db2
        return FusedDenseGeluDenseFunc._lib_backward(input, weight1, weight2, gelu_in, output1, gy)

    @staticmethod
    def _lib_backward(input, weight1, weight2, gelu_in, output1, grad_output):
        g2 = grad_output.reshape(-1, grad_output.shape[-1])
        h = output1.reshape(-1, output1.shape[-1])
        x2 = input.reshape(-1, input.shape[-1])
        dw2, db2 = _lib_wgrad(g2, h, True)
        lt = _lt(g2, weight2, gelu_in)
        gz = db1 = None
        if lt is not None:
            args = (g2.contiguous(), weight2.contiguous(), gelu_in.reshape(h.shape).contiguous())
            r = lt.dgelu_bgrad(*args, True)  # dGeLU and the bias gradient in the dgrad epilogue
            if r:
                gz, db1 = r
            else:
                r = lt.dgelu_bgrad(*args, False)  # dGeLU epilogue; db1 from the wgrad's BGRADB
                gz = r[0] if r else None
        if gz is None and (_DGELU_ROUTE == "native" and route_mode() != "library" and _native.use_native(g2) and _native.submodule("gemm") is not None
                           and g2.dtype in (torch.float16, torch.bfloat16) and weight2.dtype == g2.dtype
                           and gelu_in.dtype == g2.dtype and g2.shape[1] % 8 == 0 and weight2.shape[1] % 8 == 0):
            gz, db1 = _g().linear_dgrad_bgrad(g2.contiguous(), weight2.contiguous(), _g().EPI_DGELU,
                                              gelu_in.reshape(h.shape).contiguous(), weight1.dtype)
        if gz is None:
            dh = g2.matmul(weight2)
            z = gelu_in.reshape(h.shape)
            if (_native.use_native(dh) and _native.submodule("gemm") is not None and dh.shape[1] % 8 == 0
                    and dh.dtype in (torch.float16, torch.bfloat16) and z.dtype == dh.dtype):
                # dGeLU + bias gradient in one native pass over dh (no GeLU recompute)
                gz, db1 = _g().dgelu_column_sum(dh, z.contiguous())
            else:
                gz = torch.ops.aten.gelu_backward(dh, z, approximate="tanh")
        if db1 is None:
            dw1, db1 = _lib_wgrad(gz, x2, True)
        else:
            dw1, _ = _lib_wgrad(gz, x2, False)
        dx = gz.matmul(weight1).view(input.shape)
        return dx, dw1, db1, dw2, db2


fused_dense_function = half_function(FusedDenseFunc.apply)
dense_no_bias_function = half_function(DenseNoBiasFunc.apply)
fused_dense_gelu_dense_function = half_function(FusedDenseGeluDenseFunc.apply)


class FusedDense(nn.Module):
    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_features))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.kaiming_uniform_(self.weight, a=5 ** 0.5)
        if self.bias is not None:
            bound = 1 / (self.in_features ** 0.5)
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, input):
        if self.bias is not None:
            return fused_dense_function(input, self.weight, self.bias)
        return dense_no_bias_function(input, self.weight)


class FusedDenseGeluDense(nn.Module):
    def __init__(self, in_features, intermediate_features, out_features, bias=True):
        super().__init__()
        assert bias, "DenseGeluDense module without bias is currently not supported"
        self.in_features = in_features
        self.intermediate_features = intermediate_features
        self.out_features = out_features
        self.weight1 = nn.Parameter(torch.empty(intermediate_features, in_features))
        self.bias1 = nn.Parameter(torch.empty(intermediate_features))
        self.weight2 = nn.Parameter(torch.empty(out_features, intermediate_features))
        self.bias2 = nn.Parameter(torch.empty(out_features))
        for w, b, fan_in in ((self.weight1, self.bias1, in_features), (self.weight2, self.bias2, intermediate_features)):
            nn.init.kaiming_uniform_(w, a=5 ** 0.5)
            nn.init.uniform_(b, -1 / fan_in ** 0.5, 1 / fan_in ** 0.5)

    def forward(self, input):
        return fused_dense_gelu_dense_function(input, self.weight1, self.bias1, self.weight2, self.bias2)
