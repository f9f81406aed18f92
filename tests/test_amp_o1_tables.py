"""Table-driven O1 / O4 cast tests: what dtype every patched op produces for every input dtype,
and that gradients come back in the dtype of the input.  Capability of the reference's
tests/L0/run_amp/{test_basic_casts,test_promotion,test_rnn,test_cache}.py with the expectation
tables of tests/L0/run_amp/utils.py:3-27 (ALWAYS_LOW / ALWAYS_FLOAT / MATCH_INPUT).

Each case runs on the CPU tier and again on the GPU tier (``cuda`` parametrization, marked gpu):
the O1 patching is device-independent, the kernels behind it are not."""
import functools
import itertools
import random

import pytest
import torch
import torch.nn.functional as F
from torch import nn

from apex import amp
from apex.amp._amp_state import _amp_state

LOWS = [torch.float16, torch.bfloat16]
DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
H, B, C, K, T = 64, 16, 16, 3, 10


def always(low):
    return {torch.float32: low, low: low}


def always_float(low):
    return {torch.float32: torch.float32, low: torch.float32}


def match(low):
    return {torch.float32: torch.float32, low: low}


@pytest.fixture
def handle(request):
    low, allow = request.param if isinstance(request.param, tuple) else (request.param, False)
    h = amp.init(enabled=True, patch_type=low, allow_banned=allow)
    yield low
    h._deactivate()
    _amp_state.handle = None


def _layer_case(fns, table, shape, device, backward=True):
    for fn, (in_dt, out_dt) in itertools.product(fns, table.items()):
        x = torch.randn(shape, dtype=in_dt, device=device).requires_grad_()
        y = fn(x)
        assert y.dtype == out_dt, (fn, in_dt, y.dtype, out_dt)
        if backward:
            y.float().sum().backward()
            assert x.grad.dtype == in_dt, (fn, in_dt, x.grad.dtype)


def _cpu_low_unsupported(device, low, what):
    # CPU kernels for some half ops are missing in PyTorch; the casting logic is still exercised on
    # the GPU tier for them
    if device == "cpu" and low == torch.float16 and what in ("conv", "rnn"):
        pytest.skip("PyTorch has no fp16 CPU kernel for " + what)


# ------------------------------------------------------------------ basic casts (modules + F)
LAYER_CASES = {
    "linear": ("always", lambda d: (lambda m: [m, functools.partial(F.linear, weight=m.weight, bias=m.bias)])(
        nn.Linear(H, H).to(d)), (B, H)),
    "conv2d": ("always", lambda d: (lambda m: [m, functools.partial(F.conv2d, weight=m.weight, bias=m.bias)])(
        nn.Conv2d(C, C, K).to(d)), (B, C, H, H)),
    "softmax": ("float", lambda d: [nn.Softmax(dim=1), functools.partial(F.softmax, dim=1)], (B, H)),
    "group_norm": ("float", lambda d: [nn.GroupNorm(4, C).to(d)], (B, C, H, H)),
    "relu": ("match", lambda d: [nn.ReLU(), F.relu], (B, H)),
    "layer_norm": ("float", lambda d: [nn.LayerNorm(H).to(d)], (B, H)),
    "log_softmax": ("float", lambda d: [functools.partial(F.log_softmax, dim=1)], (B, H)),
    "gelu": ("float", lambda d: [F.gelu], (B, H)),
}


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
@pytest.mark.parametrize("case", sorted(LAYER_CASES))
def test_layer_casts(case, handle, device):
    low = handle
    kind, make, shape = LAYER_CASES[case]
    if case == "conv2d":
        _cpu_low_unsupported(device, low, "conv")
    table = {"always": always, "float": always_float, "match": match}[kind](low)
    _layer_case(make(device), table, shape, device)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
def test_mse_loss_is_float(handle, device):
    target = torch.randn(B, H, device=device)
    mod = nn.MSELoss()
    _layer_case([lambda x: mod(x, target), functools.partial(F.mse_loss, target=target)], always_float(handle),
                (B, H), device)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
def test_batch_norm_matches_input(handle, device):
    m = nn.BatchNorm2d(C).to(device)
    _layer_case([m], match(handle), (B, C, H, H), device)
    m.eval()
    f = functools.partial(F.batch_norm, running_mean=m.running_mean, running_var=m.running_var, weight=m.weight,
                          bias=m.bias, training=False)
    _layer_case([m, f], match(handle), (B, C, H, H), device, backward=False)


# ------------------------------------------------------------------ banned functions
def _bce(device, low):
    target = torch.rand(B, H, device=device)
    mod = nn.BCELoss()
    return [lambda x: mod(x, target), functools.partial(F.binary_cross_entropy, target=target)], \
        torch.rand(B, H, dtype=low, device=device)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
def test_bce_raises_by_default(handle, device):
    fns, x = _bce(device, handle)
    for fn in fns:
        with pytest.raises(NotImplementedError):
            fn(x)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", [(low, True) for low in LOWS], indirect=True)
def test_bce_is_float_with_allow_banned(handle, device):
    fns, x = _bce(device, handle)
    for fn in fns:
        assert fn(x).dtype == torch.float32


# ------------------------------------------------------------------ Tensor methods / operators
TENSOR_CASES = {
    "matmul_method": ("always", lambda o: [lambda x: x.matmul(o), lambda x: o.matmul(x)], (H, H)),
    "matmul_op": ("always", lambda o: [lambda x: x @ o, lambda x: o @ x], (H, H)),
    "pow_method": ("float", lambda o: [lambda x: x.pow(2.0)], (B, H)),
    "pow_op": ("float", lambda o: [lambda x: x ** 2.0], (B, H)),
    "sum": ("float", lambda o: [lambda x: x.sum()], (B, H)),
    "exp": ("float", lambda o: [lambda x: x.exp()], (B, H)),
}


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
@pytest.mark.parametrize("case", sorted(TENSOR_CASES))
def test_tensor_casts(case, handle, device):
    kind, make, shape = TENSOR_CASES[case]
    other = torch.randn(H, H, device=device)
    table = {"always": always, "float": always_float}[kind](handle)
    _layer_case(make(other), table, shape, device)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
def test_cpu_copy_is_float(handle, device):
    _layer_case([lambda x: x.cpu()], always_float(handle), (B, H), device)


# ------------------------------------------------------------------ promotion
def _binary_promote(fns, low, device, inplace=False):
    for fn, (xt, yt) in itertools.product(fns, itertools.product([low, torch.float32], repeat=2)):
        x_leaf = torch.randn(B, dtype=xt, device=device).requires_grad_()
        x = x_leaf.clone() if inplace else x_leaf
        y = torch.randn(B, dtype=yt, device=device)
        out = fn(x, y)
        if inplace:
            assert out.dtype == x.dtype
        else:
            assert out.dtype == (torch.float32 if torch.float32 in (xt, yt) else low), (xt, yt, out.dtype)
        out.float().sum().backward()
        assert x_leaf.grad.dtype == xt


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
@pytest.mark.parametrize("op", ["mul", "atan2", "add", "sub", "div"])
def test_binary_matches_widest(op, handle, device):
    fns = [lambda x, y: getattr(torch, op)(x, y), lambda x, y: getattr(x, op)(y)]
    _binary_promote(fns, handle, device)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
def test_inplace_add_matches_self(handle, device):
    _binary_promote([lambda x, y: x.add_(y)], handle, device, inplace=True)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
def test_cat_and_stack_match_widest(handle, device):
    ys = [torch.randn(B, dtype=handle, device=device) for _ in range(5)]
    for seq_op in (torch.cat, torch.stack):
        assert seq_op(ys + [torch.randn(B, device=device)]).dtype == torch.float32
        assert seq_op(ys + [torch.randn(B, dtype=handle, device=device)]).dtype == handle


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
def test_inplace_exp_is_error_for_low(handle, device):
    xs = torch.randn(B, device=device)
    xs.exp_()
    assert xs.dtype == torch.float32
    with pytest.raises(NotImplementedError):
        torch.randn(B, dtype=handle, device=device).exp_()


# ------------------------------------------------------------------ RNNs (O1: always low precision)
@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
@pytest.mark.parametrize("cell_type,tuple_state", [(nn.RNNCell, False), (nn.GRUCell, False), (nn.LSTMCell, True)])
def test_rnn_cells_are_low(cell_type, tuple_state, handle, device):
    low = handle
    _cpu_low_unsupported(device, low, "rnn")
    cell = cell_type(H, H).to(device)
    for typ in (torch.float32, low):
        xs = [torch.randn(B, H, dtype=typ, device=device).requires_grad_() for _ in range(T)]
        z = torch.zeros(B, H, dtype=typ, device=device)
        hidden = (z, z.clone()) if tuple_state else z
        outs = []
        for x in xs:
            hidden = cell(x, hidden)
            outs.append(hidden[0] if tuple_state else hidden)
        assert all(o.dtype == low for o in outs)
        outs[-1].float().sum().backward()
        assert all(x.grad.dtype == x.dtype for x in xs)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
@pytest.mark.parametrize("rnn_type,tuple_state", [(nn.RNN, False), (nn.GRU, False), (nn.LSTM, True)])
@pytest.mark.parametrize("layers,bidir", [(1, False), (2, False), (2, True)])
def test_rnns_are_low(rnn_type, tuple_state, layers, bidir, handle, device):
    low = handle
    _cpu_low_unsupported(device, low, "rnn")
    kw = {"nonlinearity": "relu"} if rnn_type is nn.RNN else {}
    rnn = rnn_type(input_size=H, hidden_size=H, num_layers=layers, bidirectional=bidir, **kw).to(device)
    for typ in (torch.float32, low):
        x = torch.randn(T, B, H, dtype=typ, device=device).requires_grad_()
        z = torch.zeros(layers * (2 if bidir else 1), B, H, dtype=typ, device=device)
        out, _ = rnn(x, (z, z.clone()) if tuple_state else z)
        assert out.dtype == low
        out[-1].float().sum().backward()
        assert x.grad.dtype == x.dtype


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("handle", LOWS, indirect=True)
def test_rnn_packed_sequence_is_low(handle, device):
    low = handle
    _cpu_low_unsupported(device, low, "rnn")
    rnn = nn.RNN(input_size=H, hidden_size=H, num_layers=2).to(device)
    rng = random.Random(0)
    for typ in (torch.float32, low):
        x = torch.randn(T, B, H, dtype=typ, device=device).requires_grad_()
        lens = torch.tensor(sorted((rng.randint(T // 2, T) for _ in range(B)), reverse=True), dtype=torch.int64)
        packed = nn.utils.rnn.pack_padded_sequence(x, lens)
        out, _ = rnn(packed, torch.zeros(2, B, H, dtype=typ, device=device))
        assert out.data.dtype == low
        out.data.float().sum().backward()
        assert x.grad.dtype == x.dtype


# ------------------------------------------------------------------ weight-cast cache across train/eval
class _Whitelist(nn.Module):
    def __init__(self, dtype, device):
        super().__init__()
        self.weight = nn.Parameter(torch.arange(64, device=device, dtype=dtype).view(8, 8))

    @staticmethod
    def ops(x, w):
        return x.mm(w).mm(w).sum()

    def forward(self, x):
        return self.ops(x, self.weight)


class _Blacklist(nn.Module):
    def __init__(self, dtype, device):
        super().__init__()
        self.weight = nn.Parameter(torch.arange(16, device=device, dtype=dtype).view(2, 8))

    @staticmethod
    def ops(x, w):
        return (x + torch.pow(w, 2) + torch.pow(w, 2)).sum()

    def forward(self, x):
        return self.ops(x, self.weight)


class _Promote(nn.Module):
    def __init__(self, dtype, device):
        super().__init__()
        self.weight = nn.Parameter(torch.arange(16, device=device, dtype=dtype).view(2, 8))

    @staticmethod
    def ops(x, w):
        return ((x * w) * w).sum()

    def forward(self, x):
        return self.ops(x, self.weight)


CACHE_CASES = [(mod, wdt, lvl) for lvl, low in (("O1", torch.float16), ("O4", torch.bfloat16))
               for mod in (_Whitelist, _Blacklist, _Promote) for wdt in (low, torch.float32)]


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("module,wdtype,opt_level", CACHE_CASES,
                         ids=["{}-{}-{}".format(m.__name__.strip("_"), str(w).split(".")[1], o) for m, w, o in
                              CACHE_CASES])
def test_weight_cache_train_eval_train(module, wdtype, opt_level, device):
    """The per-iteration weight-cast cache must not hand a stale cast to training after an eval
    pass (or after the weight changed): every training step's gradient matches an fp32 recompute."""
    if device == "cpu" and wdtype == torch.float16 and module is _Whitelist:
        pytest.skip("fp16 mm is slow / missing on the CPU")
    x = torch.ones(2, 8, device=device)
    model = module(wdtype, device)
    opt = torch.optim.SGD(model.parameters(), lr=1.0)
    _amp_state.allow_incoming_model_not_fp32 = True
    try:
        model, opt = amp.initialize(model, opt, opt_level=opt_level, verbosity=0)
    finally:
        _amp_state.allow_incoming_model_not_fp32 = False
    try:
        def step():
            for p in model.parameters():
                p.grad = None
            loss = model(x).sum()
            _amp_state.loss_scalers[0]._loss_scale = 4.0
            with amp.scale_loss(loss, opt) as s:
                s.backward()
            grads = [p.grad for p in model.parameters() if p.grad is not None]
            assert len(grads) == 1 and model.weight.grad.dtype == model.weight.dtype
            w32 = model.weight.detach().clone().float().requires_grad_()
            module.ops(x.detach().clone().float(), w32).backward()
            assert torch.allclose(model.weight.grad.float(), w32.grad)
            model.weight.data -= 1.0

        step()
        with torch.no_grad():
            model(x).sum()
        step()
    finally:
        _amp_state.handle._deactivate()
        _amp_state.handle = None
        _amp_state.loss_scalers = []
