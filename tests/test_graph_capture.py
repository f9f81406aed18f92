"""hipGraph capture of a whole amp training step (bench.py replays one by default): the sync-free
amp path (device loss scale, skip flag, step counter; multi-tensor tables uploaded through
kernel arguments) must replay exactly like eager steps."""
import pytest
import torch
import torch.nn.functional as F
from torch import nn

from apex import amp
from apex.amp._amp_state import _amp_state
from apex.optimizers import FusedAdam


@pytest.fixture(autouse=True)
def _clean():
    yield
    _amp_state.loss_scalers = []


def _build(seed, dev):
    from apex.models import resnet18

    torch.manual_seed(seed)
    model = resnet18(fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    opt = FusedAdam(model.parameters(), lr=1e-3, weight_decay=1e-4, materialize_master_grads=False)
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, keep_batchnorm_fp32=True,
                                verbosity=0)
    return model, opt


@pytest.mark.gpu
def test_graph_replay_matches_eager_steps():
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(16, 3, 64, 64, device=dev, generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (16,), device=dev, generator=g)

    def make_step(model, opt):
        def step():
            loss = F.cross_entropy(model(x), y)
            opt.zero_grad()
            with amp.scale_loss(loss, opt) as s:
                s.backward()
            opt.step()
            return loss
        return step

    # eager reference: 3 warm-up steps + 4 steps, twice (run-to-run spread of the eager path:
    # library conv algorithms and Adam's ~lr-sized steps on near-zero gradients)
    runs = []
    for _ in range(2):
        _amp_state.loss_scalers = []
        model_e, opt_e = _build(1, dev)
        step_e = make_step(model_e, opt_e)
        eager_losses = [float(step_e()) for _ in range(7)]
        runs.append([p.detach().float().clone() for p in model_e.parameters()])
    ref = runs[0]

    def max_rel(xs, ys):
        return max(float((a - b).norm() / b.norm().clamp_min(1e-6)) for a, b in zip(xs, ys))

    spread = max_rel(runs[1], runs[0])

    _amp_state.loss_scalers = []
    model_g, opt_g = _build(1, dev)
    step_g = make_step(model_g, opt_g)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        warm = [float(step_g()) for _ in range(3)]
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        static_loss = step_g()  # captured, not executed
    losses = []
    for _ in range(4):
        graph.replay()
        losses.append(float(static_loss))
    torch.cuda.synchronize()
    torch.testing.assert_close(torch.tensor(warm + losses), torch.tensor(eager_losses), rtol=2e-2, atol=2e-2)
    # whole-tensor relative error, bounded by the eager run-to-run spread
    got = max_rel([p.detach().float() for p in model_g.parameters()], ref)
    assert got <= max(3 * spread, 5e-3), (got, spread)
    # the device step counter advanced once per replay
    st = opt_g.param_groups[0]["_step_t"]
    assert int(st.item()) == 7
