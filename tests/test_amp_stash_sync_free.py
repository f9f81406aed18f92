"""amp O2 with materialized fp32 master grads (FusedAdam's default, the reference's path): the
scale_loss exit accumulates the fresh, still-scaled grads of fp32 params onto their stashed grads
(e.g. zeroed rather than freed by the training loop).  The sync-free scaler does that with the
device loss scale — no host read of the scale per step — and must give bitwise the result of
reading the scale on the host in the same (sync-free) run (apex/amp/_process_optimizer.py
post_backward_models_are_masters; reference apex/amp/_process_optimizer.py
post_backward_models_are_masters, scaler.loss_scale())."""
import pytest
import torch


def _run(device_scale, steps=4, guard=False):
    from apex import amp
    from apex.amp import _process_optimizer as po
    from apex.optimizers import FusedAdam

    prev = po._STASH_DEVICE_SCALE
    po._STASH_DEVICE_SCALE = device_scale
    try:
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.BatchNorm1d(128), torch.nn.ReLU(),
                                    torch.nn.Linear(128, 16)).cuda()
        opt = FusedAdam(model.parameters(), lr=1e-2, materialize_master_grads=True)
        model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16,
                                    keep_batchnorm_fp32=True, loss_scale="dynamic", verbosity=0)
        g = torch.Generator(device="cuda").manual_seed(1)
        xs = [torch.randn(32, 64, device="cuda", generator=g) for _ in range(steps)]
        ys = [torch.randint(0, 16, (32,), device="cuda", generator=g) for _ in range(steps)]
        for i in range(steps):
            for p in model.parameters():  # zeroed, not freed: the exit finds stashed fp32 grads
                if p.grad is not None:
                    p.grad.zero_()
            if guard and i >= 2:
                torch.cuda.set_sync_debug_mode("error")
            try:
                loss = torch.nn.functional.cross_entropy(model(xs[i]).float(), ys[i])
                with amp.scale_loss(loss, opt) as sl:
                    sl.backward()
                opt.step()
            finally:
                torch.cuda.set_sync_debug_mode("default")
        torch.cuda.synchronize()
        return [p.detach().float().clone() for p in model.parameters()]
    finally:
        po._STASH_DEVICE_SCALE = prev


@pytest.mark.gpu
def test_gpu_stashed_fp32_grad_exit_is_sync_free_and_bitwise_the_host_path():
    want = _run(False)
    got = _run(True, guard=True)
    assert len(got) == len(want)
    for i, (a, b) in enumerate(zip(got, want)):
        assert torch.equal(a, b), (i, float((a - b).abs().max()), float(b.abs().max()))
