"""ASP 2:4 sparsity.  Model: reference apex/contrib/sparsity/test/toy_problem.py and
checkpointing_test_*.py (train dense, prune, keep training with masks applied, masks survive a
state_dict round trip)."""
import torch

from apex.contrib.sparsity import ASP, create_mask
from apex.contrib.sparsity.sparse_masklib import valid_2d_patterns


def test_masks_have_2_of_4_structure():
    torch.manual_seed(0)
    w = torch.randn(32, 64)
    m = create_mask(w, "m4n2_1d").bool()
    assert (m.view(32, 16, 4).sum(-1) == 2).all()
    # keeps the two largest magnitudes of every group
    g = w.abs().view(32, 16, 4)
    kept_min = torch.where(m.view(32, 16, 4), g, torch.full_like(g, 1e9)).amin(-1)
    drop_max = torch.where(~m.view(32, 16, 4), g, torch.full_like(g, -1)).amax(-1)
    assert (kept_min >= drop_max).all()
    assert valid_2d_patterns(4, 2, "cpu").shape[0] == 90
    for pat in ("m4n2_2d_best", "m4n2_2d_greedy"):
        m2 = create_mask(w, pat).bool().view(8, 4, 16, 4)
        assert (m2.sum(-1) <= 2).all() and (m2.sum(1) <= 2).all()
        if pat.endswith("best"):
            assert (m2.sum(-1) == 2).all() and (m2.sum(1) == 2).all()
    conv = torch.randn(16, 32, 3, 3)
    mc = create_mask(conv).bool()
    assert (mc.permute(2, 3, 0, 1).reshape(-1, 8, 4).sum(-1) == 2).all()


def test_asp_training_flow_and_restore():
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 16),
                                torch.nn.Linear(16, 3))  # last layer: out dim 3 -> auto-skipped
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    ASP._reset()
    try:
        ASP.init_model_for_pruning(model, "m4n2_1d", verbosity=0, allow_recompute_mask=True)
        ASP.init_optimizer_for_pruning(opt)
        assert not ASP.is_sparsity_enabled()
        dense = model[0].weight.detach().clone()
        ASP.compute_sparse_masks()
        assert ASP.is_sparsity_enabled()
        w = model[0].weight
        assert float((w == 0).float().mean()) == 0.5
        for _ in range(3):
            opt.zero_grad()
            model(torch.randn(8, 32)).sum().backward()
            opt.step()
        mask = getattr(model[0], "__weight_mma_mask")
        assert (model[0].weight[~mask] == 0).all()
        sd = model.state_dict()
        assert "0.__weight_mma_mask" in sd
        ASP.restore_pruned_weights()
        assert not ASP.is_sparsity_enabled()
        # pruned entries got their dense values back
        torch.testing.assert_close(model[0].weight[~mask], dense[~mask])
    finally:
        ASP._reset()
