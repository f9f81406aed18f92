"""Weight-norm reparameterization vs torch.nn.utils.weight_norm semantics."""
import torch

from apex.reparameterization import apply_weight_norm, remove_weight_norm


def test_weight_norm_matches_definition_and_trains():
    torch.manual_seed(0)
    m = torch.nn.Linear(20, 40)
    w0 = m.weight.detach().clone()
    apply_weight_norm(m, name="weight")
    assert m.weight_g.shape == (40, 1) and m.weight_v.shape == (40, 20)
    x = torch.randn(5, 20)
    y = m(x)
    torch.testing.assert_close(y, x @ w0.t() + m.bias, atol=1e-5, rtol=1e-5)
    y.sum().backward()
    assert m.weight_g.grad is not None and m.weight_v.grad is not None
    with torch.no_grad():
        m.weight_g.mul_(2.0)
    y2 = m(x)
    torch.testing.assert_close(y2 - m.bias, 2 * (y - m.bias).detach(), atol=1e-5, rtol=1e-5)
    remove_weight_norm(m, name="weight")
    assert "weight" in dict(m.named_parameters()) and not hasattr(m, "weight_g") or "weight_g" not in m._parameters
    torch.testing.assert_close(m.weight, 2 * w0, atol=1e-5, rtol=1e-5)


def test_apply_to_all_parameters_of_a_model():
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.Conv2d(8, 4, 1))
    ref = [p.detach().clone() for p in (net[0].weight, net[2].weight)]
    apply_weight_norm(net)
    names = set(dict(net.named_parameters()).keys())
    assert {"0.weight_g", "0.weight_v", "2.weight_g", "2.weight_v", "0.bias"} <= names
    x = torch.randn(1, 3, 6, 6)
    out = net(x)
    exp = torch.nn.functional.conv2d(torch.relu(torch.nn.functional.conv2d(x, ref[0], net[0].bias)), ref[1],
                                     net[2].bias)
    torch.testing.assert_close(out, exp, atol=1e-5, rtol=1e-5)
    remove_weight_norm(net)
    assert "0.weight" in dict(net.named_parameters())
