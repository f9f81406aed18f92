"""apex.RNN vs torch.nn RNNs with copied weights (reference tests/L0/run_... had no RNN test; the
behavioural contract is torch's cells)."""
import pytest
import torch

import apex.RNN as R


def _copy(apex_rnn, torch_rnn, layers, bidir=False):
    stacks = apex_rnn.rnns if bidir else [apex_rnn]
    for d, st in enumerate(stacks):
        sfx = "_reverse" if d == 1 else ""
        for l in range(layers):
            cell = st.rnns[l]
            with torch.no_grad():
                cell.w_ih.copy_(getattr(torch_rnn, "weight_ih_l%d%s" % (l, sfx)))
                cell.w_hh.copy_(getattr(torch_rnn, "weight_hh_l%d%s" % (l, sfx)))
                cell.b_ih.copy_(getattr(torch_rnn, "bias_ih_l%d%s" % (l, sfx)))
                cell.b_hh.copy_(getattr(torch_rnn, "bias_hh_l%d%s" % (l, sfx)))


@pytest.mark.parametrize("kind", ["LSTM", "GRU", "ReLU", "Tanh"])
@pytest.mark.parametrize("bidir", [False, True])
def test_rnn_matches_torch(kind, bidir):
    torch.manual_seed(0)
    S, B, I, H = 7, 3, 10, 12
    L = 1 if bidir else 2  # apex stacks each direction independently (torch feeds 2H to layer 2)
    ours = getattr(R, kind)(I, H, L, bidirectional=bidir)
    if kind in ("LSTM", "GRU"):
        ref = getattr(torch.nn, kind)(I, H, L, bidirectional=bidir)
    else:
        ref = torch.nn.RNN(I, H, L, nonlinearity=kind.lower(), bidirectional=bidir)
    _copy(ours, ref, L, bidir)
    x = torch.randn(S, B, I, requires_grad=True)
    out, hid = ours(x)
    rout, rh = ref(x)
    torch.testing.assert_close(out, rout, atol=1e-5, rtol=1e-4)
    h_ref = rh[0] if kind == "LSTM" else rh
    if not bidir:
        torch.testing.assert_close(hid[0], h_ref, atol=1e-5, rtol=1e-4)
    g1 = torch.autograd.grad(out.sum(), x)[0]
    g2 = torch.autograd.grad(rout.sum(), x)[0]
    torch.testing.assert_close(g1, g2, atol=1e-5, rtol=1e-4)


def test_mlstm_and_collect_hidden():
    torch.manual_seed(0)
    m = R.mLSTM(8, 16, 2)
    x = torch.randn(5, 2, 8)
    out, hid = m(x, collect_hidden=True)
    assert out.shape == (5, 2, 16)
    assert len(hid) == 2 and len(hid[0]) == 5 and hid[0][0].shape == (2, 2, 16)
    out.sum().backward()
    lstm = R.LSTM(8, 16, 1, output_size=6)  # recurrent projection
    o, h = lstm(x)
    assert o.shape == (5, 2, 6) and h[1].shape == (1, 2, 16)
