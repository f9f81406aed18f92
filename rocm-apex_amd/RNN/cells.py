"""RNN cell math (reference apex/RNN/cells.py:1-84 and the torch.nn._functions.rnn cells the
reference imports, which no longer exist in current PyTorch).

Every cell takes PRE-COMPUTED input gates (``igates`` = x W_ih^T + b_ih) so the stacked RNN can
project a whole sequence with one GEMM per layer and only run h W_hh^T inside the recurrence.
"""
import torch
import torch.nn.functional as F


def lstm_cell(igates, hidden, w_hh, b_hh=None):
    hx, cx = hidden
    gates = igates + F.linear(hx, w_hh, b_hh)
    i, f, g, o = gates.chunk(4, 1)
    cy = torch.sigmoid(f) * cx + torch.sigmoid(i) * torch.tanh(g)
    hy = torch.sigmoid(o) * torch.tanh(cy)
    return hy, cy


def gru_cell(igates, hidden, w_hh, b_hh=None):
    hg = F.linear(hidden, w_hh, b_hh)
    i_r, i_z, i_n = igates.chunk(3, 1)
    h_r, h_z, h_n = hg.chunk(3, 1)
    r = torch.sigmoid(i_r + h_r)
    z = torch.sigmoid(i_z + h_z)
    n = torch.tanh(i_n + r * h_n)
    return n + z * (hidden - n)


def relu_cell(igates, hidden, w_hh, b_hh=None):
    return torch.relu(igates + F.linear(hidden, w_hh, b_hh))


def tanh_cell(igates, hidden, w_hh, b_hh=None):
    return torch.tanh(igates + F.linear(hidden, w_hh, b_hh))


# names of the reference (torch.nn._functions.rnn) kept as aliases
LSTMCell, GRUCell, RNNReLUCell, RNNTanhCell = lstm_cell, gru_cell, relu_cell, tanh_cell


def mLSTMCell(input, hidden, w_ih, w_hh, w_mih, w_mhh, b_ih=None, b_hh=None):
    """Multiplicative LSTM step (reference cells.py:61-84): m = (x W_mih^T) * (h W_mhh^T)."""
    hx, cx = hidden
    m = F.linear(input, w_mih) * F.linear(hx, w_mhh)
    gates = F.linear(input, w_ih, b_ih) + F.linear(m, w_hh, b_hh)
    i, f, g, o = gates.chunk(4, 1)
    cy = torch.sigmoid(f) * cx + torch.sigmoid(i) * torch.tanh(g)
    hy = torch.sigmoid(o) * torch.tanh(cy)
    return hy, cy
