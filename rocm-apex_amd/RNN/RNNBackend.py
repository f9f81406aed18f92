"""Stacked / bidirectional RNN driver (reference apex/RNN/RNNBackend.py:25-365).

Same module structure, stateful cells (``init_hidden`` / ``reset_hidden`` / ``detach_hidden``)
and return layout (``output`` [seq, batch, features]; hidden states per layer, optionally for
every step with ``collect_hidden``).  Different schedule: layers run one after another over the
whole sequence, so each layer's input projection is ONE GEMM over seq*batch rows instead of a
small GEMM per time step (the recurrence only multiplies by W_hh).  Results are identical —
layer l at step t only depends on layer l-1 at steps <= t."""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def is_iterable(x):
    return isinstance(x, (list, tuple))


def flatten_list(tens_list):
    if not is_iterable(tens_list):
        return tens_list
    return torch.stack(list(tens_list), 0)


class RNNCell(nn.Module):
    """One recurrent layer.  ``cell(igates, hidden, w_hh, b_hh)`` computes the new hidden
    state(s) from pre-projected input gates.  Input is never batch-first."""

    def __init__(self, gate_multiplier, input_size, hidden_size, cell, n_hidden_states=2, bias=False,
                 output_size=None):
        super().__init__()
        self.gate_multiplier = gate_multiplier
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.cell = cell
        self.bias = bias
        self.output_size = hidden_size if output_size is None else output_size
        self.gate_size = gate_multiplier * hidden_size
        self.n_hidden_states = n_hidden_states
        self.w_ih = nn.Parameter(torch.empty(self.gate_size, input_size))
        self.w_hh = nn.Parameter(torch.empty(self.gate_size, self.output_size))
        if self.output_size != hidden_size:
            self.w_ho = nn.Parameter(torch.empty(self.output_size, hidden_size))
        self.b_ih = self.b_hh = None
        if bias:
            self.b_ih = nn.Parameter(torch.empty(self.gate_size))
            self.b_hh = nn.Parameter(torch.empty(self.gate_size))
        self.hidden = [None] * n_hidden_states
        self.reset_parameters()

    def new_like(self, new_input_size=None):
        return type(self)(self.gate_multiplier, self.input_size if new_input_size is None else new_input_size,
                          self.hidden_size, self.cell, self.n_hidden_states, self.bias, self.output_size)

    def reset_parameters(self, gain=1):
        stdev = 1.0 / math.sqrt(self.hidden_size)
        for p in self.parameters():
            p.data.uniform_(-stdev, stdev)

    def init_hidden(self, bsz):
        ref = next(self.parameters())
        for i in range(self.n_hidden_states):
            if self.hidden[i] is None or self.hidden[i].size(0) != bsz:
                size = self.output_size if i == 0 else self.hidden_size
                self.hidden[i] = ref.new_zeros(bsz, size)

    def reset_hidden(self, bsz):
        self.hidden = [None] * self.n_hidden_states
        self.init_hidden(bsz)

    def detach_hidden(self):
        if any(h is None for h in self.hidden):
            raise RuntimeError("Must initialize hidden state before you can detach it")
        self.hidden = [h.detach() for h in self.hidden]

    def init_inference(self, bsz):
        self.reset_hidden(bsz)

    def project_inputs(self, seq):
        """[S, B, in] -> [S, B, gates]: the whole sequence in one GEMM."""
        return F.linear(seq, self.w_ih, self.b_ih)

    def step(self, igates):
        state = self.hidden[0] if self.n_hidden_states == 1 else tuple(self.hidden)
        new = self.cell(igates, state, self.w_hh, self.b_hh)
        self.hidden = list(new) if self.n_hidden_states > 1 else [new]
        if self.output_size != self.hidden_size:
            self.hidden[0] = F.linear(self.hidden[0], self.w_ho)
        return tuple(self.hidden)

    def forward(self, input):
        """One step (reference semantics): input [batch, in]."""
        self.init_hidden(input.size(0))
        return self.step(self.project_inputs(input))


class stackedRNN(nn.Module):
    def __init__(self, inputRNN, num_layers=1, dropout=0):
        super().__init__()
        self.dropout = dropout
        if isinstance(inputRNN, RNNCell):
            rnns = [inputRNN] + [inputRNN.new_like(inputRNN.output_size) for _ in range(num_layers - 1)]
        elif isinstance(inputRNN, list):
            assert len(inputRNN) == num_layers, "RNN list length must be equal to num_layers"
            rnns = inputRNN
        else:
            raise RuntimeError("stackedRNN expects an RNNCell or a list of them")
        self.nLayers = len(rnns)
        self.rnns = nn.ModuleList(rnns)

    def forward(self, input, collect_hidden=False, reverse=False):
        seq_len, bsz = input.size(0), input.size(1)
        steps = list(reversed(range(seq_len))) if reverse else list(range(seq_len))
        layer_in = input
        per_layer_states = []  # [layer][step-in-processing-order] -> tuple(hidden states)
        for li, rnn in enumerate(self.rnns):
            rnn.init_hidden(bsz)
            if hasattr(rnn, "project_inputs") and type(rnn).step is RNNCell.step:
                ig = rnn.project_inputs(layer_in)
                run = lambda t, rnn=rnn, ig=ig: rnn.step(ig[t])  # noqa: E731
            else:
                run = lambda t, rnn=rnn, x=layer_in: rnn(x[t])  # noqa: E731
            outs = [None] * seq_len
            states = []
            for t in steps:
                st = run(t)
                outs[t] = st[0]
                states.append(st)
            layer_in = torch.stack(outs, 0)
            if self.dropout and self.training and li + 1 < self.nLayers:
                layer_in = F.dropout(layer_in, self.dropout, True)
            per_layer_states.append(states)
        output = layer_in
        n_hid = self.rnns[0].n_hidden_states
        if collect_hidden:
            # [n_hid][seq (original order)] -> [layer, batch, feat]
            hidden = []
            for i in range(n_hid):
                seq_list = [torch.stack([per_layer_states[k][j][i] for k in range(self.nLayers)], 0)
                            for j in range(seq_len)]
                if reverse:
                    seq_list = list(reversed(seq_list))
                hidden.append(seq_list)
            return output, hidden
        hidden = [torch.stack([per_layer_states[k][-1][i] for k in range(self.nLayers)], 0) for i in range(n_hid)]
        return output, hidden

    def reset_parameters(self):
        for r in self.rnns:
            r.reset_parameters()

    def init_hidden(self, bsz):
        for r in self.rnns:
            r.init_hidden(bsz)

    def detach_hidden(self):
        for r in self.rnns:
            r.detach_hidden()

    def reset_hidden(self, bsz):
        for r in self.rnns:
            r.reset_hidden(bsz)

    def init_inference(self, bsz):
        for r in self.rnns:
            r.init_inference(bsz)


class bidirectionalRNN(nn.Module):
    def __init__(self, inputRNN, num_layers=1, dropout=0):
        super().__init__()
        self.dropout = dropout
        self.fwd = stackedRNN(inputRNN, num_layers=num_layers, dropout=dropout)
        self.bckwrd = stackedRNN(inputRNN.new_like(), num_layers=num_layers, dropout=dropout)
        self.rnns = nn.ModuleList([self.fwd, self.bckwrd])

    def forward(self, input, collect_hidden=False):
        fwd_out, fwd_h = self.fwd(input, collect_hidden=collect_hidden)
        bwd_out, bwd_h = self.bckwrd(input, reverse=True, collect_hidden=collect_hidden)
        output = torch.cat([fwd_out, bwd_out], -1)
        if collect_hidden:
            hiddens = tuple([torch.cat([a, b], -1) for a, b in zip(fh, bh)] for fh, bh in zip(fwd_h, bwd_h))
        else:
            hiddens = tuple(torch.cat([a, b], -1) for a, b in zip(fwd_h, bwd_h))
        return output, hiddens

    def reset_parameters(self):
        for r in self.rnns:
            r.reset_parameters()

    def init_hidden(self, bsz):
        for r in self.rnns:
            r.init_hidden(bsz)

    def detach_hidden(self):
        for r in self.rnns:
            r.detach_hidden()

    def reset_hidden(self, bsz):
        for r in self.rnns:
            r.reset_hidden(bsz)

    def init_inference(self, bsz):
        for r in self.rnns:
            r.init_inference(bsz)
