"""RNN model constructors (reference apex/RNN/models.py:8-54)."""
import torch.nn as nn
import torch.nn.functional as F

from .RNNBackend import RNNCell, bidirectionalRNN, stackedRNN
from .cells import gru_cell, lstm_cell, mLSTMCell, relu_cell, tanh_cell


def toRNNBackend(inputRNN, num_layers, bidirectional=False, dropout=0):
    if bidirectional:
        return bidirectionalRNN(inputRNN, num_layers, dropout=dropout)
    return stackedRNN(inputRNN, num_layers, dropout=dropout)


def LSTM(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
         output_size=None):
    return toRNNBackend(RNNCell(4, input_size, hidden_size, lstm_cell, 2, bias, output_size), num_layers,
                        bidirectional, dropout=dropout)


def GRU(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
        output_size=None):
    return toRNNBackend(RNNCell(3, input_size, hidden_size, gru_cell, 1, bias, output_size), num_layers,
                        bidirectional, dropout=dropout)


def ReLU(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
         output_size=None):
    return toRNNBackend(RNNCell(1, input_size, hidden_size, relu_cell, 1, bias, output_size), num_layers,
                        bidirectional, dropout=dropout)


def Tanh(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
         output_size=None):
    return toRNNBackend(RNNCell(1, input_size, hidden_size, tanh_cell, 1, bias, output_size), num_layers,
                        bidirectional, dropout=dropout)


class mLSTMRNNCell(RNNCell):
    """Multiplicative LSTM layer (reference apex/RNN/cells.py:12-58): the input projection
    depends on h through m, so it cannot be hoisted out of the recurrence."""

    def __init__(self, input_size, hidden_size, bias=False, output_size=None):
        super().__init__(4, input_size, hidden_size, mLSTMCell, n_hidden_states=2, bias=bias,
                         output_size=output_size)
        self.w_mih = nn.Parameter(self.w_ih.new_empty(self.output_size, self.input_size))
        self.w_mhh = nn.Parameter(self.w_ih.new_empty(self.output_size, self.output_size))
        self.reset_parameters()

    def forward(self, input):
        self.init_hidden(input.size(0))
        self.hidden = list(self.cell(input, tuple(self.hidden), self.w_ih, self.w_hh, self.w_mih, self.w_mhh,
                                     b_ih=self.b_ih, b_hh=self.b_hh))
        if self.output_size != self.hidden_size:
            self.hidden[0] = F.linear(self.hidden[0], self.w_ho)
        return tuple(self.hidden)

    def step(self, igates):  # not used: mLSTM runs through forward()
        raise NotImplementedError

    def new_like(self, new_input_size=None):
        return type(self)(self.input_size if new_input_size is None else new_input_size, self.hidden_size, self.bias,
                          self.output_size)


def mLSTM(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
          output_size=None):
    return toRNNBackend(mLSTMRNNCell(input_size, hidden_size, bias=bias, output_size=output_size), num_layers,
                        bidirectional, dropout=dropout)
