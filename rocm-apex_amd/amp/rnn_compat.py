"""RNN cast support.  The O1 TorchFunctionMode (amp.py) already casts the inputs and flat weights
of ``torch.lstm/gru/rnn_*`` and their cells to the low-precision type, which is what the
reference achieves by replacing ``torch.nn.modules.rnn._VF`` (reference apex/amp/rnn_compat.py)."""
import torch

RNN_NAMES = ["rnn_relu", "rnn_tanh", "gru", "lstm"]


def has_old_rnns():
    return False


def whitelist_rnn_cells(handle, verbose):  # pragma: no cover - handled by the cast mode
    return None
