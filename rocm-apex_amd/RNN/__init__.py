"""Python RNN backend (reference apex/RNN/__init__.py)."""
from .models import GRU, LSTM, ReLU, Tanh, mLSTM  # noqa: F401

__all__ = ["models", "LSTM", "GRU", "ReLU", "Tanh", "mLSTM"]
