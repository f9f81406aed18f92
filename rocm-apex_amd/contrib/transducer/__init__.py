"""RNN-T transducer joint / loss (reference apex/contrib/transducer/__init__.py)."""
from .transducer import TransducerJoint, TransducerLoss  # noqa: F401
