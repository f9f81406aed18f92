"""Multi-head attention modules (reference apex/contrib/multihead_attn/__init__.py)."""
from .encdec_multihead_attn import EncdecMultiheadAttn  # noqa: F401
from .mask_softmax_dropout_func import fast_mask_softmax_dropout_func  # noqa: F401
from .self_multihead_attn import SelfMultiheadAttn  # noqa: F401
