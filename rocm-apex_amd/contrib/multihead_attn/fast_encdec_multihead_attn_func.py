"""Functional encoder-decoder attention on the gfx950 flash kernel (reference
apex/contrib/multihead_attn/fast_encdec_multihead_attn_func.py: ``fast_encdec_attn_func``, no
biases, scale 1/sqrt(head_dim))."""
from ._core import FuncNamespace, encdec_attn


def fast_encdec_attn_func(use_time_mask, is_training, heads, inputs_q, inputs_kv, input_weights_q,
                          input_weights_kv, output_weights, pad_mask, dropout_prob):
    scale = (inputs_q.size(2) // heads) ** -0.5
    return encdec_attn(use_time_mask, is_training, heads, scale, inputs_q, inputs_kv, input_weights_q,
                       input_weights_kv, output_weights, None, None, None, pad_mask, dropout_prob, "fast")


class FastEncdecAttnFunc(FuncNamespace, fn=fast_encdec_attn_func):
    pass
