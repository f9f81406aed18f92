"""Functional self attention on the gfx950 flash kernel (reference
apex/contrib/multihead_attn/fast_self_multihead_attn_func.py: ``fast_self_attn_func``, the
``impl="fast"`` path; the scale is 1/sqrt(head_dim) as in the reference's C++ path)."""
from ._core import FuncNamespace, self_attn


def fast_self_attn_func(use_time_mask, is_training, heads, inputs, input_weights, output_weights, input_biases,
                        output_biases, pad_mask, mask_additive, dropout_prob):
    scale = (inputs.size(2) // heads) ** -0.5
    return self_attn(use_time_mask, is_training, heads, scale, inputs, input_weights, output_weights, input_biases,
                     output_biases, pad_mask, mask_additive, dropout_prob, "fast")


class FastSelfAttnFunc(FuncNamespace, fn=fast_self_attn_func):
    pass
