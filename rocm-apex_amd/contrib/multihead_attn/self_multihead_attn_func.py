"""Functional self attention, torch-math path (reference
apex/contrib/multihead_attn/self_multihead_attn_func.py: ``self_attn_func``, the ``impl="default"``
path of SelfMultiheadAttn).  Same argument order as the reference."""
from ._core import FuncNamespace, self_attn


def self_attn_func(use_time_mask, is_training, heads, scale, inputs, input_weights, output_weights, input_biases,
                   output_biases, mask, is_additive_mask, dropout_prob):
    return self_attn(use_time_mask, is_training, heads, scale, inputs, input_weights, output_weights, input_biases,
                     output_biases, mask, is_additive_mask, dropout_prob, "default")


class SelfAttnFunc(FuncNamespace, fn=self_attn_func):
    pass
