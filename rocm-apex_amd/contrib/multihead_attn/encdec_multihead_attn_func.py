"""Functional encoder-decoder attention, torch-math path (reference
apex/contrib/multihead_attn/encdec_multihead_attn_func.py: ``encdec_attn_func``)."""
from ._core import FuncNamespace, encdec_attn


def encdec_attn_func(use_time_mask, is_training, heads, scale, inputs_q, inputs_kv, input_weights_q,
                     input_weights_kv, output_weights, input_biases_q, input_biases_kv, output_biases, mask,
                     dropout_prob):
    return encdec_attn(use_time_mask, is_training, heads, scale, inputs_q, inputs_kv, input_weights_q,
                       input_weights_kv, output_weights, input_biases_q, input_biases_kv, output_biases, mask,
                       dropout_prob, "default")


class EncdecAttnFunc(FuncNamespace, fn=encdec_attn_func):
    pass
