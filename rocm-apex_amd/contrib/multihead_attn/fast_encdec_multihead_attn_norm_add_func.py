"""Functional pre-LayerNorm encoder-decoder attention with the residual dropout-add (reference
apex/contrib/multihead_attn/fast_encdec_multihead_attn_norm_add_func.py:
``fast_encdec_attn_norm_add_func``): out = inputs_q + dropout(attn(layer_norm(inputs_q), inputs_kv))."""
from ._core import FuncNamespace, encdec_attn


def fast_encdec_attn_norm_add_func(use_time_mask, is_training, heads, inputs_q, inputs_kv, lyr_nrm_gamma_weights,
                                   lyr_nrm_beta_weights, input_weights_q, input_weights_kv, output_weights, pad_mask,
                                   dropout_prob):
    scale = (inputs_q.size(2) // heads) ** -0.5
    return encdec_attn(use_time_mask, is_training, heads, scale, inputs_q, inputs_kv, input_weights_q,
                       input_weights_kv, output_weights, None, None, None, pad_mask, dropout_prob, "fast",
                       norm=(lyr_nrm_gamma_weights, lyr_nrm_beta_weights))


class FastEncdecAttnNormAddFunc(FuncNamespace, fn=fast_encdec_attn_norm_add_func):
    pass
