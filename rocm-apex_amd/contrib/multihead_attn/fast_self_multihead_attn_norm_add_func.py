"""Functional pre-LayerNorm self attention with the residual dropout-add (reference
apex/contrib/multihead_attn/fast_self_multihead_attn_norm_add_func.py:
``fast_self_attn_norm_add_func``): out = inputs + dropout(attn(layer_norm(inputs)))."""
from ._core import FuncNamespace, self_attn


def fast_self_attn_norm_add_func(use_time_mask, is_training, heads, inputs, lyr_nrm_gamma_weights,
                                 lyr_nrm_beta_weights, input_weights, output_weights, pad_mask, dropout_prob):
    scale = (inputs.size(2) // heads) ** -0.5
    return self_attn(use_time_mask, is_training, heads, scale, inputs, input_weights, output_weights, None, None,
                     pad_mask, False, dropout_prob, "fast", norm=(lyr_nrm_gamma_weights, lyr_nrm_beta_weights))


class FastSelfAttnNormAddFunc(FuncNamespace, fn=fast_self_attn_norm_add_func):
    pass
