"""Megatron transformer language model built on apex.transformer's TP layers
(reference apex/transformer/testing/standalone_gpt.py:54-1425, shared by the standalone GPT and
BERT).

MI355X-first differences from the reference:
  * attention is ONE fused flash kernel per direction (``apex.ops.attention``: causal for GPT,
    key-padding bias for BERT) reading Q/K/V as strided views of the fused QKV projection —
    the reference materialises [b*np, sq, sk] scores, a fused masked softmax and a dropout mask;
  * attention-probability dropout is the kernel's counter-based hash seeded per
    tensor-parallel rank (so TP ranks draw independent masks without forking a CUDA RNG);
  * LayerNorm is the gfx950 FusedLayerNorm; bias+GeLU and bias+dropout+residual are fused
    elementwise ops on the [s, b, h] activations.
Activations are [seq, batch, hidden] throughout, as in Megatron."""
import math

import torch
import torch.nn.functional as F

from ...normalization import FusedLayerNorm as LayerNorm
from ...normalization.fused_layer_norm import layer_norm_with_residual
from ...ops.attention import flash_attn_func, packed_qkv_self_attention
from ..functional.fused_bias_dropout_add import fused_bias_dropout_add
from .. import parallel_state, tensor_parallel
from ..enums import AttnMaskType, AttnType, LayerType, ModelType
from ..utils import divide
from .global_vars import get_args


def init_method_normal(sigma):
    def init_(tensor):
        return torch.nn.init.normal_(tensor, mean=0.0, std=sigma)

    return init_


def scaled_init_method_normal(sigma, num_layers):
    std = sigma / math.sqrt(2.0 * num_layers)

    def init_(tensor):
        return torch.nn.init.normal_(tensor, mean=0.0, std=std)

    return init_


def gelu_impl(x):
    return 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * x * (1.0 + 0.044715 * x * x)))


def openai_gelu(x):
    return gelu_impl(x)


def erf_gelu(x):
    return x * 0.5 * (torch.erf(x / 1.41421) + 1.0)


def bias_gelu(bias, y):
    return F.gelu(y + bias, approximate="tanh")


def bias_dropout_add(x, bias, residual, prob, training):
    if bias is not None:
        x = x + bias
    return residual + F.dropout(x, p=prob, training=training)


def get_bias_dropout_add(training):
    """The fused gfx950 epilogue (apex.transformer.functional.fused_bias_dropout_add): one kernel
    per direction, mask regenerated from the "hidden_dropout" counter stream (restored by
    activation checkpointing like the device RNG)."""
    def _f(x, bias, residual, prob):
        off = tensor_parallel.get_counter_rng_streams().next("hidden_dropout")
        return fused_bias_dropout_add(x, bias, residual, prob, training, get_args().seed, off)

    return _f


def get_linear_layer(rows, columns, init_method):
    layer = torch.nn.Linear(rows, columns)
    init_method(layer.weight)
    with torch.no_grad():
        layer.bias.zero_()
    return layer


class MegatronModule(torch.nn.Module):
    """Adds word-embedding sharing between the first and last pipeline stage
    (reference standalone_gpt.py:70-166)."""

    def __init__(self, share_word_embeddings=True):
        super().__init__()
        self.share_word_embeddings = share_word_embeddings

    def state_dict_for_save_checkpoint(self, destination=None, prefix="", keep_vars=False):
        return self.state_dict(destination=destination, prefix=prefix, keep_vars=keep_vars)

    def word_embeddings_weight(self):
        if self.pre_process:
            return self.language_model.embedding.word_embeddings.weight
        if not self.share_word_embeddings:
            raise Exception("word_embeddings_weight() called for last stage, but share_word_embeddings is false")
        return self.word_embeddings.weight

    def initialize_word_embeddings(self, init_method_normal):
        args = get_args()
        if not self.share_word_embeddings:
            raise Exception("initialize_word_embeddings() was called but share_word_embeddings is false")
        if args.pipeline_model_parallel_size == 1:
            return
        if parallel_state.is_pipeline_last_stage() and not self.pre_process:
            self.word_embeddings = tensor_parallel.VocabParallelEmbedding(
                args.padded_vocab_size, args.hidden_size, init_method=init_method_normal(args.init_method_std),
                use_cpu_initialization=args.use_cpu_initialization)
            with torch.no_grad():
                self.word_embeddings.weight.zero_()
            self.word_embeddings.weight.shared = True
        if torch.distributed.is_initialized() and (parallel_state.is_pipeline_first_stage() or
                                                   parallel_state.is_pipeline_last_stage()):
            torch.distributed.all_reduce(self.word_embeddings_weight().data,
                                         group=parallel_state.get_embedding_group())


class ParallelMLP(MegatronModule):
    """h -> 4h (column parallel) -> GeLU -> h (row parallel)."""

    def __init__(self, init_method, output_layer_init_method):
        super().__init__()
        args = get_args()
        self.dense_h_to_4h = tensor_parallel.ColumnParallelLinear(
            args.hidden_size, args.ffn_hidden_size, gather_output=False, init_method=init_method, skip_bias_add=True,
            use_cpu_initialization=args.use_cpu_initialization, params_dtype=args.params_dtype,
            sequence_parallel_enabled=args.sequence_parallel)
        self.bias_gelu_fusion = args.bias_gelu_fusion
        self.activation_func = openai_gelu if args.openai_gelu else (erf_gelu if args.onnx_safe else F.gelu)
        self.dense_4h_to_h = tensor_parallel.RowParallelLinear(
            args.ffn_hidden_size, args.hidden_size, input_is_parallel=True, init_method=output_layer_init_method,
            skip_bias_add=True, use_cpu_initialization=args.use_cpu_initialization, params_dtype=args.params_dtype,
            sequence_parallel_enabled=args.sequence_parallel)

    def _use_fused(self, x):
        from ...fused_dense.fused_dense import fused_linear_available

        w1, b1 = self.dense_h_to_4h.weight, self.dense_h_to_4h.bias
        w2, b2 = self.dense_4h_to_h.weight, self.dense_4h_to_h.bias
        return (self.bias_gelu_fusion and not self.dense_h_to_4h.sequence_parallel_enabled and b1 is not None
                and b2 is not None and fused_linear_available(x, w1, b1) and w2.dtype == x.dtype
                and b2.dtype == x.dtype and w2.shape[0] % 8 == 0 and x.is_contiguous())

    def forward(self, hidden_states):
        if self._use_fused(hidden_states):
            # one fused_dense pair on the local shard: GEMM + bias + GeLU(tanh) epilogue (aux saved for
            # the backward), then GEMM; the row-parallel bias is added after the TP reduction
            from ...fused_dense.fused_dense import FusedDenseGeluDenseFunc

            tp = parallel_state.get_tensor_model_parallel_world_size()
            x = tensor_parallel.copy_to_tensor_model_parallel_region(hidden_states) if tp > 1 else hidden_states
            b2 = self.dense_4h_to_h.bias
            out = FusedDenseGeluDenseFunc.apply(x, self.dense_h_to_4h.weight, self.dense_h_to_4h.bias,
                                                self.dense_4h_to_h.weight, b2 if tp == 1 else torch.zeros_like(b2))
            if tp > 1:
                return tensor_parallel.reduce_from_tensor_model_parallel_region(out), b2
            return out, None
        inter, bias = self.dense_h_to_4h(hidden_states)
        if self.bias_gelu_fusion:
            inter = bias_gelu(bias, inter)
        else:
            inter = self.activation_func(inter + bias)
        return self.dense_4h_to_h(inter)




class ParallelAttention(MegatronModule):
    """Self / cross attention over the local heads of this tensor-parallel rank."""

    def __init__(self, init_method, output_layer_init_method, layer_number, attention_type=AttnType.self_attn,
                 attn_mask_type=AttnMaskType.padding):
        super().__init__()
        args = get_args()
        self.layer_number = max(1, layer_number)
        self.attention_type = attention_type
        self.attn_mask_type = attn_mask_type
        self.params_dtype = args.params_dtype
        projection_size = args.kv_channels * args.num_attention_heads
        world = parallel_state.get_tensor_model_parallel_world_size()
        self.hidden_size_per_partition = divide(projection_size, world)
        self.hidden_size_per_attention_head = divide(projection_size, args.num_attention_heads)
        self.num_attention_heads_per_partition = divide(args.num_attention_heads, world)
        kw = dict(gather_output=False, init_method=init_method, use_cpu_initialization=args.use_cpu_initialization,
                  params_dtype=args.params_dtype, sequence_parallel_enabled=args.sequence_parallel)
        if attention_type == AttnType.self_attn:
            self.query_key_value = tensor_parallel.ColumnParallelLinear(args.hidden_size, 3 * projection_size, **kw)
        else:
            self.query = tensor_parallel.ColumnParallelLinear(args.hidden_size, projection_size, **kw)
            self.key_value = tensor_parallel.ColumnParallelLinear(args.hidden_size, 2 * projection_size, **kw)
        self.scale = 1.0 / math.sqrt(self.hidden_size_per_attention_head)
        self.attention_dropout = args.attention_dropout
        self.dense = tensor_parallel.RowParallelLinear(
            projection_size, args.hidden_size, input_is_parallel=True, init_method=output_layer_init_method,
            skip_bias_add=True, use_cpu_initialization=args.use_cpu_initialization, params_dtype=args.params_dtype,
            sequence_parallel_enabled=args.sequence_parallel)
        self.seed_base = (args.seed + 2718 * (parallel_state.get_tensor_model_parallel_rank() + 1)) & 0x7FFFFFFF

    def forward(self, hidden_states, attention_mask, encoder_output=None, inference_params=None):
        np_, hn = self.num_attention_heads_per_partition, self.hidden_size_per_attention_head
        causal = self.attn_mask_type == AttnMaskType.causal
        p = self.attention_dropout if self.training else 0.0
        if self.attention_type == AttnType.self_attn:
            mixed, _ = self.query_key_value(hidden_states)
            s, b = mixed.shape[:2]
            offset = tensor_parallel.get_counter_rng_streams().next("attention")
            # q / k / v stay strided views of the projection; context comes back in [s, b, h]
            ctx = packed_qkv_self_attention(mixed.view(s, b, np_, 3 * hn), self.scale, causal=causal,
                                            bias=None if causal else attention_mask, dropout_p=p,
                                            seed=self.seed_base, offset=offset)
            return self.dense(ctx)
        kv, _ = self.key_value(encoder_output)
        sk, b = kv.shape[:2]
        kv = kv.view(sk, b, np_, 2 * hn)
        k, v = kv[..., :hn], kv[..., hn:]
        q, _ = self.query(hidden_states)
        q = q.view(q.size(0), b, np_, hn)
        # [s, b, np, hn] views -> [b, s, np, hn] views (no copy)
        q4, k4, v4 = (t.permute(1, 0, 2, 3) for t in (q, k, v))
        bias = None if causal else attention_mask
        offset = tensor_parallel.get_counter_rng_streams().next("attention")
        ctx = flash_attn_func(q4, k4, v4, dropout_p=p, softmax_scale=self.scale, causal=causal, bias=bias,
                              seed=self.seed_base, offset=offset)
        sq, b = q.shape[0], q.shape[1]
        ctx = ctx.transpose(0, 1).reshape(sq, b, np_ * hn)
        return self.dense(ctx)


class ParallelTransformerLayer(MegatronModule):
    def __init__(self, init_method, output_layer_init_method, layer_number, layer_type=LayerType.encoder,
                 self_attn_mask_type=AttnMaskType.padding):
        super().__init__()
        args = get_args()
        self.layer_number = layer_number
        self.layer_type = layer_type
        self.apply_residual_connection_post_layernorm = args.apply_residual_connection_post_layernorm
        self.bf16, self.fp32_residual_connection = args.bf16, args.fp32_residual_connection
        self.input_layernorm = LayerNorm(args.hidden_size, eps=args.layernorm_epsilon)
        self.self_attention = ParallelAttention(init_method, output_layer_init_method, layer_number,
                                                attention_type=AttnType.self_attn,
                                                attn_mask_type=self_attn_mask_type)
        self.hidden_dropout = args.hidden_dropout
        self.post_attention_layernorm = LayerNorm(args.hidden_size, eps=args.layernorm_epsilon)
        if layer_type == LayerType.decoder:
            self.inter_attention = ParallelAttention(init_method, output_layer_init_method, layer_number,
                                                     attention_type=AttnType.cross_attn)
            self.post_inter_attention_layernorm = LayerNorm(args.hidden_size, eps=args.layernorm_epsilon)
        self.mlp = ParallelMLP(init_method, output_layer_init_method)

    def forward(self, hidden_states, attention_mask, encoder_output=None, enc_dec_attn_mask=None,
                inference_params=None):
        post = self.apply_residual_connection_post_layernorm
        # pre-LN: the block input feeds the norm AND the residual add; one autograd node for both
        # sums their gradients inside the LayerNorm backward kernel
        if post:
            ln_out, res_in = self.input_layernorm(hidden_states), None
        else:
            ln_out, res_in = layer_norm_with_residual(self.input_layernorm, hidden_states)
        attn_out, attn_bias = self.self_attention(ln_out, attention_mask)
        residual = ln_out if post else res_in
        bda = get_bias_dropout_add(self.training)
        ln_in = bda(attn_out, attn_bias, residual, self.hidden_dropout)
        if post or self.layer_type == LayerType.decoder:
            ln_out, ln_in_res = self.post_attention_layernorm(ln_in), ln_in
        else:
            ln_out, ln_in_res = layer_norm_with_residual(self.post_attention_layernorm, ln_in)
        if self.layer_type == LayerType.decoder:
            attn_out, attn_bias = self.inter_attention(ln_out, enc_dec_attn_mask, encoder_output=encoder_output)
            residual = ln_out if self.apply_residual_connection_post_layernorm else ln_in
            ln_in = bda(attn_out, attn_bias, residual, self.hidden_dropout)
            ln_out = self.post_inter_attention_layernorm(ln_in)
        mlp_out, mlp_bias = self.mlp(ln_out)
        if self.layer_type == LayerType.decoder:
            residual = ln_out if post else ln_in
        else:
            residual = ln_out if post else ln_in_res
        return bda(mlp_out, mlp_bias, residual, self.hidden_dropout)


class ParallelTransformer(MegatronModule):
    """This pipeline stage's share of the layers (+ final LayerNorm on the last stage)."""

    def __init__(self, init_method, output_layer_init_method, layer_type=LayerType.encoder,
                 self_attn_mask_type=AttnMaskType.padding, pre_process=True, post_process=True):
        super().__init__()
        args = get_args()
        self.pre_process, self.post_process = pre_process, post_process
        self.input_tensor = None
        self.checkpoint_activations = args.checkpoint_activations
        self.checkpoint_num_layers = args.activations_checkpoint_num_layers
        pp = parallel_state.get_pipeline_model_parallel_world_size()
        assert args.num_layers % pp == 0, "num_layers must be divisible by pipeline size"
        self.num_layers = args.num_layers // pp
        vpp = parallel_state.get_virtual_pipeline_model_parallel_world_size()
        if vpp is not None:
            assert args.num_layers % vpp == 0
            self.num_layers = self.num_layers // vpp
            offset = parallel_state.get_virtual_pipeline_model_parallel_rank() * (args.num_layers // vpp) + \
                parallel_state.get_pipeline_model_parallel_rank() * self.num_layers
        else:
            offset = parallel_state.get_pipeline_model_parallel_rank() * self.num_layers
        self.layers = torch.nn.ModuleList([
            ParallelTransformerLayer(init_method, output_layer_init_method, i + 1 + offset, layer_type=layer_type,
                                     self_attn_mask_type=self_attn_mask_type) for i in range(self.num_layers)])
        if post_process:
            self.final_layernorm = LayerNorm(args.hidden_size, eps=args.layernorm_epsilon)

    def set_input_tensor(self, input_tensor):
        self.input_tensor = input_tensor

    def _checkpointed_forward(self, hidden_states, attention_mask, encoder_output, enc_dec_attn_mask):
        def custom(start, end):
            def fwd(x, mask, enc, encmask):
                for layer in self.layers[start:end]:
                    x = layer(x, mask, encoder_output=enc, enc_dec_attn_mask=encmask)
                return x

            return fwd

        i = 0
        while i < self.num_layers:
            hidden_states = tensor_parallel.checkpoint(custom(i, i + self.checkpoint_num_layers), hidden_states,
                                                       attention_mask, encoder_output, enc_dec_attn_mask)
            i += self.checkpoint_num_layers
        return hidden_states

    def forward(self, hidden_states, attention_mask, encoder_output=None, enc_dec_attn_mask=None,
                inference_params=None):
        if not self.pre_process:
            hidden_states = self.input_tensor
        if self.checkpoint_activations and self.training:
            hidden_states = self._checkpointed_forward(hidden_states, attention_mask, encoder_output,
                                                       enc_dec_attn_mask)
        else:
            for layer in self.layers:
                hidden_states = layer(hidden_states, attention_mask, encoder_output=encoder_output,
                                      enc_dec_attn_mask=enc_dec_attn_mask)
        if self.post_process:
            hidden_states = self.final_layernorm(hidden_states)
        return hidden_states


def parallel_lm_logits(input_, word_embeddings_weight, parallel_output, bias=None):
    """[s, b, h] x [v/tp, h]^T -> vocab-parallel logits (gathered unless parallel_output)."""
    if get_args().sequence_parallel:
        input_parallel = tensor_parallel.gather_from_sequence_parallel_region(input_)
    else:
        input_parallel = tensor_parallel.copy_to_tensor_model_parallel_region(input_)
    logits = F.linear(input_parallel, word_embeddings_weight, bias)
    if parallel_output:
        return logits
    return tensor_parallel.gather_from_tensor_model_parallel_region(logits)


class Pooler(MegatronModule):
    def __init__(self, hidden_size, init_method):
        super().__init__()
        self.dense = get_linear_layer(hidden_size, hidden_size, init_method)

    def forward(self, hidden_states, sequence_index=0):
        return torch.tanh(self.dense(hidden_states[sequence_index, :, :]))


class Embedding(MegatronModule):
    """word + position (+ tokentype) embeddings, dropout; output [s, b, h]."""

    def __init__(self, hidden_size, vocab_size, max_sequence_length, embedding_dropout_prob, init_method,
                 num_tokentypes=0):
        super().__init__()
        args = get_args()
        self.hidden_size = hidden_size
        self.init_method = init_method
        self.num_tokentypes = num_tokentypes
        self.word_embeddings = tensor_parallel.VocabParallelEmbedding(
            vocab_size, hidden_size, init_method=init_method, use_cpu_initialization=args.use_cpu_initialization,
            params_dtype=args.params_dtype)
        self.position_embeddings = torch.nn.Embedding(max_sequence_length, hidden_size)
        init_method(self.position_embeddings.weight)
        if num_tokentypes > 0:
            self.tokentype_embeddings = torch.nn.Embedding(num_tokentypes, hidden_size)
            init_method(self.tokentype_embeddings.weight)
        else:
            self.tokentype_embeddings = None
        self.embedding_dropout = torch.nn.Dropout(embedding_dropout_prob)

    def zero_parameters(self):
        with torch.no_grad():
            for p in self.parameters():
                p.zero_()

    def forward(self, input_ids, position_ids, tokentype_ids=None):
        emb = self.word_embeddings(input_ids) + self.position_embeddings(position_ids)
        if tokentype_ids is not None:
            assert self.tokentype_embeddings is not None
            emb = emb + self.tokentype_embeddings(tokentype_ids)
        emb = emb.transpose(0, 1).contiguous()  # [b, s, h] -> [s, b, h]
        if get_args().sequence_parallel:
            emb = tensor_parallel.scatter_to_sequence_parallel_region(emb)
        return self.embedding_dropout(emb)


class TransformerLanguageModel(MegatronModule):
    def __init__(self, init_method, output_layer_init_method, encoder_attn_mask_type, num_tokentypes=0,
                 add_pooler=False, pre_process=True, post_process=True):
        super().__init__()
        args = get_args()
        self.pre_process, self.post_process = pre_process, post_process
        self.hidden_size = args.hidden_size
        self.num_tokentypes = num_tokentypes
        self.init_method = init_method
        self.encoder_attn_mask_type = encoder_attn_mask_type
        self.add_pooler = add_pooler
        if pre_process:
            self.embedding = Embedding(self.hidden_size, args.padded_vocab_size, args.max_position_embeddings,
                                       args.hidden_dropout, init_method, num_tokentypes)
        self.encoder = ParallelTransformer(init_method, output_layer_init_method,
                                           self_attn_mask_type=encoder_attn_mask_type, pre_process=pre_process,
                                           post_process=post_process)
        if post_process and add_pooler:
            self.pooler = Pooler(self.hidden_size, init_method)

    def set_input_tensor(self, input_tensor):
        if isinstance(input_tensor, (list, tuple)):
            input_tensor = input_tensor[0]
        self.encoder.set_input_tensor(input_tensor)

    def forward(self, enc_input_ids, enc_position_ids, enc_attn_mask, tokentype_ids=None, pooling_sequence_index=0):
        enc_in = self.embedding(enc_input_ids, enc_position_ids, tokentype_ids=tokentype_ids) \
            if self.pre_process else None
        out = self.encoder(enc_in, enc_attn_mask)
        if self.post_process and self.add_pooler:
            return out, self.pooler(out, pooling_sequence_index)
        return out


def get_language_model(num_tokentypes, add_pooler, encoder_attn_mask_type, init_method=None,
                       scaled_init_method=None, pre_process=True, post_process=True):
    args = get_args()
    if init_method is None:
        init_method = init_method_normal(args.init_method_std)
    if scaled_init_method is None:
        scaled_init_method = scaled_init_method_normal(args.init_method_std, args.num_layers)
    lm = TransformerLanguageModel(init_method, scaled_init_method, encoder_attn_mask_type,
                                  num_tokentypes=num_tokentypes, add_pooler=add_pooler, pre_process=pre_process,
                                  post_process=post_process)
    return lm, "language_model"


__all__ = ["MegatronModule", "ParallelMLP", "ParallelAttention", "ParallelTransformerLayer", "ParallelTransformer",
           "TransformerLanguageModel", "Embedding", "Pooler", "parallel_lm_logits", "get_language_model",
           "init_method_normal", "scaled_init_method_normal", "ModelType"]
