"""Standalone Megatron BERT (reference apex/transformer/testing/standalone_bert.py:10-217): the
padding-masked transformer of :mod:`.standalone_transformer_lm` + LM head (tied word
embeddings) + optional binary (NSP) head.  The [b, s] padding mask becomes a [b, 1, 1, s]
additive bias consumed by the flash-attention kernel (no [b, 1, s, s] mask tensor)."""
import torch
import torch.nn.functional as F

from ...normalization import FusedLayerNorm as LayerNorm
from .. import parallel_state, tensor_parallel
from ..enums import AttnMaskType
from .global_vars import get_args
from .standalone_transformer_lm import (MegatronModule, get_language_model, get_linear_layer, init_method_normal,
                                        parallel_lm_logits, scaled_init_method_normal)


def bert_extended_attention_mask(attention_mask):
    """[b, s] (1 = attend) -> [b, 1, 1, s] additive bias (0 / -10000), the flash kernel's input;
    the reference builds the boolean [b, 1, s, s] outer product instead."""
    return ((1.0 - attention_mask.float()) * -10000.0).unsqueeze(1).unsqueeze(1)


def bert_position_ids(token_ids):
    s = token_ids.size(1)
    return torch.arange(s, dtype=torch.long, device=token_ids.device).unsqueeze(0).expand_as(token_ids)


class BertLMHead(MegatronModule):
    def __init__(self, mpu_vocab_size, hidden_size, init_method, layernorm_epsilon, parallel_output):
        super().__init__()
        args = get_args()
        self.bias = torch.nn.Parameter(torch.zeros(mpu_vocab_size))
        tensor_parallel.set_tensor_model_parallel_attributes(self.bias, True, 0, 1)
        self.parallel_output = parallel_output
        self.dense = get_linear_layer(hidden_size, hidden_size, init_method)
        self.layernorm = LayerNorm(hidden_size, eps=layernorm_epsilon)
        self.gelu = F.gelu
        if args.openai_gelu:
            from .standalone_transformer_lm import openai_gelu

            self.gelu = openai_gelu

    def forward(self, hidden_states, word_embeddings_weight):
        h = self.layernorm(self.gelu(self.dense(hidden_states)))
        return parallel_lm_logits(h, word_embeddings_weight, self.parallel_output, bias=self.bias)


def post_language_model_processing(lm_output, pooled_output, lm_head, binary_head, lm_labels, logit_weights,
                                   fp16_lm_cross_entropy):
    lm_logits = lm_head(lm_output, logit_weights)
    binary_logits = binary_head(pooled_output) if binary_head is not None else None
    if lm_labels is None:
        return lm_logits, binary_logits
    lm_labels = lm_labels.transpose(0, 1).contiguous()
    # fp32 loss math inside either way (see standalone_gpt.post_language_model_processing)
    assert not fp16_lm_cross_entropy or lm_logits.dtype == torch.half
    lm_loss = tensor_parallel.vocab_parallel_cross_entropy(lm_logits, lm_labels)
    return lm_loss.transpose(0, 1).contiguous(), binary_logits


class BertModel(MegatronModule):
    def __init__(self, num_tokentypes=2, add_binary_head=True, parallel_output=True, pre_process=True,
                 post_process=True, cpu_offload=False):
        super().__init__()
        args = get_args()
        self.fp16_lm_cross_entropy = args.fp16_lm_cross_entropy
        self.add_binary_head = add_binary_head
        self.parallel_output = parallel_output
        self.pre_process, self.post_process = pre_process, post_process
        init_method = init_method_normal(args.init_method_std)
        self.language_model, self._language_model_key = get_language_model(
            num_tokentypes=num_tokentypes, add_pooler=add_binary_head, encoder_attn_mask_type=AttnMaskType.padding,
            init_method=init_method, scaled_init_method=scaled_init_method_normal(args.init_method_std,
                                                                                  args.num_layers),
            pre_process=pre_process, post_process=post_process)
        self.initialize_word_embeddings(init_method_normal)
        if post_process:
            self.lm_head = BertLMHead(self.word_embeddings_weight().size(0), args.hidden_size, init_method,
                                      args.layernorm_epsilon, parallel_output)
            self._lm_head_key = "lm_head"
            self.binary_head = get_linear_layer(args.hidden_size, 2, init_method) if add_binary_head else None

    def set_input_tensor(self, input_tensor):
        self.language_model.set_input_tensor(input_tensor)

    def forward(self, bert_model_input, attention_mask, tokentype_ids=None, lm_labels=None):
        ext_mask = bert_extended_attention_mask(attention_mask)
        position_ids = bert_position_ids(bert_model_input)
        lm_output = self.language_model(bert_model_input, position_ids, ext_mask, tokentype_ids=tokentype_ids)
        if self.post_process and self.add_binary_head:
            lm_output, pooled = lm_output
        else:
            pooled = None
        if self.post_process:
            return post_language_model_processing(lm_output, pooled, self.lm_head, self.binary_head, lm_labels,
                                                  self.word_embeddings_weight(), self.fp16_lm_cross_entropy)
        return lm_output


def bert_model_provider(pre_process=True, post_process=True, cpu_offload=False):
    args = get_args()
    num_tokentypes = 2 if args.bert_binary_head else 0
    model = BertModel(num_tokentypes=num_tokentypes, add_binary_head=args.bert_binary_head, parallel_output=True,
                      pre_process=pre_process, post_process=post_process)
    if torch.cuda.is_available() and not args.use_cpu_initialization:
        model = model.cuda()
    if args.params_dtype != torch.float32:
        model = model.to(args.params_dtype)
    return model


__all__ = ["BertModel", "bert_model_provider", "bert_extended_attention_mask", "bert_position_ids",
           "parallel_state"]
