"""Standalone Megatron GPT (reference apex/transformer/testing/standalone_gpt.py:1411-1504):
causal LM over the tensor/pipeline-parallel transformer of :mod:`.standalone_transformer_lm`
with the vocab-parallel cross entropy on the last stage."""
import torch

from .. import tensor_parallel
from ..enums import AttnMaskType
from .global_vars import get_args
from .standalone_transformer_lm import (MegatronModule, get_language_model, init_method_normal, parallel_lm_logits,
                                        scaled_init_method_normal)


def post_language_model_processing(lm_output, labels, logit_weights, parallel_output, fp16_lm_cross_entropy):
    output = parallel_lm_logits(lm_output, logit_weights, parallel_output)
    if labels is None:
        return output
    # labels [b, s]; logits [s, b, v/tp]
    labels = labels.transpose(0, 1).contiguous()
    # the loss math is fp32 either way: the fused kernel (unsharded vocabulary) upcasts the half
    # logits in registers and the sharded path upcasts them itself, so an fp32 copy of the
    # [tokens, vocab] logits (the reference's upcast) is never materialised;
    # fp16_lm_cross_entropy only pins the logits dtype
    assert not fp16_lm_cross_entropy or output.dtype == torch.half
    loss = tensor_parallel.vocab_parallel_cross_entropy(output, labels)
    return loss.transpose(0, 1).contiguous()  # [b, s]


class GPTModel(MegatronModule):
    def __init__(self, num_tokentypes=0, parallel_output=True, pre_process=True, post_process=True,
                 cpu_offload=False):
        super().__init__()
        args = get_args()
        self.parallel_output = parallel_output
        self.pre_process, self.post_process = pre_process, post_process
        self.fp16_lm_cross_entropy = args.fp16_lm_cross_entropy
        self.language_model, self._language_model_key = get_language_model(
            num_tokentypes=num_tokentypes, add_pooler=False, encoder_attn_mask_type=AttnMaskType.causal,
            init_method=init_method_normal(args.init_method_std),
            scaled_init_method=scaled_init_method_normal(args.init_method_std, args.num_layers),
            pre_process=pre_process, post_process=post_process)
        self.initialize_word_embeddings(init_method_normal)

    def set_input_tensor(self, input_tensor):
        self.language_model.set_input_tensor(input_tensor)

    def forward(self, input_ids, position_ids, attention_mask, labels=None, tokentype_ids=None,
                inference_params=None):
        lm_output = self.language_model(input_ids, position_ids, attention_mask)
        if self.post_process:
            return post_language_model_processing(lm_output, labels, self.word_embeddings_weight(),
                                                  self.parallel_output, self.fp16_lm_cross_entropy)
        return lm_output


def gpt_model_provider(pre_process=True, post_process=True, cpu_offload=False):
    args = get_args()
    model = GPTModel(num_tokentypes=0, parallel_output=True, pre_process=pre_process, post_process=post_process)
    if torch.cuda.is_available() and not args.use_cpu_initialization:
        model = model.cuda()
    if args.params_dtype != torch.float32:
        model = model.to(args.params_dtype)
    return model
