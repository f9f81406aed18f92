"""fast_mask_softmax_dropout_func (reference apex/contrib/multihead_attn/mask_softmax_dropout_func.py):
softmax over the last dim of [b*heads, sq, sk] scores with an optional key-padding mask
([b, sk], boolean or additive), then dropout.  Saves the softmax output (not the input) for the
backward, like the reference."""
import torch
import torch.nn.functional as F


class MaskSoftmaxDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, is_training, heads, inputs, pad_mask, mask_additive, dropout_prob):
        bh, sq, sk = inputs.shape
        x = inputs
        if pad_mask is not None:
            b = bh // heads
            x = x.view(b, heads, sq, sk)
            if mask_additive:
                x = x + pad_mask.view(b, 1, 1, sk).to(x.dtype)
            else:
                x = x.masked_fill(pad_mask.view(b, 1, 1, sk).bool(), float("-inf"))
            x = x.view(bh, sq, sk)
        sm = F.softmax(x.float(), dim=-1).to(inputs.dtype)
        if is_training and dropout_prob > 0:
            keep = (torch.rand_like(sm, dtype=torch.float32) >= dropout_prob)
            out = sm * keep.to(sm.dtype) * (1.0 / (1.0 - dropout_prob))
        else:
            keep = None
            out = sm
        ctx.save_for_backward(sm, keep)
        ctx.p = dropout_prob if is_training else 0.0
        return out.detach()

    @staticmethod
    def backward(ctx, grad):
        sm, keep = ctx.saved_tensors
        g = grad
        if keep is not None:
            g = g * keep.to(g.dtype) * (1.0 / (1.0 - ctx.p))
        gf, sf = g.float(), sm.float()
        dx = sf * (gf - (gf * sf).sum(-1, keepdim=True))
        return None, None, dx.to(grad.dtype), None, None, None


fast_mask_softmax_dropout_func = MaskSoftmaxDropout.apply
