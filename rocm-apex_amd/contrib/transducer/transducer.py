"""RNN-T transducer joint and loss (reference apex/contrib/transducer/transducer.py:5-195).

GPU tensors run the gfx950 kernels (``csrc/transducer/transducer.hip``); CPU tensors the
torch reference implementations below (the same lattice recursions, used by the CPU tests).
Dropout in the joint uses a counter-based hash (seed from torch's generator), so the mask is
reproducible and exposed through ``mask_probe`` like the reference's."""
import torch
import torch.nn.functional as F

from ... import _native


def _lib(name):
    return getattr(_native.require("transducer"), name)


_dropout_calls = [0]


# ------------------------------------------------------------------------------------------
# CPU reference math
# ------------------------------------------------------------------------------------------
def _joint_ref(f, g, f_len, g_len, pack_output, relu, dropout, batch_offset, packed_batch, p):
    B, T, H = f.shape
    U = g.size(1)
    h = f.unsqueeze(2) + g.unsqueeze(1)  # [B, T, U, H]
    valid = (torch.arange(T).view(1, T, 1) < f_len.view(B, 1, 1)) & \
            (torch.arange(U).view(1, 1, U) < g_len.view(B, 1, 1))
    mask = valid.unsqueeze(-1).expand_as(h).clone()
    if relu:
        mask &= h > 0
    if dropout:
        mask &= torch.rand(h.shape) >= p
        h = h / (1 - p)
    out = torch.where(mask, h, torch.zeros_like(h))
    out = torch.where(valid.unsqueeze(-1), out, torch.full_like(out, -1.0))
    if pack_output:
        rows = [out[b, :int(f_len[b]), :int(g_len[b])].reshape(-1, H) for b in range(B)]
        mrows = [mask[b, :int(f_len[b]), :int(g_len[b])].reshape(-1, H) for b in range(B)]
        return torch.cat(rows, 0), torch.cat(mrows, 0)
    return out, mask


def _loss_ref(x, label, f_len, y_len, blank_idx):
    """Negative log-likelihood per batch element; x = log-probs [B, T, U+1, V]."""
    B = x.size(0)
    losses = []
    for b in range(B):
        T, U = int(f_len[b]), int(y_len[b]) + 1
        lp = x[b]
        alpha = [[None] * U for _ in range(T)]
        alpha[0][0] = lp.new_zeros(())
        for t in range(T):
            for u in range(U):
                if t == 0 and u == 0:
                    continue
                cands = []
                if t > 0:
                    cands.append(alpha[t - 1][u] + lp[t - 1, u, blank_idx])
                if u > 0:
                    cands.append(alpha[t][u - 1] + lp[t, u - 1, label[b, u - 1]])
                alpha[t][u] = torch.logsumexp(torch.stack(cands), 0)
        losses.append(-(alpha[T - 1][U - 1] + lp[T - 1, U - 1, blank_idx]))
    return torch.stack(losses)


# ------------------------------------------------------------------------------------------
class TransducerJoint(torch.nn.Module):
    def __init__(self, pack_output=False, relu=False, dropout=False, opt=1, fwd_tile_size=4, dropout_prob=0,
                 probe_mask=False):
        super().__init__()
        self.pack_output = pack_output
        self.relu = relu
        self.dropout = dropout
        self.dropout_prob = dropout_prob
        self.opt = opt
        self.fwd_tile_size = fwd_tile_size
        self.dummy_batch_offset = torch.empty(0)
        masked = relu or dropout
        self.mask_probe = [] if masked and probe_mask else None
        if masked and opt != 1:
            raise NotImplementedError("ReLU and dropout fusion is only supported with opt=1")

    def forward(self, f, g, f_len, g_len, batch_offset=None, packed_batch=0):
        my_batch_offset = batch_offset if self.pack_output else self.dummy_batch_offset
        if self.pack_output and (batch_offset is None or packed_batch == 0):
            raise Exception("Please specify batch_offset and packed_batch when packing is enabled")
        dropout = self.dropout and self.training
        return TransducerJointFunc.apply(f, g, f_len, g_len, self.pack_output, self.relu, dropout, my_batch_offset,
                                         packed_batch, self.opt, self.fwd_tile_size, self.dropout_prob,
                                         self.mask_probe)


class TransducerLoss(torch.nn.Module):
    def __init__(self, fuse_softmax_backward=True, opt=1, packed_input=False):
        super().__init__()
        self.fuse_softmax_backward = fuse_softmax_backward
        self.opt = opt
        self.packed_input = packed_input
        self.dummy_batch_offset = torch.empty(0)

    def forward(self, x, label, f_len, y_len, blank_idx, batch_offset=None, max_f_len=None, debug_list=None):
        if self.packed_input:
            if batch_offset is None or max_f_len is None:
                raise Exception("Please specify batch_offset and max_f_len when packing is enabled")
            my_batch_offset, my_max_f_len = batch_offset, max_f_len
        else:
            my_batch_offset, my_max_f_len = self.dummy_batch_offset, x.size(1)
        return TransducerLossFunc.apply(x, label, f_len, y_len, my_batch_offset, my_max_f_len, blank_idx,
                                        self.fuse_softmax_backward, debug_list, self.opt, self.packed_input)


class TransducerLossFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, label, f_len, y_len, batch_offset, max_f_len, blank_idx, fuse_softmax_backward, debug_list,
                opt, packed_input):
        ctx.native = x.is_cuda
        if not ctx.native:
            with torch.enable_grad():
                xr = x.detach().requires_grad_(True)
                if packed_input:
                    raise NotImplementedError("packed transducer loss runs on the GPU kernels only")
                loss = _loss_ref(F.log_softmax(xr.float(), -1), label, f_len, y_len, blank_idx)
            ctx.ref = (xr, loss)
            return loss.detach().to(x.dtype)
        if fuse_softmax_backward:
            lp = F.log_softmax(x, dim=-1)
        else:
            with torch.enable_grad():
                xr = x.detach().requires_grad_(True)
                lp = F.log_softmax(xr, dim=-1)
            ctx.xr = xr
        alpha, beta, loss = _lib("transducer_loss_cuda").forward(lp.detach(), label, f_len, y_len, batch_offset,
                                                                  max_f_len, blank_idx, opt, packed_input)
        if debug_list == []:
            debug_list += [alpha, beta]
        ctx.save_for_backward(lp, alpha, beta, f_len, y_len, label, batch_offset)
        ctx.blank_idx = blank_idx
        ctx.fuse_softmax_backward = fuse_softmax_backward
        ctx.opt = opt
        ctx.packed_input = packed_input
        ctx.max_f_len = max_f_len
        return loss

    @staticmethod
    def backward(ctx, loss_grad):
        if not ctx.native:
            xr, loss = ctx.ref
            (g,) = torch.autograd.grad(loss, [xr], loss_grad.float())
            return g, None, None, None, None, None, None, None, None, None, None
        lp, alpha, beta, f_len, y_len, label, batch_offset = ctx.saved_tensors
        x_grad = _lib("transducer_loss_cuda").backward(lp.detach(), loss_grad, alpha, beta, f_len, y_len, label,
                                                       batch_offset, ctx.max_f_len, ctx.blank_idx, ctx.opt,
                                                       ctx.fuse_softmax_backward, ctx.packed_input)
        if not ctx.fuse_softmax_backward:
            (x_grad,) = torch.autograd.grad(lp, [ctx.xr], x_grad)
        return x_grad, None, None, None, None, None, None, None, None, None, None


class TransducerJointFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f, g, f_len, g_len, pack_output, relu, dropout, batch_offset, packed_batch, opt, fwd_tile_size,
                dropout_prob, mask_probe):
        masked = relu or dropout
        ctx.native = f.is_cuda
        if ctx.native:
            seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if dropout else 0
            _dropout_calls[0] += 1
            out, mask = _lib("transducer_joint_cuda").forward(f, g, f_len, g_len, batch_offset, packed_batch, opt,
                                                               pack_output, relu, dropout, float(dropout_prob),
                                                               fwd_tile_size, seed, _dropout_calls[0])
        else:
            out, mask = _joint_ref(f, g, f_len, g_len, pack_output, relu, dropout, batch_offset, packed_batch,
                                   dropout_prob)
        if masked:
            ctx.save_for_backward(mask, f_len, g_len, batch_offset, f, g)
            if mask_probe is not None:
                mask_probe.append(mask)
        else:
            ctx.save_for_backward(f_len, g_len, batch_offset, f, g)
        ctx.pack_output = pack_output
        ctx.masked = masked
        ctx.max_f_len = f.size(1)
        ctx.max_g_len = g.size(1)
        ctx.scale = 1 / (1 - dropout_prob) if dropout and dropout_prob != 1 else 1
        return out

    @staticmethod
    def backward(ctx, grad):
        if ctx.masked:
            mask, f_len, g_len, batch_offset, f, g = ctx.saved_tensors
            inp = [grad, mask]
        else:
            f_len, g_len, batch_offset, f, g = ctx.saved_tensors
            inp = [grad]
        if ctx.native:
            f_grad, g_grad = _lib("transducer_joint_cuda").backward(inp, f_len, g_len, batch_offset, ctx.max_f_len,
                                                                     ctx.max_g_len, ctx.pack_output, ctx.scale, f, g)
        else:
            B, T, H = f.shape
            U = g.size(1)
            if ctx.pack_output:
                full = grad.new_zeros(B, T, U, H)
                fm = grad.new_zeros(B, T, U, H, dtype=torch.bool)
                off = 0
                for b in range(B):
                    n = int(f_len[b]) * int(g_len[b])
                    full[b, :int(f_len[b]), :int(g_len[b])] = grad[off:off + n].view(int(f_len[b]), int(g_len[b]), H)
                    if ctx.masked:
                        fm[b, :int(f_len[b]), :int(g_len[b])] = mask[off:off + n].view(int(f_len[b]), int(g_len[b]),
                                                                                        H)
                    off += n
                gr, m = full, (fm if ctx.masked else None)
            else:
                gr, m = grad, (mask if ctx.masked else None)
            valid = (torch.arange(T).view(1, T, 1) < f_len.view(B, 1, 1)) & \
                    (torch.arange(U).view(1, 1, U) < g_len.view(B, 1, 1))
            gr = gr * valid.unsqueeze(-1)
            if m is not None:
                gr = gr * m * ctx.scale
            f_grad, g_grad = gr.sum(2), gr.sum(1)
        return f_grad, g_grad, None, None, None, None, None, None, None, None, None, None, None
