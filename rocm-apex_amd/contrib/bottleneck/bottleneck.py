"""ResNet bottleneck with frozen BN, optionally split spatially over ranks
(reference apex/contrib/bottleneck/bottleneck.py:10-520).

The reference's fast path (``use_cudnn=True``) is a cuDNN-frontend fused graph of
conv -> scale/bias -> ReLU chains (apex/contrib/csrc/bottleneck/bottleneck.cpp).  Here every
stage is ONE native implicit-GEMM launch (``apex.ops.conv.conv_bn_act``,
csrc/conv/conv_igemm.hip) whose epilogue applies the frozen-BN scale / bias, the residual add of
the last stage and the ReLU to the fp32 accumulator — channels_last bf16/fp16, C and K multiples
of 64.  Other shapes / dtypes fold the frozen BN into the convolution (w * s, bias b) inside the
autograd graph — exact for frozen statistics, the raw-weight gradient flows through the fold —
and run one MIOpen conv-with-bias per stage.  ``explicit_nhwc``
tensors ([N, H, W, C] inputs, [K, R, S, C] weights) are consumed as zero-copy channels_last
views.  ``SpatialBottleneck`` splits H over ``spatial_group_size`` ranks with a 1-row halo
exchange before the 3x3 conv (see :mod:`.halo_exchangers`)."""
import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from ...ops.conv import conv_bn_act, conv_bn_act_supported
from .halo_exchangers import halo_pad, make_exchanger


def kaiming_uniform_(tensor, a=0, mode="fan_in", nonlinearity="leaky_relu"):
    nn.init.kaiming_uniform_(tensor, a=a, mode=mode, nonlinearity=nonlinearity)


class FrozenBatchNorm2d(nn.Module):
    """BatchNorm2d with fixed statistics and affine parameters (buffers)."""

    def __init__(self, n):
        super().__init__()
        self.register_buffer("weight", torch.ones(n))
        self.register_buffer("bias", torch.zeros(n))
        self.register_buffer("running_mean", torch.zeros(n))
        self.register_buffer("running_var", torch.ones(n))

    def get_scale_bias(self, nhwc=False):
        scale = self.weight * self.running_var.rsqrt()
        bias = self.bias - self.running_mean * scale
        shape = (1, 1, 1, -1) if nhwc else (1, -1, 1, 1)
        return scale.reshape(shape), bias.reshape(shape)

    def forward(self, x):
        scale, bias = self.get_scale_bias()
        return x * scale + bias


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation, groups=groups,
                     bias=False, dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


def _fold(w, bn, explicit_nhwc):
    """conv weight with the frozen BN scale folded in (NCHW-shaped view) and the BN bias."""
    s, b = bn.get_scale_bias(False)
    if explicit_nhwc:  # stored [K, R, S, C] -> channels_last [K, C, R, S] view
        w = w.permute(0, 3, 1, 2)
    return w * s.reshape(-1, 1, 1, 1).to(w.dtype), b.reshape(-1).to(w.dtype)


class _FusedBottleneckFn(torch.autograd.Function):
    """The whole frozen-BN bottleneck as one autograd node on the native kernels.

    Forward: one implicit-GEMM launch per stage with the scale / bias (/ residual) / ReLU epilogue.
    Backward, stage by stage from the block output: a single ReLU-mask pass on the incoming
    gradient (the block output's own ReLU), then per stage ONE data-gradient launch that does
    dconv + dReLU + dscale together — the frozen-BN scale is folded into the (tiny) weight
    (``W * s``), and the previous stage's ReLU mask is applied in the dconv epilogue from that
    stage's saved output (the 1x1 GEMM's DReLU epilogue / the tap kernel's mask epilogue) — the
    capability of the reference's cudnn-frontend dconv + drelu + dscale graphs
    (apex/contrib/csrc/bottleneck/bottleneck.cpp:760, :1287-1534).  Weight gradients: MIOpen on
    the masked gradient, post-scaled per output channel."""

    @staticmethod
    def forward(ctx, x, w1, w2, w3, wd, s1, b1, s2, b2, s3, b3, sd, bd, stride):
        if wd is not None:
            identity = conv_bn_act(x, wd, sd, bd, None, False, stride, (0, 0))
        else:
            identity = x
        y1 = conv_bn_act(x, w1, s1, b1, None, True, stride, (0, 0))
        y2 = conv_bn_act(y1, w2, s2, b2, None, True, 1, (1, 1))
        out = conv_bn_act(y2, w3, s3, b3, identity, True, 1, (0, 0))
        ctx.save_for_backward(x, w1, w2, w3, wd, s1, s2, s3, sd, y1, y2, out)
        ctx.stride = stride
        return out

    @staticmethod
    def backward(ctx, gy):
        x, w1, w2, w3, wd, s1, s2, s3, sd, y1, y2, out = ctx.saved_tensors
        stride = ctx.stride
        from ...ops.conv import conv_tap_dgrad
        from ... import _native

        gmm = _native.require("fused bottleneck backward").gemm
        gy = gy.contiguous(memory_format=torch.channels_last)
        g3 = torch.where(out > 0, gy, torch.zeros((), dtype=gy.dtype, device=gy.device))

        def wgrad(g, inp, w, s, st, pad):
            dw = torch.ops.aten.convolution_backward(g, inp, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                                     [False, True, False])[1]
            return dw * s.to(dw.dtype).view(-1, 1, 1, 1)

        def scaled(w, s):
            return (w * s.to(w.dtype).view(-1, 1, 1, 1)).contiguous(memory_format=torch.channels_last)

        def dgrad_1x1(g, w, s, mask):
            n, k, h, wdt = g.shape
            c = w.shape[1]
            g2 = g.permute(0, 2, 3, 1).reshape(-1, k)
            ws = scaled(w, s).view(k, c)
            aux = None if mask is None else mask.permute(0, 2, 3, 1).reshape(-1, c)
            epi = gmm.EPI_NONE if mask is None else gmm.EPI_DRELU
            return gmm.linear_dgrad(g2, ws, epi, aux).view(n, h, wdt, c).permute(0, 3, 1, 2)

        dw3 = wgrad(g3, y2, w3, s3, 1, 0)
        g2 = dgrad_1x1(g3, w3, s3, y2)                      # dconv3 + dReLU(y2) + dscale3
        dw2 = wgrad(g2, y1, w2, s2, 1, 1)
        g1 = conv_tap_dgrad(g2, scaled(w2, s2), y1.shape, 1, 1, mask=y1)  # dconv2 + dReLU(y1) + dscale2
        dw1 = wgrad(g1, x, w1, s1, stride, 0)
        if stride == 1:
            dx = dgrad_1x1(g1, w1, s1, None)
        else:
            dx = conv_tap_dgrad(g1, scaled(w1, s1), x.shape, stride, 0)
        dwd = None
        if wd is not None:
            dwd = wgrad(g3, x, wd, sd, stride, 0)
            if stride == 1:
                dx = dx + dgrad_1x1(g3, wd, sd, None)
            else:
                dx = dx + conv_tap_dgrad(g3, scaled(wd, sd), x.shape, stride, 0)
        else:
            dx = dx + g3
        return dx, dw1, dw2, dw3, dwd, None, None, None, None, None, None, None, None, None


class Bottleneck(nn.Module):
    def __init__(self, in_channels, bottleneck_channels, out_channels, stride=1, groups=1, dilation=1,
                 norm_func=None, use_cudnn=False, explicit_nhwc=False):
        super().__init__()
        if groups != 1:
            raise RuntimeError("Only support groups == 1")
        if dilation != 1:
            raise RuntimeError("Only support dilation == 1")
        if norm_func is not None:
            raise RuntimeError("Only support frozen BN now.")
        norm_func = FrozenBatchNorm2d
        if stride != 1 or in_channels != out_channels:
            self.downsample = nn.Sequential(conv1x1(in_channels, out_channels, stride), norm_func(out_channels))
        else:
            self.downsample = None
        # stride on the first 1x1 (ResNet v1), like the reference
        self.conv1 = conv1x1(in_channels, bottleneck_channels, stride)
        self.conv2 = conv3x3(bottleneck_channels, bottleneck_channels)
        self.conv3 = conv1x1(bottleneck_channels, out_channels)
        self.relu = nn.ReLU(inplace=True)
        self.stride = stride
        self.bn1 = norm_func(bottleneck_channels)
        self.bn2 = norm_func(bottleneck_channels)
        self.bn3 = norm_func(out_channels)
        self.use_cudnn = use_cudnn
        self.w_conv = [self.conv1.weight, self.conv2.weight, self.conv3.weight]
        if self.downsample is not None:
            self.w_conv.append(self.downsample[0].weight)
        for w in self.w_conv:
            kaiming_uniform_(w, a=1)
        self.explicit_nhwc = explicit_nhwc
        # native conv + scale/bias/residual/ReLU kernels on the fused path (False: MIOpen with the
        # BN folded into the weights; the A/B switch)
        self.use_native = True
        if explicit_nhwc:
            for p in self.parameters():
                with torch.no_grad():
                    p.data = p.data.permute(0, 2, 3, 1).contiguous()

    # ---- plain module path (reference "native ops" fallback) ----
    def _forward_modules(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self._conv2_plain(out)
        out = self.relu(self.bn2(out))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)

    def _conv2_plain(self, out):
        return self.conv2(out)

    def _conv2_input(self, out):
        """(input, padding) of the 3x3 conv (the spatial variant pads H with neighbour halos)."""
        return out, (1, 1)

    def _stage(self, x, conv, bn, residual=None, relu=True, stride=1, padding=(0, 0)):
        """act(conv(x) * s + b [+ residual]) for a frozen BN (s, b): one native conv launch with
        the scale / bias / residual / ReLU epilogue where supported, else the BN folded into a
        MIOpen conv-with-bias."""
        w = conv.weight.permute(0, 3, 1, 2) if self.explicit_nhwc else conv.weight
        if self.use_native and conv_bn_act_supported(x, w, residual):
            s, b = bn.get_scale_bias(False)
            return conv_bn_act(x, w, s.reshape(-1), b.reshape(-1), residual, relu, stride, padding)
        wf, bf = _fold(conv.weight, bn, self.explicit_nhwc)
        y = F.conv2d(x, wf, bf, stride=stride, padding=padding)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y

    def _weights(self):
        ws = [c.weight.permute(0, 3, 1, 2) if self.explicit_nhwc else c.weight
              for c in (self.conv1, self.conv2, self.conv3)]
        wd = None
        if self.downsample is not None:
            wd = self.downsample[0].weight
            wd = wd.permute(0, 3, 1, 2) if self.explicit_nhwc else wd
        return ws, wd

    def _single_node_ok(self, x):
        """One fused autograd node (native forward stages + dconv/dReLU/dscale backward launches)
        for the whole block: every stage on the native kernels, no spatial halo."""
        if not self.use_native or getattr(self, "spatial_group_size", 1) > 1:
            return False
        (w1, w2, w3), wd = self._weights()
        ws = (w1, w2, w3) + ((wd,) if wd is not None else ())
        return (conv_bn_act_supported(x, w1) and (wd is None or conv_bn_act_supported(x, wd))
                and all(t.dtype == x.dtype and t.is_contiguous(memory_format=torch.channels_last) for t in ws)
                and all(t.shape[0] % 64 == 0 and t.shape[1] % 64 == 0 for t in ws))

    # ---- fused path: conv -> frozen-BN scale/bias -> (+ residual) -> ReLU per stage ----
    def _forward_fused(self, x):
        nhwc = self.explicit_nhwc
        if nhwc:
            x = x.permute(0, 3, 1, 2)  # [N, H, W, C] -> channels_last NCHW view
        if self._single_node_ok(x) and torch.is_grad_enabled():
            (w1, w2, w3), wd = self._weights()
            sb = [bn.get_scale_bias(False) for bn in (self.bn1, self.bn2, self.bn3)]
            sb = [(s.reshape(-1).float().contiguous(), b.reshape(-1).float().contiguous()) for s, b in sb]
            sd = bd = None
            if wd is not None:
                s_, b_ = self.downsample[1].get_scale_bias(False)
                sd, bd = s_.reshape(-1).float().contiguous(), b_.reshape(-1).float().contiguous()
            out = _FusedBottleneckFn.apply(x, w1, w2, w3, wd, sb[0][0], sb[0][1], sb[1][0], sb[1][1], sb[2][0],
                                           sb[2][1], sd, bd, self.stride)
            return out.permute(0, 2, 3, 1) if nhwc else out
        if self.downsample is not None:
            identity = self._stage(x, self.downsample[0], self.downsample[1], relu=False, stride=self.stride)
        else:
            identity = x
        out = self._stage(x, self.conv1, self.bn1, stride=self.stride)
        inp, pad = self._conv2_input(out)
        out = self._stage(inp, self.conv2, self.bn2, padding=pad)
        out = self._stage(out, self.conv3, self.bn3, residual=identity)
        return out.permute(0, 2, 3, 1) if nhwc else out

    def forward(self, x):
        if self.use_cudnn or self.explicit_nhwc:
            return self._forward_fused(x)
        return self._forward_modules(x)


class SpatialBottleneck(Bottleneck):
    def __init__(self, in_channels, bottleneck_channels, out_channels, stride=1, groups=1, dilation=1,
                 norm_func=None, use_cudnn=False, explicit_nhwc=False, spatial_group_size=1, communicator=None,
                 halo_ex="sendrecv"):
        super().__init__(in_channels, bottleneck_channels, out_channels, stride, groups, dilation, norm_func,
                         use_cudnn, explicit_nhwc)
        self.spatial_group_size = spatial_group_size
        if spatial_group_size > 1:
            world = dist.get_world_size()
            assert world % spatial_group_size == 0, "world size must be a multiple of spatial_group_size"
            rank = dist.get_rank()
            self.local_rank = rank % spatial_group_size
            if communicator is None:
                for gi in range(world // spatial_group_size):
                    ranks = list(range(gi * spatial_group_size, (gi + 1) * spatial_group_size))
                    comm = dist.new_group(ranks=ranks)
                    if rank in ranks:
                        self.communicator = comm
            else:
                self.communicator = communicator
        else:
            self.local_rank = 0
            self.communicator = None
        # "sendrecv" (neighbour P2P over xGMI, default), "allgather", "nocomm" or a HaloExchanger
        self.halo_ex = make_exchanger(halo_ex, self.communicator, self.local_rank, spatial_group_size) \
            if spatial_group_size > 1 else None

    def _halo(self, out):
        return halo_pad(out, 1, self.communicator, self.local_rank, self.spatial_group_size, self.halo_ex)

    def _conv2_plain(self, out):
        if self.spatial_group_size == 1:
            return self.conv2(out)
        return F.conv2d(self._halo(out), self.conv2.weight, None, padding=(0, 1))

    def _conv2_input(self, out):
        if self.spatial_group_size == 1:
            return out, (1, 1)
        return self._halo(out), (0, 1)
