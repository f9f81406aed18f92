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

    # ---- fused path: conv -> frozen-BN scale/bias -> (+ residual) -> ReLU per stage ----
    def _forward_fused(self, x):
        nhwc = self.explicit_nhwc
        if nhwc:
            x = x.permute(0, 3, 1, 2)  # [N, H, W, C] -> channels_last NCHW view
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
