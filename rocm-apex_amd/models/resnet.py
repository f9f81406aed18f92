"""ResNet family (He et al. 2015; v1.5 stride placement), the architecture behind the reference's
headline ImageNet benchmark (reference examples/imagenet/main_amp.py uses torchvision's
``resnet50``; torchvision is not a dependency here, so the architecture is defined directly).

Layout notes for MI355X: build with ``memory_format=torch.channels_last`` — MIOpen's NHWC
convolution kernels and our NHWC batch-norm kernels are the fast path on gfx950.

``fused_bn=True`` also routes the bottleneck 1x1 convolutions through ``ops.conv.Conv1x1NHWC``
(native MFMA GEMM where it beats MIOpen for the shape) and swaps every BatchNorm (+ReLU) (+residual add +ReLU) group for
``apex.contrib.groupbn.BatchNorm2d_NHWC`` with the ReLU / add fused in (reference capability:
apex/contrib/groupbn, the NHWC BN with fused add+ReLU used for ResNet-50).  Parameters, buffers
and state_dict keys are identical to the torch.nn.BatchNorm2d model; the math is the same
training-mode batch norm, computed by the gfx950 kernels in fewer HBM passes.

``bn_group=N`` (fused only) makes every batch norm a synchronized one over groups of N adjacent
ranks (the reference's groupbn ``bn_group``; ``bn_group=world`` is SyncBatchNorm over the whole
job): same fused kernels, statistics exchanged over xGMI peer memory (or RCCL).

In the fused model every block but the last hands its output on as a ``(main, shortcut)`` pair of
aliases (``BatchNorm2d_NHWC(..., fork=True)``): the next block's conv1 reads one and its shortcut
the other, so the two gradients of the block output reach the producing batch norm separately
and are summed inside its backward reduction instead of by an autograd add over the activation."""
import os

import torch
import torch.nn as nn

from ..ops.conv import ChannelPadConv2d, Conv1x1NHWC, Conv2dNHWC
from ..ops.pooling import MaxPool2dNHWC

__all__ = ["ResNet", "BasicBlock", "Bottleneck", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152"]


def conv3x3(cin, cout, stride=1, groups=1, dilation=1, native=False):
    # native: the gfx950 implicit-GEMM NHWC kernels where they beat MIOpen (ops/conv.py tap_route)
    if native and groups == 1 and dilation == 1:
        return Conv2dNHWC(cin, cout, 3, stride)
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=dilation, groups=groups, bias=False,
                     dilation=dilation)


def conv1x1(cin, cout, stride=1, native=False):
    # native: per-shape routing of the NHWC GEMM / implicit-GEMM kernels to the gfx950 MFMA
    # kernels (ops/conv.py); same parameters / state_dict as nn.Conv2d
    if native:
        return Conv1x1NHWC(cin, cout, stride) if stride == 1 else Conv2dNHWC(cin, cout, 1, stride)
    return nn.Conv2d(cin, cout, kernel_size=1, stride=stride, bias=False)


def _bn_add_bn_relu(x, z, bn_x, bn_z, fork):
    from ..contrib.groupbn import bn_add_bn_relu

    return bn_add_bn_relu(x, z, bn_x, bn_z, fork=fork)


def _fused_bn(planes, relu, bn_group=1):
    from ..contrib.groupbn import BatchNorm2d_NHWC

    return BatchNorm2d_NHWC(planes, fuse_relu=relu, torch_channels_last=True, bn_group=bn_group)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, fused_bn=False, bn_group=1):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self.fused_bn = fused_bn
        self.conv1 = conv3x3(inplanes, planes, stride, native=fused_bn)
        self.bn1 = _fused_bn(planes, True, bn_group) if fused_bn else norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes, native=fused_bn)
        self.bn2 = _fused_bn(planes, True, bn_group) if fused_bn else norm_layer(planes)
        self.downsample = downsample
        self.stride = stride
        self.fork_out = False

    def forward(self, x):
        if self.fused_bn:
            xm, xr = x if isinstance(x, tuple) else (x, x)
            zds = None if self.downsample is None else self.downsample[0](xr)
            out = self.bn1(self.conv1(xm))
            if zds is not None:
                return _bn_add_bn_relu(self.conv2(out), zds, self.bn2, self.downsample[1], self.fork_out)
            return self.bn2(self.conv2(out), xr, fork=self.fork_out)
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, fused_bn=False, bn_group=1):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self.fused_bn = fused_bn
        width = int(planes * (base_width / 64.0)) * groups
        nl = (lambda c, relu: _fused_bn(c, relu, bn_group)) if fused_bn else (lambda c, relu: norm_layer(c))  # noqa: E731
        self.conv1 = conv1x1(inplanes, width, native=fused_bn)
        self.bn1 = nl(width, True)
        self.conv2 = conv3x3(width, width, stride, groups, dilation, native=fused_bn)
        self.bn2 = nl(width, True)
        self.conv3 = conv1x1(width, planes * self.expansion, native=fused_bn)
        self.bn3 = nl(planes * self.expansion, True)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self.fork_out = False

    def forward_linked(self, x, link_in, nxt=None):
        """Fused-node forward that chains with its neighbours (``ops.bottleneck_bn.BlockLink``):
        returns ``(out, link_out)``; falls back to ``forward`` (and no link) off the node path.
        ``nxt``: the block that consumes the output (it may take over the output pass).

        Only ``run_linked`` may call this: with a deferring ``link_out`` the returned tensor is
        EMPTY until ``nxt``'s conv1 (or ``BlockLink.materialize``) writes it, and ``run_linked``
        is what guarantees one of the two runs before anything else reads it."""
        from ..ops import bottleneck_bn

        if self.fused_bn and not isinstance(x, tuple) and self.training and bottleneck_bn.block_supported(self, x):
            n, _, h, w = x.shape
            s = self.conv2.stride[0]
            oh, ow = (h - 1) // s + 1, (w - 1) // s + 1
            defer = nxt is not None and bottleneck_bn.takes_deferred_input(
                nxt, (n, self.conv3.out_channels, oh, ow), x.dtype)
            link_out = bottleneck_bn.BlockLink(defer)
            return bottleneck_bn.bottleneck_forward(self, x, link_in, link_out), link_out
        if link_in is not None:
            link_in.materialize()
        return self.forward(x), None

    def forward(self, x):
        if self.fused_bn:
            from ..ops import bottleneck_bn

            if not isinstance(x, tuple) and self.training and bottleneck_bn.block_supported(self, x):
                # the whole block as one node: BN statistics in the 1x1 conv epilogues, bn2's
                # apply+ReLU as conv3's operand prologue (ops/bottleneck_bn.py)
                return bottleneck_bn.bottleneck_forward(self, x)
            xm, xr = x if isinstance(x, tuple) else (x, x)
            # downsampling block: the shortcut's conv output goes straight into the fused
            # relu(bn3(.) + bn_ds(.)) pass (contrib.groupbn.bn_add_bn_relu) — its normalized
            # tensor is never written
            zds = None if self.downsample is None else self.downsample[0](xr)
            out = self.bn1(self.conv1(xm))
            out = self.bn2(self.conv2(out))
            if zds is not None:
                return _bn_add_bn_relu(self.conv3(out), zds, self.bn3, self.downsample[1], self.fork_out)
            return self.bn3(self.conv3(out), xr, fork=self.fork_out)
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + identity)


def run_linked(blocks, x):
    """Run consecutive fused-BN blocks as chained bottleneck nodes: block i hands block i+1 its
    output BN's state (ops/bottleneck_bn.py BlockLink), so block i+1's conv1 data gradient does
    block i's bn3 backward reduction.  Blocks off the node path run unlinked."""
    link = None
    for i, blk in enumerate(blocks):
        nxt = blocks[i + 1] if i + 1 < len(blocks) and isinstance(blocks[i + 1], Bottleneck) else None
        if isinstance(blk, Bottleneck):
            x, link = blk.forward_linked(x, link, nxt)
        else:
            if link is not None:
                link.materialize()
            x, link = blk(x), None
    if link is not None:
        link.materialize()
    # the hand-off contract: no block output is left deferred (uninitialised) once the walk ends
    assert link is None or link.pend is None, "run_linked: a deferred block output was never computed"
    return x


def _has_hooks(layers):
    from torch.nn.modules import module as _m

    if any(getattr(_m, n, None) for n in ("_global_forward_hooks", "_global_forward_pre_hooks",
                                         "_global_backward_hooks", "_global_backward_pre_hooks")):
        return True
    for layer in layers:
        for mod in (layer, *layer):
            if (mod._forward_hooks or mod._forward_pre_hooks or mod._backward_hooks
                    or getattr(mod, "_backward_pre_hooks", None)):
                return True
    return False


class _SpatialMeanNHWC(torch.autograd.Function):
    """Global average pool of a channels_last [N, C, H, W] activation to [N, C] whose gradient is
    produced directly in channels_last memory: nn.AdaptiveAvgPool2d's backward hands the last
    bottleneck node an NCHW-contiguous gradient, and making it channels_last cost a strided
    83 us copy per ResNet-50 step (tools/find_copies.py); here it is one broadcast write."""

    @staticmethod
    def forward(ctx, x):
        n, c, h, w = x.shape
        ctx.geo = (n, c, h, w)
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, g):
        n, c, h, w = ctx.geo
        from .. import _native

        ext = _native.submodule("conv")
        if (ext is not None and hasattr(ext, "spatial_broadcast") and g.is_cuda and c % 8 == 0
                and g.dtype in (torch.bfloat16, torch.float16)):
            # one 16-byte store per 8 channels (layout.hip spatial_broadcast; torch's expand copy
            # took 38 us per ResNet-50 step)
            return ext.spatial_broadcast(g.contiguous(), h, w, 1.0 / (h * w))
        gx = (g * (1.0 / (h * w))).view(n, 1, 1, c).expand(n, h, w, c).contiguous()
        return gx.permute(0, 3, 1, 2)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, zero_init_residual=False, groups=1, width_per_group=64,
                 norm_layer=None, fused_bn=False, bn_group=1):
        super().__init__()
        self._norm_layer = norm_layer or nn.BatchNorm2d
        self.fused_bn = fused_bn
        self.bn_group = bn_group
        self.inplanes = 64
        self.dilation = 1
        self.groups = groups
        self.base_width = width_per_group
        # fused path: stem input channels padded 3 -> 4 on the GPU (MIOpen's NHWC kernels, ops/conv.py)
        stem = ChannelPadConv2d if fused_bn else nn.Conv2d
        self.conv1 = stem(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = _fused_bn(self.inplanes, True, bn_group) if fused_bn else self._norm_layer(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        # fused path (channels_last): gfx950 NHWC max pool with 1-byte indices
        self.maxpool = MaxPool2dNHWC(kernel_size=3, stride=2, padding=1) if fused_bn else \
            nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)) or hasattr(m, "running_mean"):
                if getattr(m, "weight", None) is not None:
                    nn.init.constant_(m.weight, 1)
                    nn.init.constant_(m.bias, 0)
        if fused_bn:
            blocks = [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]
            for b in blocks[:-1]:
                b.fork_out = True
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            bn = (_fused_bn(planes * block.expansion, False, self.bn_group) if self.fused_bn
                  else norm_layer(planes * block.expansion))
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride, native=self.fused_bn),
                                       bn)
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width, self.dilation,
                        norm_layer, fused_bn=self.fused_bn, bn_group=self.bn_group)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                dilation=self.dilation, norm_layer=norm_layer, fused_bn=self.fused_bn,
                                bn_group=self.bn_group))
        return nn.Sequential(*layers)

    @property
    def _amp_casts_input(self):
        # amp O2 hands the fused-BN model its fp32 batch: the native stem casts it in its padding
        # pass (forward below), every other path casts it first
        return self.fused_bn and os.environ.get("APEX_AMD_STEM_INPUT_CAST", "1") != "0"

    def forward(self, x):
        amp_dt = getattr(self, "_amp_input_dtype", None)
        if self.fused_bn:
            # stem: BN statistics, then normalize + ReLU + 3x3/2 max pool in one pass
            from ..contrib.groupbn import bn_relu_maxpool
            from ..ops import stem

            self.conv1._amp_input_fp32_ok = amp_dt is not None and amp_dt == self.conv1.weight.dtype
            if not (stem.stem_supported(self.conv1, self.bn1, self.maxpool, x) and not _has_hooks(())):
                if amp_dt is not None and torch.is_tensor(x) and x.is_floating_point() and x.dtype != amp_dt:
                    x = x.to(amp_dt)
            if stem.stem_supported(self.conv1, self.bn1, self.maxpool, x) and not _has_hooks(()):
                # conv + BN statistics, BN + ReLU + pool, and the fused backward (ops/stem.py)
                x = stem.stem_forward(self.conv1, self.bn1, self.maxpool, x)
            else:
                x = bn_relu_maxpool(self.conv1(x), self.bn1, self.maxpool)
            # bottleneck nodes hand each other their output BN's state (ops/bottleneck_bn.py
            # BlockLink): block i+1's conv1 dgrad does block i's bn3 backward reduction.  The
            # linked walk calls the blocks directly and hands block i the ReLU-MASKED gradient of
            # its output, so with any module hook on the layers / blocks (forward or backward,
            # global ones included) the model runs each layer through ``__call__`` unlinked.
            layers = (self.layer1, self.layer2, self.layer3, self.layer4)
            if _has_hooks(layers):
                for layer in layers:
                    x = layer(x)
            else:
                x = run_linked([blk for layer in layers for blk in layer], x)
        else:
            x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
            x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if isinstance(x, tuple):
            x = x[0]
        if (self.fused_bn and x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
                and isinstance(self.avgpool, nn.AdaptiveAvgPool2d) and self.avgpool.output_size in ((1, 1), 1)
                and not self.avgpool._forward_hooks and not self.avgpool._forward_pre_hooks):
            x = _SpatialMeanNHWC.apply(x)
        else:
            x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)
