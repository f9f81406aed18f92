"""Print memory formats along the ResNet-50 fused stem under amp O2 (diagnostic)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import apex
from apex import amp
from apex.models import resnet50
from apex.optimizers import FusedAdam

m = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
opt = FusedAdam(m.parameters(), lr=1e-3)
m, opt = amp.initialize(m, opt, opt_level="O2", cast_model_type=torch.bfloat16, keep_batchnorm_fp32=True, verbosity=0)
x = torch.randn(8, 3, 224, 224, device="cuda").to(memory_format=torch.channels_last)
def hook(name):
    def f(mod, inp, out):
        i = inp[0]
        print(name, "in", tuple(i.shape), i.dtype, i.stride(), "cl" if i.is_contiguous(memory_format=torch.channels_last) else "NOT-cl",
              "| out", tuple(out.shape), out.stride(), "cl" if out.is_contiguous(memory_format=torch.channels_last) else "NOT-cl", flush=True)
    return f
base = m
base.conv1.register_forward_hook(hook("conv1"))
base.bn1.register_forward_hook(hook("bn1"))
base.maxpool.register_forward_hook(hook("maxpool"))
base.layer1[0].conv1.register_forward_hook(hook("layer1.0.conv1"))
base.fc.register_forward_hook(hook("fc"))
y = m(x)
y.float().sum().backward()
print("done")
