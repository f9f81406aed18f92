import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, apex
from apex import amp
from apex.models import resnet50
from apex.optimizers import FusedAdam
from apex.ops import conv as C
m = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
o = FusedAdam(m.parameters(), materialize_master_grads=False)
m, o = amp.initialize(m, o, opt_level='O2', cast_model_type=torch.bfloat16, keep_batchnorm_fp32=True, verbosity=0)
for name, mod in m.named_modules():
    if isinstance(mod, C.Conv2dNHWC):
        def hook(mod, inp, name=name):
            x = inp[0]
            print(name, "native_ok", mod._native_ok(x), x.dtype, mod.weight.dtype, x.is_contiguous(memory_format=torch.channels_last),
                  mod.weight.is_contiguous(memory_format=torch.channels_last), C.tap_route(mod.in_channels, mod.out_channels, mod.kernel_size[0], mod.stride[0], x.shape[2]))
        mod.register_forward_pre_hook(hook)
x = torch.randn(8, 3, 224, 224, device="cuda").to(memory_format=torch.channels_last)
y = m(x)
print("ok", y.shape)
