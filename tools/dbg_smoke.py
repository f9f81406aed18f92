import torch, sys
sys.path.insert(0, '.')
import apex
from apex import amp
from apex.models import resnet50
from apex.optimizers import FusedAdam
import apex.amp_C as amp_C
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = resnet50().to(dev).to(memory_format=torch.channels_last)
opt = FusedAdam(model.parameters(), lr=1e-3, materialize_master_grads=False)
model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
x = torch.randn(4, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (4,), device=dev)
names = [n for n, _ in model.named_parameters()]
loss = torch.nn.functional.cross_entropy(model(x), y)
(loss * 32768.0).backward()
bad = [(n, p.dtype, p.grad.is_contiguous(), p.grad.is_contiguous(memory_format=torch.channels_last) if p.grad.dim()==4 else None) for n, p in zip(names, model.parameters()) if not torch.isfinite(p.grad).all()]
print("nonfinite grads:", bad)
for dt in (torch.bfloat16, torch.float32):
    gs = [p.grad for p in model.parameters() if p.grad.dtype == dt]
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    amp_C.multi_tensor_check_finite(65536, flag, [gs])
    print(dt, "check_finite flag", flag.item(), len(gs))
    for i, g in enumerate(gs):
        f = torch.zeros(1, dtype=torch.int32, device=dev)
        amp_C.multi_tensor_check_finite(65536, f, [[g]])
        if f.item():
            print("  flagged", i, g.shape, g.stride(), g.dtype, g.data_ptr() % 32, float(g.float().abs().max()))
