"""Weight normalisation w = g v / ||v|| (reference apex/reparameterization/weight_norm.py:8-78).
The recompute is torch's fused ``_weight_norm`` kernel (fp32 norm accumulation for 16-bit v)."""
import torch
from torch.nn.parameter import Parameter

from .reparameterization import Reparameterization


def _norm(p, dim):
    """Norm over every dimension except ``dim`` (``None``: whole tensor)."""
    if dim is None:
        return p.norm()
    if dim == 0:
        return p.contiguous().view(p.size(0), -1).norm(dim=1).view((p.size(0),) + (1,) * (p.dim() - 1))
    if dim == p.dim() - 1:
        return p.contiguous().view(-1, p.size(-1)).norm(dim=0).view((1,) * (p.dim() - 1) + (p.size(-1),))
    return _norm(p.transpose(0, dim), 0).transpose(0, dim)


class WeightNorm(Reparameterization):
    def compute_weight(self, module=None, name=None):
        module = self.module if module is None else module
        name = self.name if name is None else name
        module, name = Reparameterization.get_module_and_name(module, name)
        g = getattr(module, name + "_g")
        v = getattr(module, name + "_v").contiguous()
        if self.dim is None:
            return v * (g / v.float().norm().to(v.dtype))
        return torch._weight_norm(v, g, self.dim)

    def reparameterize(self, name, weight, dim):
        names = [name + "_g", name + "_v"]
        params = [Parameter(_norm(weight, dim).data), Parameter(weight.data)]
        return names, params
