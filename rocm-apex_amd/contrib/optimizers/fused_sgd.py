"""Legacy contrib FusedSGD (reference apex/contrib/optimizers/fused_sgd.py:7-211), the optimizer behind
``apex.contrib.optimizers.FP16_Optimizer``; shared plumbing in ``_legacy_common.py``."""

import torch

from ... import amp_C
from ._legacy_common import _groupify, _split_by


class FusedSGD(torch.optim.Optimizer):
    """SGD for ``FP16_Optimizer`` (reference contrib fused_sgd.py): ``grads`` and ``output_params``
    are mandatory; fp16 model params get their copy written by the same launch."""

    def __init__(self, params, lr=0.1, momentum=0, dampening=0, weight_decay=0, nesterov=False,
                 wd_after_momentum=False, materialize_master_grads=True):
        if momentum < 0.0 or weight_decay < 0.0 or lr < 0.0:
            raise ValueError("invalid hyper-parameter")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))
        self.wd_after_momentum = wd_after_momentum

    def get_momentums(self, params):
        first_run = True
        moms = []
        for p in params:
            st = self.state[p]
            if "momentum_buffer" not in st:
                st["momentum_buffer"] = torch.zeros_like(p)
            else:
                first_run = False
            moms.append(st["momentum_buffer"])
        return moms, first_run

    def step(self, closure=None, grads=None, output_params=None, scale=1.0, grad_norms=None):
        if hasattr(self, "_amp_stash"):
            raise RuntimeError("apex.contrib.optimizers.FusedSGD should not be used with AMP.")
        loss = closure() if closure is not None else None
        if grads is None or output_params is None:
            raise RuntimeError("apex.contrib.optimizers.FusedSGD must be wrapped with "
                               "apex.contrib.optimizers.FP16_Optimizer which provides grads and output_params.")
        n = len(self.param_groups)
        for group, g_this, o_this in zip(self.param_groups, _groupify(grads, n), _groupify(output_params, n)):
            if g_this is None or o_this is None:
                raise RuntimeError("apex.contrib.optimizers.FusedSGD only works when all parameters require grad.")
            masters = group["params"]
            keys = [(g.dtype, o.dtype) for g, o in zip(g_this, o_this)]
            for (gdt, odt), (g_l, p_l, o_l) in _split_by(keys, list(g_this), list(masters), list(o_this)).items():
                moms, first = self.get_momentums(p_l)
                dev = p_l[0].device
                noop = torch.zeros(1, dtype=torch.int32, device=dev)
                tl = [g_l, p_l, moms] + ([o_l] if odt != p_l[0].dtype else [])
                amp_C.multi_tensor_sgd(65536, noop, tl, group["weight_decay"], group["momentum"],
                                       group["dampening"], group["lr"], group["nesterov"], first,
                                       self.wd_after_momentum, 1.0 / scale)
                if odt == p_l[0].dtype:
                    for o, p in zip(o_l, p_l):
                        if o.data_ptr() != p.data_ptr():
                            o.data.copy_(p.data)
        return loss
