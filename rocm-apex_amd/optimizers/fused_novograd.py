"""FusedNovoGrad (reference apex/optimizers/fused_novograd.py:4-214).

Per-tensor second moment kept as a norm in ``group['exp_avg_sq'] = [low_precision_norms,
fp32_norms]``; each step blends the new per-tensor grad norms in-kernel (single-pass reduction,
no cleanup launch) and then applies the moment update."""
import torch

from .. import amp_C


class FusedNovoGrad(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, reg_inside_moment=False, grad_averaging=True, norm_type=2, init_zero=False,
                 set_grad_none=True):
        if amsgrad:
            raise RuntimeError("FusedNovoGrad does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        grad_averaging=grad_averaging, norm_type=norm_type, init_zero=init_zero)
        super(FusedNovoGrad, self).__init__(params, defaults)
        self.moment_mode = 0 if reg_inside_moment else 1
        self.set_grad_none = set_grad_none
        self._dummy_overflow_buf = None

    def zero_grad(self, set_to_none=None):
        if self.set_grad_none if set_to_none is None else set_to_none:
            for group in self.param_groups:
                for p in group["params"]:
                    p.grad = None
        else:
            super(FusedNovoGrad, self).zero_grad(set_to_none=False)

    def load_state_dict(self, state_dict):
        super(FusedNovoGrad, self).load_state_dict(state_dict)
        for group in self.param_groups:
            if len(group["params"]) > 0 and "exp_avg_sq" in group:
                dev = group["params"][0].device
                group["exp_avg_sq"] = [t.to(dev) for t in group["exp_avg_sq"]]

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            grad_averaging = 1 if group["grad_averaging"] else 0
            group["step"] = group.get("step", 0) + 1
            g_16, p_16, m_16, g_32, p_32, m_32 = [], [], [], [], [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedNovoGrad does not support sparse gradients")
                state = self.state[p]
                if len(state) == 0:
                    state["exp_avg"] = torch.zeros_like(p)
                if p.dtype in (torch.float16, torch.bfloat16):
                    g_16.append(p.grad)
                    p_16.append(p)
                    m_16.append(state["exp_avg"])
                elif p.dtype == torch.float32:
                    g_32.append(p.grad)
                    p_32.append(p)
                    m_32.append(state["exp_avg"])
                else:
                    raise RuntimeError("FusedNovoGrad only support fp16, bfloat16 and fp32.")
            device = self.param_groups[0]["params"][0].device
            if self._dummy_overflow_buf is None:
                self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int32, device=device)
            if "exp_avg_sq" not in group:
                if group["init_zero"]:
                    v16 = torch.zeros(len(g_16), device=device)
                    v32 = torch.zeros(len(g_32), device=device)
                else:  # initialize with the first step's norms so the first blend is a no-op
                    if group["norm_type"] == 0:
                        f = lambda g: g.float().abs().max()  # noqa: E731
                    elif group["norm_type"] == 2:
                        f = lambda g: g.float().pow(2).sum().sqrt()  # noqa: E731
                    else:
                        raise RuntimeError("FusedNovoGrad only support l2/inf norm now.")
                    v16 = torch.stack([f(g) for g in g_16]).float() if g_16 else torch.zeros(0, device=device)
                    v32 = torch.stack([f(g) for g in g_32]).float() if g_32 else torch.zeros(0, device=device)
                group["exp_avg_sq"] = [v16.to(device), v32.to(device)]
            else:
                assert len(g_16) == group["exp_avg_sq"][0].numel()
                assert len(g_32) == group["exp_avg_sq"][1].numel()
            for gs, ps, ms, norms in ((g_16, p_16, m_16, group["exp_avg_sq"][0]),
                                      (g_32, p_32, m_32, group["exp_avg_sq"][1])):
                if gs:
                    amp_C.multi_tensor_novograd(65536, self._dummy_overflow_buf, [gs, ps, ms], norms, group["lr"],
                                                beta1, beta2, group["eps"], group["step"], bias_correction,
                                                group["weight_decay"], grad_averaging, self.moment_mode,
                                                group["norm_type"])
        return loss
