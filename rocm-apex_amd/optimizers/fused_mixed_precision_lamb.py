"""FusedMixedPrecisionLamb (reference apex/optimizers/fused_mixed_precision_lamb.py:8-256).

LAMB with device-resident ``lr`` and ``step`` and native ``torch.cuda.amp.GradScaler``
integration (``_step_supports_amp_scaling``): ``found_inf`` skips the update on device and
``inv_scale`` unscales inside the kernel, so the step never syncs with the host.  With
``reduced_precision_dtype`` the optimizer keeps fp32 masters and writes the low-precision params
in the same kernel pass."""
from collections import defaultdict
from copy import deepcopy
from itertools import chain

import torch

from .. import amp_C


class FusedMixedPrecisionLamb(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, step=0, bias_correction=True, betas=(0.9, 0.999), eps=1e-6,
                 weight_decay=0.01, amsgrad=False, adam_w_mode=True, grad_averaging=True, max_grad_norm=1.0,
                 use_nvlamb=False, reduced_precision_dtype=None):
        if amsgrad:
            raise RuntimeError("FusedLAMB does not support the AMSGrad variant.")
        defaults = dict(lr=torch.tensor(lr, dtype=torch.float32), step=torch.tensor([step], dtype=torch.int),
                        bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        grad_averaging=grad_averaging, max_grad_norm=max_grad_norm)
        super(FusedMixedPrecisionLamb, self).__init__(params, defaults)
        device = self.param_groups[0]["params"][0].device
        for group in self.param_groups:
            for item in ("lr", "step"):
                group[item] = group[item].to(device=device)
        self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int32, device=device)
        self.reduced_precision_dtype = reduced_precision_dtype
        self.param_groups_full_precision = []
        self._step_supports_amp_scaling = True
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.use_nvlamb = use_nvlamb

    def load_state_dict(self, state_dict):
        """Like torch's, but state tensors keep their own dtype/device (fp32 moments for
        reduced-precision params)."""
        state_dict = deepcopy(state_dict)
        groups = self.param_groups
        saved_groups = state_dict["param_groups"]
        if len(groups) != len(saved_groups):
            raise ValueError("loaded state dict has a different number of parameter groups")
        if any(len(g["params"]) != len(s["params"]) for g, s in zip(groups, saved_groups)):
            raise ValueError("loaded state dict contains a parameter group that doesn't match the size of "
                             "optimizer's group")
        id_map = {old: p for old, p in zip(chain.from_iterable(g["params"] for g in saved_groups),
                                           chain.from_iterable(g["params"] for g in groups))}

        def cast(param, value):
            if isinstance(value, torch.Tensor):
                return value.to(param.device)
            if isinstance(value, dict):
                return {k: cast(param, v) for k, v in value.items()}
            return value

        state = defaultdict(dict)
        for k, v in state_dict["state"].items():
            if k in id_map:
                state[id_map[k]] = cast(id_map[k], v)
            else:
                state[k] = v
        param_groups = []
        for g, ng in zip(groups, saved_groups):
            ng["params"] = g["params"]
            for item in ("lr", "step"):
                if isinstance(ng.get(item), torch.Tensor):
                    ng[item] = ng[item].to(g["params"][0].device)
            param_groups.append(ng)
        self.__setstate__({"state": state, "param_groups": param_groups})

    def _setup_full_precision_params(self):
        for pg in self.param_groups:
            self.param_groups_full_precision.append({"params": [
                p.clone().detach().to(dtype=torch.float32)
                if (self.reduced_precision_dtype is not None) and (p.dtype == self.reduced_precision_dtype) else None
                for p in pg["params"]]})

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        for name, default in self.defaults.items():
            if isinstance(default, torch.Tensor):
                self.param_groups[-1][name] = default.clone().to(self.param_groups[0]["params"][0].device)

    @torch.no_grad()
    def step(self, closure=None, grad_scaler=None):
        loss = closure() if closure is not None else None
        if len(self.param_groups_full_precision) == 0:
            self._setup_full_precision_params()
        grad_list = []
        for group in self.param_groups:
            for p in group["params"]:
                assert group["params"][0].dtype == p.dtype, \
                    "Error: Parameters are not of the identical type: {} != {}".format(group["params"][0].dtype,
                                                                                       p.dtype)
                if p.grad is not None:
                    grad_list.append(p.grad)
        device = self.param_groups[0]["params"][0].device
        found_inf = (grad_scaler._check_inf_per_device(self)[device] if grad_scaler is not None
                     else torch.zeros((1,), device=device))
        self._dummy_overflow_buf.copy_(found_inf)
        if grad_scaler:
            scale = grad_scaler._get_scale_async()
            inv_scale = scale.double().reciprocal().float()
        else:
            scale = torch.ones((1,), device=device)
            inv_scale = torch.ones((1,), device=device)
        max_grad_norm = (self.defaults["max_grad_norm"] * scale).reshape(1).float()
        grad_norm = amp_C.multi_tensor_l2norm_mp(65536, self._dummy_overflow_buf, [grad_list], False)[0]
        for group, group_full in zip(self.param_groups, self.param_groups_full_precision):
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            grad_averaging = 1 if group["grad_averaging"] else 0
            group["step"] += (self._dummy_overflow_buf != 1).to(torch.int)
            lists = [[], [], [], []]
            if self.reduced_precision_dtype is not None:
                lists.append([])
            for p, p_full in zip(group["params"], group_full["params"]):
                if p.grad is None:
                    continue
                assert not p.grad.is_sparse
                state = self.state[p]
                if len(state) == 0:
                    dtype = torch.float32 if (self.reduced_precision_dtype is not None and
                                              p.dtype == self.reduced_precision_dtype) else p.dtype
                    state["exp_avg"] = torch.zeros_like(p, dtype=dtype)
                    state["exp_avg_sq"] = torch.zeros_like(p, dtype=dtype)
                lists[0].append(p.grad)
                lists[2].append(state["exp_avg"])
                lists[3].append(state["exp_avg_sq"])
                if self.reduced_precision_dtype is not None:
                    lists[1].append(p_full if p_full is not None else p)
                    lists[4].append(p)
                else:
                    lists[1].append(p)
            if not lists[0]:
                continue
            if self.reduced_precision_dtype is not None and any(x is y for x, y in zip(lists[1], lists[4])):
                lists = lists[:4]  # params already full precision: no copy-out
            amp_C.multi_tensor_lamb_mp(65536, self._dummy_overflow_buf, lists, group["lr"].float().reshape(1),
                                       beta1, beta2, group["eps"], group["step"], bias_correction,
                                       group["weight_decay"], grad_averaging, self.adam_w_mode, grad_norm,
                                       max_grad_norm, self.use_nvlamb, found_inf, inv_scale)
        return loss
