"""Automatic SParsity (reference apex/contrib/sparsity/asp.py:21-217).

Same class-level API: ``init_model_for_pruning`` registers a boolean ``__<param>_mma_mask``
buffer per eligible weight (plus a CPU ``__<param>_mma_pruned_p`` stash with
``allow_recompute_mask``), ``init_optimizer_for_pruning`` wraps ``optimizer.step`` so gradients
are masked before and weights after the step, ``compute_sparse_masks`` /
``restore_pruned_weights`` / ``is_sparsity_enabled`` / ``prune_trained_model``.

The masking around the step is two ``torch._foreach_mul_`` calls over every sparse tensor
(one fused multi-tensor launch each) rather than one kernel per layer.  Eligibility follows
MFMA-friendly shapes: output dim % 8 and input dim % 16 (the sparse-MFMA 4:2 tile)."""
import types

import torch

from .sparse_masklib import create_mask


def eligible_modules(model, whitelist_layer_types, allowed_layer_names, disallowed_layer_names):
    out = []
    for name, mod in model.named_modules():
        if isinstance(mod, whitelist_layer_types) and name not in disallowed_layer_names:
            if allowed_layer_names is not None and name not in allowed_layer_names:
                continue
            out.append((name, mod))
    return out


class ASP:
    __model = None
    __verbosity = 0
    __optimizer = None
    __sparse_parameters = []
    __calculate_mask = None

    @classmethod
    def init_model_for_pruning(cls, model, mask_calculator="m4n2_1d", verbosity=3,
                               whitelist=(torch.nn.Linear, torch.nn.Conv1d, torch.nn.Conv2d, torch.nn.Conv3d),
                               allowed_layer_names=None, disallowed_layer_names=(), allow_recompute_mask=False,
                               custom_layer_dict=None):
        assert cls.__model is None, "ASP has been initialized already."
        cls.__model = model
        cls.__verbosity = verbosity
        if isinstance(mask_calculator, str):
            pattern = mask_calculator
            cls.__calculate_mask = lambda p: create_mask(p, pattern).bool()
        else:
            cls.__calculate_mask = mask_calculator
        params_of = {torch.nn.Linear: ["weight"], torch.nn.Conv1d: ["weight"], torch.nn.Conv2d: ["weight"],
                     torch.nn.Conv3d: ["weight"]}
        whitelist = list(whitelist)
        if custom_layer_dict:
            params_of.update(custom_layer_dict)
            whitelist += list(custom_layer_dict.keys())
        for t in whitelist:
            assert t in params_of, "Module {} :: Don't know how to sparsify module.".format(t)

        def add(module_name, module):
            names = params_of[type(module)]
            for p_name, p in module.named_parameters():
                if p_name not in names or not p.requires_grad:
                    continue
                if p.dim() >= 2 and (p.size(0) % 8 != 0 or p.size(1) % 16 != 0):
                    if cls.__verbosity >= 1:
                        print("[ASP] Auto skipping pruning {}::{} of size={} and type={} for sparsity".format(
                            module_name, p_name, tuple(p.shape), p.dtype))
                    continue
                if cls.__verbosity >= 3:
                    print("[ASP] Sparsifying {}::{} of size={} and type={} for sparsity".format(
                        module_name, p_name, tuple(p.shape), p.dtype))
                mask = torch.ones_like(p, dtype=torch.bool)
                buf = p_name.split(".")[-1]
                module.register_buffer("__%s_mma_mask" % buf, mask)
                pruned = None
                if allow_recompute_mask:
                    pruned = torch.zeros_like(p, device="cpu")
                    module.register_buffer("__%s_mma_pruned_p" % buf, pruned)
                cls.__sparse_parameters.append((module_name, module, p_name, p, mask, pruned))

        for name, mod in eligible_modules(model, tuple(whitelist), allowed_layer_names, disallowed_layer_names):
            add(name, mod)

    @classmethod
    def _masked(cls):
        ps, ms = [], []
        for _, _, _, p, mask, _ in cls.__sparse_parameters:
            ps.append(p)
            ms.append(mask)
        return ps, ms

    @classmethod
    def init_optimizer_for_pruning(cls, optimizer):
        assert cls.__optimizer is None, "ASP has initialized optimizer already."
        assert cls.__calculate_mask is not None, \
            "Called ASP.init_optimizer_for_pruning before ASP.init_model_for_pruning."
        cls.__optimizer = optimizer
        optimizer.__asp_step = optimizer.step

        def step(opt_self, *args, **kwargs):
            ps, ms = cls._masked()
            with torch.no_grad():
                gl = [(p.grad, m) for p, m in zip(ps, ms) if p.grad is not None]
                if gl:
                    torch._foreach_mul_([g for g, _ in gl], [m.to(g.dtype) for g, m in gl])
            rval = opt_self.__asp_step(*args, **kwargs)
            with torch.no_grad():
                if ps:
                    torch._foreach_mul_(ps, [m.to(p.dtype) for p, m in zip(ps, ms)])
            return rval

        optimizer.step = types.MethodType(step, optimizer)

    @classmethod
    def compute_sparse_masks(cls):
        with torch.no_grad():
            for module_name, module, p_name, p, mask, pruned in cls.__sparse_parameters:
                if mask.sum() < mask.numel():  # recomputing: restore the dense weight first
                    assert pruned is not None, "Unable to restore dense parameter because allow_recompute_mask == False"
                    p.add_(pruned.to(p.device))
                mask.set_(cls.__calculate_mask(p).to(mask.device))
                if pruned is not None:
                    pruned.set_((p * (~mask)).cpu())
                p.mul_(mask)
                if cls.__verbosity >= 2:
                    print("[ASP] Enabled {:.2f}% sparsity for {}::{} of size={} and type={}".format(
                        100.0 * float(mask.sum()) / mask.numel(), module_name, p_name, tuple(p.shape), p.dtype))

    @classmethod
    def restore_pruned_weights(cls):
        with torch.no_grad():
            for module_name, module, p_name, p, mask, pruned in cls.__sparse_parameters:
                if mask.sum() < mask.numel():
                    assert pruned is not None, "Unable to restore dense parameter because allow_recompute_mask == False"
                    p.add_(pruned.to(p.device))
                    mask.fill_(1)
                    pruned.zero_()
                    if cls.__verbosity >= 2:
                        print("[ASP] Disabled sparsity for {}::{} (dense weights restored)".format(module_name, p_name))

    @classmethod
    def is_sparsity_enabled(cls):
        total = sp100 = sp50 = 0
        for _, _, _, p, mask, _ in cls.__sparse_parameters:
            total += 1
            s, n = int(mask.sum()), mask.numel()
            if s == n:
                sp100 += 1
            elif s * 2 == n:
                sp50 += 1
        assert total == sp100 or total == sp50, "Inconsistent model sparsity"
        return total == sp50 and total > 0

    @classmethod
    def prune_trained_model(cls, model, optimizer):
        cls.init_model_for_pruning(model, mask_calculator="m4n2_1d", verbosity=2,
                                   whitelist=[torch.nn.Linear, torch.nn.Conv2d], allow_recompute_mask=False)
        cls.init_optimizer_for_pruning(optimizer)
        cls.compute_sparse_masks()

    @classmethod
    def _reset(cls):
        """Forget the registered model / optimizer (tests; the reference has no equivalent)."""
        cls.__model = None
        cls.__optimizer = None
        cls.__sparse_parameters = []
        cls.__calculate_mask = None
