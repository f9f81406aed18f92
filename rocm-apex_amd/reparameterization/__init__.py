"""Weight reparameterizations (reference apex/reparameterization/__init__.py:4-127)."""
from .reparameterization import Reparameterization
from .weight_norm import WeightNorm


def apply_weight_norm(module, name="", dim=0, hook_child=True):
    """Replace ``name`` (or every >1-D parameter when empty) by ``<name>_g`` / ``<name>_v``."""
    return apply_reparameterization(module, reparameterization=WeightNorm, hook_child=hook_child, name=name, dim=dim)


def remove_weight_norm(module, name="", remove_all=False):
    return remove_reparameterization(module, reparameterization=WeightNorm, name=name, remove_all=remove_all)


def apply_reparameterization(module, reparameterization=None, name="", dim=0, hook_child=True):
    assert reparameterization is not None
    if name != "":
        Reparameterization.apply(module, name, dim, reparameterization, hook_child)
    else:
        for n in list(module.state_dict().keys()):
            apply_reparameterization(module, reparameterization, n, dim, hook_child)
    return module


def remove_reparameterization(module, reparameterization=Reparameterization, name="", remove_all=False):
    if name != "" or remove_all:
        to_remove = [k for k, hook in module._forward_pre_hooks.items()
                     if isinstance(hook, reparameterization) and (hook.name == name or remove_all)]
        for k in to_remove:
            module._forward_pre_hooks[k].remove(module)
            del module._forward_pre_hooks[k]
        if to_remove or remove_all:
            return module
        raise ValueError("reparameterization of '{}' not found in {}".format(name, module))
    for m in [module] + list(module.modules()):
        remove_reparameterization(m, reparameterization=reparameterization, remove_all=True)
    return module


__all__ = ["Reparameterization", "WeightNorm", "apply_weight_norm", "remove_weight_norm",
           "apply_reparameterization", "remove_reparameterization"]
