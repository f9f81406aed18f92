"""Generic parameter reparameterization via forward pre-hooks
(reference apex/reparameterization/reparameterization.py:4-151)."""
import torch
from torch.nn.parameter import Parameter


class Reparameterization(object):
    """Hook object: recomputes ``module.<name>`` from its reparameterization parameters before
    forward.  Subclasses implement ``reparameterize`` (create the new parameters) and
    ``compute_weight`` (rebuild the weight).  The weight is rebuilt on every forward while
    autograd is recording (each backward needs its own graph) and cached otherwise."""

    def __init__(self, name, dim, module, retain_forward=True):
        self.name = name
        self.dim = dim
        self.evaluated = False
        self.retain_forward = retain_forward
        self.reparameterization_names = []
        self.module = module

    def compute_weight(self, module=None, name=None):
        raise NotImplementedError

    def reparameterize(self, name, weight, dim):
        raise NotImplementedError

    @staticmethod
    def apply(module, name, dim, reparameterization=None, hook_child=True):
        reparameterization = reparameterization or Reparameterization
        module2use, name2use = Reparameterization.get_module_and_name(module, name)
        if name2use is None or isinstance(module2use, (torch.nn.Embedding, torch.nn.EmbeddingBag)):
            return None
        weight = getattr(module2use, name2use)
        if weight is None or weight.dim() <= 1:
            return None
        fn = reparameterization(name2use, dim, module2use) if hook_child else reparameterization(name, dim, module)
        del module2use._parameters[name2use]
        names, params = fn.reparameterize(name2use, weight, dim)
        for n, p in zip(names, params):
            module2use.register_parameter(n, p)
        fn.reparameterization_names = names
        setattr(module2use, name2use, None)
        (module2use if hook_child else module).register_forward_pre_hook(fn)
        return fn

    @staticmethod
    def get_module_and_name(module, name):
        parts = name.split(".")
        if len(parts) == 1 and parts[0] != "":
            return module, parts[0]
        if len(parts) > 1:
            m = module
            for p in parts[:-1]:
                m = getattr(m, p)
            return m, parts[-1]
        return None, None

    def get_params(self, module):
        return [getattr(module, n) for n in self.reparameterization_names]

    def remove(self, module):
        """Fold the reparameterization back into a plain parameter (forward hook removed by caller)."""
        module2use, name2use = Reparameterization.get_module_and_name(module, self.name)
        for p in self.get_params(module2use):
            p.requires_grad = False
        weight = self.compute_weight(module2use, name2use)
        delattr(module2use, name2use)
        for n in self.reparameterization_names:
            del module2use._parameters[n]
        module2use.register_parameter(name2use, Parameter(weight.data))

    def __call__(self, module, inputs):
        module2use, name2use = Reparameterization.get_module_and_name(module, self.name)
        w = getattr(module2use, name2use)
        if not self.evaluated or w is None or torch.is_grad_enabled():
            setattr(module2use, name2use, self.compute_weight(module2use, name2use))
            self.evaluated = not torch.is_grad_enabled()
