"""Version helpers kept for API parity (reference apex/amp/compat.py)."""
import torch


def variable_is_tensor():
    return True


def tensor_is_variable():
    return True


def tensor_is_float_tensor():
    return torch.is_floating_point(torch.zeros(1))


def is_tensor_like(x):
    return torch.is_tensor(x)


def is_floating_point(x):
    return torch.is_floating_point(x)


def scalar_python_val(x):
    if hasattr(x, "item"):
        return x.item()
    return x


def filter_attrs(module, attrs):
    return [a for a in attrs if hasattr(module, a)]
