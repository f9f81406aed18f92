"""Cast helpers for O1/O4 (reference apex/amp/utils.py:14-227)."""
import torch


def is_cuda_enabled():
    return torch.version.cuda is not None or torch.version.hip is not None


def get_cuda_version():
    return tuple(int(x) for x in (torch.version.hip or "0.0.0").split(".")[:3] if x.isdigit())


def is_fp_tensor(x):
    return isinstance(x, torch.Tensor) and x.is_floating_point()


def is_nested(x):
    return isinstance(x, (tuple, list))


def should_cache(x):
    # leaf parameters (weights) are cast once per iteration
    return isinstance(x, torch.Tensor) and x.is_leaf and x.requires_grad and x.is_floating_point()


def collect_fp_tensor_types(args, kwargs):
    types = set()

    def visit(a):
        if isinstance(a, torch.Tensor) and a.is_floating_point():
            types.add(a.dtype)
        elif isinstance(a, (list, tuple)):
            for y in a:
                visit(y)

    for a in args:
        visit(a)
    for a in kwargs.values():
        visit(a)
    return types


def type_string(x):
    return x.type().split(".")[-1]


def maybe_half(x, name="", verbose=False):
    if is_nested(x):
        return type(x)([maybe_half(y) for y in x])
    if not is_fp_tensor(x) or x.dtype == torch.half:
        return x
    if verbose:
        print("Float->Half ({})".format(name))
    return x.half()


def maybe_bfloat16(x, name="", verbose=False):
    if is_nested(x):
        return type(x)([maybe_bfloat16(y) for y in x])
    if not is_fp_tensor(x) or x.dtype == torch.bfloat16:
        return x
    if verbose:
        print("Float->BFloat16 ({})".format(name))
    return x.bfloat16()


def maybe_float(x, name="", verbose=False):
    if is_nested(x):
        return type(x)([maybe_float(y) for y in x])
    if not is_fp_tensor(x) or x.dtype == torch.float32:
        return x
    if verbose:
        print("Half->Float ({})".format(name))
    return x.float()


def cached_cast(cast_fn, x, cache):
    """Cast with a per-iteration cache for leaf weights (reference apex/amp/utils.py:101-133).

    The cache key is the parameter object; an entry is reused only while the parameter has not
    been modified in place (``_version``) and grad mode agrees, so an optimizer step or a
    ``no_grad`` eval pass never sees a stale or graph-less copy."""
    if is_nested(x):
        return type(x)([cached_cast(cast_fn, y, cache) for y in x])
    if not is_fp_tensor(x):
        return x
    if should_cache(x):
        ent = cache.get(id(x))
        grad_on = torch.is_grad_enabled()
        if ent is not None:
            src, ver, gmode, casted = ent
            if src is x and ver == x._version and gmode == grad_on:
                return casted
        casted = cast_fn(x)
        cache[id(x)] = (x, x._version, grad_on, casted)
        return casted
    return cast_fn(x)


def casted_args(cast_fn, args, kwargs):
    new_args = [cast_fn(a) if (is_fp_tensor(a) or is_nested(a)) else a for a in args]
    new_kwargs = {k: (cast_fn(v) if (is_fp_tensor(v) or is_nested(v)) else v) for k, v in kwargs.items()}
    return new_args, new_kwargs


def verbosify(cast_fn, fn_name, verbose):
    if verbose:
        return lambda x: cast_fn(x, fn_name, verbose)
    return cast_fn


def as_inplace(fns):
    for x in fns:
        yield x + "_"


def has_func(mod, fn):
    if isinstance(mod, dict):
        return fn in mod
    return hasattr(mod, fn)


def get_func(mod, fn):
    if isinstance(mod, dict):
        return mod[fn]
    return getattr(mod, fn)


def set_func(mod, fn, new_fn):
    if isinstance(mod, dict):
        mod[fn] = new_fn
    else:
        setattr(mod, fn, new_fn)


def set_func_save(handle, mod, fn, new_fn):
    cur_fn = get_func(mod, fn)
    handle._save_func(mod, fn, cur_fn)
    set_func(mod, fn, new_fn)
