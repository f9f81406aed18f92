"""Op-level markers for rocprofv3 (reference apex/pyprof/nvtx/nvmarker.py:1-222).

``init()`` monkey-patches ``torch.*``, ``torch.Tensor.*``, ``torch.nn.functional.*`` and the
``forward`` of every ``torch.nn`` module class so each call pushes a ROCTX range (the ROCm
build of ``torch.cuda.nvtx`` emits roctx, which ``rocprofv3 --marker-trace`` records) whose
text is a python-literal dict: ``{'mod': ..., 'op': ..., 'args': [...], 'traceMarker': [...]}``
with the shapes / dtypes / scalar values of the arguments.  ``apex.pyprof.parse`` attaches the
innermost enclosing marker to every kernel and ``apex.pyprof.prof`` turns the argument shapes
into FLOP / byte counts.  Without roctx (CPU builds) the ranges go to
``torch.autograd.profiler.record_function`` instead."""
import functools
import inspect
import traceback

import torch

try:  # roctx on ROCm builds
    from torch.cuda import nvtx as _nvtx

    _nvtx.range_push("apex.pyprof probe")
    _nvtx.range_pop()
    _HAVE_MARKERS = True
except Exception:  # pragma: no cover - depends on the build
    _nvtx = None
    _HAVE_MARKERS = False

_SKIP = {"__all__", "__array__", "__array_priority__", "__array_wrap__", "__bool__", "__builtins__", "__cached__",
         "__class__", "__deepcopy__", "__delattr__", "__delitem__", "__dict__", "__dir__", "__doc__", "__file__",
         "__format__", "__getattribute__", "__getitem__", "__hash__", "__index__", "__init__", "__init_subclass__",
         "__iter__", "__len__", "__loader__", "__module__", "__name__", "__new__", "__nonzero__", "__package__",
         "__path__", "__reduce__", "__reduce_ex__", "__repr__", "__reversed__", "__setattr__", "__setitem__",
         "__setstate__", "__sizeof__", "__spec__", "__str__", "__subclasshook__", "__version__", "__weakref__",
         "size", "tolist", "dim", "is_storage", "item", "data_ptr", "stride", "numel", "element_size",
         "is_contiguous", "storage_offset", "__torch_function__", "type", "get_device"}

_depth = [0]
_wrapped = set()


def isfunc(mod, f):
    if not hasattr(mod, f):
        return False
    if len(f) >= 2 and f[0] == "_" and f[1] != "_":
        return False
    if f in _SKIP:
        return False
    attr = getattr(mod, f)
    return inspect.ismethod(attr) or inspect.isfunction(attr) or inspect.ismethoddescriptor(attr) or \
        inspect.isbuiltin(attr)


def describe(x, name=""):
    if isinstance(x, torch.Tensor):
        return {"name": name, "type": "tensor", "shape": tuple(x.shape), "dtype": str(x.dtype).split(".")[-1]}
    if isinstance(x, (int, float, bool)):
        return {"name": name, "type": type(x).__name__, "value": x}
    if isinstance(x, (list, tuple)):
        return {"name": name, "type": type(x).__name__, "value": [describe(e) for e in x]}
    if x is None:
        return {"name": name, "type": "NoneType", "value": None}
    if isinstance(x, torch.dtype):
        return {"name": name, "type": "dtype", "value": str(x).split(".")[-1]}
    return {"name": name, "type": type(x).__name__}


def _push(text):
    if _HAVE_MARKERS:
        _nvtx.range_push(text)
        return None
    rf = torch.autograd.profiler.record_function(text[:200])
    rf.__enter__()
    return rf


def _pop(handle):
    if handle is not None:
        handle.__exit__(None, None, None)
    elif _HAVE_MARKERS:
        _nvtx.range_pop()


def add_wrapper(mod, fn_name):
    """Wrap ``mod.fn_name`` so each call is one marker range carrying its argument description."""
    key = (id(mod), fn_name)
    if key in _wrapped:
        return
    func = getattr(mod, fn_name)
    mod_name = getattr(mod, "__name__", type(mod).__name__)

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        if _depth[0] > 0:  # only the outermost torch call of a nest is annotated
            return func(*args, **kwargs)
        stack = traceback.extract_stack()[:-1]
        trace = ["{}:{}".format(f.filename, f.lineno) for f in stack[-4:]]
        desc = {"mod": mod_name, "op": fn_name, "args": [describe(a) for a in args] +
                [describe(v, k) for k, v in kwargs.items()], "traceMarker": trace}
        if fn_name == "forward" and args and hasattr(args[0], "extra_repr"):
            desc["strRepr"] = args[0].extra_repr()
            desc["args"] = desc["args"][1:]
        h = _push(str(desc))
        _depth[0] += 1
        try:
            return func(*args, **kwargs)
        finally:
            _depth[0] -= 1
            _pop(h)

    setattr(mod, fn_name, wrapper)
    _wrapped.add(key)


def init():
    """Patch torch / Tensor / functional / nn module forwards (idempotent)."""
    for mod in (torch, torch.Tensor, torch.nn.functional):
        for f in dir(mod):
            if isfunc(mod, f):
                try:
                    add_wrapper(mod, f)
                except (TypeError, AttributeError):
                    pass
    for name in dir(torch.nn):
        cls = getattr(torch.nn, name)
        if inspect.isclass(cls) and issubclass(cls, torch.nn.Module) and "forward" in cls.__dict__:
            add_wrapper(cls, "forward")
