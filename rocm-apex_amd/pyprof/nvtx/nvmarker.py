"""Op-level markers for rocprofv3 (reference apex/pyprof/nvtx/nvmarker.py:1-222).

``init()`` monkey-patches ``torch.*``, ``torch.Tensor.*``, ``torch.nn.functional.*`` and the
``forward`` of every ``torch.nn`` module class so each call pushes a ROCTX range (the ROCm
build of ``torch.cuda.nvtx`` emits roctx, which ``rocprofv3 --marker-trace`` records) whose
text is a python-literal dict::

    {'mod': 'torch.nn.functional', 'op': 'linear', 'dir': 'fprop', 'seqId': 17,
     'args': [{'name': '', 'type': 'tensor', 'shape': (64, 128), 'dtype': 'bfloat16'}, ...],
     'traceMarker': ['train.py:42', ...]}

Backward attribution (the reference leans on PyTorch's autograd ``seq=`` NVTX ranges and
matches sequence numbers afterwards, prof.py:171-256): here the wrapper registers a pre-hook and
a post-hook on the ``grad_fn`` of the op's outputs, so the backward node runs inside a range
with the SAME description, ``'dir': 'bprop'`` and the same ``seqId``.  The kernels the autograd
thread launches for it are therefore attributed directly, with no sequence matching.

``layer(name)`` (context manager / decorator) pushes ``layer:<name>`` ranges and records the
layer path in every op marker opened inside it, so backward kernels (which run outside the
user's ``with`` block) still report the layer of their forward op (reference "layer" column).  ``wrap(mod, fn)``
annotates a user function the same way (reference ``pyprof.nvtx.wrap``).  Without roctx (CPU
builds) the ranges go to ``torch.autograd.profiler.record_function`` instead."""
import contextlib
import functools
import inspect
import itertools
import threading
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
         "is_contiguous", "storage_offset", "__torch_function__", "type", "get_device", "register_hook",
         "requires_grad_", "backward", "register_post_accumulate_grad_hook"}

_grad_enabled = torch.is_grad_enabled  # captured before init() patches torch.*
_local = threading.local()
_seq = itertools.count(1)
_wrapped = set()
BACKWARD_MARKERS = True


def _depth():
    return getattr(_local, "depth", 0)


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
    """Argument description carried in the marker (shapes, dtypes, scalar values)."""
    if isinstance(x, torch.Tensor):
        return {"name": name, "type": "tensor", "shape": tuple(x.shape), "dtype": str(x.dtype).split(".")[-1]}
    if isinstance(x, (bool, int, float)):
        return {"name": name, "type": type(x).__name__, "value": x}
    if isinstance(x, str):
        return {"name": name, "type": "str", "value": x}
    if isinstance(x, (list, tuple, torch.Size)):
        return {"name": name, "type": "tuple" if isinstance(x, (tuple, torch.Size)) else "list",
                "value": [describe(e) for e in x]}
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


def _outputs(out):
    if isinstance(out, torch.Tensor):
        yield out
    elif isinstance(out, (list, tuple)):
        for o in out:
            yield from _outputs(o)


def _attach_backward(out, desc):
    """Bracket the backward node(s) that produce this op's input grads with a bprop range."""
    seen = set()
    text = str(dict(desc, dir="bprop"))
    for t in _outputs(out):
        fn = t.grad_fn if t.requires_grad else None
        if fn is None or id(fn) in seen:
            continue
        seen.add(id(fn))
        handles = []

        def pre(_grad_outputs, _handles=handles):
            _handles.append(_push(text))

        def post(_grad_inputs, _grad_outputs, _handles=handles):
            if _handles:
                _pop(_handles.pop())

        try:
            fn.register_prehook(pre)
            fn.register_hook(post)
        except (AttributeError, RuntimeError):  # pragma: no cover - exotic grad_fns
            pass


def add_wrapper(mod, fn_name):
    """Wrap ``mod.fn_name`` so each call is one marker range carrying its argument description
    (and, when its outputs require grad, a matching backward range)."""
    key = (id(mod), fn_name)
    if key in _wrapped:
        return
    func = getattr(mod, fn_name)
    mod_name = getattr(mod, "__name__", type(mod).__name__)

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        if _depth() > 0:  # only the outermost torch call of a nest is annotated
            return func(*args, **kwargs)
        stack = traceback.extract_stack()[:-1]
        trace = ["{}:{}".format(f.filename, f.lineno) for f in stack[-4:]]
        desc = {"mod": mod_name, "op": fn_name, "dir": "fprop", "seqId": next(_seq),
                "layer": list(getattr(_local, "layers", ())),
                "args": [describe(a) for a in args] + [describe(v, k) for k, v in kwargs.items()],
                "traceMarker": trace}
        if fn_name == "forward" and args and hasattr(args[0], "extra_repr"):
            desc["strRepr"] = args[0].extra_repr()
            desc["args"] = desc["args"][1:]
        h = _push(str(desc))
        _local.depth = _depth() + 1
        try:
            out = func(*args, **kwargs)
        finally:
            _local.depth -= 1
            _pop(h)
        if BACKWARD_MARKERS and _grad_enabled():
            _attach_backward(out, desc)
        return out

    setattr(mod, fn_name, wrapper)
    _wrapped.add(key)


def wrap(mod, fn_name):
    """Annotate a user function / custom module function (reference ``pyprof.nvtx.wrap``)."""
    add_wrapper(mod, fn_name)


class layer(contextlib.ContextDecorator):
    """``with layer("encoder.3"):`` or ``@layer("attn")``: a user annotation that the parse
    stage reports as the kernel's layer path."""

    def __init__(self, name):
        self.name = name
        self._h = None

    def __enter__(self):
        self._h = _push("layer:" + str(self.name))
        _local.layers = getattr(_local, "layers", ()) + (str(self.name),)
        return self

    def __exit__(self, *exc):
        _local.layers = getattr(_local, "layers", ())[:-1]
        _pop(self._h)
        return False


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
    # this package's multi-tensor entry points (fused optimizers, amp unscale, norms): their
    # markers carry the tensor lists, which the optim models price
    from ... import amp_C

    for name in getattr(amp_C, "__all__", []):
        if name.startswith("multi_tensor"):
            add_wrapper(amp_C, name)
