"""Data-parallel gradient reduction (reference apex/parallel/distributed.py:36-640).

MI355X design (not a port of the reference's flatten / side-stream / unflatten pattern):

* **Persistent flat buckets.**  Parameters are grouped by dtype into contiguous bucket tensors of
  at least ``message_size`` elements (default 1e7 = 20 MB bf16: a few large collectives, which
  is what a ring over point-to-point xGMI links wants).  After a gradient is accumulated, its
  ``.grad`` is re-pointed at its slot of the bucket (``as_strided`` with the param's own strides,
  so channels_last weights keep their layout) — from then on autograd accumulates straight into
  the bucket and there is no flatten/unflatten copy.  A freshly created grad (first use, or after
  ``zero_grad(set_to_none=True)`` / amp resetting it) is copied into its slot once.
* **Overlap via RCCL's own stream.**  A full bucket is all-reduced with ``async_op=True``: the
  process group's HIP stream waits on the producing (compute) stream with an event and runs
  while backward continues; the end-of-backward callback only makes the compute stream wait on
  the outstanding works.  Buckets are issued in a fixed order on every rank (required for
  matching collectives); out-of-order readiness is held back until predecessors fire.
* **Averaging in the collective** with ``ReduceOp.AVG`` (ncclAvg) when no predivide factor is
  requested; otherwise pre/post scaling as in the reference.
* **Zero-copy under amp.**  A DDP-owned parameter carries a weak back-reference to its DDP; amp's
  ``zero_grad`` / post-``step`` reset call :func:`zero_bucketed_grads`, which zeroes each bucket
  with ONE memset and re-attaches every gradient as its bucket view (instead of setting grads to
  None), so the next backward accumulates straight into the buckets: no per-parameter copy and no
  allocation per step.  Buckets already known to be zero are not cleared twice.
* Bucket membership defaults to reverse registration order (a good proxy for backward order,
  identical on every rank with no communication); after the first iteration it is re-derived
  from rank 0's observed gradient-arrival order, broadcast to all ranks (reference behaviour,
  :284-317).
"""
import warnings
import weakref

import torch
import torch.distributed as dist
from torch.nn.modules import Module

from . import comm_timing


def _world(group=None):
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _supports_avg(group=None):
    try:
        return dist.get_backend(group) == "nccl" and hasattr(dist.ReduceOp, "AVG")
    except Exception:
        return False


def flatten(bucket):
    return torch._utils._flatten_dense_tensors(bucket)


def unflatten(coalesced, bucket):
    return torch._utils._unflatten_dense_tensors(coalesced, bucket)


def split_by_type(tensors):
    buckets = {}
    for t in tensors:
        buckets.setdefault(t.dtype, []).append(t)
    return buckets


def apply_flat_dist_call(bucket, call, extra_args=None):
    """Flatten ``bucket``, run ``call`` on it, copy results back (reference :36-49)."""
    coalesced = flatten(bucket)
    if extra_args is not None:
        call(coalesced, *extra_args)
    else:
        call(coalesced)
    if call is dist.all_reduce:
        coalesced /= _world()
    for buf, synced in zip(bucket, unflatten(coalesced, bucket)):
        buf.copy_(synced)


def flat_dist_call(tensors, call, extra_args=None):
    for tensors_of_type in split_by_type(tensors).values():
        apply_flat_dist_call(tensors_of_type, call, extra_args)


def extract_tensors(maybe_tensor, tensor_list):
    if torch.is_tensor(maybe_tensor):
        tensor_list.append(maybe_tensor)
    else:
        try:
            for item in maybe_tensor:
                extract_tensors(item, tensor_list)
        except TypeError:
            return


class Reducer(object):
    """Manual all-reduce helper (reference :89-126): syncs params at construction (module form)
    and averages gradients across ranks when ``reduce()`` is called."""

    def __init__(self, module_or_grads_list):
        if isinstance(module_or_grads_list, Module):
            self.module = module_or_grads_list
            flat_dist_call([p.data for p in self.module.parameters()], dist.broadcast, (0,))
        else:
            self.module = None
            self.grads = []
            extract_tensors(module_or_grads_list, self.grads)

    def reduce(self):
        if self.module:
            grads = [p.grad.data for p in self.module.parameters() if p.grad is not None]
            flat_dist_call(grads, dist.all_reduce)
        else:
            flat_dist_call(self.grads, dist.all_reduce)


def _owner(param):
    ref = getattr(param, "_apex_ddp_owner", None)
    return ref() if ref is not None else None


def zero_bucketed_grads(params):
    """Zero the gradients of the DDP-owned ``params`` in place (views re-attached); returns the
    set of ``id(param)`` handled — the caller resets the others.

    Only the gradients of ``params`` are touched: a bucket is cleared with one memset when every
    parameter in it belongs to ``params``, otherwise just the views of the listed parameters are
    zeroed, so a second optimizer over the same DDP model keeps its not-yet-consumed gradients."""
    done, owners = set(), {}
    for p in params:
        d = _owner(p)
        if d is not None:
            owners.setdefault(id(d), (d, set()))[1].add(id(p))
            done.add(id(p))
    for d, ids in owners.values():
        d.zero_grad_buckets(ids)
    return done


def zeroed_bucket_params(params):
    """``id(param)`` of the DDP-owned ``params`` whose gradient is a bucket view known to be zero."""
    out = set()
    for p in params:
        d = _owner(p)
        if d is not None and p.grad is not None:
            b, i = d._slot[id(p)]
            known_zero = b.zeroed or id(p) in b.zeroed_ids
            if known_zero and p.grad.data_ptr() == b.buffer.data_ptr() + b.offsets[i] * b.buffer.element_size():
                out.add(id(p))
    return out


class _Bucket(object):
    __slots__ = ("index", "params", "offsets", "numel", "dtype", "buffer", "fp32_buffer", "ready", "fired",
                 "work", "group", "zeroed", "zeroed_ids")

    def __init__(self, index, params, dtype, device, group, fp32_copy):
        self.index = index
        self.params = params
        self.dtype = dtype
        self.offsets = []
        n = 0
        for p in params:
            self.offsets.append(n)
            n += p.numel()
        self.numel = n
        self.buffer = torch.zeros(n, dtype=dtype, device=device)
        self.fp32_buffer = torch.zeros(n, dtype=torch.float32, device=device) if (
            fp32_copy and dtype != torch.float32) else None
        self.ready = 0
        self.fired = False
        self.work = None
        self.group = group
        self.zeroed = True
        self.zeroed_ids = set()  # params zeroed one by one since the bucket was last written

    def dirty(self):
        self.zeroed = False
        self.zeroed_ids.clear()

    def view_for(self, i):
        p = self.params[i]
        return torch.as_strided(self.buffer, p.size(), p.stride(), self.offsets[i])


class DistributedDataParallel(Module):
    """Wraps ``module``; broadcasts its parameters from rank 0 at construction and averages
    gradients across ranks during ``backward()``, overlapped with the backward computation.

    Arguments follow the reference (message_size, delay_allreduce, allreduce_trigger_params,
    retain_allreduce_buffers, allreduce_always_fp32, num_allreduce_streams,
    allreduce_communicators, gradient_average, gradient_predivide_factor, prof)."""

    def __init__(self, module, message_size=10000000, delay_allreduce=False, shared_param=None,
                 allreduce_trigger_params=None, retain_allreduce_buffers=False, allreduce_always_fp32=False,
                 num_allreduce_streams=1, allreduce_communicators=None, gradient_average=True,
                 gradient_predivide_factor=1.0, gradient_average_split_factor=None, prof=False,
                 rebucket_by_arrival=True, process_group=None):
        super(DistributedDataParallel, self).__init__()
        if shared_param is not None:
            raise ValueError("shared_param is no longer supported as an option.  Overlapping communication with "
                             "computation works fine with shared parameters; use delay_allreduce to delay it.")
        if gradient_average_split_factor is not None:
            warnings.warn("gradient_average_split_factor has been renamed to gradient_predivide_factor.")
            gradient_predivide_factor = gradient_average_split_factor
        self.module = module
        self.process_group = process_group
        self._backend = dist.get_backend(process_group)
        self.prof = prof
        self.num_allreduce_streams = num_allreduce_streams
        self.allreduce_different_streams = num_allreduce_streams > 1
        if self.allreduce_different_streams and delay_allreduce:
            raise ValueError("self.allreduce_different_streams may only be used if delay_allreduce=False.")
        self.world_size = float(_world(process_group))
        self.retain_allreduce_buffers = retain_allreduce_buffers
        self.allreduce_always_fp32 = allreduce_always_fp32
        self.gradient_average = gradient_average
        self.gradient_predivide_factor = gradient_predivide_factor
        self.custom_allreduce_triggers = allreduce_trigger_params is not None
        if self.custom_allreduce_triggers:
            if delay_allreduce:
                raise ValueError("Setting allreduce_trigger_params is only valid if delay_allreduce=False.")
            self.allreduce_trigger_params = set(id(p) for p in allreduce_trigger_params)
        self.delay_allreduce = delay_allreduce
        self.message_size = int(message_size)
        self.rebucket_by_arrival = rebucket_by_arrival and not self.custom_allreduce_triggers
        self._disable_allreduce = False
        if self._backend == "gloo":
            for p in module.parameters():
                if p.dtype in (torch.float16, torch.bfloat16):
                    warnings.warn("DDP with the gloo backend reduces half-precision gradients on the CPU path; "
                                  "use the nccl (RCCL) backend on GPUs.")
                    break
        if self._backend == "nccl":
            for p in module.parameters():
                assert p.is_cuda, "NCCL backend only supports model parameters to be on GPU."

        if allreduce_communicators is not None:
            self._groups = list(allreduce_communicators[0])
        elif self.allreduce_different_streams:
            self._groups = [dist.new_group(ranks=list(range(int(self.world_size))))
                            for _ in range(num_allreduce_streams)]
        else:
            self._groups = [process_group]

        self._params = [p for p in module.parameters() if p.requires_grad]
        self._param_index = {id(p): i for i, p in enumerate(self._params)}
        self._arrival = []
        self._iteration = 0
        self._hooks = []
        self._callback_queued = False
        self._sync_enabled = True
        self.grad_copies = 0  # grads that arrived outside their bucket and were copied in
        self._build_buckets(list(reversed(range(len(self._params)))))
        self._create_hooks()
        me = weakref.ref(self)
        for p in self._params:
            p._apex_ddp_owner = me
        flat_dist_call([p.data for p in module.parameters()], dist.broadcast, (0,))

    # ------------------------------------------------------------------------------ buckets
    def _build_buckets(self, order):
        self._buckets = []
        self._slot = {}
        cur = {}
        for idx in order:
            p = self._params[idx]
            lst = cur.setdefault(p.dtype, [])
            lst.append(p)
            trigger = (self.custom_allreduce_triggers and id(p) in self.allreduce_trigger_params)
            if trigger or (not self.custom_allreduce_triggers and sum(x.numel() for x in lst) >= self.message_size):
                self._emit_bucket(lst)
                cur[p.dtype] = []
        for lst in cur.values():
            if lst:
                self._emit_bucket(lst)

    def _emit_bucket(self, params):
        dev = params[0].device
        b = _Bucket(len(self._buckets), list(params), params[0].dtype, dev,
                    self._groups[len(self._buckets) % len(self._groups)], self.allreduce_always_fp32)
        for i, p in enumerate(params):
            self._slot[id(p)] = (b, i)
        self._buckets.append(b)

    def _rebucket_from_arrival(self):
        """Re-derive bucket membership from rank 0's gradient arrival order (reference :284-317)."""
        order = [self._param_index[pid] for pid in self._arrival if pid in self._param_index]
        seen = set(order)
        order += [i for i in reversed(range(len(self._params))) if i not in seen]
        t = torch.tensor(order, dtype=torch.int64,
                         device=self._params[0].device if self._backend == "nccl" else "cpu")
        dist.broadcast(t, 0, group=self.process_group)
        old = {id(p): (b, i) for b in self._buckets for i, p in enumerate(b.params)}
        self._build_buckets(t.tolist())
        # move existing grads into the new bucket storage
        for p in self._params:
            if p.grad is not None and id(p) in old:
                b, i = self._slot[id(p)]
                v = b.view_for(i)
                v.copy_(p.grad)
                p.grad = v
                b.dirty()

    # ------------------------------------------------------------------------------ hooks
    def _create_hooks(self):
        for p in self._params:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(p)))

    def _make_hook(self, p):
        pid = id(p)

        def hook(param):
            if self._disable_allreduce or not self._sync_enabled:
                return
            if not self._callback_queued:
                torch.autograd.Variable._execution_engine.queue_callback(self._epilogue)
                self._callback_queued = True
            if self._iteration == 0 and self.rebucket_by_arrival:
                self._arrival.append(pid)
            b, i = self._slot[pid]
            b.dirty()
            g = param.grad
            if g.data_ptr() != b.buffer.data_ptr() + b.offsets[i] * b.buffer.element_size():
                # a freshly allocated grad (first iteration, or grads reset to None): one copy
                v = b.view_for(i)
                v.copy_(g)
                param.grad = v
                self.grad_copies += 1
            b.ready += 1
            if self.delay_allreduce or (self._iteration == 0 and self.rebucket_by_arrival):
                return
            if b.ready == len(b.params):
                self._fire_ready_in_order()

        return hook

    def _fire_ready_in_order(self):
        for b in self._buckets:
            if b.fired:
                continue
            if b.ready < len(b.params):
                break
            self._allreduce_bucket(b)

    def _allreduce_bucket(self, b):
        b.fired = True
        buf = b.buffer
        if b.fp32_buffer is not None:
            b.fp32_buffer.copy_(buf)
            buf = b.fp32_buffer
        ws = _world(b.group)
        if self.gradient_predivide_factor != 1.0:
            buf.mul_(1.0 / self.gradient_predivide_factor)
        if self.gradient_average and self.gradient_predivide_factor == 1.0 and _supports_avg(b.group):
            b.work = dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=b.group, async_op=True)
            b.work = (b.work, None)
        else:
            w = dist.all_reduce(buf, group=b.group, async_op=True)
            post = (self.gradient_predivide_factor / ws) if self.gradient_average else None
            b.work = (w, post)

    def _finish_bucket(self, b):
        w, post = b.work
        w.wait()
        buf = b.fp32_buffer if b.fp32_buffer is not None else b.buffer
        if post is not None and post != 1.0:
            buf.mul_(post)
        if b.fp32_buffer is not None:
            b.buffer.copy_(b.fp32_buffer)
        b.work = None

    def _epilogue(self):
        self._callback_queued = False
        try:
            if self._iteration == 0 and self.rebucket_by_arrival and _world(self.process_group) > 1:
                self._rebucket_from_arrival()
                for b in self._buckets:
                    b.ready = sum(1 for p in b.params if p.grad is not None)
            # params that got no gradient on this rank: contribute zeros so every rank joins
            for b in self._buckets:
                if b.ready < len(b.params):
                    for i, p in enumerate(b.params):
                        v = b.view_for(i)
                        if p.grad is None:
                            v.zero_()
                            p.grad = v
                            b.dirty()
                        elif p.grad.data_ptr() != v.data_ptr():
                            v.copy_(p.grad)
                            p.grad = v
                    b.ready = len(b.params)
            # exposed communication: from here (every backward kernel is enqueued) to the last
            # bucket's completion on the compute stream (parallel.comm_timing, bench JSON)
            with comm_timing.span("allreduce_exposed", self._buckets[0].buffer.device if self._buckets else None):
                for b in self._buckets:
                    if not b.fired:
                        self._allreduce_bucket(b)
                for b in self._buckets:
                    if b.work is not None:
                        self._finish_bucket(b)
        finally:
            for b in self._buckets:
                b.ready = 0
                b.fired = False
            self._iteration += 1

    # ------------------------------------------------------------------------------ API
    def zero_grad_buckets(self, only=None):
        """Zero the buckets (one memset each, skipped when already zero) and attach each
        parameter's gradient as its bucket view, so backward accumulates in place.

        ``only``: a set of ``id(param)``; a bucket holding parameters outside it is not cleared
        as a whole — only the listed parameters' views are zeroed (and re-attached)."""
        for b in self._buckets:
            whole = only is None or all(id(p) in only for p in b.params)
            if whole:
                if not b.zeroed:
                    b.buffer.zero_()
                    b.zeroed = True
                b.zeroed_ids.clear()
            for i, p in enumerate(b.params):
                if not whole and id(p) not in only:
                    continue
                g = p.grad
                attached = g is not None and g.data_ptr() == b.buffer.data_ptr() + b.offsets[i] * b.buffer.element_size()
                if not attached:
                    p.grad = b.view_for(i)
                if not whole and not b.zeroed and id(p) not in b.zeroed_ids:
                    p.grad.zero_()
                    b.zeroed_ids.add(id(p))

    def forward(self, *inputs, **kwargs):
        if self.prof:
            torch.cuda.nvtx.range_push("forward pass DDP logic")
        out = self.module(*inputs, **kwargs)
        if self.prof:
            torch.cuda.nvtx.range_pop()
        return out

    def disable_allreduce(self):
        self._disable_allreduce = True

    def enable_allreduce(self):
        self._disable_allreduce = False

    class _NoSync(object):
        def __init__(self, ddp):
            self.ddp = ddp

        def __enter__(self):
            self.prev = self.ddp._sync_enabled
            self.ddp._sync_enabled = False

        def __exit__(self, *a):
            self.ddp._sync_enabled = self.prev

    def no_sync(self):
        """Context manager: accumulate gradients locally without all-reducing them."""
        return DistributedDataParallel._NoSync(self)

    @property
    def buckets(self):
        return [[self._param_index[id(p)] for p in b.params] for b in self._buckets]

    def __setstate__(self, state):
        super(DistributedDataParallel, self).__setstate__(state)

    def __getstate__(self):
        attrs = dict(self.__dict__)
        for k in ("_hooks", "_buckets", "_slot", "_groups"):
            attrs.pop(k, None)
        return attrs
