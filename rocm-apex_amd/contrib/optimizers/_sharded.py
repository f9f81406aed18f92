"""Flat, sharded parameter / gradient storage shared by DistributedFusedAdam and
DistributedFusedLAMB (ZeRO-2 style).

Reference: apex/contrib/optimizers/distributed_fused_adam.py:128-371 (flat fp16 grad buffer split
[block x chunk x shard], per-param hooks copying grads in, reduce-scatter per block on
``dwu_num_rs_pg`` streams, inter-group all-reduce, all-gather of the updated params with the
NVIDIA-only ``no_copy=True`` kwarg).

MI355X design:
  * ONE contiguous model-dtype parameter buffer and ONE gradient buffer; every parameter's
    ``.data`` and ``.grad`` are views into them, so autograd accumulates straight into the
    buffer (no per-parameter copy hooks, no flatten/unflatten).  288 GB of HBM per GPU makes the
    extra full-size gradient buffer free.
  * the buffer is cut into ``num_blocks`` equal blocks in reverse registration order (the order
    gradients become ready in backward); each block is ``world`` equal shards.  When the last
    parameter of a block has its gradient (``register_post_accumulate_grad_hook``) the block is
    reduce-scattered on a side stream, overlapping the rest of backward.  Blocks are sized so a
    reduce-scatter moves >= a few MB per rank (RCCL over xGMI is per-link bound; small messages
    are latency bound).
  * each rank keeps fp32 master params and optimizer moments ONLY for its shards
    (``[num_blocks, shard]``), updates them with one fused multi-tensor launch that also writes
    the model-dtype copy in place, and the updated shards are all-gathered per block
    (``all_gather_into_tensor`` — stock RCCL, no ``no_copy`` extension).
  * optional fp8 all-gather compression (e5m2 as in the reference, or e4m3): the optimizer
    kernel's epilogue converts the updated fp32 master straight into this rank's slice of an
    fp8 gather buffer (gfx950 ``v_cvt_pk_bf8/fp8_f32``), the uint8 buffer is all-gathered in
    place, and one multi-tensor cast (``v_cvt_pk_f32_bf8/fp8``) expands every block into the
    model-dtype parameters — no torch casts, no staging copies.  Every rank (the owner
    included) ends up with the same dequantised weights.  Global grad-norm clipping and
    sync-free overflow handling (device skip flag + inverse scale consumed by the kernels).
  * two-level data parallelism (reference ``dwu_group_size``: shard within groups of G ranks,
    replicate across the world/G groups): each block is reduce-scattered inside the group, then
    this rank's shard is all-reduced across the groups over ``ar_group`` (the ranks holding the
    same shard index; reference :409-418).  Optional fp32 accumulation (``reduce_dtype``) and
    pre-division by the data-parallel size before the sum (``predivide``).
  * ``mode="ar"`` (reference v3): all-reduce the whole block, keep this rank's slice.
"""
import math

import torch
import torch.distributed as dist

from ... import amp_C

_ALIGN = 128  # elements; keeps every param / shard 16-byte aligned for the vector kernels


class FlatShardedBuffers:
    def __init__(self, params, process_group=None, num_blocks=4, min_block_elems=1 << 20, grad_dtype=None,
                 overlap_reductions=True, ar_group=None, reduce_dtype=None, predivide=False, mode="rs"):
        params = [p for p in params if p.requires_grad]
        assert params, "no trainable parameters"
        dtypes = {p.dtype for p in params}
        if len(dtypes) != 1:
            raise RuntimeError("Distributed fused optimizers need parameters of one dtype; got {}".format(dtypes))
        self.dtype = params[0].dtype
        self.grad_dtype = grad_dtype or self.dtype
        self.device = params[0].device
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.params = params
        self.overlap = overlap_reductions
        self._gloo = dist.is_initialized() and dist.get_backend(process_group) == "gloo"
        assert mode in ("rs", "ar"), mode
        self.mode = mode
        self.ar_pg = ar_group
        self.ar_world = dist.get_world_size(ar_group) if (ar_group is not None and dist.is_initialized()) else 1
        self.dp_size = self.world * self.ar_world  # ranks whose gradients are averaged
        self.reduce_dtype = reduce_dtype or self.grad_dtype
        self.predivide = bool(predivide)

        # layout: reverse order (gradients arrive roughly last-layer-first)
        order = list(reversed(range(len(params))))
        offsets = [0] * len(params)
        cur = 0
        for i in order:
            offsets[i] = cur
            cur += int(math.ceil(params[i].numel() / _ALIGN)) * _ALIGN
        used = cur
        unit = self.world * _ALIGN
        nb = max(1, min(num_blocks, int(math.ceil(used / max(min_block_elems, unit)))))
        block = int(math.ceil(used / (nb * unit))) * unit
        self.num_blocks = nb
        self.block = block
        self.shard = block // self.world
        self.total = nb * block
        self.offsets = offsets

        self.flat_param = torch.zeros(self.total, dtype=self.dtype, device=self.device)
        self.flat_grad = torch.zeros(self.total, dtype=self.grad_dtype, device=self.device)
        with torch.no_grad():
            for p, off in zip(params, offsets):
                n = p.numel()
                self.flat_param[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat_param[off:off + n].view_as(p)
        self.attach_grads()

        # parameters per block (a param belongs to every block it overlaps)
        self.block_params = [set() for _ in range(nb)]
        for i, (p, off) in enumerate(zip(params, offsets)):
            first, last = off // block, (off + max(p.numel(), 1) - 1) // block
            for b in range(first, last + 1):
                self.block_params[b].add(i)
        self.param_blocks = [[b for b in range(nb) if i in self.block_params[b]] for i in range(len(params))]

        # this rank's shards: [num_blocks, shard] fp32 masters + reduced-grad staging
        self.shard_grad = torch.zeros(nb, self.shard, dtype=self.reduce_dtype, device=self.device)
        self.master = torch.empty(nb, self.shard, dtype=torch.float32, device=self.device)
        with torch.no_grad():
            for b in range(nb):
                self.master[b].copy_(self.param_shard(b).float())

        self._pending = [len(s) for s in self.block_params]
        self._ready = [0] * nb
        self._handles = [None] * nb
        self._fired = [False] * len(params)
        self._dirty = set()
        self._stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        self.is_accumulation_step = False
        self.generation = 0  # bumped whenever a reduction (re)writes shard_grad
        self._hooks = []
        if overlap_reductions:
            for i, p in enumerate(params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))

    # ---- views ----
    def attach_grads(self):
        for p, off in zip(self.params, self.offsets):
            n = p.numel()
            p.grad = self.flat_grad[off:off + n].view_as(p)

    def _adopt_grad(self, i):
        """Put a gradient autograd allocated outside the flat buffer (after a user
        ``zero_grad(set_to_none=True)``) back into the buffer."""
        p, off = self.params[i], self.offsets[i]
        view = self.flat_grad[off:off + p.numel()]
        g = p.grad
        if g is not None and g.data_ptr() != view.data_ptr():
            view.copy_(g.reshape(-1))
            p.grad = view.view_as(p)

    def block_view(self, buf, b):
        return buf[b * self.block:(b + 1) * self.block]

    def param_shard(self, b, rank=None):
        r = self.rank if rank is None else rank
        s = b * self.block + r * self.shard
        return self.flat_param[s:s + self.shard]

    # ---- compressed all-gather payload ----
    def payload(self, dtype):
        """fp8 gather buffer laid out like ``flat_param`` (allocated on first use, with this rank's
        shards already holding its current master weights: see ``refresh_payload``)."""
        buf = getattr(self, "_payload", None)
        if buf is None or buf.dtype != dtype:
            buf = torch.zeros(self.total, dtype=dtype, device=self.device)
            self._payload = buf
            self._fill_payload(buf)
        return buf

    def refresh_payload(self, dtype):
        """Write this rank's master shards into its slice of the fp8 gather payload.  The step's
        epilogue normally writes that slice, but a skipped (overflow) step leaves it untouched and
        the all-gather still runs (the skip flag stays on the device), so the slice must always
        hold the current weights: at allocation (not zeros) and after a checkpoint load (not the
        pre-load weights)."""
        if dtype is None or self.world == 1:
            return
        buf = getattr(self, "_payload", None)
        if buf is None or buf.dtype != dtype:
            self.payload(dtype)  # allocates and fills
        else:
            self._fill_payload(buf)

    def _fill_payload(self, buf):
        for b in range(self.num_blocks):
            s = b * self.block + self.rank * self.shard
            buf[s:s + self.shard].copy_(self.master[b].to(buf.dtype))

    def out_shards(self, gather_dtype=None):
        """Where the optimizer epilogue writes this rank's updated weights: the model-dtype
        shards of ``flat_param``, or the fp8 payload shards when gathering compressed."""
        src = self.flat_param if gather_dtype is None or self.world == 1 else self.payload(gather_dtype)
        return [src[b * self.block + self.rank * self.shard:][:self.shard] for b in range(self.num_blocks)]

    def out_fragments(self, frags, gather_dtype=None):
        rows = self.out_shards(gather_dtype)
        return [rows[b][lo:hi] for (_, b, lo, hi) in frags]

    def grad_shard_views(self):
        return [self.shard_grad[b] for b in range(self.num_blocks)]

    def fragments(self):
        """(param index, block, start, end) of every parameter fragment inside this rank's shards,
        as offsets into the shard row ``[0, shard)`` of block ``block``."""
        out = []
        for i, (p, off) in enumerate(zip(self.params, self.offsets)):
            n = p.numel()
            for b in self.param_blocks[i]:
                s0 = b * self.block + self.rank * self.shard
                lo, hi = max(off, s0), min(off + n, s0 + self.shard)
                if lo < hi:
                    out.append((i, b, lo - s0, hi - s0))
        return out

    # ---- reductions ----
    def _make_hook(self, i):
        def hook(param):
            self._adopt_grad(i)
            if self.is_accumulation_step:
                return
            if self._fired[i]:
                # a shared parameter accumulated again after its block may have been reduced:
                # reduce those blocks once more at the end (same decision on every rank)
                self._dirty.update(b for b in self.param_blocks[i] if self._handles[b] is not None)
                return
            self._fired[i] = True
            for b in self.param_blocks[i]:
                self._ready[b] += 1
                if self._ready[b] == self._pending[b]:
                    self._reduce_block(b)
        return hook

    def _issue_block(self, b, again=False):
        """Queue block ``b``'s reduction; returns (pending works, reduced shard tensor)."""
        src = self.block_view(self.flat_grad, b)
        dst = self.shard_grad[b]
        # the gradient buffer itself is never modified (a shared parameter can make a block be
        # reduced twice); scaling / widening / the in-place all-reduce work on a copy
        pre = self.predivide and self.dp_size > 1
        red = src
        if self.reduce_dtype != src.dtype:
            red = src.to(self.reduce_dtype)
            if pre:
                red.mul_(1.0 / self.dp_size)
        elif pre:
            red = src * (1.0 / self.dp_size)
        elif again or self.mode == "ar":
            red = src.clone()
        if self.world == 1:
            out = red
        elif self.mode == "rs":
            out = dst if dst.dtype == red.dtype else torch.empty(self.shard, dtype=red.dtype, device=self.device)
            w = dist.reduce_scatter_tensor(out, red, group=self.pg, async_op=True)
            if self.ar_pg is None:
                return [w], out
            w.wait()  # NCCL: the issuing (side) stream waits on the reduce-scatter, not the host
        else:  # "ar" (reference v3): whole-block all-reduce, keep this rank's slice
            w = dist.all_reduce(red, group=self.pg, async_op=True)
            out = red[self.rank * self.shard:(self.rank + 1) * self.shard]
            if self.ar_pg is None:
                return [w], out
            w.wait()
        if self.ar_pg is not None:
            # inter-group: the same shard index of every group (reference :409-418)
            return [dist.all_reduce(out, group=self.ar_pg, async_op=True)], out
        return [], out

    def _reduce_block(self, b, again=False):
        if self._handles[b] is not None:
            return
        self.generation += 1  # shard_grad is about to be overwritten
        dst = self.shard_grad[b]
        if self.dp_size == 1:
            dst.copy_(self.block_view(self.flat_grad, b))
            self._handles[b] = True
            return
        if self._stream is not None:
            self._stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self._stream):
                works, out = self._issue_block(b, again)
        else:
            works, out = self._issue_block(b, again)
        self._handles[b] = (works, out, dst)

    def _finish(self, h):
        works, out, dst = h
        for w in works:
            w.wait()
        if out is not dst:
            dst.copy_(out)

    def complete_reductions(self):
        """Reduce every block not reduced yet and wait for all of them."""
        if not self.overlap:
            for i in range(len(self.params)):
                self._adopt_grad(i)
        for b in range(self.num_blocks):
            if self._handles[b] is None:
                self._reduce_block(b)
        for b in range(self.num_blocks):
            h = self._handles[b]
            if isinstance(h, tuple):
                self._finish(h)
        if self._stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._stream)
        for b in sorted(self._dirty):
            self._handles[b] = None
            self._reduce_block(b, again=True)
            if isinstance(self._handles[b], tuple):
                self._finish(self._handles[b])
        if self._dirty and self._stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._stream)
        self._dirty = set()
        self._handles = [None] * self.num_blocks
        self._ready = [0] * self.num_blocks
        self._fired = [False] * len(self.params)

    def zero_grad(self):
        self.flat_grad.zero_()
        self.attach_grads()

    # ---- parameter all-gather ----
    def all_gather_params(self, gather_dtype=None):
        """Gather every rank's updated shards.  ``gather_dtype`` (an fp8 dtype) means the
        optimizer wrote fp8 shards into ``payload``; they are gathered as bytes and expanded
        into ``flat_param`` by one multi-tensor cast."""
        if self.world == 1:
            return
        src_buf = self.flat_param if gather_dtype is None else self.payload(gather_dtype)
        for b in range(self.num_blocks):
            full = self.block_view(src_buf, b)
            mine = full[self.rank * self.shard:(self.rank + 1) * self.shard]
            if gather_dtype is not None:
                full, mine = full.view(torch.uint8), mine.view(torch.uint8)
            # RCCL gathers in place when the input is this rank's slice of the output
            dist.all_gather_into_tensor(full, mine.clone() if self._gloo else mine, group=self.pg)
        if gather_dtype is not None:
            noop = torch.zeros(1, dtype=torch.int32, device=self.device)
            amp_C.multi_tensor_cast(65536, noop, [[self.block_view(src_buf, b) for b in range(self.num_blocks)],
                                                  [self.block_view(self.flat_param, b)
                                                   for b in range(self.num_blocks)]])

    def state_dict_shards(self):
        return {"rank": self.rank, "world": self.world, "block": self.block, "num_blocks": self.num_blocks,
                "master": self.master.clone()}
