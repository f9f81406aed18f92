"""Peer-memory exchange over xGMI for tiny, latency-bound collectives (``csrc/comm/peer.hip``).

The reference's groupbn exchanges CUDA-IPC handles with ``all_gather`` and has its NHWC batch-norm
kernel write its statistics straight into the partner GPUs' memory (apex/contrib/groupbn/
batch_norm.py:179-226, csrc/groupbn/ipc.cu); on HIP that path is compiled out and ``bn_group > 1``
is unavailable.  Here the same idea is a standalone primitive: every member of a process group
exports one device buffer with ``hipIpcGetMemHandle``, the handles are all-gathered once, and each
exchange is ONE single-workgroup kernel that pushes this rank's payload into every member's buffer
over xGMI and waits (bounded) for the others' epoch flags — no RCCL launch / protocol round trip
per batch-norm layer.  ``all_gather`` / ``all_reduce_sum`` keep the stream order of the calling
stream, like the collectives they replace.

Use: ``enable_peer_memory(group)`` once (collective over ``group``, all members on one node), after
which SyncBatchNorm / BatchNorm2d_NHWC(bn_group>1) statistics over ``group`` take this path.

Failure detection (no silent corruption, no device sync on the hot path): a member that does not
arrive within ``timeout_s`` (30 s default — far beyond any legitimate skew such as a first-step
convolution search) makes the kernel give up, fill the output with NaN and bump an error counter.
The NaN statistics poison the loss, so a dynamic loss scaler skips that step; the counter is
copied to pinned host memory asynchronously every ``poll_every`` exchanges and the NEXT poll
raises ``PeerExchangeTimeout`` once the copy has landed.  ``check()`` is the blocking variant."""
import torch
import torch.distributed as dist

from .. import _native

_REGISTRY = {}
_HANDLE_BYTES = 64


def _ext():
    return _native.require("peer_memory").peer_memory


class PeerExchangeTimeout(RuntimeError):
    pass


class PeerExchange(object):
    """Collective constructor over ``group``: allocates, exports and opens the exchange buffers."""

    def __init__(self, group=None, max_floats=4104, timeout_s=30.0, poll_every=16):
        ext = _ext()
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > ext.max_group():
            raise ValueError("peer memory exchange supports at most {} ranks".format(ext.max_group()))
        self.nmax = int(max_floats)
        self.device = torch.device("cuda", torch.cuda.current_device())
        nbytes = 2 * self.world * (self.nmax + 4) * 4
        self.local_ptr = ext.alloc(nbytes)
        handle = bytes(ext.handle(self.local_ptr))
        assert len(handle) == _HANDLE_BYTES
        on_gpu = dist.get_backend(group) == "nccl"
        ht = torch.tensor(list(handle), dtype=torch.uint8, device=self.device if on_gpu else "cpu")
        parts = [torch.empty_like(ht) for _ in range(self.world)]
        dist.all_gather(parts, ht, group=group)
        self.ptrs = []
        self._opened = []
        for r, part in enumerate(parts):
            if r == self.rank:
                self.ptrs.append(self.local_ptr)
            else:
                p = ext.open(bytes(part.cpu().tolist()))
                self.ptrs.append(p)
                self._opened.append(p)
        self.epoch = 0
        self.timeout_s = float(timeout_s)
        self.poll_every = max(1, int(poll_every))
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._err_event = None
        dist.barrier(group=group)  # every member has opened every buffer before the first exchange

    def all_gather(self, local):
        """[world, n] fp32: every member's ``local`` (1-D, n <= max_floats)."""
        flat = local.reshape(-1).float().contiguous()
        if flat.numel() > self.nmax:
            raise ValueError("payload of {} floats exceeds the exchange slot ({})".format(flat.numel(), self.nmax))
        self.epoch += 1
        out = torch.empty(self.world, flat.numel(), dtype=torch.float32, device=flat.device)
        _ext().allgather(flat, self.ptrs, self.nmax, self.rank, self.epoch, out, self.err, self.timeout_s)
        if self.epoch % self.poll_every == 0:
            self.poll()
        return out

    def all_reduce_sum(self, t):
        return self.all_gather(t).sum(0).view(t.shape).to(t.dtype)

    def _raise(self, n):
        raise PeerExchangeTimeout("peer memory exchange timed out {} time(s): a member of the group did not arrive "
                                  "within {:.1f} s (the affected outputs were poisoned with NaN)".format(n, self.timeout_s))

    def poll(self):
        """Sync-free error check: inspect the host copy enqueued by the previous poll once it has
        landed, then enqueue a fresh one."""
        ev = self._err_event
        if ev is not None:
            if not ev.query():
                return
            n = int(self._err_host[0])
            self._err_event = None
            if n != 0:
                self._raise(n)
        self._err_host.copy_(self.err, non_blocking=True)
        self._err_event = torch.cuda.Event()
        self._err_event.record()

    def check(self):
        """Blocking check (synchronizes with the device)."""
        n = int(self.err.item())
        if n != 0:
            self._raise(n)

    def close(self):
        ext = _ext()
        for p in self._opened:
            ext.close(p)
        self._opened = []
        ext.free(self.local_ptr)


def _key(group):
    return id(group) if group is not None else 0


def enable_peer_memory(group=None, max_floats=4104, timeout_s=30.0):
    """Create (collectively) and register the exchange for ``group``; returns it, or None (with the
    RCCL path kept) when peer memory is unavailable (no native extension / no GPU / IPC failure)."""
    key = _key(group)
    if key in _REGISTRY:
        return _REGISTRY[key]
    if not torch.cuda.is_available() or _native.submodule("peer_memory") is None:
        return None
    ex = PeerExchange(group, max_floats, timeout_s)
    _REGISTRY[key] = ex
    return ex


def get_peer_exchange(group=None):
    return _REGISTRY.get(_key(group))


def disable_peer_memory(group=None):
    ex = _REGISTRY.pop(_key(group), None)
    if ex is not None:
        ex.close()
