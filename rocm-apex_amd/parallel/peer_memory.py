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

Use: ``enable_peer_memory(group)`` once (collective over ``group``), after which SyncBatchNorm /
BatchNorm2d_NHWC(bn_group>1) statistics over ``group`` take this path.  Construction is safe by
design: the buffers are uncached device memory (what RCCL uses for cross-GPU flags), the group
agrees collectively on every step (size <= 8, one host, allocation, IPC open), and a handshake
exchange with a 2 s bound must deliver every word to every member — otherwise every member gets
None and stays on RCCL, in-process (no restart).

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


class PeerExchangeUnavailable(RuntimeError):
    """Raised (on every member alike) when the group cannot use peer memory; callers keep RCCL."""


_ALLOC_KINDS = {2: "uncached", 1: "fine-grained", 0: "coarse-grained"}


def _agree(ok, group, device):
    """Collective AND of a per-rank flag over ``group`` (every member gets the same answer, so a
    failure on one rank can never leave the others waiting in a later collective)."""
    on_gpu = dist.get_backend(group) == "nccl"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device if on_gpu else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


class PeerExchange(object):
    """Collective constructor over ``group``: allocates, exports and opens the exchange buffers,
    then proves the protocol with one handshake exchange.  Every step ends in a group-wide
    agreement, so either every member gets a working exchange or every member gets
    :class:`PeerExchangeUnavailable` (and keeps the RCCL path) — no member can hang the others.

    Preconditions checked collectively: group size <= ``max_group()``, every member on this host
    (hipIpc handles only open on the same node), the native extension present on every member."""

    def __init__(self, group=None, max_floats=4104, timeout_s=30.0, poll_every=16, handshake_timeout_s=2.0,
                 _fail_handshake=False):
        import socket

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device("cuda", torch.cuda.current_device())
        self._opened = []
        self.local_ptr = None
        ext = _native.submodule("peer_memory")
        ext = getattr(ext, "peer_memory", ext) if ext is not None else None
        hosts = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        ok = ext is not None and self.world <= (ext.max_group() if ext is not None else 0) and len(set(hosts)) == 1
        if not _agree(ok, group, self.device):
            raise PeerExchangeUnavailable("peer memory needs <= {} ranks on one host with the native extension "
                                          "(hosts: {})".format(ext.max_group() if ext else "?", sorted(set(hosts))))
        self.nmax = int(max_floats)
        nbytes = 2 * self.world * (self.nmax + 4) * 4
        handle, err = bytes(_HANDLE_BYTES), None
        try:
            self.local_ptr, kind = ext.alloc(nbytes)
            self.alloc_kind = _ALLOC_KINDS.get(int(kind), str(kind))
            handle = bytes(ext.handle(self.local_ptr))
            assert len(handle) == _HANDLE_BYTES
        except Exception as e:  # noqa: BLE001 - any local failure is agreed on below
            err = e
        on_gpu = dist.get_backend(group) == "nccl"
        ht = torch.tensor(list(handle), dtype=torch.uint8, device=self.device if on_gpu else "cpu")
        parts = [torch.empty_like(ht) for _ in range(self.world)]
        dist.all_gather(parts, ht, group=group)
        if not _agree(err is None, group, self.device):
            self._release()
            raise PeerExchangeUnavailable("peer buffer allocation / export failed: {!r}".format(err))
        self.ptrs = []
        try:
            for r, part in enumerate(parts):
                if r == self.rank:
                    self.ptrs.append(self.local_ptr)
                else:
                    q = ext.open(bytes(part.cpu().tolist()))
                    self.ptrs.append(q)
                    self._opened.append(q)
        except Exception as e:  # noqa: BLE001
            err = e
        if not _agree(err is None, group, self.device):
            self._release()
            raise PeerExchangeUnavailable("opening the peers' IPC handles failed: {!r}".format(err))
        self.epoch = 0
        self.poll_every = max(1, int(poll_every))
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._err_event = None
        dist.barrier(group=group)  # every member has opened every buffer before the first exchange
        # handshake: one exchange with a short bound; every member checks every word it received
        self.timeout_s = float(handshake_timeout_s)
        probe = torch.arange(64, dtype=torch.float32, device=self.device) + 1000.0 * (self.rank + 1)
        got = self.all_gather(probe)
        torch.cuda.synchronize()
        expect = torch.stack([torch.arange(64, dtype=torch.float32, device=self.device) + 1000.0 * (r + 1)
                              for r in range(self.world)])
        good = int(self.err.item()) == 0 and torch.equal(got, expect) and not _fail_handshake
        if not _agree(good, group, self.device):
            self._release()
            raise PeerExchangeUnavailable("peer-memory handshake failed (cross-device visibility within {:.1f} s)"
                                          .format(self.timeout_s))
        self.timeout_s = float(timeout_s)

    def _release(self):
        ext = _ext()
        for q in self._opened:
            ext.close(q)
        self._opened = []
        if self.local_ptr is not None:
            ext.free(self.local_ptr)
            self.local_ptr = None

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
        self._release()


def _key(group):
    return id(group) if group is not None else 0


_FAILED = {}


def enable_peer_memory(group=None, max_floats=4104, timeout_s=30.0, _fail_handshake=False):
    """Create (collectively) and register the exchange for ``group``; returns it, or None with the
    RCCL path kept when peer memory is unavailable on ANY member (no GPU / extension, more than
    ``max_group()`` ranks, ranks on several hosts, an IPC failure, or a failed handshake) — the
    decision is agreed by the whole group, so all members take the same path."""
    key = _key(group)
    if key in _REGISTRY:
        return _REGISTRY[key]
    if key in _FAILED or not torch.cuda.is_available():
        return None
    try:
        ex = PeerExchange(group, max_floats, timeout_s, _fail_handshake=_fail_handshake)
    except PeerExchangeUnavailable as e:
        _FAILED[key] = str(e)
        return None
    _REGISTRY[key] = ex
    return ex


def exchange_path(group=None):
    """"peer" when ``group``'s statistics exchange runs over peer memory, else "rccl"."""
    return "peer" if _key(group) in _REGISTRY else "rccl"


def get_peer_exchange(group=None):
    return _REGISTRY.get(_key(group))


def disable_peer_memory(group=None):
    _FAILED.pop(_key(group), None)
    ex = _REGISTRY.pop(_key(group), None)
    if ex is not None:
        ex.close()
