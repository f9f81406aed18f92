"""ZeRO-2 style distributed Adam (reference apex/contrib/optimizers/distributed_fused_adam.py:9-636,
distributed_fused_adam_v2.py, distributed_fused_adam_v3.py).

Gradients are reduce-scattered per block while backward runs (see :mod:`._sharded`), every rank
updates only its fp32 master shard with one fused multi-tensor Adam launch (which also writes
the model-dtype copy), and the new parameters are all-gathered.  Loss scaling is sync-free: the
inverse scale (and the global-norm clip factor) is a device scalar folded into the kernel and an
overflow anywhere skips the step on every rank through a device flag.

Constructor keywords of the reference that only tune its CUDA pipeline (``dwu_num_rs_pg``,
``dwu_num_ar_pg``, ``dwu_num_ag_pg``, ``dwu_num_chunks``, ``flat_mt``, ``do_not_flatten_model``,
``num_process_groups``...) are accepted and ignored; ``dwu_num_blocks`` sets the number of
reduce-scatter blocks and ``dwu_group_size`` / ``current_process_group`` the sharding group.

``dwu_group_size = G < world`` (reference :306-371, :397-441): optimizer state is sharded over
groups of G consecutive ranks and replicated across the world/G groups; every block is
reduce-scattered inside the group and the shard is then all-reduced across groups (ranks with
the same index in their group), so every replica trains on the gradient of the whole job.
``reduce_dtype=torch.float32`` accumulates the reduction in fp32 (bf16/fp16 grads are widened
before the collective); ``predivide`` divides by the data-parallel size before the sum."""
import torch
import torch.distributed as dist

from ... import amp_C
from ._sharded import FlatShardedBuffers

_TWO_LEVEL = {}


def two_level_groups(group_size):
    """(intra-group, inter-group) process groups for sharding over ``group_size`` consecutive
    ranks: the caller's block of ranks, and the ranks that hold the same shard index in every
    block.  Collective (every rank creates every group, same order); cached per size."""
    if group_size in _TWO_LEVEL:
        return _TWO_LEVEL[group_size]
    world, rank = dist.get_world_size(), dist.get_rank()
    assert world % group_size == 0, "world size must be a multiple of dwu_group_size"
    intra = inter = None
    for start in range(0, world, group_size):
        g = dist.new_group(list(range(start, start + group_size)))
        if start <= rank < start + group_size:
            intra = g
    for k in range(group_size):
        g = dist.new_group(list(range(k, world, group_size)))
        if rank % group_size == k:
            inter = g
    _TWO_LEVEL[group_size] = (intra, inter)
    return intra, inter


class DistributedFusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, eps_inside_sqrt=False,
                 weight_decay=0.0, max_grad_norm=0.0, amsgrad=False, flat_mt=False, overlap_reductions=True,
                 compute_L2_grad_norm=False, dwu_group_size=0, dwu_num_blocks=4, dwu_num_chunks=4, dwu_num_rs_pg=1,
                 dwu_num_ar_pg=4, dwu_num_ag_pg=0, predivide=True, e5m2_allgather=False, do_not_flatten_model=False,
                 step_supports_amp_scaling=True, num_process_groups=1, current_process_group=None,
                 process_group_id=0, process_group_size=0, clip_grad_norm=True, model_parallel=False,
                 adam_w_mode=True, min_block_elems=1 << 22, reduce_dtype=None, grad_sync_dtype=None,
                 allgather_dtype=None, _reduction_mode="rs"):
        if amsgrad:
            raise RuntimeError("DistributedFusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        if eps_inside_sqrt:
            raise RuntimeError("eps_inside_sqrt is not supported; eps is added to sqrt(v_hat)")
        self.adam_w_mode = 1 if adam_w_mode else 0
        self._predivide = predivide
        self._e5m2_allgather = e5m2_allgather
        # fp8 parameter all-gather (reference e5m2_allgather; e4m3 also accepted): the Adam
        # epilogue writes the fp8 payload directly (see _sharded.py)
        self._ag_dtype = allgather_dtype if allgather_dtype is not None else (
            torch.float8_e5m2 if e5m2_allgather else None)
        if self._ag_dtype not in (None, torch.float8_e5m2, torch.float8_e4m3fn):
            raise ValueError("allgather_dtype must be torch.float8_e5m2 or torch.float8_e4m3fn")
        self._compute_L2_grad_norm = compute_L2_grad_norm
        self._clip_grad_norm = clip_grad_norm
        self._step_supports_amp_scaling = step_supports_amp_scaling
        self._L2_grad_norm = None
        self._global_scale = None
        self._last_step = False
        pg, ar_pg = current_process_group, None
        if pg is None and dwu_group_size and dist.is_initialized() and dwu_group_size < dist.get_world_size():
            pg, ar_pg = two_level_groups(dwu_group_size)
        all_params = [p for g in self.param_groups for p in g["params"]]
        self._flat = FlatShardedBuffers(all_params, pg, num_blocks=dwu_num_blocks, min_block_elems=min_block_elems,
                                        overlap_reductions=overlap_reductions, ar_group=ar_pg,
                                        reduce_dtype=reduce_dtype or grad_sync_dtype, predivide=predivide,
                                        mode=_reduction_mode)
        self._pg = pg
        self._ar_pg = ar_pg
        dev = self._flat.device
        self._m = torch.zeros_like(self._flat.master)
        self._v = torch.zeros_like(self._flat.master)
        self._step_t = torch.zeros(1, dtype=torch.float32, device=dev)
        self._lr_t = torch.zeros(1, dtype=torch.float32, device=dev)
        self._inv = torch.ones(1, dtype=torch.float32, device=dev)
        self._skip = torch.zeros(1, dtype=torch.int32, device=dev)
        self._group_of = {}
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                self._group_of[id(p)] = gi
        if len({(g["lr"], g["betas"], g["eps"], g["weight_decay"], g["bias_correction"])
                for g in self.param_groups}) > 1:
            raise RuntimeError("DistributedFusedAdam: all param groups must share hyper-parameters "
                               "(the shards mix parameters of every group)")

    # ---- reference API ----
    def set_last_step(self, last_step):
        self._last_step = last_step

    def set_is_accumulation_step(self, is_accumulation_step):
        self._flat.is_accumulation_step = is_accumulation_step

    def set_global_scale(self, global_scale):
        self._global_scale = global_scale

    @property
    def global_scale(self):
        return self._global_scale

    @property
    def L2_grad_norm(self):
        return self._L2_grad_norm

    @property
    def has_overflow(self):
        return bool(self._skip.item())

    @property
    def peek_overflow(self):
        return bool(self._skip.item())

    def complete_reductions(self):
        self._flat.complete_reductions()

    def zero_grad(self, set_to_none=False):
        self._flat.zero_grad()

    # ---- step ----
    def _prepare_step(self, grad_scaler=None):
        flat = self._flat
        flat.complete_reductions()
        grads = flat.grad_shard_views()
        dev = flat.device
        inv = torch.ones(1, dtype=torch.float32, device=dev)
        if not flat.predivide and flat.dp_size > 1:
            inv = inv / flat.dp_size  # average over every data-parallel rank (both levels)
        scale = None
        if grad_scaler is not None and grad_scaler.is_enabled():
            scale = grad_scaler._get_scale_async()
        elif getattr(self, "grad_scale", None) is not None:
            scale = self.grad_scale
        elif self._global_scale is not None:
            scale = torch.tensor([float(self._global_scale)], device=dev)
        if scale is not None:
            inv = inv / scale.float().reshape(1).to(dev)
        # overflow: any non-finite reduced grad on any rank skips the step everywhere
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        amp_C.multi_tensor_check_finite(65536, flag, [grads])
        if flat.world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self._pg)
        self._skip.copy_(flag)
        found_inf = getattr(self, "found_inf", None)
        if found_inf is not None:
            self._skip.copy_(torch.maximum(self._skip, (found_inf.reshape(1) > 0).to(torch.int32).to(dev)))
        # global grad norm (of the unscaled, averaged gradient) and clipping
        max_norm = self.defaults["max_grad_norm"]
        if self._compute_L2_grad_norm or (self._clip_grad_norm and max_norm > 0):
            noop = torch.zeros(1, dtype=torch.int32, device=dev)
            nrm, _ = amp_C.multi_tensor_l2norm(65536, noop, [grads], False)
            sq = (nrm.float() * inv) ** 2
            if flat.world > 1:
                dist.all_reduce(sq, group=self._pg)
            gnorm = sq.sqrt()
            self._L2_grad_norm = gnorm
            if self._clip_grad_norm and max_norm > 0:
                clip = torch.clamp(max_norm / (gnorm + 1e-6), max=1.0)
                inv = inv * clip
        self._inv.copy_(inv.reshape(1))
        return grads

    def step(self, closure=None, grad_scaler=None):
        loss = closure() if closure is not None else None
        flat = self._flat
        grads = self._prepare_step(grad_scaler)
        g0 = self.param_groups[0]
        beta1, beta2 = g0["betas"]
        self._lr_t.fill_(float(g0["lr"]))
        self._step_t.add_(1 - self._skip.float())
        for g in self.param_groups:
            g["step"] = g.get("step", 0) + 1
        nb = flat.num_blocks
        amp_C.multi_tensor_adam_capturable(65536, self._skip, self._adam_lists(grads), self._lr_t, beta1, beta2,
                                           g0["eps"], self._step_t, self.adam_w_mode,
                                           1 if g0["bias_correction"] else 0, g0["weight_decay"], self._inv)
        self._stepped_generation = flat.generation
        flat.all_gather_params(self._ag_dtype)
        flat.zero_grad()
        if grad_scaler is not None and grad_scaler.is_enabled():
            _record_found_inf(grad_scaler, self, self._skip)
        return loss

    def _adam_lists(self, grads):
        flat, nb = self._flat, self._flat.num_blocks
        return [grads, [flat.master[b] for b in range(nb)], [self._m[b] for b in range(nb)],
                [self._v[b] for b in range(nb)], flat.out_shards(self._ag_dtype)]

    # ---- checkpointing (sharded, like the reference :598-636) ----
    def state_dict(self):
        sd = super().state_dict()
        sd["distributed_shard"] = {"rank": self._flat.rank, "world": self._flat.world, "block": self._flat.block,
                                   "num_blocks": self._flat.num_blocks, "master": self._flat.master.clone(),
                                   "exp_avg": self._m.clone(), "exp_avg_sq": self._v.clone(),
                                   "step": self._step_t.clone()}
        return sd

    def load_state_dict(self, state_dict):
        shard = state_dict.get("distributed_shard")
        base = {k: v for k, v in state_dict.items() if k != "distributed_shard"}
        super().load_state_dict(base)
        if shard is not None:
            assert shard["world"] == self._flat.world and shard["block"] == self._flat.block, \
                "checkpoint was written with a different sharding layout"
            self._flat.master.copy_(shard["master"])
            self._m.copy_(shard["exp_avg"])
            self._v.copy_(shard["exp_avg_sq"])
            self._step_t.copy_(shard["step"])
            for b in range(self._flat.num_blocks):
                self._flat.param_shard(b).copy_(self._flat.master[b].to(self._flat.dtype))
            self._flat.all_gather_params()
            # a skipped first step after the load gathers the fp8 payload: it must hold the loaded
            # weights, not the ones this optimizer held before
            self._flat.refresh_payload(self._ag_dtype)


def _record_found_inf(grad_scaler, optimizer, skip):
    """Tell a torch GradScaler that this optimizer found (or not) an overflow, so update()
    backs off / grows the scale exactly as for a stock optimizer."""
    st = grad_scaler._per_optimizer_states[id(optimizer)]
    dev = grad_scaler._scale.device
    st["found_inf_per_device"] = {dev: skip.float().to(dev)}
