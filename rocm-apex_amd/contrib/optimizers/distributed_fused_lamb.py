"""ZeRO-2 style distributed LAMB (reference apex/contrib/optimizers/distributed_fused_lamb.py:10-900).

Same flat/sharded storage and overlapped reduce-scatter as :class:`DistributedFusedAdam`.  LAMB
needs the L2 norm of every *whole* parameter and of its update, while each rank only owns
fragments of parameters: each rank computes per-fragment squared norms with one multi-tensor
launch, scatters them into a ``[num_params]`` vector, and ONE all-reduce of that small vector
gives every rank the full per-parameter norms (reference :673-692 does the same with its
contrib fragments).  Update term and trust-ratio update are the legacy two-stage kernels
(``multi_tensor_lamb_stage1_cuda`` / ``_stage2_cuda``) over the shard rows / fragments.
"""
import torch
import torch.distributed as dist

from ... import amp_C
from .distributed_fused_adam import DistributedFusedAdam, _record_found_inf


class DistributedFusedLAMB(DistributedFusedAdam):
    def __init__(self, params, lr=1e-3, bias_correction=True, grad_averaging=True, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, max_grad_norm=0.0, adam_w_mode=True, use_nvlamb=False,
                 step_supports_amp_scaling=True, overlap_reductions=True, dwu_group_size=0, dwu_num_blocks=4,
                 dwu_num_chunks=4, dwu_num_rs_pg=1, dwu_num_ar_pg=4, dwu_num_ag_pg=0, e5m2_allgather=False,
                 verbose=False, clip_after_ar=True, min_block_elems=1 << 22, current_process_group=None,
                 reduce_dtype=None, predivide=True, allgather_dtype=None):
        super().__init__(params, lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                         weight_decay=weight_decay, max_grad_norm=max_grad_norm, overlap_reductions=overlap_reductions,
                         compute_L2_grad_norm=True, dwu_group_size=dwu_group_size, dwu_num_blocks=dwu_num_blocks,
                         e5m2_allgather=e5m2_allgather, step_supports_amp_scaling=step_supports_amp_scaling,
                         clip_grad_norm=clip_after_ar, adam_w_mode=adam_w_mode, min_block_elems=min_block_elems,
                         current_process_group=current_process_group, reduce_dtype=reduce_dtype, predivide=predivide,
                         allgather_dtype=allgather_dtype)
        for g in self.param_groups:
            g["grad_averaging"] = grad_averaging
        self._use_nvlamb = use_nvlamb
        self._grad_averaging = grad_averaging
        flat = self._flat
        self._frags = flat.fragments()
        dev = flat.device
        self._frag_param = torch.tensor([f[0] for f in self._frags], dtype=torch.long, device=dev)
        self._num_params = len(flat.params)
        self._u = torch.zeros_like(flat.master)
        self._decay = torch.full((flat.num_blocks,), float(weight_decay) if adam_w_mode else 0.0,
                                 dtype=torch.float32, device=dev)

    def _frag_views(self, buf2d):
        return [buf2d[b, lo:hi] for (_, b, lo, hi) in self._frags]

    def _param_norms(self, p_frags, u_frags):
        """Full-parameter L2 norms of the master weights and of the LAMB update from this rank's
        fragments: both squared-norm vectors in ONE [2, num_params] buffer and ONE all-reduce
        (two latency-bound collectives per step were one too many at BERT-large's ~400 params)."""
        dev = self._flat.device
        sq = torch.zeros(2, self._num_params, dtype=torch.float32, device=dev)
        if p_frags:
            noop = torch.zeros(1, dtype=torch.int32, device=dev)
            for row, frags in ((0, p_frags), (1, u_frags)):
                _, per = amp_C.multi_tensor_l2norm(65536, noop, [frags], True)
                sq[row].index_add_(0, self._frag_param, per.float() ** 2)
        if self._flat.world > 1:
            dist.all_reduce(sq, group=self._pg)
        nrm = sq.sqrt()
        return nrm[0], nrm[1]

    def step(self, closure=None, grad_scaler=None):
        """One LAMB step with no host synchronization: the overflow flag, step count and learning
        rate stay on the device and gate / parameterize the two stage launches (reference
        apex/contrib/optimizers/distributed_fused_lamb.py:702-712)."""
        loss = closure() if closure is not None else None
        flat = self._flat
        self._prepare_step(grad_scaler)
        g0 = self.param_groups[0]
        beta1, beta2 = g0["betas"]
        wd = g0["weight_decay"]
        self._lr_t.fill_(float(g0["lr"]))
        self._step_t.add_(1 - self._skip.float())
        for g in self.param_groups:
            g["step"] = g.get("step", 0) + 1
        grads = flat.shard_grad
        grads.mul_(self._inv)  # unscale, average over ranks, clip (folded into one factor)
        if not self.adam_w_mode and wd != 0:
            grads.add_(flat.master, alpha=wd)  # L2 mode: decay enters the moments
        nb = flat.num_blocks
        rows = lambda t: [t[b] for b in range(nb)]  # noqa: E731
        noclip = torch.zeros(1, dtype=torch.float32, device=flat.device)
        beta3 = (1.0 - beta1) if self._grad_averaging else 1.0
        amp_C.multi_tensor_lamb_stage1_capturable(65536, self._skip, [rows(grads), rows(flat.master), rows(self._m),
                                                                      rows(self._v), rows(self._u)],
                                                  self._decay, self._step_t, bool(g0["bias_correction"]), beta1,
                                                  beta2, g0["eps"], noclip, 1.0, beta3)
        p_frags = self._frag_views(flat.master)
        u_frags = self._frag_views(self._u)
        pn, un = self._param_norms(p_frags, u_frags)
        if p_frags:
            # stage 2 also writes the model-dtype (or fp8 gather payload) copy of each fragment
            out_frags = flat.out_fragments(self._frags, self._ag_dtype)
            amp_C.multi_tensor_lamb_stage2_capturable(65536, self._skip, [p_frags, u_frags, out_frags],
                                                      pn[self._frag_param], un[self._frag_param], self._lr_t, wd,
                                                      self._use_nvlamb)
        # a skipped step leaves the shards (and so the gathered weights) as they were
        flat.all_gather_params(self._ag_dtype)
        flat.zero_grad()
        if grad_scaler is not None and grad_scaler.is_enabled():
            _record_found_inf(grad_scaler, self, self._skip)
        return loss

    def state_dict(self):
        # the step count lives on the device (DistributedFusedAdam's "step" entry of the shard)
        return super().state_dict()

    def load_state_dict(self, state_dict):
        shard = state_dict.get("distributed_shard", {})
        if "step_host" in shard and "step" not in shard:  # checkpoints of the host-counted step
            shard["step"] = torch.tensor([float(shard["step_host"])])
        super().load_state_dict(state_dict)
