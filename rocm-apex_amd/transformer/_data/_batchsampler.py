"""Megatron-style data-parallel batch samplers (reference
apex/transformer/_data/_batchsampler.py:16-180).

Iterating yields this data-parallel rank's LOCAL mini-batch (a list of dataset indices, global
batch / dp of them); the pipeline schedules then cut it into micro-batches.

* ``MegatronPretrainingSampler``: global batch g covers the consecutive indices
  ``[consumed + g*B*dp, consumed + (g+1)*B*dp)``; this rank takes its contiguous B-slice.  The
  index ranges are computed arithmetically (no per-index list building).  (The reference builds
  only B indices and then slices ``[rank*B:(rank+1)*B]`` out of them, which leaves every rank but
  0 with an empty batch; the Megatron-LM semantics are kept here instead.)
* ``MegatronPretrainingRandomSampler``: each rank owns a contiguous bucket of the dataset and
  walks a permutation of it drawn from a generator seeded with the epoch number, so resuming at
  ``consumed_samples`` replays exactly the remaining batches."""
import torch


def _check(total, consumed, local_bs, rank, dp, err=ValueError, strict_consumed=False):
    if total <= 0:
        raise err("no sample to consume: {}".format(total))
    if strict_consumed and consumed >= total:
        raise err("no samples left to consume: {}, {}".format(consumed, total))
    if local_bs <= 0:
        raise err("local minibatch size must be greater than 0: {}".format(local_bs))
    if dp <= 0:
        raise err("data parallel size must be greater than 0: {}".format(dp))
    if rank >= dp:
        raise err("data_parallel_rank should be smaller than data parallel size: {}, {}".format(rank, dp))


class _SamplerBase:
    def __init__(self, total_samples, consumed_samples, local_minibatch_size, data_parallel_rank,
                 data_parallel_size):
        self.total_samples = total_samples
        self.consumed_samples = consumed_samples
        self.data_parallel_rank = data_parallel_rank
        self.data_parallel_size = data_parallel_size
        self._local_minibatch_size = local_minibatch_size

    def __len__(self):
        return self.total_samples

    @property
    def local_minibatch_size(self):
        return self._local_minibatch_size

    @local_minibatch_size.setter
    def local_minibatch_size(self, value):
        self._local_minibatch_size = value

    @property
    def local_minibatch_times_data_parallel_size(self):
        return self._local_minibatch_size * self.data_parallel_size


class MegatronPretrainingSampler(_SamplerBase):
    def __init__(self, total_samples, consumed_samples, local_minibatch_size, data_parallel_rank, data_parallel_size,
                 drop_last=True):
        _check(total_samples, consumed_samples, local_minibatch_size, data_parallel_rank, data_parallel_size,
               RuntimeError, strict_consumed=True)
        super().__init__(total_samples, consumed_samples, local_minibatch_size, data_parallel_rank,
                         data_parallel_size)
        self.drop_last = drop_last

    def get_start_end_idx(self):
        lo = self.data_parallel_rank * self.local_minibatch_size
        return lo, lo + self.local_minibatch_size

    def __iter__(self):
        span = self.local_minibatch_times_data_parallel_size
        lo, hi = self.get_start_end_idx()
        first = self.consumed_samples
        full = (self.total_samples - first) // span
        for g in range(full):
            base = first + g * span
            yield list(range(base + lo, base + hi))
        tail = first + full * span
        if tail < self.total_samples and not self.drop_last:
            yield list(range(min(tail + lo, self.total_samples), min(tail + hi, self.total_samples)))


class MegatronPretrainingRandomSampler(_SamplerBase):
    def __init__(self, total_samples, consumed_samples, local_minibatch_size, data_parallel_rank,
                 data_parallel_size):
        _check(total_samples, consumed_samples, local_minibatch_size, data_parallel_rank, data_parallel_size)
        super().__init__(total_samples, consumed_samples, local_minibatch_size, data_parallel_rank,
                         data_parallel_size)

    @property
    def last_batch_size(self):
        return self.total_samples % self.local_minibatch_times_data_parallel_size

    def __iter__(self):
        span = self.local_minibatch_times_data_parallel_size
        usable = self.total_samples - self.last_batch_size       # whole global batches per epoch
        self.epoch, in_epoch = divmod(self.consumed_samples, usable)
        bucket = (self.total_samples // span) * self.local_minibatch_size  # this rank's share
        g = torch.Generator()
        g.manual_seed(self.epoch)
        order = torch.randperm(bucket, generator=g) + self.data_parallel_rank * bucket
        done = in_epoch // self.data_parallel_size                # already consumed from the bucket
        order = order[done:]
        bs = self.local_minibatch_size
        for k in range(order.numel() // bs):
            self.consumed_samples += span
            yield order[k * bs:(k + 1) * bs].tolist()
