"""Number-of-microbatches calculators (reference apex/transformer/microbatches.py:21-172):
constant, or a linear global-batch-size ramp-up."""
from abc import ABC, abstractmethod
from typing import List, Optional


def build_num_microbatches_calculator(rank: int, rampup_batch_size: Optional[List[int]], global_batch_size: int,
                                      micro_batch_size: int, data_parallel_size: int):
    if rampup_batch_size is None:
        calc = ConstantNumMicroBatches(global_batch_size, micro_batch_size, data_parallel_size)
        if rank == 0:
            print("setting number of micro-batches to constant {}".format(calc.get()), flush=True)
        return calc
    assert len(rampup_batch_size) == 3, ("expected the following format: --rampup-batch-size <start batch size> "
                                         "<batch size incerement> <ramp-up samples>")
    start, inc, samples = (int(v) for v in rampup_batch_size)
    if rank == 0:
        print("will use batch size rampup starting from global batch size {} to global batch size {} with batch "
              "size increments {} over {} samples.".format(start, global_batch_size, inc, samples), flush=True)
    return RampupBatchsizeNumMicroBatches(start, inc, samples, global_batch_size, micro_batch_size,
                                          data_parallel_size)


class NumMicroBatchesCalculator(ABC):
    def __init__(self):
        self.num_micro_batches = None
        self.current_global_batch_size = None

    def get(self):
        return self.num_micro_batches

    def get_current_global_batch_size(self):
        return self.current_global_batch_size

    @abstractmethod
    def update(self, consumed_samples, consistency_check):
        pass


class ConstantNumMicroBatches(NumMicroBatchesCalculator):
    def __init__(self, global_batch_size, micro_batch_size, data_parallel_size):
        super().__init__()
        per = micro_batch_size * data_parallel_size
        assert global_batch_size % per == 0, ("global batch size ({}) is not divisible by micro batch size ({}) "
                                              "times data parallel size ({})".format(global_batch_size,
                                                                                     micro_batch_size,
                                                                                     data_parallel_size))
        self.num_micro_batches = global_batch_size // per
        assert self.num_micro_batches >= 1
        self.current_global_batch_size = global_batch_size
        self.micro_batch_size = micro_batch_size

    def update(self, consumed_samples, consistency_check):
        pass


class RampupBatchsizeNumMicroBatches(NumMicroBatchesCalculator):
    """Global batch grows from ``start_batch_size`` to ``global_batch_size`` in steps of
    ``batch_size_increment``, one step every ``ramup_samples / num_increments`` samples."""

    def __init__(self, start_batch_size, batch_size_increment, ramup_samples, global_batch_size, micro_batch_size,
                 data_parallel_size):
        super().__init__()
        self.micro_batch_size = micro_batch_size
        self.data_parallel_size = data_parallel_size
        self.micro_batch_times_data_parallel_size = micro_batch_size * data_parallel_size
        assert self.micro_batch_times_data_parallel_size > 0
        assert start_batch_size > 0 and global_batch_size > 0 and batch_size_increment > 0
        self.start_batch_size = start_batch_size
        self.global_batch_size = global_batch_size
        diff = global_batch_size - start_batch_size
        assert diff >= 0
        assert diff % batch_size_increment == 0, ("expected global batch size interval ({}) to be divisible by "
                                                  "global batch size increment ({})".format(diff, batch_size_increment))
        self.batch_size_increment = batch_size_increment
        num_increments = diff // batch_size_increment
        self.ramup_samples = ramup_samples
        assert self.ramup_samples >= 0
        self.rampup_samples_per_increment = self.ramup_samples / num_increments if num_increments else float("inf")
        self.update(0, False)

    def update(self, consumed_samples, consistency_check):
        if consumed_samples > self.ramup_samples:
            self.current_global_batch_size = self.global_batch_size
        else:
            steps = int(consumed_samples / self.rampup_samples_per_increment)
            self.current_global_batch_size = self.start_batch_size + steps * self.batch_size_increment
            assert self.current_global_batch_size <= self.global_batch_size
        if consistency_check:
            assert self.current_global_batch_size % self.micro_batch_times_data_parallel_size == 0, (
                "current global batch size ({}) is not divisible by micro-batch-size ({}) times data parallel size "
                "({})".format(self.current_global_batch_size, self.micro_batch_size, self.data_parallel_size))
        self.num_micro_batches = self.current_global_batch_size // self.micro_batch_times_data_parallel_size
