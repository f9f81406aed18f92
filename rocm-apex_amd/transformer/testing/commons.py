"""Shared helpers of the transformer tests (reference apex/transformer/testing/commons.py:31-123)."""
import os
import random

import numpy
import torch
import torch.nn as nn

from .. import parallel_state, tensor_parallel


TEST_SUCCESS_MESSAGE = ">> passed the test :-)"  # reference commons.py:27 (test harness banner)


class MyLayer(nn.Module):
    def __init__(self, hidden_size, pre_process, post_process):
        super().__init__()
        self.pre_process, self.post_process = pre_process, post_process
        self.layer = nn.Linear(hidden_size, hidden_size)

    def forward(self, x):
        return self.layer(x)


class MyModel(nn.Module):
    def __init__(self, hidden_size, pre_process=False, post_process=False):
        super().__init__()
        self.pre_process, self.post_process = pre_process, post_process
        self.layer = MyLayer(hidden_size, pre_process, post_process)
        self.input_tensor = None

    def set_input_tensor(self, input_tensor):
        self.input_tensor = input_tensor[0] if isinstance(input_tensor, (list, tuple)) else input_tensor

    def forward(self, x):
        return self.layer(self.input_tensor if self.input_tensor is not None else x)


def model_provider_func(hidden_size, pre_process, post_process):
    return MyModel(hidden_size, pre_process, post_process)


class IdentityLayer(nn.Module):
    def __init__(self, size, scale=1.0):
        super().__init__()
        self.weight = nn.Parameter(scale * torch.randn(size))

    def forward(self):
        return self.weight


def set_random_seed(seed):
    random.seed(seed)
    numpy.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available() and parallel_state.model_parallel_is_initialized():
        tensor_parallel.model_parallel_cuda_manual_seed(seed)


def initialize_distributed(backend="nccl"):
    """One process per GPU, env:// rendezvous (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT)."""
    if torch.distributed.is_initialized():
        return
    rank = int(os.getenv("RANK", "0"))
    world = int(os.getenv("WORLD_SIZE", "1"))
    local = int(os.getenv("LOCAL_RANK", str(rank)))
    if backend == "nccl" and torch.cuda.is_available():
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "6000")
    torch.distributed.init_process_group(backend=backend, world_size=world, rank=rank)


def print_separator(message):
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
    filler = "-" * max(0, (78 - len(message)) // 2)
    if not torch.distributed.is_initialized() or torch.distributed.get_rank() == 0:
        print("\n" + filler + " " + message + " " + filler, flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
