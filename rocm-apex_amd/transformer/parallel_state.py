"""Tensor / pipeline / data-parallel process-group state (reference apex/transformer/parallel_state.py:26-396).

Rank layout (same as the reference so existing launch scripts keep their meaning):
``rank = pp_rank * (dp * tp) + dp_rank * tp + tp_rank`` — tensor-parallel ranks are adjacent.
On an MI355X node the 8 GPUs are fully connected by point-to-point xGMI links, so a TP group of
2/4/8 adjacent ranks always sits on direct links; keep TP inside one node and let DP/PP span nodes.

The layout math lives in :class:`ParallelTopology` (pure python, unit-testable without any
process group); :func:`initialize_model_parallel` instantiates it and creates the RCCL groups.
"""
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from .utils import ensure_divisibility

_TENSOR_MODEL_PARALLEL_GROUP = None
_PIPELINE_MODEL_PARALLEL_GROUP = None
_MODEL_PARALLEL_GROUP = None
_EMBEDDING_GROUP = None
_POSITION_EMBEDDING_GROUP = None
_DATA_PARALLEL_GROUP = None

_VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = None
_VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
_PIPELINE_MODEL_PARALLEL_SPLIT_RANK = None

_MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE = None
_MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
_MPU_TENSOR_MODEL_PARALLEL_RANK = None
_MPU_PIPELINE_MODEL_PARALLEL_RANK = None

_EMBEDDING_GLOBAL_RANKS = None
_POSITION_EMBEDDING_GLOBAL_RANKS = None
_PIPELINE_GLOBAL_RANKS = None
_DATA_PARALLEL_GLOBAL_RANKS = None
_TOPOLOGY = None


@dataclass(frozen=True)
class ParallelTopology:
    world_size: int
    tensor_model_parallel_size: int = 1
    pipeline_model_parallel_size: int = 1

    def __post_init__(self):
        ensure_divisibility(self.world_size, self.tensor_model_parallel_size * self.pipeline_model_parallel_size)

    @property
    def data_parallel_size(self) -> int:
        return self.world_size // (self.tensor_model_parallel_size * self.pipeline_model_parallel_size)

    def coords(self, rank: int) -> Tuple[int, int, int]:
        """(tp_rank, pp_rank, dp_rank) of a global rank."""
        tp = self.tensor_model_parallel_size
        dp = self.data_parallel_size
        return rank % tp, rank // (tp * dp), (rank // tp) % dp

    def rank_of(self, tp_rank: int, pp_rank: int, dp_rank: int) -> int:
        tp = self.tensor_model_parallel_size
        return pp_rank * (self.data_parallel_size * tp) + dp_rank * tp + tp_rank

    def tensor_groups(self) -> List[List[int]]:
        tp = self.tensor_model_parallel_size
        return [list(range(i * tp, (i + 1) * tp)) for i in range(self.world_size // tp)]

    def data_groups(self) -> List[List[int]]:
        tp, pp, dp = self.tensor_model_parallel_size, self.pipeline_model_parallel_size, self.data_parallel_size
        return [[self.rank_of(t, p, d) for d in range(dp)] for p in range(pp) for t in range(tp)]

    def pipeline_groups(self) -> List[List[int]]:
        n = self.world_size // self.pipeline_model_parallel_size
        return [list(range(i, self.world_size, n)) for i in range(n)]

    def model_groups(self) -> List[List[int]]:
        tp, pp = self.tensor_model_parallel_size, self.pipeline_model_parallel_size
        return [[self.rank_of(t, p, d) for p in range(pp) for t in range(tp)] for d in range(self.data_parallel_size)]

    @staticmethod
    def embedding_ranks(pipeline_ranks: List[int], split_rank: Optional[int] = None) -> List[int]:
        if len(pipeline_ranks) == 1:
            return list(pipeline_ranks)
        ranks = [pipeline_ranks[0], pipeline_ranks[-1]]
        if split_rank is not None and pipeline_ranks[split_rank] not in ranks:
            ranks = [pipeline_ranks[0], pipeline_ranks[split_rank], pipeline_ranks[-1]]
        return ranks


def is_unitialized():
    """Useful for code segments that may be accessed with or without mpu initialization."""
    return _DATA_PARALLEL_GROUP is None


def initialize_model_parallel(tensor_model_parallel_size_=1, pipeline_model_parallel_size_=1,
                              virtual_pipeline_model_parallel_size_=None, pipeline_model_parallel_split_rank_=None,
                              *, default_backend=None, p2p_backend=None):
    """Create the TP / PP / DP / model-parallel / embedding groups for this process.

    With 16 ranks, tp=2 and pp=4: 8 TP groups [g0,g1],[g2,g3],...; 8 DP groups [g0,g2],[g1,g3],
    [g4,g6],...; 4 PP groups [g0,g4,g8,g12],... (reference docstring :66-84)."""
    assert torch.distributed.is_initialized()
    world_size = torch.distributed.get_world_size()
    tp = min(tensor_model_parallel_size_, world_size)
    pp = min(pipeline_model_parallel_size_, world_size)
    topo = ParallelTopology(world_size, tp, pp)
    if torch.distributed.get_rank() == 0:
        print("> initializing tensor model parallel with size {}".format(tp))
        print("> initializing pipeline model parallel with size {}".format(pp))
        print("> initializing data parallel with size {}".format(topo.data_parallel_size))

    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK, _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    if virtual_pipeline_model_parallel_size_ is not None:
        assert pp > 2, "pipeline-model-parallel size should be greater than 2 with interleaved schedule"
        _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = 0
        _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = virtual_pipeline_model_parallel_size_
    global _PIPELINE_MODEL_PARALLEL_SPLIT_RANK
    if pipeline_model_parallel_split_rank_ is not None:
        _PIPELINE_MODEL_PARALLEL_SPLIT_RANK = pipeline_model_parallel_split_rank_

    rank = torch.distributed.get_rank()
    new_group = lambda ranks, backend=default_backend: torch.distributed.new_group(ranks, backend=backend)  # noqa: E731

    global _DATA_PARALLEL_GROUP, _DATA_PARALLEL_GLOBAL_RANKS
    assert _DATA_PARALLEL_GROUP is None, "data parallel group is already initialized"
    for ranks in topo.data_groups():  # every rank must take part in every new_group call
        g = new_group(ranks)
        if rank in ranks:
            _DATA_PARALLEL_GROUP = g
            _DATA_PARALLEL_GLOBAL_RANKS = ranks

    global _MODEL_PARALLEL_GROUP
    assert _MODEL_PARALLEL_GROUP is None, "model parallel group is already initialized"
    for ranks in topo.model_groups():
        g = new_group(ranks)
        if rank in ranks:
            _MODEL_PARALLEL_GROUP = g

    global _TENSOR_MODEL_PARALLEL_GROUP
    assert _TENSOR_MODEL_PARALLEL_GROUP is None, "tensor model parallel group is already initialized"
    for ranks in topo.tensor_groups():
        g = new_group(ranks)
        if rank in ranks:
            _TENSOR_MODEL_PARALLEL_GROUP = g

    global _PIPELINE_MODEL_PARALLEL_GROUP, _PIPELINE_GLOBAL_RANKS
    global _EMBEDDING_GROUP, _EMBEDDING_GLOBAL_RANKS, _POSITION_EMBEDDING_GROUP, _POSITION_EMBEDDING_GLOBAL_RANKS
    assert _PIPELINE_MODEL_PARALLEL_GROUP is None, "pipeline model parallel group is already initialized"
    assert _EMBEDDING_GROUP is None, "embedding group is already initialized"
    for ranks in topo.pipeline_groups():
        g = new_group(ranks, p2p_backend if p2p_backend is not None else default_backend)
        if rank in ranks:
            _PIPELINE_MODEL_PARALLEL_GROUP = g
            _PIPELINE_GLOBAL_RANKS = ranks
        emb = topo.embedding_ranks(ranks, _PIPELINE_MODEL_PARALLEL_SPLIT_RANK)
        g = new_group(emb)
        if rank in emb:
            _EMBEDDING_GROUP = g
        if rank in ranks:
            _EMBEDDING_GLOBAL_RANKS = emb
        pos = ranks[:1]
        if _PIPELINE_MODEL_PARALLEL_SPLIT_RANK is not None and len(ranks) > 1:
            pos = [ranks[0], ranks[_PIPELINE_MODEL_PARALLEL_SPLIT_RANK]]
        g = new_group(pos)
        if rank in pos:
            _POSITION_EMBEDDING_GROUP = g
        if rank in ranks:
            _POSITION_EMBEDDING_GLOBAL_RANKS = pos
    global _TOPOLOGY
    _TOPOLOGY = topo


def get_topology() -> Optional[ParallelTopology]:
    return _TOPOLOGY


def get_rank_info() -> Tuple[int, int, int]:
    """(tensor, pipeline, data)-parallel rank of this process, for the logger."""
    if model_parallel_is_initialized():
        return (get_tensor_model_parallel_rank(), get_pipeline_model_parallel_rank(), get_data_parallel_rank())
    return (0, 0, 0)


def model_parallel_is_initialized():
    return not (_TENSOR_MODEL_PARALLEL_GROUP is None or _PIPELINE_MODEL_PARALLEL_GROUP is None
                or _DATA_PARALLEL_GROUP is None)


def get_model_parallel_group():
    assert _MODEL_PARALLEL_GROUP is not None, "model parallel group is not initialized"
    return _MODEL_PARALLEL_GROUP


def get_tensor_model_parallel_group():
    assert _TENSOR_MODEL_PARALLEL_GROUP is not None, "intra_layer_model parallel group is not initialized"
    return _TENSOR_MODEL_PARALLEL_GROUP


def get_pipeline_model_parallel_group():
    assert _PIPELINE_MODEL_PARALLEL_GROUP is not None, "pipeline_model parallel group is not initialized"
    return _PIPELINE_MODEL_PARALLEL_GROUP


def get_data_parallel_group():
    assert _DATA_PARALLEL_GROUP is not None, "data parallel group is not initialized"
    return _DATA_PARALLEL_GROUP


def get_embedding_group():
    assert _EMBEDDING_GROUP is not None, "embedding group is not initialized"
    return _EMBEDDING_GROUP


def get_position_embedding_group():
    assert _POSITION_EMBEDDING_GROUP is not None, "position embedding group is not initialized"
    return _POSITION_EMBEDDING_GROUP


def is_rank_in_embedding_group(ignore_virtual=False):
    rank = torch.distributed.get_rank()
    if ignore_virtual:
        return rank in _EMBEDDING_GLOBAL_RANKS
    if rank in _EMBEDDING_GLOBAL_RANKS:
        if rank == _EMBEDDING_GLOBAL_RANKS[0]:
            return is_pipeline_first_stage(ignore_virtual=False)
        if rank == _EMBEDDING_GLOBAL_RANKS[-1]:
            return is_pipeline_last_stage(ignore_virtual=False)
        return True
    return False


def is_rank_in_position_embedding_group():
    return torch.distributed.get_rank() in (_POSITION_EMBEDDING_GLOBAL_RANKS or [])


def is_pipeline_stage_before_split(rank=None):
    if get_pipeline_model_parallel_world_size() == 1:
        return True
    if rank is None:
        rank = get_pipeline_model_parallel_rank()
    if _PIPELINE_MODEL_PARALLEL_SPLIT_RANK is None:
        return True
    return rank < _PIPELINE_MODEL_PARALLEL_SPLIT_RANK


def is_pipeline_stage_after_split(rank=None):
    if get_pipeline_model_parallel_world_size() == 1:
        return True
    if rank is None:
        rank = get_pipeline_model_parallel_rank()
    if _PIPELINE_MODEL_PARALLEL_SPLIT_RANK is None:
        return True
    return rank >= _PIPELINE_MODEL_PARALLEL_SPLIT_RANK


def set_tensor_model_parallel_world_size(world_size):
    global _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE
    _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE = world_size


def set_pipeline_model_parallel_world_size(world_size):
    global _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = world_size


def get_tensor_model_parallel_world_size():
    if _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE is not None:
        return _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE
    return torch.distributed.get_world_size(group=get_tensor_model_parallel_group())


def get_pipeline_model_parallel_world_size():
    if _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE is not None:
        return _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    return torch.distributed.get_world_size(group=get_pipeline_model_parallel_group())


def set_tensor_model_parallel_rank(rank):
    global _MPU_TENSOR_MODEL_PARALLEL_RANK
    _MPU_TENSOR_MODEL_PARALLEL_RANK = rank


def set_pipeline_model_parallel_rank(rank):
    global _MPU_PIPELINE_MODEL_PARALLEL_RANK
    _MPU_PIPELINE_MODEL_PARALLEL_RANK = rank


def get_tensor_model_parallel_rank():
    if _MPU_TENSOR_MODEL_PARALLEL_RANK is not None:
        return _MPU_TENSOR_MODEL_PARALLEL_RANK
    return torch.distributed.get_rank(group=get_tensor_model_parallel_group())


def get_pipeline_model_parallel_rank():
    if _MPU_PIPELINE_MODEL_PARALLEL_RANK is not None:
        return _MPU_PIPELINE_MODEL_PARALLEL_RANK
    return torch.distributed.get_rank(group=get_pipeline_model_parallel_group())


def get_pipeline_model_parallel_split_rank():
    return _PIPELINE_MODEL_PARALLEL_SPLIT_RANK


def set_pipeline_model_parallel_split_rank(rank):
    global _PIPELINE_MODEL_PARALLEL_SPLIT_RANK
    _PIPELINE_MODEL_PARALLEL_SPLIT_RANK = rank


def is_pipeline_first_stage(ignore_virtual=False):
    if not ignore_virtual:
        if (get_virtual_pipeline_model_parallel_world_size() is not None
                and get_virtual_pipeline_model_parallel_rank() != 0):
            return False
    return get_pipeline_model_parallel_rank() == 0


def is_pipeline_last_stage(ignore_virtual=False):
    if not ignore_virtual:
        vws = get_virtual_pipeline_model_parallel_world_size()
        if vws is not None and get_virtual_pipeline_model_parallel_rank() != (vws - 1):
            return False
    return get_pipeline_model_parallel_rank() == (get_pipeline_model_parallel_world_size() - 1)


def get_virtual_pipeline_model_parallel_rank():
    return _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK


def set_virtual_pipeline_model_parallel_rank(rank):
    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK
    _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = rank


def get_virtual_pipeline_model_parallel_world_size():
    return _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE


def set_virtual_pipeline_model_parallel_world_size(size):
    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = size


def get_tensor_model_parallel_src_rank():
    """Global rank of the first rank of this process's TP group."""
    global_rank = torch.distributed.get_rank()
    local_world_size = get_tensor_model_parallel_world_size()
    return (global_rank // local_world_size) * local_world_size


def get_data_parallel_src_rank():
    assert _DATA_PARALLEL_GLOBAL_RANKS is not None, "data parallel group is not initialized"
    return _DATA_PARALLEL_GLOBAL_RANKS[0]


def get_pipeline_model_parallel_first_rank():
    assert _PIPELINE_GLOBAL_RANKS is not None, "Pipeline parallel group is not initialized"
    return _PIPELINE_GLOBAL_RANKS[0]


def get_pipeline_model_parallel_last_rank():
    assert _PIPELINE_GLOBAL_RANKS is not None, "Pipeline parallel group is not initialized"
    return _PIPELINE_GLOBAL_RANKS[get_pipeline_model_parallel_world_size() - 1]


def get_pipeline_model_parallel_next_rank():
    assert _PIPELINE_GLOBAL_RANKS is not None, "Pipeline parallel group is not initialized"
    rank_in_pipeline = get_pipeline_model_parallel_rank()
    world_size = get_pipeline_model_parallel_world_size()
    return _PIPELINE_GLOBAL_RANKS[(rank_in_pipeline + 1) % world_size]


def get_pipeline_model_parallel_prev_rank():
    assert _PIPELINE_GLOBAL_RANKS is not None, "Pipeline parallel group is not initialized"
    rank_in_pipeline = get_pipeline_model_parallel_rank()
    world_size = get_pipeline_model_parallel_world_size()
    return _PIPELINE_GLOBAL_RANKS[(rank_in_pipeline - 1) % world_size]


def get_data_parallel_world_size():
    return torch.distributed.get_world_size(group=get_data_parallel_group())


def get_data_parallel_rank():
    return torch.distributed.get_rank(group=get_data_parallel_group())


def destroy_model_parallel():
    """Forget every group (the process groups themselves are owned by torch.distributed)."""
    global _MODEL_PARALLEL_GROUP, _TENSOR_MODEL_PARALLEL_GROUP, _PIPELINE_MODEL_PARALLEL_GROUP
    global _DATA_PARALLEL_GROUP, _EMBEDDING_GROUP, _POSITION_EMBEDDING_GROUP
    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK, _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    global _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE, _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    global _MPU_TENSOR_MODEL_PARALLEL_RANK, _MPU_PIPELINE_MODEL_PARALLEL_RANK, _PIPELINE_MODEL_PARALLEL_SPLIT_RANK
    global _EMBEDDING_GLOBAL_RANKS, _POSITION_EMBEDDING_GLOBAL_RANKS, _PIPELINE_GLOBAL_RANKS
    global _DATA_PARALLEL_GLOBAL_RANKS, _TOPOLOGY
    _MODEL_PARALLEL_GROUP = None
    _TENSOR_MODEL_PARALLEL_GROUP = None
    _PIPELINE_MODEL_PARALLEL_GROUP = None
    _DATA_PARALLEL_GROUP = None
    _EMBEDDING_GROUP = None
    _POSITION_EMBEDDING_GROUP = None
    _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = None
    _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
    _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE = None
    _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
    _MPU_TENSOR_MODEL_PARALLEL_RANK = None
    _MPU_PIPELINE_MODEL_PARALLEL_RANK = None
    _PIPELINE_MODEL_PARALLEL_SPLIT_RANK = None
    _EMBEDDING_GLOBAL_RANKS = None
    _POSITION_EMBEDDING_GLOBAL_RANKS = None
    _PIPELINE_GLOBAL_RANKS = None
    _DATA_PARALLEL_GLOBAL_RANKS = None
    _TOPOLOGY = None
