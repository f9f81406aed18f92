"""Pipeline-parallel utilities (reference apex/transformer/pipeline_parallel/utils.py:41-333):
micro-batch calculator globals, micro-batch slicing, timers, parameter-norm / loss averaging
over the model / data-parallel groups, memory report, left-to-right masks."""
from typing import List, Optional, Union

import torch
from torch.nn.parallel import DistributedDataParallel

from ... import amp_C
from .. import parallel_state
from ..microbatches import build_num_microbatches_calculator
from ..tensor_parallel.layers import param_is_not_tensor_parallel_duplicate
from ..utils import comm_device
from ._timers import _Timers

_GLOBAL_ARGS = None
_GLOBAL_NUM_MICROBATCHES_CALCULATOR = None
_GLOBAL_TOKENIZER = None
_GLOBAL_TENSORBOARD_WRITER = None
_GLOBAL_AUTORESUME = None
_GLOBAL_TIMERS = None

Shape = Union[List[int], torch.Size]


def listify_model(model: Union[torch.nn.Module, List[torch.nn.Module]]) -> List[torch.nn.Module]:
    if isinstance(model, list):
        return model
    return [model]


def _ensure_var_is_initialized(var, name):
    assert var is not None, "{} is not initialized.".format(name)


def _ensure_var_is_not_initialized(var, name):
    assert var is None, "{} is already initialized.".format(name)


def setup_microbatch_calculator(rank: int, rampup_batch_size: Optional[List[int]], global_batch_size: int,
                                micro_batch_size: int, data_parallel_size: int) -> None:
    global _GLOBAL_NUM_MICROBATCHES_CALCULATOR
    _ensure_var_is_not_initialized(_GLOBAL_NUM_MICROBATCHES_CALCULATOR, "num microbatches calculator")
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR = build_num_microbatches_calculator(
        rank, rampup_batch_size, global_batch_size, micro_batch_size, data_parallel_size)


def _reconfigure_microbatch_calculator(rank: int, rampup_batch_size: Optional[List[int]], global_batch_size: int,
                                       micro_batch_size: int, data_parallel_size: int) -> None:
    """For tests: replace the calculator unconditionally."""
    global _GLOBAL_NUM_MICROBATCHES_CALCULATOR
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR = build_num_microbatches_calculator(
        rank, rampup_batch_size, global_batch_size, micro_batch_size, data_parallel_size)


def destroy_microbatch_calculator():
    global _GLOBAL_NUM_MICROBATCHES_CALCULATOR
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR = None


def get_micro_batch_size():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.micro_batch_size


def get_num_microbatches():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get()


def get_current_global_batch_size():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get_current_global_batch_size()


def update_num_microbatches(consumed_samples, consistency_check=True):
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR.update(consumed_samples, consistency_check)


def _split_batch_into_microbatch(batch: List[torch.Tensor], *, _micro_batch_size: Optional[int] = None,
                                 _global_batch_size: Optional[int] = None):
    micro_batch_size = _micro_batch_size if _micro_batch_size is not None else get_micro_batch_size()
    global_batch_size = _global_batch_size if _global_batch_size is not None else get_current_global_batch_size()
    for i in range(0, global_batch_size // micro_batch_size):
        yield [x[i * micro_batch_size:(i + 1) * micro_batch_size] for x in batch]


def get_kth_microbatch(batch: List[torch.Tensor], k: int) -> List[torch.Tensor]:
    """The k-th micro-batch of a local mini-batch (``global_batch / dp`` samples)."""
    if batch is None or not isinstance(batch, (list, tuple)):
        return batch
    micro_batch_size = get_micro_batch_size()
    return [x[k * micro_batch_size:(k + 1) * micro_batch_size] for x in batch]


def get_autoresume():
    return _GLOBAL_AUTORESUME


def _set_timers():
    global _GLOBAL_TIMERS
    _ensure_var_is_not_initialized(_GLOBAL_TIMERS, "timers")
    _GLOBAL_TIMERS = _Timers()


def get_timers():
    global _GLOBAL_TIMERS
    if _GLOBAL_TIMERS is None:
        _GLOBAL_TIMERS = _Timers()
    return _GLOBAL_TIMERS


def print_rank_0(message: str) -> None:
    if torch.distributed.is_initialized():
        if torch.distributed.get_rank() == 0:
            print(message, flush=True)
    else:
        print(message, flush=True)


def is_last_rank():
    return torch.distributed.get_rank() == (torch.distributed.get_world_size() - 1)


def print_rank_last(message):
    if torch.distributed.is_initialized():
        if is_last_rank():
            print(message, flush=True)
    else:
        print(message, flush=True)


def param_is_not_shared(param: torch.nn.Parameter) -> bool:
    return not getattr(param, "shared", False)


def unwrap_model(model, module_instances=(DistributedDataParallel,)):
    return_list = True
    if not isinstance(model, list):
        model = [model]
        return_list = False
    unwrapped = []
    for m in model:
        while isinstance(m, module_instances):
            m = m.module
        unwrapped.append(m)
    return unwrapped if return_list else unwrapped[0]


def calc_params_l2_norm(model: torch.nn.Module, bf16: bool):
    """L2 norm of the (non-duplicated) parameters across the model-parallel group: one fused
    multi-tensor l2norm per dtype + one all-reduce."""
    if not isinstance(model, list):
        model = [model]
    by_dtype = {}
    for model_ in model:
        for param in model_.parameters():
            if param_is_not_shared(param) and param_is_not_tensor_parallel_duplicate(param):
                data = param.data.float() if bf16 else param.data
                by_dtype.setdefault(data.dtype, []).append(data)
    dev = comm_device()
    norm_2 = torch.zeros(1, dtype=torch.float32, device=dev)
    for params in by_dtype.values():
        flag = torch.zeros(1, dtype=torch.int32, device=params[0].device)
        norm, _ = amp_C.multi_tensor_l2norm(65536, flag, [params], False)
        norm_2 += (norm.float() * norm.float()).to(dev)
    torch.distributed.all_reduce(norm_2, op=torch.distributed.ReduceOp.SUM,
                                 group=parallel_state.get_model_parallel_group())
    return norm_2.item() ** 0.5


def average_losses_across_data_parallel_group(losses):
    averaged = torch.cat([loss.clone().detach().view(1) for loss in losses])
    torch.distributed.all_reduce(averaged, group=parallel_state.get_data_parallel_group())
    return averaged / torch.distributed.get_world_size(group=parallel_state.get_data_parallel_group())


def report_memory(name):
    mega_bytes = 1024.0 * 1024.0
    string = name + " memory (MB)"
    string += " | allocated: {}".format(torch.cuda.memory_allocated() / mega_bytes)
    string += " | max allocated: {}".format(torch.cuda.max_memory_allocated() / mega_bytes)
    string += " | reserved: {}".format(torch.cuda.memory_reserved() / mega_bytes)
    string += " | max reserved: {}".format(torch.cuda.max_memory_reserved() / mega_bytes)
    if parallel_state.get_data_parallel_rank() == 0:
        print("[Rank {}] {}".format(torch.distributed.get_rank(), string), flush=True)


def print_params_min_max_norm(optimizer, iteration):
    index = 0
    rank = torch.distributed.get_rank()
    string = "iteration, rank, index, tensor-model-parallel, min, max, norm\n"
    optimizer_ = getattr(optimizer, "optimizer", optimizer)
    for param_group in optimizer_.param_groups:
        for param in param_group["params"]:
            index += 1
            string += "{:7d}, {:4d}, {:4d}, {:2d}, ".format(iteration, rank, index,
                                                           int(getattr(param, "tensor_model_parallel", False)))
            string += "{:.6E}, {:.6E}, {:.6E}\n".format(param.data.min(), param.data.max(),
                                                         torch.linalg.norm(param.data))
    print(string, flush=True)


def get_ltor_masks_and_position_ids(data, eod_token, reset_position_ids, reset_attention_mask, eod_mask_loss):
    """Causal attention mask (True = masked), loss mask and position ids for a left-to-right LM."""
    micro_batch_size, seq_length = data.size()
    att_mask_batch = micro_batch_size if reset_attention_mask else 1
    attention_mask = torch.tril(torch.ones((att_mask_batch, seq_length, seq_length), device=data.device)).view(
        att_mask_batch, 1, seq_length, seq_length)
    loss_mask = torch.ones(data.size(), dtype=torch.float, device=data.device)
    if eod_mask_loss:
        loss_mask[data == eod_token] = 0.0
    position_ids = torch.arange(seq_length, dtype=torch.long, device=data.device)
    position_ids = position_ids.unsqueeze(0).expand_as(data)
    if reset_position_ids:
        position_ids = position_ids.clone()
    if reset_position_ids or reset_attention_mask:
        for b in range(micro_batch_size):
            eod_index = position_ids[b, data[b] == eod_token]
            if reset_position_ids:
                eod_index = eod_index.clone()
            prev_index = 0
            for j in range(eod_index.size()[0]):
                i = eod_index[j]
                if reset_attention_mask:
                    attention_mask[b, 0, (i + 1):, :(i + 1)] = 0
                if reset_position_ids:
                    position_ids[b, (i + 1):] -= i + 1 - prev_index
                    prev_index = i + 1
    attention_mask = attention_mask < 0.5
    return attention_mask, loss_mask, position_ids
