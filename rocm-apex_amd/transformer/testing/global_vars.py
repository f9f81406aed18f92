"""Megatron global singletons for the standalone models (reference
apex/transformer/testing/global_vars.py:34-270): args, microbatch calculator, tensorboard
writer, autoresume and timers."""
import time

import torch

from ..microbatches import build_num_microbatches_calculator
from .arguments import parse_args

_GLOBAL_ARGS = None
_GLOBAL_NUM_MICROBATCHES_CALCULATOR = None
_GLOBAL_TENSORBOARD_WRITER = None
_GLOBAL_ADLR_AUTORESUME = None
_GLOBAL_TIMERS = None


def _ensure_var_is_initialized(var, name):
    assert var is not None, "{} is not initialized.".format(name)


def _ensure_var_is_not_initialized(var, name):
    assert var is None, "{} is already initialized.".format(name)


def get_args():
    _ensure_var_is_initialized(_GLOBAL_ARGS, "args")
    return _GLOBAL_ARGS


def get_num_microbatches():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get()


def get_current_global_batch_size():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get_current_global_batch_size()


def update_num_microbatches(consumed_samples, *, consistency_check=True):
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR.update(consumed_samples, consistency_check)


def get_tensorboard_writer():
    return _GLOBAL_TENSORBOARD_WRITER


def get_adlr_autoresume():
    return _GLOBAL_ADLR_AUTORESUME


def get_timers():
    _ensure_var_is_initialized(_GLOBAL_TIMERS, "timers")
    return _GLOBAL_TIMERS


def set_global_variables(extra_args_provider=None, args_defaults=None, override_args=None, ignore_unknown_args=False,
                         argv=None):
    global _GLOBAL_ARGS, _GLOBAL_NUM_MICROBATCHES_CALCULATOR, _GLOBAL_TIMERS
    args = parse_args(extra_args_provider, args_defaults or {}, override_args or {}, ignore_unknown_args, argv)
    _GLOBAL_ARGS = args
    if args.micro_batch_size is not None and args.global_batch_size is not None:
        _GLOBAL_NUM_MICROBATCHES_CALCULATOR = build_num_microbatches_calculator(
            args.rank, args.rampup_batch_size, args.global_batch_size, args.micro_batch_size, args.data_parallel_size)
    _set_tensorboard_writer(args)
    _GLOBAL_TIMERS = Timers()
    return args


def destroy_global_vars():
    global _GLOBAL_ARGS, _GLOBAL_NUM_MICROBATCHES_CALCULATOR, _GLOBAL_TENSORBOARD_WRITER, _GLOBAL_TIMERS
    _GLOBAL_ARGS = _GLOBAL_NUM_MICROBATCHES_CALCULATOR = _GLOBAL_TENSORBOARD_WRITER = _GLOBAL_TIMERS = None


def _set_tensorboard_writer(args):
    global _GLOBAL_TENSORBOARD_WRITER
    if getattr(args, "tensorboard_dir", None) and args.rank == args.world_size - 1:
        try:
            from torch.utils.tensorboard import SummaryWriter

            _GLOBAL_TENSORBOARD_WRITER = SummaryWriter(log_dir=args.tensorboard_dir,
                                                       max_queue=args.tensorboard_queue_size)
        except Exception:  # tensorboard not installed
            _GLOBAL_TENSORBOARD_WRITER = None


class _Timer:
    """Device-synchronised wall timer."""

    def __init__(self, name):
        self.name_ = name
        self.elapsed_ = 0.0
        self.started_ = False
        self.start_time = time.time()

    def _sync(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def start(self):
        assert not self.started_, "timer has already been started"
        self._sync()
        self.start_time = time.time()
        self.started_ = True

    def stop(self):
        assert self.started_, "timer is not started"
        self._sync()
        self.elapsed_ += time.time() - self.start_time
        self.started_ = False

    def reset(self):
        self.elapsed_ = 0.0
        self.started_ = False

    def elapsed(self, reset=True):
        started = self.started_
        if started:
            self.stop()
        e = self.elapsed_
        if reset:
            self.reset()
        if started:
            self.start()
        return e


class Timers:
    def __init__(self):
        self.timers = {}

    def __call__(self, name):
        if name not in self.timers:
            self.timers[name] = _Timer(name)
        return self.timers[name]

    def write(self, names, writer, iteration, normalizer=1.0, reset=False):
        for n in names:
            writer.add_scalar(n + "-time", self.timers[n].elapsed(reset=reset) / normalizer, iteration)

    def log(self, names, normalizer=1.0, reset=True):
        s = "time (ms)"
        for n in names:
            s += " | {}: {:.2f}".format(n, self.timers[n].elapsed(reset=reset) * 1000.0 / normalizer)
        if not torch.distributed.is_initialized() or torch.distributed.get_rank() == torch.distributed.get_world_size() - 1:
            print(s, flush=True)
