"""Process-global amp state shared by the amp modules (reference apex/amp/_amp_state.py:1-57)."""
import collections.abc as container_abcs  # noqa: F401  (re-exported for compat)
import os

import torch


class AmpState(object):
    def __init__(self):
        self.hard_override = False
        self.allow_incoming_model_not_fp32 = False
        self.verbosity = 1
        # MI355X addition: keep the dynamic loss scaler on the device (no per-step .item()) when
        # every optimizer handed to amp can consume a device skip flag.
        # "0" = reference (sync) scaler; "force" = sync-free even without a GPU (the device-side
        # scaler then runs its torch reference ops on the CPU: used by the CPU test tier)
        self.sync_free_requested = os.environ.get("APEX_AMD_AMP_SYNC_FREE", "1") != "0"
        self.sync_free_force = os.environ.get("APEX_AMD_AMP_SYNC_FREE", "1") == "force"
        self.sync_free = False
        self.loss_scalers = []


_amp_state = AmpState()


def warn_or_err(msg):
    if _amp_state.hard_override:
        print("Warning:  " + msg)
    else:
        raise RuntimeError(msg)


def _is_distributed():
    return (torch.distributed.is_available() and torch.distributed.is_initialized()
            and torch.distributed.get_world_size() > 1)


def maybe_print(msg, rank0=False):
    if _amp_state.verbosity > 0:
        if rank0 and _is_distributed():
            if torch.distributed.get_rank() == 0:
                print(msg)
        else:
            print(msg)


def master_params(optimizer):
    """Iterates over the params owned by ``optimizer`` (fp32 masters under O2/O5)."""
    for group in optimizer.param_groups:
        for p in group["params"]:
            yield p
