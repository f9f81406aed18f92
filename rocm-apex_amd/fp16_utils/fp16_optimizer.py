"""Legacy ``FP16_Optimizer`` (reference apex/fp16_utils/fp16_optimizer.py:13-554).

Wraps any optimizer: fp16/bf16 params are swapped for fp32 masters, ``backward()`` scales the
loss, ``update_master_grads()`` unscales into the masters with overflow detection (the
multi-tensor kernels on GPU, torch reference on CPU), ``step()`` skips on overflow and copies the
masters back.  ``state_dict()`` saves the scaler state and the fp32 masters.
Works on CPU tensors too (BASELINE config #1 runs it without a GPU)."""
import torch

from ..amp._amp_state import maybe_print
from ..amp.scaler import LossScaler
from .. import amp_C
from .fp16util import clip_grad_norm, master_params_to_model_params

_LOW = (torch.float16, torch.bfloat16)


class FP16_Optimizer(object):
    def __init__(self, init_optimizer, static_loss_scale=1.0, dynamic_loss_scale=False, dynamic_loss_args=None,
                 verbose=True):
        print("Warning:  FP16_Optimizer is deprecated and dangerous, and will be deleted soon.  "
              "If it still works, you're probably getting lucky.  "
              "For mixed precision, use amp.initialize with opt_level=O1/O2/O5.")
        self.verbose = verbose
        self.optimizer = init_optimizer
        self.fp16_groups = []
        self.fp32_from_fp16_groups = []
        self.fp32_from_fp32_groups = []
        for i, param_group in enumerate(self.optimizer.param_groups):
            self.maybe_print("FP16_Optimizer processing param group {}:".format(i))
            fp16_this, fp32_this, fp32_from_fp16_this = [], [], []
            for j, param in enumerate(param_group["params"]):
                if not param.requires_grad:
                    continue
                if param.dtype in _LOW:
                    self.maybe_print("FP16_Optimizer received {} with {}".format(param.type(), param.size()))
                    fp16_this.append(param)
                    master = param.detach().clone().float()
                    master.requires_grad = True
                    param_group["params"][j] = master
                    fp32_from_fp16_this.append(master)
                    if param in self.optimizer.state:
                        self.optimizer.state[master] = self.optimizer.state.pop(param)
                elif param.dtype == torch.float32:
                    self.maybe_print("FP16_Optimizer received {} with {}".format(param.type(), param.size()))
                    fp32_this.append(param)
                    param_group["params"][j] = param
                else:
                    raise TypeError("Wrapped parameters must be float32, float16 or bfloat16. "
                                    "Received {}".format(param.type()))
            self.fp16_groups.append(fp16_this)
            self.fp32_from_fp16_groups.append(fp32_from_fp16_this)
            self.fp32_from_fp32_groups.append(fp32_this)
        self.all_fp16_params = [p for g in self.fp16_groups for p in g]
        self.all_fp32_from_fp16_params = [p for g in self.fp32_from_fp16_groups for p in g]
        self.all_fp32_from_fp32_params = [p for g in self.fp32_from_fp32_groups for p in g]
        self.optimizer.load_state_dict(self.optimizer.state_dict())
        if dynamic_loss_scale:
            self.dynamic_loss_scale = True
            self.loss_scaler = LossScaler("dynamic", **(dynamic_loss_args or {}))
        else:
            self.dynamic_loss_scale = False
            self.loss_scaler = LossScaler(static_loss_scale)
        self.overflow = False
        self.first_closure_call_this_step = True
        self.clip_grad_norm = clip_grad_norm
        dev = self.all_fp16_params[0].device if self.all_fp16_params else (
            self.all_fp32_from_fp32_params[0].device if self.all_fp32_from_fp32_params else "cpu")
        self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int32, device=dev)

    def maybe_print(self, msg):
        if self.verbose:
            print(msg)

    def __getstate__(self):
        raise RuntimeError("FP16_Optimizer should be serialized using state_dict().")

    def __setstate__(self, state):
        raise RuntimeError("FP16_Optimizer should be deserialized using load_state_dict().")

    def zero_grad(self, set_grads_to_None=False):
        groups = [g["params"] for g in self.optimizer.param_groups] + self.fp16_groups
        for params in groups:
            for p in params:
                if set_grads_to_None:
                    p.grad = None
                elif p.grad is not None:
                    if p.grad.grad_fn is not None:
                        p.grad.detach_()  # grads may be DDP bucket views
                    else:
                        p.grad.requires_grad_(False)
                    p.grad.zero_()

    def _master_params_to_model_params(self):
        if self.all_fp16_params:
            amp_C.multi_tensor_scale(65536, self._dummy_overflow_buf,
                                     [self.all_fp32_from_fp16_params, self.all_fp16_params], 1.0)

    def clip_master_grads(self, max_norm, norm_type=2):
        if self.overflow:
            return -1
        fp32_params = [p for g in self.optimizer.param_groups for p in g["params"]]
        return self.clip_grad_norm(fp32_params, max_norm, norm_type)

    def state_dict(self):
        return {
            "loss_scaler": {"loss_scale": self.loss_scaler.loss_scale(), "unskipped": self.loss_scaler._unskipped,
                            "dynamic": self.loss_scaler.dynamic},
            "dynamic_loss_scale": self.dynamic_loss_scale,
            "overflow": self.overflow,
            "first_closure_call_this_step": self.first_closure_call_this_step,
            "optimizer_state_dict": self.optimizer.state_dict(),
            "fp32_from_fp16": self.fp32_from_fp16_groups,
        }

    def load_state_dict(self, state_dict):
        ls = state_dict["loss_scaler"]
        if isinstance(ls, LossScaler):
            self.loss_scaler = ls
        else:
            self.loss_scaler.load(ls["loss_scale"], ls["unskipped"])
        self.dynamic_loss_scale = state_dict["dynamic_loss_scale"]
        self.overflow = state_dict["overflow"]
        self.first_closure_call_this_step = state_dict["first_closure_call_this_step"]
        self.optimizer.load_state_dict(state_dict["optimizer_state_dict"])
        for current_group, saved_group in zip(self.fp32_from_fp16_groups, state_dict["fp32_from_fp16"]):
            for current, saved in zip(current_group, saved_group):
                current.data.copy_(saved.data)

    def step(self, closure=None):
        if self.overflow:
            maybe_print("Gradient overflow.  Skipping step, reducing loss scale to {}".format(
                self.loss_scaler.loss_scale()))
            return
        retval = self._step_with_closure(closure) if closure is not None else self.optimizer.step()
        self._master_params_to_model_params()
        return retval

    def _step_with_closure(self, closure):
        def wrapped_closure():
            if self.first_closure_call_this_step:
                self.first_closure_call_this_step = False
            else:
                self._master_params_to_model_params()
            temp_loss = closure()
            while self.overflow:
                print("OVERFLOW within closure! Skipping step, reducing loss scale to {}".format(
                    self.loss_scaler.loss_scale()))
                temp_loss = closure()
            return temp_loss

        retval = self.optimizer.step(wrapped_closure)
        self.first_closure_call_this_step = True
        return retval

    def backward(self, loss, update_master_grads=True, retain_graph=False):
        scaled_loss = loss.float() * self.loss_scaler.loss_scale()
        scaled_loss.backward(retain_graph=retain_graph)
        if update_master_grads:
            self.update_master_grads()

    def update_master_grads(self):
        self.loss_scaler.clear_overflow_state()
        if self.all_fp16_params:
            model_grads, master_grads = [], []
            for model_param, master_param in zip(self.all_fp16_params, self.all_fp32_from_fp16_params):
                if model_param.grad is not None:
                    model_grads.append(model_param.grad)
                    if master_param.grad is None:
                        master_param.grad = torch.empty_like(master_param)
                    master_grads.append(master_param.grad)
            self.loss_scaler.unscale(model_grads, master_grads, self.loss_scaler.loss_scale())
        if self.all_fp32_from_fp32_params:
            grads = [p.grad for p in self.all_fp32_from_fp32_params if p.grad is not None]
            self.loss_scaler.unscale(grads, grads, self.loss_scaler.loss_scale())
        self.overflow = self.loss_scaler.update_scale()

    def inspect_master_grad_data(self):
        if self.overflow:
            print("Warning:  calling FP16_Optimizer.inspect_master_grad_data while in an overflow state.  "
                  "Gradients are currently invalid (may be inf, nan, or stale).  Returning None.")
            return None
        return [[p.grad.data if p.grad is not None else None for p in g["params"]]
                for g in self.optimizer.param_groups]

    def _get_loss_scale(self):
        return self.loss_scaler.loss_scale()

    def _set_loss_scale(self, value):
        self.loss_scaler._loss_scale = value

    loss_scale = property(_get_loss_scale, _set_loss_scale)

    def _get_state(self):
        return self.optimizer.state

    def _set_state(self, value):
        self.optimizer.state = value

    state = property(_get_state, _set_state)

    def _get_param_groups(self):
        return self.optimizer.param_groups

    def _set_param_groups(self, value):
        self.optimizer.param_groups = value

    param_groups = property(_get_param_groups, _set_param_groups)
