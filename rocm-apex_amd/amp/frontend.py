"""``amp.initialize`` / ``amp.state_dict`` / ``amp.load_state_dict`` and the O0–O5 presets
(reference apex/amp/frontend.py:7-467).  The ``amp.state_dict()`` format is kept exactly:
``OrderedDict({'loss_scaler%d': {'loss_scale': float, 'unskipped': int}})``."""
from collections import OrderedDict

import torch

from ._amp_state import _amp_state, maybe_print, warn_or_err
from ._initialize import _initialize


class Properties(object):
    """Option bag whose setters validate combinations against the chosen opt_level."""

    def __init__(self):
        self.options = {
            "enabled": False,
            "opt_level": None,
            "cast_model_type": None,
            "patch_torch_functions": False,
            "patch_torch_functions_type": None,
            "keep_batchnorm_fp32": None,
            "master_weights": None,
            "loss_scale": 1.0,
        }

    def _update_options_dict(self, new_options):
        for k, v in new_options:
            if k in self.options:
                self.options[k] = v
            else:
                raise ValueError("Tried to set unexpected option {}".format(k))

    def __getattr__(self, name):
        if "options" in self.__dict__:
            options = self.__dict__["options"]
            if name in options:
                return options[name]
        raise AttributeError("'{}' object has no attribute '{}'".format(type(self).__name__, name))

    def __setattr__(self, name, value):
        if "options" not in self.__dict__:
            return super(Properties, self).__setattr__(name, value)
        if name not in self.options:
            return super(Properties, self).__setattr__(name, value)
        lvl = self.opt_level
        if name == "cast_model_type":
            if lvl in {"O1", "O4"} and value is not None and value is not False and value is not torch.float32:
                warn_or_err("O1 inserts casts around Torch functions rather than model weights, so with O1, "
                            "the model weights themselves should remain FP32. If you wish to cast the model "
                            "to a different type, use opt_level='O2' or 'O3'. cast_model_type was {}".format(value))
            self.options[name] = value
        elif name == "patch_torch_functions":
            if lvl not in {"O1", "O4"} and value:
                warn_or_err("Currently, patch_torch_functions=True should only be set by selecting "
                            "opt_level='O1' or 'O4'.")
            self.options[name] = value
        elif name == "patch_torch_functions_type":
            if lvl not in {"O1", "O4"} and value is not None:
                warn_or_err("Currently, patch_torch_functions_type should only be set by selecting "
                            "opt_level='O1' or 'O4'.")
            elif lvl == "O1" and value != torch.float16:
                warn_or_err("patch_torch_functions_type should only be set to torch.float16 for opt_level='O1.")
            elif lvl == "O4" and value != torch.bfloat16:
                warn_or_err("patch_torch_functions_type should only be set to torch.bfloat16 for opt_level='O4.")
            else:
                self.options[name] = value
        elif name == "keep_batchnorm_fp32":
            if lvl in {"O1", "O4"} and value is not None:
                warn_or_err("With opt_level O1 or O4, batchnorm functions are automatically patched to run in "
                            "FP32, so keep_batchnorm_fp32 should be None. keep_batchnorm_fp32 was {}".format(value))
            if value == "False":
                self.options[name] = False
            elif value == "True":
                self.options[name] = True
            else:
                assert value is True or value is False or value is None, \
                    "keep_batchnorm_fp32 must be a boolean, the string 'True' or 'False', or None, " \
                    "found keep_batchnorm_fp32={}".format(value)
                self.options[name] = value
        elif name == "master_weights":
            if lvl in {"O1", "O4"} and value is not None:
                warn_or_err("It doesn't make sense to use master_weights with O1 and O4 . With O1 and O4, your "
                            "model weights themselves should be FP32.")
            self.options[name] = value
        elif name == "loss_scale":
            self.options[name] = value if value == "dynamic" else float(value)
        else:
            self.options[name] = value


class _Preset(object):
    brief = ""
    more = ""
    values = {}

    def __call__(self, properties):
        for k, v in self.values:
            setattr(properties, k, v)
        return properties


class O3(_Preset):
    brief = "O3:  Pure FP16 training."
    more = ("Calls .half() on your model, converting the entire model to FP16. A casting operation is also "
            "inserted to cast incoming Tensors to FP16. Useful for establishing a performance ceiling.")
    values = (("enabled", True), ("opt_level", "O3"), ("cast_model_type", torch.float16),
              ("patch_torch_functions", False), ("patch_torch_functions_type", None),
              ("keep_batchnorm_fp32", False), ("master_weights", False), ("loss_scale", 1.0))


class O2(_Preset):
    brief = "O2:  FP16 training with FP32 batchnorm and FP32 master weights.\n"
    more = ("Converts the model (except batchnorms) to FP16, casts inputs to FP16, keeps FP32 master weights "
            "in the optimizer and copies them back into the model after each step.")
    values = (("enabled", True), ("opt_level", "O2"), ("cast_model_type", torch.float16),
              ("patch_torch_functions", False), ("patch_torch_functions_type", None),
              ("keep_batchnorm_fp32", True), ("master_weights", True), ("loss_scale", "dynamic"))


class O1(_Preset):
    brief = "O1:  Insert automatic casts around Pytorch functions and Tensor methods.\n"
    more = ("Model weights stay FP32; matmul/conv-like ops run in FP16 and numerically sensitive ops are "
            "forced to FP32.  The safest way to try mixed precision.")
    values = (("enabled", True), ("opt_level", "O1"), ("cast_model_type", None),
              ("patch_torch_functions", True), ("patch_torch_functions_type", torch.float16),
              ("keep_batchnorm_fp32", None), ("master_weights", None), ("loss_scale", "dynamic"))


class O0(_Preset):
    brief = "O0:  Pure FP32 training.\n"
    more = "Parameters are checked to be FP32; no casts are inserted."
    values = (("enabled", True), ("opt_level", "O0"), ("cast_model_type", torch.float32),
              ("patch_torch_functions", False), ("patch_torch_functions_type", None),
              ("keep_batchnorm_fp32", None), ("master_weights", False), ("loss_scale", 1.0))


class O4(_Preset):
    brief = "O4:  Insert automatic casts around Pytorch functions and Tensor methods.\n"
    more = ("As O1 with BFLOAT16 as the low-precision type.  Loss scaling is not required since bfloat16 "
            "has the same dynamic range as fp32.")
    values = (("enabled", True), ("opt_level", "O4"), ("cast_model_type", None),
              ("patch_torch_functions", True), ("patch_torch_functions_type", torch.bfloat16),
              ("keep_batchnorm_fp32", None), ("master_weights", None), ("loss_scale", 1))


class O5(_Preset):
    brief = "O5:  BFLOAT16 training with FP32 batchnorm and FP32 master weights.\n"
    more = ("As O2 with BFLOAT16 model weights: FP32 batchnorm, FP32 master weights, static loss scale 1.")
    values = (("enabled", True), ("opt_level", "O5"), ("cast_model_type", torch.bfloat16),
              ("patch_torch_functions", None), ("patch_torch_functions_type", None),
              ("keep_batchnorm_fp32", True), ("master_weights", True), ("loss_scale", 1))


opt_levels = {"O3": O3(), "O2": O2(), "O1": O1(), "O0": O0(), "O4": O4(), "O5": O5()}


def initialize(models, optimizers=None, enabled=True, opt_level="O1", cast_model_type=None,
               patch_torch_functions=None, patch_torch_functions_type=None, keep_batchnorm_fp32=None,
               master_weights=None, loss_scale=None, cast_model_outputs=None, num_losses=1, verbosity=1,
               min_loss_scale=None, max_loss_scale=2.0 ** 24):
    """Initialize models, optimizers and (for O1/O4) the cast policy for ``opt_level``.

    Any property keyword that is not None overrides the preset.  Must be called before wrapping
    the model in a DistributedDataParallel.  Returns model(s) and optimizer(s) in the shape they
    were passed (single object or list).  See reference apex/amp/frontend.py:258-425."""
    _amp_state.opt_properties = Properties()
    _amp_state.verbosity = verbosity
    if not enabled:
        return models if optimizers is None else (models, optimizers)
    if opt_level not in opt_levels:
        raise RuntimeError("Unexpected optimization level {}. Options are 'O0', 'O1', 'O2', 'O3', 'O4', 'O5'.  "
                           "Note that in `O0`, `O1`, etc., the prefix O is the letter O, not the number zero."
                           .format(opt_level))
    _amp_state.opt_properties = opt_levels[opt_level](_amp_state.opt_properties)
    maybe_print("Selected optimization level {}".format(opt_levels[opt_level].brief), True)
    maybe_print("Defaults for this optimization level are:", True)
    for k, v in _amp_state.opt_properties.options.items():
        maybe_print("{:26} : {}".format(k, v), True)
    _amp_state.min_loss_scale = min_loss_scale
    _amp_state.max_loss_scale = max_loss_scale
    maybe_print("Processing user overrides (additional kwargs that are not None)...", True)
    props = _amp_state.opt_properties
    for name, val in (("enabled", enabled), ("opt_level", opt_level), ("cast_model_type", cast_model_type),
                      ("patch_torch_functions", patch_torch_functions),
                      ("patch_torch_functions_type", patch_torch_functions_type),
                      ("keep_batchnorm_fp32", keep_batchnorm_fp32), ("master_weights", master_weights),
                      ("loss_scale", loss_scale)):
        if val is not None:
            setattr(props, name, val)
    maybe_print("After processing overrides, optimization options are:", True)
    for k, v in props.options.items():
        maybe_print("{:26} : {}".format(k, v), True)
    return _initialize(models, optimizers, props, num_losses, cast_model_outputs)


def state_dict(destination=None):
    if destination is None:
        destination = OrderedDict()
    for idx, loss_scaler in enumerate(_amp_state.loss_scalers):
        st = loss_scaler.state()
        destination["loss_scaler%d" % idx] = {"loss_scale": st["loss_scale"], "unskipped": st["unskipped"]}
    return destination


def load_state_dict(state_dict):
    if len(state_dict) != len(_amp_state.loss_scalers):
        print("Warning: state_dict contains {} entries, while {} loss_scalers are used".format(
            len(state_dict), len(_amp_state.loss_scalers)))
    state_dict = state_dict.copy()
    nb = len(_amp_state.loss_scalers)
    unexpected = []
    idx = 0
    for key in state_dict:
        if "loss_scaler" not in key:
            unexpected.append(key)
        else:
            if idx > nb - 1:
                print("Skipping loss_scaler[{}], since num_losses was set to {}".format(idx, nb))
                break
            _amp_state.loss_scalers[idx].load(state_dict[key]["loss_scale"], state_dict[key]["unskipped"])
            idx += 1
    if unexpected:
        raise RuntimeError("Error(s) in loading state_dict. Unexpected key(s) in state_dict: {}. ".format(
            ", ".join('"{}"'.format(k) for k in unexpected)))
