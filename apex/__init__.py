"""Import shim: ``import apex`` loads the framework that lives in ``rocm-apex_amd/``.

The source tree is laid out as ``rocm-apex_amd/{models,ops,parallel,utils,amp,optimizers,...}``;
the directory name is not a valid Python identifier, so this package re-points its own
``__path__`` there.  Every submodule (``apex.amp``, ``apex.optimizers``, ``apex.parallel``, ...)
is therefore the file under ``rocm-apex_amd/`` imported under the familiar ``apex`` name.
"""
import os as _os

_ROOT = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "rocm-apex_amd")
__path__ = [_ROOT]
__file__ = _os.path.join(_ROOT, "__init__.py")
with open(__file__) as _f:
    exec(compile(_f.read(), __file__, "exec"))
