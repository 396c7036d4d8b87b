"""Import alias for the framework.

The framework's source tree lives in the directory
``vt-cluster--parallel-and-distributed-programming-of-machine-learning-models_amd/``
(the layout the project requires).  That name is not a valid Python
identifier, so this tiny package re-roots its ``__path__`` there: every
``mift.<sub>`` import (``mift.models``, ``mift.ops``, ``mift.parallel`` ...)
resolves to the real directory, and the real ``__init__.py`` runs in this
module's namespace.
"""
import os as _os

PKG_DIRNAME = "vt-cluster--parallel-and-distributed-programming-of-machine-learning-models_amd"
_REAL = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), PKG_DIRNAME)
__path__ = [_REAL]  # noqa: F821 - package path re-rooting
__file__ = _os.path.join(_REAL, "__init__.py")
with open(__file__, "r", encoding="utf-8") as _fh:
    exec(compile(_fh.read(), __file__, "exec"))
