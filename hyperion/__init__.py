"""Import alias for the Hyperion-MI355X package.

The package source lives in
``hyperion-accelerated-deep-learning-and-distributed-performance-on-mi250x_amd/``
(a directory name that is not a valid Python identifier).  This shim points the
``hyperion`` package's ``__path__`` at that directory, so ``import hyperion.models``
and friends resolve there, and then runs the real ``__init__``.
"""
import os as _os

_SRC = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "hyperion-accelerated-deep-learning-and-distributed-performance-on-mi250x_amd",
)
__path__ = [_SRC]  # noqa: F811 - submodules resolve inside the source directory
__file__ = _os.path.join(_SRC, "__init__.py")

with open(__file__, "r", encoding="utf-8") as _f:
    exec(compile(_f.read(), __file__, "exec"))
