"""Import alias for the framework package.

The framework lives in the directory
``sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/`` (the name the
project layout prescribes).  A hyphenated directory is not a valid Python
identifier, so this shim makes it importable as ``spmm_amd``: it points the
package search path at that directory and executes its ``__init__``.
"""
import os as _os

_REAL = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd",
)
__path__ = [_REAL]
__file__ = _os.path.join(_REAL, "__init__.py")
with open(__file__) as _f:
    exec(compile(_f.read(), __file__, "exec"))
