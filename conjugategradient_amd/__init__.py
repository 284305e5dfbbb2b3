"""conjugategradient_amd — MI355X-native conjugate-gradient solver.

A from-scratch gfx950 engine (libcgx.so: HIP kernels + C ABI, include/cgx.h)
behind the interfaces of XeniaHerr/ConjugateGradient:

* C++: include/CG.hpp, include/VectorOperations.hpp,
  include/LinearAlgebraTypes.hpp (drop-in for src/*.hpp);
* Python: the same classes in ``conjugategradient_amd.core``.
"""
from ._native import CgxError, device_count, header_symbols, lib  # noqa: F401
from .core import (CG, DeviceArray, Debuglevel, Event, Matrix, Queue, Scalar,  # noqa: F401
                   Vector, VectorOperations)

__all__ = ["CG", "CgxError", "Debuglevel", "DeviceArray", "Event", "Matrix", "Queue", "Scalar",
           "Vector", "VectorOperations", "device_count", "header_symbols", "lib"]
