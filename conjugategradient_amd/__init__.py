"""conjugategradient_amd — MI355X-native conjugate-gradient solver.

A from-scratch gfx950 engine (libcgx.so: HIP kernels + C ABI, include/cgx.h)
behind the interfaces of XeniaHerr/ConjugateGradient:

* C++: include/CG.hpp, include/VectorOperations.hpp,
  include/LinearAlgebraTypes.hpp (drop-in for src/*.hpp);
* Python: the same classes in ``conjugategradient_amd.core``; the
  Matrix-Market loader (test/mm_reader.cpp read_file) in ``.mtx``.
"""
from ._native import CgxError, device_count, header_symbols, lib  # noqa: F401
from .core import (CG, DeviceArray, Debuglevel, Event, Matrix, Queue, Scalar,  # noqa: F401
                   Vector, VectorOperations)
from .mtx import read_file, write_mtx_lower  # noqa: F401

__all__ = ["CG", "CgxError", "Debuglevel", "DeviceArray", "Event", "Matrix", "Queue", "Scalar",
           "Vector", "VectorOperations", "device_count", "header_symbols", "lib", "read_file",
           "write_mtx_lower"]
