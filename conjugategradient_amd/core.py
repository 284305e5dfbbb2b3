"""Python mirror of the reference's C++ API, on top of libcgx.so.

Same class and method names, argument meaning and error behaviour as
/root/reference/src (cited per method), so parity tests read like the
reference's own driver (test/Tester.cpp). The C++ drop-in for the same API is
include/CG.hpp, include/VectorOperations.hpp, include/LinearAlgebraTypes.hpp.

Everything here is a thin wrapper: every computation runs in libcgx.so's HIP
kernels on a gfx950 device; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import enum

import numpy as np

from . import _native as N
from ._native import CgxError, check, lib

_vp = C.c_void_p


class Debuglevel(enum.IntEnum):
    """LinearAlgebraTypes.hpp:26-30"""
    None_ = 0
    Verbose = 1


def _dtype_code(dtype) -> int:
    dt = np.dtype(dtype)
    if dt == np.float64:
        return N.F64
    if dt == np.float32:
        return N.F32
    raise TypeError(f"unsupported dtype {dt} (float64 or float32)")


class Queue:
    """The sycl::queue of the reference (CG.hpp:61,70-77): one device, one
    in-order HIP stream. ``wait()`` is ``executeQueue`` (CG.hpp:561-578)."""

    def __init__(self, device: int = 0):
        h = _vp()
        check(lib().cgx_create(device, C.byref(h)))
        self._h = h
        self.device = device

    @property
    def handle(self):
        return self._h

    def wait(self) -> None:
        check(lib().cgx_sync(self._h))

    wait_and_throw = wait

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().cgx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


class DeviceArray:
    """A device allocation released when the last reference goes away (the
    shared_ptr + Asycl_deleter of LinearAlgebraTypes.hpp:43-49)."""

    def __init__(self, queue: Queue, n: int, dtype=np.float64):
        self.queue = queue
        self.n = int(n)
        self.dtype = np.dtype(dtype)
        p = _vp()
        check(lib().cgx_alloc(queue.handle, max(self.n, 1) * self.dtype.itemsize, C.byref(p)))
        self.ptr = p.value

    @property
    def nbytes(self) -> int:
        return self.n * self.dtype.itemsize

    def upload(self, host) -> "DeviceArray":
        a = np.ascontiguousarray(host, dtype=self.dtype)
        if a.size != self.n:
            raise ValueError(f"size {a.size} != {self.n}")
        check(lib().cgx_h2d(self.queue.handle, self.ptr, a.ctypes.data, a.nbytes))
        return self

    def download(self) -> np.ndarray:
        out = np.empty(self.n, self.dtype)
        check(lib().cgx_d2h(self.queue.handle, out.ctypes.data, self.ptr, out.nbytes))
        return out

    def fill(self, value: float) -> None:
        check(lib().cgx_fill(self.queue.handle, _dtype_code(self.dtype), self.ptr,
                             float(value), self.n))

    def __del__(self):  # pragma: no cover
        try:
            if self.ptr and self.queue.handle:
                lib().cgx_free(self.queue.handle, self.ptr)
        except Exception:
            pass
        self.ptr = None


class Matrix:
    """CSR matrix on the device (LinearAlgebraTypes.hpp:57-132)."""

    def __init__(self, queue: Queue, data=None, cols=None, rows=None, dtype=np.float64):
        self._queue = queue
        self.dtype = np.dtype(dtype)
        self._N = 0
        self._NNZ = 0
        self._data = self._columns = self._rows = None
        self._csr = None
        self._host_rows = None
        if data is not None:
            self.init(data, cols, rows)

    def init(self, data, cols, rows) -> None:
        """LinearAlgebraTypes.hpp:101-121: upload a CSR triple."""
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        data = np.ascontiguousarray(data, dtype=self.dtype)
        self._N = len(rows) - 1
        self._NNZ = len(data)
        self._data = DeviceArray(self._queue, self._NNZ, self.dtype).upload(data)
        self._columns = DeviceArray(self._queue, self._NNZ, np.int32).upload(cols)
        self._rows = DeviceArray(self._queue, self._N + 1, np.int32).upload(rows)
        self._host_rows = rows
        self._drop_schedule()

    @classmethod
    def poisson(cls, queue: Queue, dim: int, nx: int, ny: int, nz: int = 1,
                dtype=np.float64) -> "Matrix":
        """Dirichlet Poisson CSR generated on the device."""
        m = cls(queue, dtype=dtype)
        zz = nz if dim == 3 else 1
        n = nx * ny * zz
        nnz = lib().cgx_poisson_nnz(dim, nx, ny, zz, 0, n)
        m._N, m._NNZ = n, nnz
        m._data = DeviceArray(queue, nnz, dtype)
        m._columns = DeviceArray(queue, nnz, np.int32)
        m._rows = DeviceArray(queue, n + 1, np.int32)
        check(lib().cgx_poisson_fill(queue.handle, _dtype_code(dtype), dim, nx, ny, zz, 0, n,
                                     m._rows.ptr, m._columns.ptr, m._data.ptr))
        queue.wait()
        return m

    def _drop_schedule(self):
        # libcgx refcounts the context from the handle, so this is valid after
        # the queue was closed (interpreter shutdown, a fixture closing first)
        if self._csr:
            lib().cgx_csr_destroy(self._csr)
        self._csr = None

    def schedule(self):
        """The cgx_csr handle (row-block schedule), built on first use."""
        if self._csr is None:
            if self._rows is None:
                raise CgxError("No Matrix given")
            h = _vp()
            hr = self._host_rows.ctypes.data if self._host_rows is not None else None
            check(lib().cgx_csr_create(self._queue.handle, self._N, self._NNZ, self._rows.ptr,
                                       self._columns.ptr, self._data.ptr,
                                       _dtype_code(self.dtype), hr, C.byref(h)))
            self._csr = h
        return self._csr

    def data(self):
        return self._data

    def columns(self):
        return self._columns

    def rows(self):
        return self._rows

    def N(self) -> int:
        return self._N

    def NNZ(self) -> int:
        return self._NNZ

    def __del__(self):  # pragma: no cover
        try:
            self._drop_schedule()
        except Exception:
            pass


class Vector:
    """Vector on the device (LinearAlgebraTypes.hpp:143-203)."""

    def __init__(self, queue: Queue, arg=None, dtype=np.float64):
        self._q = queue
        self.dtype = np.dtype(dtype)
        self._N = 0
        self._ptr = None
        if isinstance(arg, (int, np.integer)):
            self._N = int(arg)
            self.init_empty(self._N)
        elif arg is not None:
            self.init(arg)

    def init_empty(self, size: int = 0) -> None:
        """:160-171 — allocate and zero (asserts a non-zero size)."""
        if size != 0 and self._N == 0:
            self._N = int(size)
        assert self._N != 0
        self._ptr = DeviceArray(self._q, self._N, self.dtype)
        self._ptr.fill(0.0)

    def init(self, data) -> None:
        """:177-183 — copy a host vector (the size is not recorded, as in the
        reference, unless it was never set)."""
        a = np.ascontiguousarray(data, dtype=self.dtype)
        self._ptr = DeviceArray(self._q, a.size, self.dtype).upload(a)
        if self._N == 0:
            self._N = a.size

    def data(self):
        return self._ptr

    def ptr(self):
        return self._ptr.ptr if self._ptr is not None else None

    def N(self) -> int:
        return self._N

    def to_numpy(self) -> np.ndarray:
        return self._ptr.download()


class Scalar:
    """Device-resident scalar (LinearAlgebraTypes.hpp:210-250)."""

    def __init__(self, queue: Queue, value: float = 0.0, dtype=np.float64):
        self._q = queue
        self.dtype = np.dtype(dtype)
        self.init(value)

    def init(self, value: float) -> None:
        self._v = DeviceArray(self._q, 1, self.dtype).upload(np.array([value], self.dtype))

    def ptr(self):
        return self._v.ptr

    def get(self) -> float:
        return float(self._v.download()[0])


class Event:
    """Stand-in for sycl::event: the queue is in order, so an event only
    names the point in the stream (VectorOperations methods return one)."""

    def __init__(self, queue: Queue):
        self.queue = queue

    def wait(self) -> None:
        self.queue.wait()


class VectorOperations:
    """src/VectorOperations.hpp:39-488. Methods are asynchronous and return an
    Event; scalars are device pointers (Scalar.ptr()) as in the reference."""

    def __init__(self, queue: Queue, dtype=np.float64, debug=Debuglevel.None_):
        self._queue = queue
        self.dtype = np.dtype(dtype)
        self._dt = _dtype_code(dtype)
        self.vector_size = 0
        self.workgroupsize = 128  # calculateWorkgroupSize :478-487 (min(128, max))

    def setVectorSize(self, size: int) -> None:
        self.vector_size = int(size)

    @staticmethod
    def _p(x):
        if isinstance(x, (Vector, Scalar)):
            return x.ptr()
        if isinstance(x, DeviceArray):
            return x.ptr
        return x

    def spmv(self, A: Matrix, vec, Result, NNZ=None, events=(), count=0) -> Event:
        """:438-466 — ignores NNZ, honours count, asserts A.N() == count."""
        self.vector_size = count if count else self.vector_size
        assert self.vector_size != 0 and A.N() == self.vector_size
        check(lib().cgx_spmv(self._queue.handle, A.schedule(), self._p(vec), self._p(Result),
                             self.vector_size))
        return Event(self._queue)

    def dot_product_trivial(self, left, right, result, dependencies=(), size=0) -> Event:
        """:287-309 — *result += left.right over vector_size (size ignored, Q7)."""
        check(lib().cgx_dot_acc(self._queue.handle, self._dt, self.vector_size, self._p(left),
                                self._p(right), self._p(result)))
        return Event(self._queue)

    def norm(self, vector, result, dependencies=(), size=0) -> Event:
        """:311-331 — *result += sum x^2 (no sqrt)."""
        check(lib().cgx_norm_acc(self._queue.handle, self._dt, self.vector_size,
                                 self._p(vector), self._p(result)))
        return Event(self._queue)

    def dot_product(self, left, right, result, dependencies=(), vec_size=0) -> Event:
        """:212-285 (deprecated in the reference) — *result += left.right."""
        self.vector_size = vec_size if vec_size else self.vector_size
        assert self.vector_size != 0
        return self.dot_product_trivial(left, right, result)

    def dot_product_optimised(self, Left, Right, result, dependencies=(), count=0) -> Event:
        """:110-208 — *result += Left.Right. The reference's multi-level tree
        indexes the wrong offsets beyond wg^2 groups (SURVEY §2 C2'); this one
        is the exact deterministic reduction for every size."""
        self.vector_size = count if count else self.vector_size
        assert self.vector_size != 0
        return self.dot_product_trivial(Left, Right, result)

    def saxpby(self, X, Y, a, b, Result, events=(), vec_size=0) -> Event:
        """:349-367 — Result = (*a) X + (*b) Y."""
        self.vector_size = vec_size if vec_size else self.vector_size
        check(lib().cgx_saxpby(self._queue.handle, self._dt, self.vector_size, self._p(X),
                               self._p(Y), self._p(a), self._p(b), self._p(Result)))
        return Event(self._queue)

    def sambx(self, X, Y, b, Result, events=(), count=0) -> Event:
        """:380-397 — Result = X - (*b) Y over vector_size (count ignored, Q7)."""
        check(lib().cgx_sambx(self._queue.handle, self._dt, self.vector_size, self._p(X),
                              self._p(Y), self._p(b), self._p(Result)))
        return Event(self._queue)

    def sapbx(self, X, Y, b, Result, events=(), count=0) -> Event:
        """:410-428 — Result = X + (*b) Y over vector_size (count ignored, Q7)."""
        check(lib().cgx_sapbx(self._queue.handle, self._dt, self.vector_size, self._p(X),
                              self._p(Y), self._p(b), self._p(Result)))
        return Event(self._queue)


class CG:
    """CGSolver::CG<DT, Debuglevel> (src/CG.hpp:53-601)."""

    def __init__(self, queue: Queue, dtype=np.float64, debug=Debuglevel.None_):
        self._queue = queue
        self.dtype = np.dtype(dtype)
        self.debug = debug
        self.A = Matrix(queue, dtype=dtype)
        self.x = Vector(queue, dtype=dtype)
        self.b = Vector(queue, dtype=dtype)
        self.is_solved = False
        self._cg = None
        self._cg_for = None
        self.iterations = 0       # extension: loop bodies of the last solve
        self.final_rxr = float("nan")  # extension: rxr after the last body
        self.poll_every = 32
        self.use_graph = True
        self.mode = 0  # cgx_cg_set_mode: 0 auto (5, 4, 6 or 3), 1 three kernels, 2 fused,
        # 3 deferred x, 4 fused + deferred x, 5 persistent body, 6 deferred x with Ap
        # recomputed (lean walk), 7 fused + deferred x with Ap recomputed (tile walk)

    @classmethod
    def createCG(cls, dtype=np.float64, debug=Debuglevel.None_, device: int = 0) -> "CG":
        """:70-77 — a CG with its own default queue."""
        return cls(Queue(device), dtype, debug)

    # -- inputs ---------------------------------------------------------
    def setMatrix(self, data, columns=None, rows=None) -> None:
        """:87-93 (host CSR triple) and :102 (a device Matrix, moved)."""
        if isinstance(data, Matrix):
            self.A = data
        else:
            self.A.init(data, columns, rows)
        self._drop_solver()

    def getDimension(self) -> int:
        """:156"""
        return self.A.N()

    def setTarget(self, data) -> None:
        """:164-170 (host vector) and :206 (a device Vector)."""
        if isinstance(data, Vector):
            self.b = data
        else:
            self.b.init(data)
            self._queue.wait()

    def setInital(self, data) -> None:
        """:215-219 (sic) — initial guess from a host vector."""
        self.x.init(data)
        self._queue.wait()

    def setInitial(self, V) -> None:
        """:244 — initial guess from a device Vector (moved)."""
        if isinstance(V, Vector):
            self.x = V
        else:
            self.setInital(V)

    def calculateExpectedStepCount(self, accuracy) -> None:
        """:235 (empty in the reference)."""
        return None

    # -- solve ----------------------------------------------------------
    def _drop_solver(self):
        if self._cg:  # valid after Queue.close (see Matrix._drop_schedule)
            lib().cgx_cg_destroy(self._cg)
        self._cg = None
        self._cg_for = None

    def _solver(self):
        sched = self.A.schedule()
        if self._cg is None or self._cg_for != sched:
            self._drop_solver()
            h = _vp()
            check(lib().cgx_cg_create(self._queue.handle, sched, C.byref(h)))
            self._cg = h
            self._cg_for = sched
            check(lib().cgx_cg_config(self._cg, self.poll_every, 1 if self.use_graph else 0))
            check(lib().cgx_cg_set_mode(self._cg, self.mode))
        return self._cg

    def solve(self, improvement: float = 0.0, max_iter: int = -1) -> None:
        """:255-454. Throws RuntimeError for a missing b or A (:266-272).
        max_iter caps the loop bodies (extension; -1 keeps the cap N+1)."""
        if self.b.ptr() is None:
            raise RuntimeError("No right hand side to solve for")
        if self.A.columns() is None:
            raise RuntimeError("No Matrix given")
        n = self.A.N()
        if self.x.ptr() is None:  # :291-297
            self.x = Vector(self._queue, n, dtype=self.dtype)
        bodies = C.c_int64(0)
        rxr = C.c_double(0)
        check(lib().cgx_cg_solve(self._solver(), self.b.ptr(), self.x.ptr(), float(improvement),
                                 int(max_iter), C.byref(bodies), C.byref(rxr)))
        self.iterations = bodies.value
        self.final_rxr = rxr.value
        self.is_solved = True

    # -- outputs --------------------------------------------------------
    def accuracy(self) -> float:
        """:463-515 — |sum (b - A x)^2 / sum x^2| (squared norms, Q6)."""
        out = C.c_double(0)
        check(lib().cgx_accuracy(self._queue.handle, self.A.schedule(), self.b.ptr(),
                                 self.x.ptr(), C.byref(out)))
        return out.value

    def extract(self) -> np.ndarray:
        """:517-523"""
        return self.x.data().download()[: self.A.N()]

    def extractTo(self, result: list) -> None:
        """:529-532 — resizes `result` to N and copies x into it."""
        v = self.extract()
        result[:] = v.tolist()

    def memoryFootprint(self) -> int:
        """:555-558"""
        it = self.dtype.itemsize
        return (2 * self.A.NNZ() + 4 * self.A.N()) * it + 2 * self.A.N() * 4

    def __del__(self):  # pragma: no cover
        try:
            self._drop_solver()
        except Exception:
            pass
