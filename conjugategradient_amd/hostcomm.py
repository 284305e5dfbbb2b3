"""Host-staged transport for libcgx's partitioned solver
(cgx_dist_init_host, include/cgx.h) over torch.distributed (gloo).

RCCL refuses two ranks on one GPU; with this transport several ranks can
share a device, so the multi-rank device path (halo plan, ghost area, pack
kernel, all-reduce points, stop rule) runs on a single-GPU box. Every
collective stages through host memory: correct, not fast. Production runs use
RCCL (cgx_dist_init).
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.distributed as dist

from ._native import check, lib

AG = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
AR = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int)
EX = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_void_p),
                 C.POINTER(C.c_size_t), C.POINTER(C.c_void_p), C.POINTER(C.c_size_t))


def _bytes_tensor(ptr, n):
    t = torch.empty(n, dtype=torch.uint8)
    if n:
        C.memmove(t.data_ptr(), ptr, n)
    return t


class HostTransport:
    """Owns the ctypes callbacks (they must outlive the communicator)."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.calls = {"allgather": 0, "allreduce": 0, "exchange": 0}

        def allgather(user, send, nbytes, recv):
            try:
                self.calls["allgather"] += 1
                t = _bytes_tensor(send, nbytes)
                out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
                dist.all_gather(out, t, group=self.group)
                for r, o in enumerate(out):
                    if nbytes:
                        C.memmove(recv + r * nbytes, o.data_ptr(), nbytes)
                return 0
            except Exception:  # pragma: no cover - reported as a libcgx error
                return 1

        def allreduce(user, vals, count):
            try:
                self.calls["allreduce"] += 1
                t = torch.tensor([vals[i] for i in range(count)], dtype=torch.float64)
                dist.all_reduce(t, group=self.group)
                for i in range(count):
                    vals[i] = float(t[i])
                return 0
            except Exception:  # pragma: no cover
                return 1

        def exchange(user, n, peers, send, sbytes, recv, rbytes):
            try:
                self.calls["exchange"] += 1
                reqs, bufs = [], []
                for i in range(n):
                    if sbytes[i]:
                        reqs.append(dist.isend(_bytes_tensor(send[i], sbytes[i]), peers[i],
                                               group=self.group))
                    if rbytes[i]:
                        b = torch.empty(rbytes[i], dtype=torch.uint8)
                        bufs.append((i, b))
                        reqs.append(dist.irecv(b, peers[i], group=self.group))
                for q in reqs:
                    q.wait()
                for i, b in bufs:
                    C.memmove(recv[i], b.data_ptr(), rbytes[i])
                return 0
            except Exception:  # pragma: no cover
                return 1

        self._cbs = (AG(allgather), AR(allreduce), EX(exchange))

    def attach(self, queue, overlap: bool = False) -> None:
        """overlap: run the halo exchange on libcgx's comm stream
        (cgx_dist_host_async): the exchange callback then runs on the HIP
        runtime's callback thread while the interior slices compute. Only one
        thread of a rank issues collectives at a time: the solver stream
        waits for the exchange before the next all-reduce is staged."""
        check(lib().cgx_dist_init_host(queue.handle, self.rank, self.world,
                                       C.cast(self._cbs[0], C.c_void_p),
                                       C.cast(self._cbs[1], C.c_void_p),
                                       C.cast(self._cbs[2], C.c_void_p), None))
        if overlap:
            check(lib().cgx_dist_host_async(queue.handle, 1))
