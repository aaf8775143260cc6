"""In-process loopback backend: P ranks as threads of one process (SURVEY §4
"pluggable backend": ``rccl`` real, ``mpi-host`` staged, ``loopback`` for
unit tests; §5.6 ``--comm loopback``).

The reference's ranks exchange partials with blocking MPI_Send / MPI_Recv
(sparse_matrix_mult.cu:466-553).  Here ``LoopbackComm`` implements the same
point-to-point contract as :class:`parallel.comm.Comm` (``send_bsr`` /
``recv_bsr`` in per-(src, dst) FIFO order, ``barrier``, ``allreduce_max``)
over thread-safe queues, so the distributed chain code (the binomial tree
with row-panel splits) runs unchanged at any P in one process: no launcher,
no sockets, and a failing rank surfaces as an exception in the caller.
A sent matrix is cloned, so sender and receiver never share storage.

    results = run_loopback(world, lambda comm: run_chain(folder, comm, ...))
"""
from __future__ import annotations

import queue
import threading
from typing import Callable, List

import torch

from ..ops.bsr import BSR
from .comm import Comm


class _Hub:
    def __init__(self, world: int, timeout_s: float):
        self.world = world
        self.timeout_s = timeout_s
        self.q = {(s, d): queue.Queue() for s in range(world) for d in range(world)}
        self.barrier = threading.Barrier(world, timeout=timeout_s)
        self.slots = [0.0] * world


class LoopbackComm(Comm):
    """One rank of an in-process group (``backend == "loopback"``)."""

    def __init__(self, rank: int, world: int, device: torch.device, hub: _Hub):
        super().__init__(rank, world, rank, device, "loopback")
        self._hub = hub

    def send_bsr(self, M: BSR, dst: int) -> None:
        self._hub.q[(self.rank, dst)].put(BSR(M.rows, M.cols, M.k, M.keys.clone(), M.vals.clone()))

    def recv_bsr(self, src: int) -> BSR:
        try:
            M = self._hub.q[(src, self.rank)].get(timeout=self._hub.timeout_s)
        except queue.Empty:
            raise TimeoutError(f"loopback rank {self.rank}: nothing from rank {src} "
                               f"in {self._hub.timeout_s} s") from None
        return M.to(self.device)

    def barrier(self) -> None:
        self._hub.barrier.wait()

    def allreduce_max(self, x: float) -> float:
        self._hub.slots[self.rank] = x
        self._hub.barrier.wait()
        m = max(self._hub.slots)
        self._hub.barrier.wait()   # everyone read before the slots are reused
        return m

    def close(self) -> None:
        pass


def run_loopback(world: int, fn: Callable[[LoopbackComm], object], device: str = "cpu",
                 timeout_s: float = 300.0) -> List[object]:
    """Run ``fn(comm)`` on ``world`` ranks (threads) and return their results
    in rank order; the first rank failure is re-raised here (the other ranks
    are released by aborting the barrier)."""
    hub = _Hub(world, timeout_s)
    dev = torch.device(device)
    out: List[object] = [None] * world
    errs: List[BaseException] = []

    def body(r: int) -> None:
        try:
            out[r] = fn(LoopbackComm(r, world, dev, hub))
        except BaseException as e:   # noqa: BLE001  (re-raised in the caller)
            errs.append(e)
            hub.barrier.abort()

    threads = [threading.Thread(target=body, args=(r,), name=f"loopback-rank{r}") for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errs:
        raise errs[0]
    return out
