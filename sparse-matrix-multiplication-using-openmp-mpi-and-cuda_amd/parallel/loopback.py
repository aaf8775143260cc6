"""In-process loopback backend: P ranks as threads of one process (SURVEY §4
"pluggable backend": ``rccl`` real, ``mpi-host`` staged, ``loopback`` for
unit tests; §5.6 ``--comm loopback``).

The reference's ranks exchange partials with blocking MPI_Send / MPI_Recv
(sparse_matrix_mult.cu:466-553).  ``LoopbackComm`` implements the whole
:class:`parallel.comm.Comm` contract — point-to-point (``send`` / ``recv``,
``send_bsr`` / ``recv_bsr`` in per-(src, dst) FIFO order) and every
collective the models use (``all_gather[_async]``, ``all_to_all_v``,
``all_reduce_``, ``reduce_scatter``, ``barrier``) — over a shared hub, so
the distributed code runs unchanged at any P in one process: no launcher,
no sockets, and a failing rank surfaces as an exception in the caller.

On a GPU (``run_loopback(..., device="cuda")``) every rank is a thread on
the same card and ``device_collectives`` is True: the models take exactly
the branches they take under RCCL (padded device payloads, device-side
unpacking), which a single-GPU box cannot otherwise run at P > 1 (RCCL does
not put two ranks of one communicator on one device).  Stream safety: a
posting rank records an event on its current stream and every consumer's
stream waits on it before reading, as RCCL orders its kernels.

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
        self.cv = threading.Condition()
        self.slots = {}     # collective sequence number -> [posted objects], readers left
        self.failed = False

    def post(self, seq: int, rank: int, obj) -> None:
        with self.cv:
            slot = self.slots.setdefault(seq, [[None] * self.world, 0, self.world])
            slot[0][rank] = obj
            slot[1] += 1
            self.cv.notify_all()

    def collect(self, seq: int, rank: int) -> list:
        with self.cv:
            ok = self.cv.wait_for(lambda: self.failed or (seq in self.slots and self.slots[seq][1] == self.world),
                                  timeout=self.timeout_s)
            if self.failed:
                raise RuntimeError(f"loopback rank {rank}: another rank failed")
            if not ok:
                raise TimeoutError(f"loopback rank {rank}: collective #{seq} incomplete after {self.timeout_s} s")
            slot = self.slots[seq]
            out = list(slot[0])
            slot[2] -= 1
            if slot[2] == 0:
                del self.slots[seq]
            return out

    def fail(self) -> None:
        with self.cv:
            self.failed = True
            self.cv.notify_all()
        self.barrier.abort()


def _mark(t: torch.Tensor):
    """(tensor, event recorded after its producer on the current stream)."""
    if t.device.type == "cuda":
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(t.device))
        return t, ev
    return t, None


def _take(item, device: torch.device) -> torch.Tensor:
    t, ev = item
    if ev is not None and device.type == "cuda":
        cur = torch.cuda.current_stream(device)
        cur.wait_event(ev)
        if t.device == device:   # the poster's block stays allocated until this stream has read it
            t.record_stream(cur)
    elif ev is not None:
        ev.synchronize()
    return t.to(device)


class LoopbackComm(Comm):
    """One rank of an in-process group (``backend == "loopback"``)."""

    def __init__(self, rank: int, world: int, device: torch.device, hub: _Hub):
        super().__init__(rank, world, rank, device, "loopback")
        self._hub = hub
        self._seq = 0

    @property
    def device_collectives(self) -> bool:
        return self.device.type == "cuda"

    def _exchange(self, obj) -> list:
        seq = self._seq
        self._seq += 1
        self._hub.post(seq, self.rank, obj)
        return self._hub.collect(seq, self.rank)

    def _post(self, obj) -> Callable[[], list]:
        """Post now, collect later (once: the result is kept, like a finished
        RCCL work object that can be waited on again)."""
        seq = self._seq
        self._seq += 1
        self._hub.post(seq, self.rank, obj)
        got = []

        def collect():
            if not got:
                got.append(self._hub.collect(seq, self.rank))
            return got[0]
        return collect

    # --- collectives -------------------------------------------------------
    def all_gather_async(self, t: torch.Tensor) -> Callable[[], torch.Tensor]:
        flat = t.reshape(-1)
        dev = t.device
        # posted as a copy: a rank returns once every rank has POSTED, not once
        # every peer has read, so the caller may reuse its buffer right away
        # (RCCL's stream-ordered collective gives the caller the same freedom)
        got = self._post(_mark(flat.clone()))
        return lambda: torch.cat([_take(x, dev) for x in got()])

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor) -> Callable[[], None]:
        got = self.all_gather_async(t)
        return lambda: (out.copy_(got()), None)[1]

    def all_to_all_v(self, x: torch.Tensor, send: List[int], recv: List[int]) -> torch.Tensor:
        got = self._exchange((_mark(x.clone()), list(send)))   # (a copy: see all_gather_async)
        parts = []
        for src, (item, ssend) in enumerate(got):
            off = sum(ssend[:self.rank])
            if ssend[self.rank] != recv[src]:
                raise RuntimeError(f"loopback all_to_all_v: rank {src} sends {ssend[self.rank]} to rank "
                                   f"{self.rank}, which expects {recv[src]}")
            parts.append(_take(item, x.device)[off:off + ssend[self.rank]])
        return torch.cat(parts) if parts else x[:0]

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        got = [_take(x, t.device) for x in self._exchange(_mark(t.clone()))]
        acc = got[0].clone()
        for g in got[1:]:
            if op == "sum":
                acc += g
            elif op == "max":
                acc = torch.maximum(acc, g)
            else:
                acc = torch.minimum(acc, g)
        t.copy_(acc)
        return t

    def reduce_scatter(self, full: torch.Tensor) -> torch.Tensor:
        c = full.shape[0] // self.world
        s = self.all_reduce_(full.clone())
        return s[self.rank * c:(self.rank + 1) * c].clone()

    def send(self, t: torch.Tensor, dst: int) -> None:
        self._hub.q[(self.rank, dst)].put(_mark(t.clone()))

    def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
        try:
            item = self._hub.q[(src, self.rank)].get(timeout=self._hub.timeout_s)
        except queue.Empty:
            raise TimeoutError(f"loopback rank {self.rank}: nothing from rank {src} "
                               f"in {self._hub.timeout_s} s") from None
        x = _take(item, t.device)
        if x.shape != t.shape:
            raise RuntimeError(f"loopback recv: got {tuple(x.shape)}, expected {tuple(t.shape)}")
        t.copy_(x)
        return t

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

    def _allreduce_scalar(self, x: float, op: str) -> float:
        vals = self._exchange(float(x))
        return max(vals) if op == "max" else (min(vals) if op == "min" else float(sum(vals)))

    def gather_ints(self, x: int) -> List[int]:
        return [int(v) for v in self._exchange(int(x))]

    def close(self) -> None:
        pass


def run_loopback(world: int, fn: Callable[[LoopbackComm], object], device: str = "cpu",
                 timeout_s: float = 300.0) -> List[object]:
    """Run ``fn(comm)`` on ``world`` ranks (threads) and return their results
    in rank order; the first rank failure is re-raised here (the other ranks
    are released by aborting the barrier and failing pending collectives)."""
    hub = _Hub(world, timeout_s)
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    out: List[object] = [None] * world
    errs: List[BaseException] = []

    def body(r: int) -> None:
        try:
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            out[r] = fn(LoopbackComm(r, world, dev, hub))
        except BaseException as e:   # noqa: BLE001  (re-raised in the caller)
            errs.append(e)
            hub.fail()

    threads = [threading.Thread(target=body, args=(r,), name=f"loopback-rank{r}") for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if errs:
        raise errs[0]
    return out


class PanelComm(Comm):
    """Rank ``rank`` of ``world`` in ONE thread, for the row-block step's
    operand gathers only (``models.spgemm.RowblockGraph``: the panel sizes,
    row counts and the two payload gathers, plus agreements): the other ranks'
    contributions are computed from ``panels`` (every rank's B row panel) by
    the payload builders the step binds (``bind_payloads``: packed columns,
    value bits), so rank r's whole step runs on one GPU with no peer threads.
    ``gbps`` > 0 delivers each payload late: a "wire" stream runs a
    stream-ordered delay of (bytes this rank receives) / gbps per payload, in
    RCCL's issue order (columns, then values), while a "link" stream writes the
    payloads (the HBM traffic of the incoming data); a payload is delivered
    when both are done.  ``prefill``: the payloads are written once, at the
    first gather into each buffer, and later gathers only run the delay --
    the panels' data must then not change -- i.e. the link model of a real
    node, where the peers' RCCL kernels push the bytes into this GPU's memory
    and none of this GPU's CUs copy them.  ``tools/rank_emulate.py`` models a
    rank of an N-GPU node with it; tests drive the W-rank branches with it."""

    def __init__(self, rank: int, world: int, dev: torch.device, panels, gbps: float = 0.0, link_priority: int = 0,
                 prefill: bool = False):
        super().__init__(rank, world, rank, dev, "panels")
        if len(panels) != world:
            raise ValueError("PanelComm: one B panel per rank")
        self.panels, self.gbps, self.prefill = panels, gbps, prefill
        self._filled = set()
        # (``link_priority`` -1: high-priority streams, whose work the dispatcher puts
        # ahead of the compute stream's large grids; tools/rank_emulate.py --link-priority)
        self.link = torch.cuda.Stream(dev, priority=link_priority) if dev.type == "cuda" else None
        self.wire = torch.cuda.Stream(dev, priority=link_priority) if dev.type == "cuda" else None
        self._n = 0
        self._payloads = None

    def bind_payloads(self, cols, vals) -> None:
        """``cols(panel, out)`` / ``vals(panel, out)`` write one rank's send
        buffer of the column / value gather (the step's own builders)."""
        self._payloads = (cols, vals)

    @property
    def device_collectives(self) -> bool:
        return self.device.type == "cuda"

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if t.numel() == 2:   # [m, nnz] of every panel
            return torch.tensor([[p.m, p.nnz] for p in self.panels], dtype=torch.int64, device=t.device).view(-1)
        out = torch.zeros(self.world, t.numel(), dtype=t.dtype, device=t.device)   # row counts, padded
        for r, p in enumerate(self.panels):
            out[r, :p.m] = p.rowptr[1:] - p.rowptr[:-1]
        return out.view(-1)

    def _allreduce_scalar(self, x: float, op: str) -> float:
        return x * self.world if op == "sum" else x

    def barrier(self) -> None:
        pass

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor) -> Callable[[], None]:
        if self._payloads is None:
            raise RuntimeError("PanelComm: the step did not bind its payload builders")
        which = self._n % 2   # RowblockGraph's order: columns, then value bits
        self._n += 1
        per = t.numel()
        if out.numel() != self.world * per:
            raise ValueError(f"PanelComm: receive buffer of {out.numel()} for {self.world} payloads of {per}")
        cur = torch.cuda.current_stream(self.device)
        evs = []
        if self.gbps > 0:
            from .. import _native

            self.wire.wait_stream(cur)   # (RCCL: a collective starts after the producer of its input)
            recv_bytes = (self.world - 1) * per * t.element_size()
            with torch.cuda.stream(self.wire):
                _native.check(_native.hip().spmm_prim_spin(recv_bytes / (self.gbps * 1e3),
                                                           _native.stream_ptr(self.device)), "prim_spin")
            evs.append(torch.cuda.Event())
            evs[-1].record(self.wire)
        key = (out.data_ptr(), which)
        if not (self.prefill and key in self._filled):
            self._filled.add(key)
            self.link.wait_stream(cur)
            with torch.cuda.stream(self.link):
                for r, p in enumerate(self.panels):   # every rank's payload from its panel's current data
                    self._payloads[which](p, out[r * per:(r + 1) * per])
            evs.append(torch.cuda.Event())
            evs[-1].record(self.link)

        def wait() -> None:
            for e in evs:
                cur.wait_event(e)
        return wait
