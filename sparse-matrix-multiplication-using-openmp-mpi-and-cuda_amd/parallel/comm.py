"""Process-group bootstrap, collectives and BSR point-to-point transport.

Parity: the reference bootstraps with MPI_Init (sparse_matrix_mult.cu:404-409)
and moves partial products with blocking MPI_Send/MPI_Recv of host-serialised
maps in three messages (header tag 0, keys tag 1 in 256 Ki chunks, values tag
2 in 4 Mi chunks; :466-553), with ``int`` counts that overflow past 2^31.

Here one process drives one GPU (``torch.cuda.set_device(LOCAL_RANK)`` — the
reference never calls cudaSetDevice, so all its ranks share device 0) and
``torch.distributed`` carries the data:

* backend ``nccl`` — RCCL on ROCm: device-to-device over xGMI, straight from
  HBM, no host staging, no chunking (RCCL pipelines internally), 64-bit
  counts;
* backend ``gloo`` — CPU tensors; used for the CPU backend, for
  multi-process tests without GPUs and for rehearsing several ranks on one
  card (device tensors are staged through the host by this class).

Every collective the models use is a method here (``all_gather``,
``all_gather_async``, ``all_to_all_v``, ``all_reduce_``, ``reduce_scatter``,
``send`` / ``recv``): callers hand in tensors on their compute device and get
results on that device, whatever the wire is.  The in-process loopback
backend (``parallel.loopback``) implements the same methods for P ranks as
threads of one process, so the device-resident code paths that run under
RCCL at P > 1 run at any P on a single GPU in tests.

A matrix travels as a fixed 4-int64 header (rows, cols, nb, k) followed, when
nb > 0, by the key and value tensors.  The receiver learns the payload size
from the header before posting the payload receives, so variable-size
partials need no padding.

Launchers (torchrun, mpirun/mpiexec) are recognised from their environment
variables; with none present the job is a single process.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

from ..ops.bsr import BSR


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return int(v)
    return default


def launcher_env():
    """(rank, world, local_rank) from torchrun / MPICH (PMI_*) / Open MPI /
    Slurm variables."""
    rank = _env_int("RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK", "SLURM_PROCID", default=0)
    world = _env_int("WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "SLURM_NTASKS", default=1)
    local = _env_int("LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID",
                     default=rank)
    return rank, world, local


_REDUCE_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


@dataclass
class Comm:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: Optional[str]   # None for a single process

    @property
    def is_dist(self) -> bool:
        return self.backend is not None

    @property
    def device_collectives(self) -> bool:
        """True when collectives move device tensors directly (RCCL over
        xGMI): no host staging, so device-side packing / unpacking pays."""
        return self.backend == "nccl"

    # --- helpers -----------------------------------------------------------
    def _wire_device(self) -> torch.device:
        return self.device if self.device_collectives else torch.device("cpu")

    def _wire(self, t: torch.Tensor) -> torch.Tensor:
        return t.to(self._wire_device()).contiguous()

    # --- collectives (results on the input's device) ------------------------
    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world * t.numel()] concatenation of every rank's equally sized
        tensor, rank order."""
        return self.all_gather_async(t)()

    def all_gather_async(self, t: torch.Tensor) -> Callable[[], torch.Tensor]:
        """Start an all-gather of equally sized tensors; the returned function
        waits for it (the current stream waits, not the host, under RCCL) and
        yields the flat [world * numel] result in rank order."""
        flat = t.reshape(-1)
        if not self.is_dist:
            return lambda: flat
        dev = t.device
        src = self._wire(flat)
        if self.device_collectives:
            out = torch.empty(self.world * flat.numel(), dtype=t.dtype, device=src.device)
            work = dist.all_gather_into_tensor(out, src, async_op=True)

            def finish():
                work.wait()
                return out.to(dev)
            return finish
        parts = [torch.empty_like(src) for _ in range(self.world)]
        work = dist.all_gather(parts, src, async_op=True)

        def finish_host():
            work.wait()
            return torch.cat(parts).to(dev)
        return finish_host

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor) -> Callable[[], None]:
        """Start an all-gather of equally sized ``t`` into the preallocated
        ``out`` ([world * t.numel()], rank order) and return the function
        that makes the current stream wait for it (RCCL: a stream wait, no
        host wait).  Persistent buffers, so a captured HIP graph can read the
        result every step (``models.spgemm.RowblockGraph``)."""
        flat = t.reshape(-1)
        if out.numel() != self.world * flat.numel():
            raise ValueError(f"all_gather_into: {out.numel()} != {self.world} x {flat.numel()}")
        if not self.is_dist:
            out.copy_(flat)
            return lambda: None
        if self.device_collectives and out.device == self.device and out.is_contiguous():
            work = dist.all_gather_into_tensor(out, flat.contiguous(), async_op=True)
            return lambda: (work.wait(), None)[1]
        got = self.all_gather_async(t)
        return lambda: (out.copy_(got()), None)[1]

    def all_to_all_v(self, x: torch.Tensor, send: List[int], recv: List[int]) -> torch.Tensor:
        """Rank r sends x[sum(send[:p]) : sum(send[:p + 1])] to rank p and
        receives recv[p] elements from each rank p (concatenated, rank
        order).  1-D tensors; counts are in elements."""
        if not self.is_dist:
            return x
        src = self._wire(x)
        out = torch.empty(sum(recv), dtype=x.dtype, device=src.device)
        dist.all_to_all_single(out, src, list(recv), list(send))
        return out.to(x.device)

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place reduction over ranks."""
        if not self.is_dist:
            return t
        if self.device_collectives and t.device == self.device and t.is_contiguous():
            dist.all_reduce(t, op=_REDUCE_OPS[op])
            return t
        w = self._wire(t).clone()
        dist.all_reduce(w, op=_REDUCE_OPS[op])
        t.copy_(w)
        return t

    def reduce_scatter(self, full: torch.Tensor) -> torch.Tensor:
        """Sum of every rank's ``full`` [world * c, ...], block ``rank``
        ([c, ...]) of it on this rank."""
        if not self.is_dist:
            return full
        c = full.shape[0] // self.world
        if self.device_collectives:
            src = self._wire(full)
            out = torch.empty((c,) + tuple(full.shape[1:]), dtype=full.dtype, device=src.device)
            dist.reduce_scatter_tensor(out, src)
            return out.to(full.device)
        w = self._wire(full).clone()   # gloo has no reduce-scatter: all-reduce, keep this rank's block
        dist.all_reduce(w)
        return w[self.rank * c:(self.rank + 1) * c].to(full.device)

    def send(self, t: torch.Tensor, dst: int) -> None:
        dist.send(self._wire(t), dst)

    def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
        """Receive into ``t`` (any device) and return it."""
        w = t if (self.device_collectives and t.device == self.device and t.is_contiguous()) else \
            torch.empty(t.shape, dtype=t.dtype, device=self._wire_device())
        dist.recv(w, src)
        if w is not t:
            t.copy_(w)
        return t

    def allreduce_max(self, x: float) -> float:
        return self._allreduce_scalar(x, "max")

    def allreduce_sum(self, x: float) -> float:
        return self._allreduce_scalar(x, "sum")

    def _allreduce_scalar(self, x: float, op: str) -> float:
        if not self.is_dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self._wire_device())
        self.all_reduce_(t, op)
        return float(t.item())

    def gather_ints(self, x: int) -> List[int]:
        """Every rank's integer, rank order (small host-visible exchange)."""
        if not self.is_dist:
            return [int(x)]
        return [int(v) for v in self.all_gather(torch.tensor([int(x)], dtype=torch.int64,
                                                             device=self._wire_device())).tolist()]

    # --- BSR transport -------------------------------------------------------
    def send_bsr(self, M: BSR, dst: int) -> None:
        hdr = torch.tensor([M.rows, M.cols, M.nb, M.k], dtype=torch.int64, device=self._wire_device())
        self.send(hdr, dst)
        if M.nb:
            self.send(M.keys, dst)
            self.send(M.vals, dst)

    def recv_bsr(self, src: int) -> BSR:
        hdr = self.recv(torch.empty(4, dtype=torch.int64, device=self._wire_device()), src)
        rows, cols, nb, k = (int(x) for x in hdr.tolist())
        keys = torch.empty((nb, 2), dtype=torch.int32, device=self.device)
        vals = torch.empty((nb, k, k), dtype=torch.int64, device=self.device)
        if nb:
            self.recv(keys, src)
            self.recv(vals, src)
        return BSR(rows, cols, k, keys, vals)

    def barrier(self) -> None:
        if self.is_dist:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def close(self) -> None:
        if self.is_dist and dist.is_initialized():
            dist.destroy_process_group()


def init(backend: str = "auto", device: str = "auto", timeout_s: Optional[float] = None) -> Comm:
    """Create the process group for this launch.

    backend: ``auto`` (nccl when GPUs are visible, else gloo), ``nccl``,
    ``gloo``.  device: ``auto`` (cuda:LOCAL_RANK when available, else cpu),
    ``cuda`` or ``cpu``.

    timeout_s (default ``CONFIG.comm_timeout_s``, env ``SPMM_COMM_TIMEOUT``,
    600 s; the test suite sets 120 s): a collective that has not completed by then raises (gloo) or
    aborts the communicator and the process (RCCL watchdog), so a stuck rank
    names itself instead of hanging the job past a launcher's silence window.
    The reference's blocking MPI calls have no timeout at all
    (sparse_matrix_mult.cu:474-537).

    Single-node jobs rendezvous on the loopback interface: gloo binds to
    ``lo`` (``GLOO_SOCKET_IFNAME``) unless the caller chose an interface,
    because its default resolves the host name, which a container may not
    resolve or may map to an address its peers cannot reach (a pair connect
    then waits out the whole timeout).
    """
    from ..utils.config import CONFIG

    if timeout_s is None:
        timeout_s = CONFIG.comm_timeout_s
    rank, world, local = launcher_env()
    use_gpu = torch.cuda.is_available() if device == "auto" else device.startswith("cuda")
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", local % max(ndev, 1))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if world <= 1 and not os.environ.get("SPMM_FORCE_DIST"):
        return Comm(0, 1, 0, dev, None)
    # SPMM_FORCE_DIST=1: a one-rank process group, so the collective code paths
    # (RCCL on a GPU box with a single card) run for real in tests
    if backend == "auto":
        backend = "nccl" if use_gpu else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    if backend == "gloo" and os.environ["MASTER_ADDR"] in ("127.0.0.1", "localhost") and \
            not os.environ.get("GLOO_SOCKET_IFNAME"):
        os.environ["GLOO_SOCKET_IFNAME"] = "lo"
    kw = dict(backend=backend, rank=rank, world_size=world,
              timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        kw["device_id"] = dev
    if not dist.is_initialized():
        dist.init_process_group(**kw)
    return Comm(rank, world, local, dev, backend)
