"""Process-group bootstrap and BSR point-to-point transport.

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
* backend ``gloo`` — CPU tensors; used for the CPU backend and for
  multi-process tests without GPUs.

A matrix travels as a fixed 4-int64 header (rows, cols, nb, k) followed, when
nb > 0, by the key and value tensors.  The receiver learns the payload size
from the header before posting the payload receives, so variable-size
partials need no padding.

Launchers (torchrun, mpirun/mpiexec) are recognised from their environment
variables; with none present the job is a single process (loopback).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

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

    # --- transport -------------------------------------------------------
    def _wire_device(self) -> torch.device:
        return self.device if self.backend == "nccl" else torch.device("cpu")

    def send_bsr(self, M: BSR, dst: int) -> None:
        wd = self._wire_device()
        hdr = torch.tensor([M.rows, M.cols, M.nb, M.k], dtype=torch.int64, device=wd)
        dist.send(hdr, dst)
        if M.nb:
            dist.send(M.keys.to(wd).contiguous(), dst)
            dist.send(M.vals.to(wd).contiguous(), dst)

    def recv_bsr(self, src: int) -> BSR:
        wd = self._wire_device()
        hdr = torch.empty(4, dtype=torch.int64, device=wd)
        dist.recv(hdr, src)
        rows, cols, nb, k = (int(x) for x in hdr.tolist())
        keys = torch.empty((nb, 2), dtype=torch.int32, device=wd)
        vals = torch.empty((nb, k, k), dtype=torch.int64, device=wd)
        if nb:
            dist.recv(keys, src)
            dist.recv(vals, src)
        return BSR(rows, cols, k, keys.to(self.device), vals.to(self.device))

    def barrier(self) -> None:
        if self.is_dist:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def allreduce_max(self, x: float) -> float:
        if not self.is_dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self._wire_device())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def close(self) -> None:
        if self.is_dist and dist.is_initialized():
            dist.destroy_process_group()


def init(backend: str = "auto", device: str = "auto", timeout_s: float = 600.0) -> Comm:
    """Create the process group for this launch.

    backend: ``auto`` (nccl when GPUs are visible, else gloo), ``nccl``,
    ``gloo``.  device: ``auto`` (cuda:LOCAL_RANK when available, else cpu),
    ``cuda`` or ``cpu``.
    """
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
    kw = dict(backend=backend, rank=rank, world_size=world,
              timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        kw["device_id"] = dev
    if not dist.is_initialized():
        dist.init_process_group(**kw)
    return Comm(rank, world, local, dev, backend)
