"""Ordered chain product  A_1 . A_2 . ... . A_N  of block-sparse uint64 matrices.

This is the reference's whole workload:

* ``extract`` (sparse_matrix_mult.cu:328-401): OpenMP tasks parse the rank's
  files, then ``helper2`` (:287-327) reduces them with a level-by-level
  pairwise tree, printing ``multiplying <i> <i+1>`` per product.
* ``main`` (:437-571): contiguous chain ranges per MPI rank, linear gather of
  the partials to rank 0, a second pairwise tree on rank 0's GPU, zero-tile
  prune, ``./matrix`` writer.

MI355X design:

* Loading is pipelined: a loader thread parses files (all host threads per
  file, libspmm_host.so) into pinned memory and DMAs them to HBM on a copy
  stream while the compute stream is already multiplying the first pairs of
  the tree's first level.
* The tree has the reference's shape (its association order is part of the
  exact arithmetic), but every product runs on the GPU with no host round
  trip; independent products of one level overlap on separate HIP streams.
* The cross-rank reduction is a distributed binomial tree over RCCL (see
  :mod:`..parallel.comm`), so no single GPU funnels all partials, and each
  tree product is row-panel split over the ranks its step leaves idle.
"""
from __future__ import annotations

import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import torch

from ..ops.bsr import BSR, bsr_matmul, prune_zero_tiles, tile_pair_count
from ..parallel.comm import Comm
from ..parallel.partition import chain_ranges, chain_ranges_balanced
from ..utils import refio

Log = Callable[[str], None]


@dataclass
class ChainStats:
    products: int = 0
    tile_pairs: int = 0            # 2*k^3 integer ops each
    t_load: float = 0.0
    t_reduce: float = 0.0
    t_comm: float = 0.0
    t_write: float = 0.0
    bytes_h2d: int = 0
    bytes_p2p: int = 0
    log: List[str] = field(default_factory=list)

    def as_dict(self, k: int) -> dict:
        ops = self.tile_pairs * 2 * k ** 3
        t = self.t_reduce
        return dict(products=self.products, tile_pairs=self.tile_pairs, int_ops=ops,
                    t_load_s=self.t_load, t_reduce_s=self.t_reduce, t_comm_s=self.t_comm,
                    t_write_s=self.t_write, bytes_h2d=self.bytes_h2d, bytes_p2p=self.bytes_p2p,
                    reduce_gops=(ops / t / 1e9) if t > 0 else None)


class _Loader(threading.Thread):
    """Parses matrix files in order and stages them onto the device."""

    def __init__(self, folder: str, lo: int, hi: int, k: int, device: torch.device, nthreads: int):
        super().__init__(daemon=True)
        self.folder, self.lo, self.hi, self.k = folder, lo, hi, k
        self.device, self.nthreads = device, nthreads
        self.q: "queue.Queue" = queue.Queue()
        self.bytes = 0

    def run(self) -> None:
        try:
            use_gpu = self.device.type == "cuda"
            stream = torch.cuda.Stream(self.device) if use_gpu else None
            for i in range(self.lo, self.hi + 1):
                M = refio.read_matrix(refio.matrix_path(self.folder, i + 1), self.k, self.nthreads, pin=use_gpu)
                self.bytes += M.nbytes()
                ev = None
                if use_gpu:
                    with torch.cuda.stream(stream):
                        M = M.to(self.device, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(stream)
                self.q.put((M, ev))
        except BaseException as e:  # surfaced in the consumer
            self.q.put(e)

    def get(self) -> BSR:
        item = self.q.get()
        if isinstance(item, BaseException):
            raise item
        M, ev = item
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        return M


def reduce_tree(mats: List[BSR], start: int, log: Optional[Log], stats: Optional[ChainStats] = None,
                source=None, streams: int = 1) -> BSR:
    """``helper2``: pairwise tree, level by level, odd tail carried.

    ``mats`` may be shorter than the chain when ``source`` (a loader) is given:
    level 0 pulls matrices from it as they land, so products start before the
    last file is parsed.  ``streams`` > 1 (GPU): the independent products of a
    level are issued round-robin on a pool of HIP streams (``a4 --streams``),
    so one product's kernels overlap the next one's host-side planning.
    """
    n = len(mats) if source is None else (source.hi - source.lo + 1)
    arr: List[Optional[BSR]] = list(mats) if source is None else []
    pool = _StreamPool(streams, mats[0].device if mats else (source.device if source is not None else None))
    if source is not None:
        level0: List[BSR] = []
        for j, ind in enumerate(range(0, n - 1, 2)):
            a = source.get()
            b = source.get()
            if log:
                log(f"multiplying {start + ind} {start + ind + 1}")
            level0.append(pool.mul(j, a, b, stats))
        if n % 2 == 1:
            level0.append(source.get())
        pool.join(level0)
        if n == 1:
            return level0[0]
        arr = level0
    while len(arr) > 1:
        nxt = []
        for j, ind in enumerate(range(0, len(arr) - 1, 2)):
            if log:
                log(f"multiplying {start + ind} {start + ind + 1}")
            nxt.append(pool.mul(j, arr[ind], arr[ind + 1], stats))
        if len(arr) % 2 == 1:
            nxt.append(arr[-1])
        pool.join(nxt)
        arr = nxt
    return arr[0]


class _StreamPool:
    """Round-robin HIP streams for the products of one tree level.  Every
    product's stream waits for the issuing stream first; operands are recorded
    on the stream that reads them and results on the issuing stream, so the
    caching allocator never hands a block to one stream while another still
    uses it."""

    def __init__(self, streams: int, device):
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.on = streams > 1 and dev.type == "cuda"
        self.dev = dev
        self.pool = [torch.cuda.Stream(dev) for _ in range(streams)] if self.on else []
        self.used = set()

    def mul(self, j: int, a: BSR, b: BSR, stats: Optional[ChainStats]) -> BSR:
        if not self.on:
            return _mul(a, b, stats)
        st = self.pool[j % len(self.pool)]
        st.wait_stream(torch.cuda.current_stream(self.dev))
        self.used.add(j % len(self.pool))
        with torch.cuda.stream(st):
            c = _mul(a, b, stats)
        for t in (a.keys, a.vals, b.keys, b.vals):
            t.record_stream(st)
        return c

    def join(self, results: List[BSR]) -> None:
        if not self.on:
            return
        cur = torch.cuda.current_stream(self.dev)
        for i in sorted(self.used):
            cur.wait_stream(self.pool[i])
        self.used.clear()
        for M in results:
            M.keys.record_stream(cur)
            M.vals.record_stream(cur)


def _mul(a: BSR, b: BSR, stats: Optional[ChainStats]) -> BSR:
    if stats is not None:
        stats.products += 1
        stats.tile_pairs += tile_pair_count(a, b)
    return bsr_matmul(a, b, prune=True)


def _sync(dev: torch.device) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def run_chain(folder: str, comm: Comm, out_path: Optional[str] = "matrix", log: Optional[Log] = print,
              nthreads: int = 0, stats: Optional[ChainStats] = None, split: bool = True,
              fast: bool = False, streams: int = 1) -> Optional[BSR]:
    """The full reference pipeline on this rank.  Returns the final product on
    rank 0 (pruned), None elsewhere.  Writes ``out_path`` on rank 0 unless None.
    ``fast``: chain ranges balanced on the matrix files' sizes instead of the
    reference's count split (re-associates the chain: identical output unless
    a partial sum hits the 2^64-1 collapse)."""
    stats = stats if stats is not None else ChainStats()
    n, k = refio.read_size(folder)
    if fast and n >= comm.world:
        import os

        costs = [os.path.getsize(refio.matrix_path(folder, i + 1)) for i in range(n)]
        ranges = chain_ranges_balanced(costs, comm.world)
    else:
        ranges = chain_ranges(n, comm.world)
    my = ranges[comm.rank]
    dev = comm.device
    part: Optional[BSR] = None
    if my is not None:
        t0 = time.perf_counter()
        loader = _Loader(folder, my[0], my[1], k, dev, nthreads)
        loader.start()
        part = reduce_tree([], my[0], log, stats, source=loader, streams=streams)
        _sync(dev)
        loader.join()
        stats.bytes_h2d += loader.bytes
        stats.t_reduce += time.perf_counter() - t0

    if n // comm.world != 0 and comm.world > 1:
        t0 = time.perf_counter()
        part = _binomial_reduce(part, comm, log, stats, split=split)
        _sync(dev)
        stats.t_comm += time.perf_counter() - t0

    if comm.rank != 0:
        return None
    final = prune_zero_tiles(part)
    if out_path is not None:
        t0 = time.perf_counter()
        refio.write_matrix(out_path, final, nthreads)
        stats.t_write += time.perf_counter() - t0
    return final


def row_cuts(keys: torch.Tensor, parts: int) -> List[int]:
    """parts + 1 tile offsets cutting sorted tiles into panels of whole tile
    rows, balanced by tile count (output tile (i, c) only needs tile row i of
    the left operand)."""
    nb = int(keys.shape[0])
    rows = keys[:, 0].tolist()
    cut = [0]
    for i in range(1, parts):
        t = max(cut[-1], nb * i // parts)
        while 0 < t < nb and rows[t] == rows[t - 1]:
            t += 1
        cut.append(t)
    cut.append(nb)
    return cut


def _slice(M: BSR, t0: int, t1: int) -> BSR:
    return BSR(M.rows, M.cols, M.k, M.keys[t0:t1].contiguous(), M.vals[t0:t1].contiguous())


def _binomial_reduce(part: Optional[BSR], comm: Comm, log: Optional[Log], stats: ChainStats,
                     split: bool = True) -> Optional[BSR]:
    """Cross-rank tree with the shape of the reference's helper2 over the P
    partials (:569-571): at step s, the partial of rank g0 (g0 % 2s == 0) is
    multiplied by rank g0+s's.  With ``split`` the product is shared by every
    rank of the group [g0, g0 + 2s) (they would idle otherwise): g0 sends each
    a row panel of its partial, g0+s sends its partial to all, each returns its
    panel of the product and g0 concatenates the panels (disjoint tile-row
    ranges in order: the same bytes as the unsplit product).  Every member
    receives its panel before R, so blocking transports cannot deadlock.
    Printed indices are the reference's level-relative ones."""
    r, p = comm.rank, comm.world
    s = 1
    while s < p:
        g0 = r - r % (2 * s)
        partner = g0 + s
        gend = min(p, g0 + 2 * s)
        if partner >= p:
            s *= 2
            continue
        if not split:
            if r == g0:
                other = comm.recv_bsr(partner)
                stats.bytes_p2p += other.nbytes()
                if log:
                    log(f"multiplying {g0 // s} {g0 // s + 1}")
                part = _mul(part, other, stats)
            elif r == partner:
                comm.send_bsr(part, g0)
                stats.bytes_p2p += part.nbytes()
                part = None
        elif r == g0:
            if log:
                log(f"multiplying {g0 // s} {g0 // s + 1}")
            cut = row_cuts(part.keys, gend - g0)
            for i in range(1, gend - g0):
                piece = _slice(part, cut[i], cut[i + 1])
                comm.send_bsr(piece, g0 + i)
                stats.bytes_p2p += piece.nbytes()
            R = comm.recv_bsr(partner)
            panels = [_mul(_slice(part, cut[0], cut[1]), R, stats)]
            panels += [comm.recv_bsr(g0 + i) for i in range(1, gend - g0)]
            part = BSR(panels[0].rows, panels[0].cols, part.k, torch.cat([q.keys for q in panels]),
                       torch.cat([q.vals for q in panels]))
        elif r < gend:
            L = comm.recv_bsr(g0)
            if r == partner:
                for h in list(range(g0 + 1, gend)) + [g0]:
                    if h != partner:
                        comm.send_bsr(part, h)
                        stats.bytes_p2p += part.nbytes()
                R, part = part, None
            else:
                R = comm.recv_bsr(partner)
            C = _mul(L, R, stats)
            comm.send_bsr(C, g0)
            stats.bytes_p2p += C.nbytes()
        s *= 2
    return part if r == 0 else None


def chain_product(mats: List[BSR], log: Optional[Log] = None, streams: int = 1) -> BSR:
    """In-memory chain product with the single-rank tree (P = 1 association)."""
    if not mats:
        raise ValueError("empty chain")
    return prune_zero_tiles(reduce_tree(mats, 0, log, streams=streams))
