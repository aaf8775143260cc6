"""Distributed CSR SpGEMM: 1D row-block decomposition over RCCL / xGMI.

North-star config "1M x 1M CSR SpGEMM at 0.01 % density, 1D row-block over
8 x MI355X" (BASELINE.json).  The reference distributes a *chain* over MPI
ranks (sparse_matrix_mult.cu:437-456) and funnels partials to rank 0
(:466-571); it has no decomposition of a single product.  Here:

* rank r owns row panel r of A and of B (contiguous rows, chunk-aligned so the
  synthetic matrices do not depend on P);
* B's row panels are all-gathered (row counts first, then columns + values in
  one packed ``all_gather_into_tensor`` over the xGMI ring that overlaps the
  local product counting — B is ~0.9 GB for the 1M config, small against
  288 GB of HBM, so replicating it is the right trade);
* each rank computes its C row panel = A_panel . B with the local gfx950
  SpGEMM; C stays distributed (no reduce needed: rows are disjoint).

``innerdim_spgemm`` is the other 1D decomposition (north-star "reduce-scatter
of C"): rank r holds A's COLUMN panel r and B's row panel r (the same slice
of the inner dimension), computes a full-height sparse partial
C_r = A[:, K_r] . B[K_r, :], and a sparse reduce-scatter sums the partials
into C's row panels: an all-to-all-v over RCCL moves row panel p of every
partial to rank p, which merges the P sorted partial panels with the SpGEMM
kernel itself (``ops.spgemm.csr_sum``: [I .. I] . [C_0; ..; C_{P-1}]).  No
operand is replicated; traffic is the partials' nnz, so it pays when B is
large relative to C (deep inner dimension, few products per output).

``gather_rows`` reassembles a distributed CSR on one rank (tests, output).
"""
from __future__ import annotations

import itertools
import threading
from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

import torch

from ..ops.csr import CSR
from ..ops.spgemm import SpgemmInfo, csr_sum, spgemm
from ..parallel.comm import Comm
from ..parallel.partition import row_panels, weighted_row_panels
from ..utils.gen_csr import pattern_csr, rmat_edges, rmat_nchunks, rmat_perm, uniform_csr


def allgather_csr_rows(panel: CSR, comm: Comm) -> CSR:
    """Concatenate every rank's row panel (same column space) in rank order."""
    if not comm.is_dist:
        return panel
    B_meta, ready = allgather_operand_async(panel, comm)
    return ready()


def gather_rows(panel: CSR, comm: Comm, dst: int = 0) -> Optional[CSR]:
    full = allgather_csr_rows(panel, comm)
    return full if comm.rank == dst else None


class OperandReady:
    """``ready()`` of :func:`allgather_operand_async`: the full right operand.
    ``cols()`` returns it with columns only (values empty) as soon as the
    first of the two payload collectives has landed: the SpGEMM's window
    splits and count kernel read only B's columns, so they run while the
    values are still crossing xGMI."""

    def __init__(self, full: Callable[[], CSR], cols: Optional[Callable[[], CSR]] = None, local: bool = False):
        self._full, self._cols = full, cols
        self.local = local   # the operand never left this rank: its values are already readable

    def __call__(self) -> CSR:
        return self._full()

    def cols(self) -> CSR:
        return self._cols() if self._cols is not None else self._full()


class GatherStats:
    """Observability of the right operand's all-gather (``bench.py`` JSON):
    bytes received per call and the time from issuing the payload
    collectives to the moment the compute stream may read the operand (device
    events on the current stream, read after the timed loop; host clock for
    host panels).  Off unless ``enabled``; recording adds no host sync."""

    def __init__(self):
        self.enabled = False
        self.calls = []   # (bytes, start, end): torch.cuda.Event pairs or perf_counter floats

    def reset(self, enabled: bool = True) -> None:
        self.enabled = enabled
        self.calls = []

    def mark(self, dev: torch.device):
        if dev.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        import time
        return time.perf_counter()

    def summary(self):
        """(total bytes, total ms) over the recorded calls (synchronises)."""
        tot_b, tot_ms = 0, 0.0
        for b, t0, t1 in self.calls:
            tot_b += b
            if t1 is None:
                continue
            if isinstance(t0, float):
                tot_ms += (t1 - t0) * 1e3
            else:
                t1.synchronize()
                tot_ms += t0.elapsed_time(t1)
        return tot_b, tot_ms


GATHER_STATS = GatherStats()


def col_bits(n: int) -> int:
    """Bits per column index of an n-column operand on the wire (32: sent raw)."""
    b = max(1, (n - 1).bit_length())
    return b if b < 30 else 32


def packed_words(entries: int, bits: int) -> int:
    """Words of one rank's column payload (packed: one spare word, the
    unpacker reads two words an entry)."""
    return entries if bits >= 32 else (entries * bits + 31) // 32 + 1


def pack_cols(col: torch.Tensor, bits: int, out: torch.Tensor) -> None:
    """This rank's columns -> its send buffer ``out`` (int32[packed_words]):
    packed to ``bits`` bits each (csr_bitmap_layout.hip bm_pack_bits), or
    copied and zero-padded when sent raw."""
    from ..ops.spgemm import _native as _nat

    n = col.numel()
    if bits >= 32:
        out[:n].copy_(col)
        out[n:].zero_()
        return
    _nat.check(_nat.hip().spmm_pack_bits(_nat.ptr(col), n, bits, _nat.ptr(out), out.numel(),
                                         _nat.stream_ptr(out.device)), "pack_bits")


def unpack_gathered(gc, gv, W: int, gstride: int, cstride: int, bits: int, base: torch.Tensor, max_n: int,
                    col: torch.Tensor, val=None, cv=None) -> None:
    """[W, stride] gathered payloads -> contiguous columns / values
    (csr_bitmap_layout.hip bm_unpack_gathered; see there)."""
    from ..ops.spgemm import _native as _nat

    P = _nat.ptr
    _nat.check(_nat.hip().spmm_spgemm_bm_unpack_gathered(
        P(gc) if gc is not None else None, P(gv) if gv is not None else None, W, gstride, cstride, bits, P(base),
        max_n, P(col), P(val) if val is not None else None, P(cv) if cv is not None else None,
        _nat.stream_ptr(col.device)), "spgemm_bm_unpack_gathered")


def allgather_operand_async(panel: CSR, comm: Comm) -> Tuple[CSR, Callable[[], CSR]]:
    """Right operand of the row-block SpGEMM (every rank's B row panel), in
    stages so the gather overlaps the SpGEMM's setup.

    1. sizes, then the row counts of every panel (small collectives): B's row
       pointer is complete, which is all the product-count / binning / memory
       planning phase of ``spgemm`` reads;
    2. device panels: the columns, then the value bits, as two collectives
       started asynchronously (they run in issue order): the row plan overlaps
       the columns, the window splits and count kernel (columns only) overlap
       the values; each lands in a padded [world, emax] buffer and one native
       pass unpacks it.  Host panels (gloo on CPUs): one
       packed [cols | values] collective and host-side concatenation.

    The collectives are ``comm`` methods, so the device branch is the one
    RCCL runs at P ranks, and the in-process loopback backend drives the same
    branch at any P on one GPU (tests/test_dist_device.py).

    Returns (B with row pointer only, ready): ``ready()`` makes the current
    stream wait for the payload and returns the full CSR; ``ready.cols()``
    the columns-only operand (see :class:`OperandReady`).
    """
    if not comm.is_dist:
        return panel, OperandReady(lambda: panel, local=True)
    dev = panel.device
    W = comm.world
    meta = comm.all_gather(torch.tensor([panel.m, panel.nnz], dtype=torch.int64, device=dev)).view(-1, 2)
    ms, nnzs = meta[:, 0].tolist(), meta[:, 1].tolist()
    mmax, emax = max(ms), max(nnzs)
    cbuf = torch.zeros(mmax, dtype=torch.int64, device=dev)
    cbuf[:panel.m] = panel.rowptr[1:] - panel.rowptr[:-1]
    # counts first: collectives of one group run in issue order, so the small
    # one must not queue behind the payload
    cnt = comm.all_gather(cbuf).view(W, mmax)
    counts = cnt.reshape(-1) if all(x == mmax for x in ms) else torch.cat([cnt[r, :ms[r]] for r in range(W)])
    m = sum(ms)
    rowptr = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    torch.cumsum(counts, 0, out=rowptr[1:])
    nnz = sum(nnzs)
    empty_c = torch.empty(0, dtype=panel.col.dtype, device=dev)
    empty_v = torch.empty(0, dtype=panel.val.dtype, device=dev)
    meta_B = CSR(m, panel.n, rowptr, empty_c, empty_v)
    meta_B._nnz_total = nnz   # the payload is in flight: CSR.nnz (= len(col)) is 0 here
    if emax == 0:
        return meta_B, OperandReady(lambda: CSR(m, panel.n, rowptr, empty_c, empty_v))

    if dev.type == "cuda" and panel.col.dtype == torch.int32 and panel.val.dtype == torch.float32:
        # columns cross the links packed to ceil(log2 n) bits (1M columns: 20 of 32)
        bits = col_bits(panel.n)
        cw = packed_words(emax, bits)
        cb = torch.empty(cw, dtype=torch.int32, device=dev)
        pack_cols(panel.col, bits, cb)
        vb = torch.zeros(emax, dtype=torch.int32, device=dev)
        vb[:panel.nnz] = panel.val.view(torch.int32)
        rec = None
        if GATHER_STATS.enabled:   # bytes this rank receives: row counts + columns + values
            rec = [W * (mmax * 8 + (cw + emax) * 4), GATHER_STATS.mark(dev), None]
            GATHER_STATS.calls.append(rec)
        pay_c = comm.all_gather_async(cb)
        pay_v = comm.all_gather_async(vb)
        base = torch.tensor([0] + list(itertools.accumulate(nnzs)), dtype=torch.int64, device=dev)
        got = {}

        def unpack(gc, gv, col, val, cv):
            unpack_gathered(gc, gv, W, emax, cw, bits, base, emax, col, val, cv)

        def cols() -> CSR:
            if "col" not in got:
                g = pay_c()
                if g.numel() != W * cw:
                    raise RuntimeError(f"operand gather: {g.numel()} column words, expected {W * cw}")
                col = torch.empty(nnz, dtype=torch.int32, device=dev)
                unpack(g, None, col, None, None)
                got["col"] = col
                got["gc"] = g   # the unpack kernel is still reading it (stream order)
            return CSR(m, panel.n, rowptr, got["col"], empty_v)

        def full() -> CSR:
            if "B" not in got:
                col = cols().col
                g = pay_v()
                if g.numel() != W * emax:
                    raise RuntimeError(f"operand gather: {g.numel()} value words, expected {W * emax}")
                val = torch.empty(nnz, dtype=torch.float32, device=dev)
                if rec is not None:
                    rec[2] = GATHER_STATS.mark(dev)   # the compute stream may read the payload from here
                # (no interleaved copy here: the bitmap kernels read B through its
                # padded pair layout, built from col / val by the SpGEMM itself,
                # csr_bitmap_plan.hip)
                unpack(None, g, col, val, None)
                B = CSR(m, panel.n, rowptr, col, val)
                got["B"] = B
                got["gv"] = g
            return got["B"]
        return meta_B, OperandReady(full, cols)

    # generic (host panels, other dtypes): columns and value bits padded per rank
    vbits = {2: torch.int16, 4: torch.int32, 8: torch.int64}[panel.val.element_size()]
    cb = torch.zeros(emax, dtype=panel.col.dtype, device=dev)
    cb[:panel.nnz] = panel.col
    vb = torch.zeros(emax, dtype=vbits, device=dev)
    vb[:panel.nnz] = panel.val.view(vbits)
    rec = None
    if GATHER_STATS.enabled:
        rec = [W * (mmax * 8 + emax * (cb.element_size() + vb.element_size())), GATHER_STATS.mark(dev), None]
        GATHER_STATS.calls.append(rec)
    pay_c = comm.all_gather_async(cb)
    pay_v = comm.all_gather_async(vb)

    done = []

    def ready() -> CSR:
        if not done:
            Gc = pay_c().view(W, emax)
            Gv = pay_v().view(W, emax)
            if rec is not None:
                rec[2] = GATHER_STATS.mark(dev)
            col = torch.cat([Gc[r, :nnzs[r]] for r in range(W)])
            val = torch.cat([Gv[r, :nnzs[r]] for r in range(W)]).view(panel.val.dtype)
            done.append(CSR(m, panel.n, rowptr, col, val))
        return done[0]
    return meta_B, OperandReady(ready)


def allgather_operand(panel: CSR, comm: Comm) -> CSR:
    """Every rank's B row panel as one CSR (blocking form of
    :func:`allgather_operand_async`)."""
    _, ready = allgather_operand_async(panel, comm)
    return ready()


def rowblock_spgemm(A_panel: CSR, B_panel: CSR, comm: Comm, info: Optional[SpgemmInfo] = None) -> CSR:
    """C_panel = A_panel . B, where B = rows of every rank's B_panel; the
    payload of B's all-gather is in flight while the local product counts
    and row binning run."""
    B_meta, ready = allgather_operand_async(B_panel, comm)
    return spgemm(A_panel, B_meta, info, B_ready=ready)


_CAPTURE_LOCK = threading.Lock()   # one graph capture at a time per process (loopback ranks are threads)


def _agree(comm: Comm, ok: bool) -> bool:
    """True on every rank iff ``ok`` on every rank (the ranks must take the
    same collective sequence afterwards)."""
    return comm.allreduce_sum(1.0 if ok else 0.0) == comm.world


class RowblockGraph:
    """The row-block SpGEMM step (B's panels all-gathered over RCCL, then
    C_panel = A_panel . B on the bitmap-rank kernels) with NO host
    synchronisation inside the step, for operands of fixed structure: the
    reference's per-rank product + merge (sparse_matrix_mult.cu:437-571) as
    an inspector / executor pair.

    Built once per operand structure (collective: every rank constructs it):
    the panel sizes and row counts are gathered here, once (the only host
    read-backs), B's full row pointer is formed, the bitmap plan is made from
    A's row plan against it, and every buffer the step touches is allocated
    -- the send buffers, the [world, emax] receive buffers, B's unpacked
    columns and values, the plan's workspace, C at its product-count bound.
    Two HIP graphs are captured on a side stream:

      graph 1: B's column layouts (window splits, packed bounds, padded count
               columns), count kernel, unit scan;
      graph 2: padded pairs, numeric + reload.

    The layout passes read B in place from the gathered [world, stride]
    buffers (columns unpacked from their 20-bit packing on the fly) when the
    plan's kernels read B only through its padded layouts (the 1M config:
    ``ops.spgemm.bitmap_gathered_ok``); otherwise graph 1 / graph 2 first
    unpack the gathered columns / values into B's arrays.

    ``run()`` = copy this rank's B panel (columns packed to ceil(log2 n) bits,
    value bits) into the send
    buffers, start the two payload all-gathers (RCCL runs them in issue order
    on its own stream), make the compute stream wait for the columns and
    replay graph 1 -- the count kernel runs while the values cross xGMI --
    then wait for the values and replay graph 2.  Every step re-gathers and
    recomputes everything from the panels' current columns and values (only
    the row counts are fixed); :meth:`result` reads the nnz and error bits
    of the last step once.  A product that does not take the bitmap-rank
    path raises ``ValueError`` on every rank (the caller runs the eager
    ``rowblock_spgemm``)."""

    def __init__(self, A_panel: CSR, B_panel: CSR, comm: Comm):
        from ..ops import spgemm as SG

        dev = A_panel.device
        local_ok = (dev.type == "cuda" and comm.device_collectives and B_panel.col.dtype == torch.int32
                    and B_panel.val.dtype == torch.float32 and A_panel.val.dtype == torch.float32)
        if not _agree(comm, local_ok):
            raise ValueError("RowblockGraph: fp32 / int32 GPU operands and device collectives on every rank")
        W = comm.world
        self.A, self.Bp, self.comm = A_panel, B_panel, comm
        # ---- the operand structure: gathered once ---------------------------
        meta = comm.all_gather(torch.tensor([B_panel.m, B_panel.nnz], dtype=torch.int64, device=dev)).view(-1, 2)
        ms, nnzs = meta[:, 0].tolist(), meta[:, 1].tolist()
        mmax, emax = max(ms), max(nnzs)
        cbuf = torch.zeros(max(mmax, 1), dtype=torch.int64, device=dev)
        cbuf[:B_panel.m] = B_panel.rowptr[1:] - B_panel.rowptr[:-1]
        cnt = comm.all_gather(cbuf).view(W, -1)
        m, nnz = sum(ms), sum(nnzs)
        rowptr = torch.zeros(m + 1, dtype=torch.int64, device=dev)
        torch.cumsum(torch.cat([cnt[r, :ms[r]] for r in range(W)]), 0, out=rowptr[1:])
        self.B = CSR(m, B_panel.n, rowptr, torch.zeros(nnz, dtype=torch.int32, device=dev),
                     torch.zeros(nnz, dtype=torch.float32, device=dev))
        self.emax = emax
        # ---- the plan (A's row plan reads only B's row pointer) --------------
        plan = None
        info = SG.SpgemmInfo()
        if emax > 0 and A_panel.n == m and A_panel.nnz > 0:
            nprod, _, st = SG.row_plan(A_panel, self.B)
            tot, mx, nz, light, _h1, _h2, _h4, _h8, amax = st.tolist()[:9]
            pre = dict(max=mx, nonempty=nz, light=light, amax=amax)
            info.flops, info.mean_seg = 2 * tot, tot / max(A_panel.nnz, 1)
            if SG._bitmap_ok(A_panel, self.B, tot, pre):
                plan = SG._bitmap_plan(A_panel, self.B, info, pre)
                if plan is not None and plan.det:
                    plan = None
        if not _agree(comm, plan is not None):
            raise ValueError("RowblockGraph: the product does not take the bitmap-rank path on every rank")
        self.plan, self.flops = plan, info.flops
        # send buffers: columns packed to ceil(log2 n) bits, value bits raw
        self.bits = col_bits(B_panel.n)
        self.cw = packed_words(emax, self.bits)
        self.cb = torch.zeros(self.cw, dtype=torch.int32, device=dev)
        self.vb = torch.zeros(emax, dtype=torch.int32, device=dev)
        self.gc = torch.empty(W * self.cw, dtype=torch.int32, device=dev)
        self.gv = torch.empty(W * emax, dtype=torch.int32, device=dev)
        self.base = torch.tensor([0] + list(itertools.accumulate(nnzs)), dtype=torch.int64, device=dev)
        self.bufs = SG.bitmap_buffers(plan, dev, cap=max(plan.raw.tot, 1))
        self.bufs["n"] = B_panel.n
        self.gather_bytes = W * (self.cw + emax) * 4
        if hasattr(comm, "bind_payloads"):   # (an emulated group: it builds the peers' payloads the same way)
            comm.bind_payloads(self._col_payload, self._val_payload)
        # B read in place from the gathered panels by the layout passes when the plan's kernels
        # read B only through its padded layouts (the 1M config): no unpack passes, and B's
        # column / value arrays are never formed
        self.gview = None
        if SG.bitmap_gathered_ok(plan):
            P = SG._native.ptr
            self.rbase = torch.tensor([0] + list(itertools.accumulate(ms)), dtype=torch.int64, device=dev)
            mk = lambda gv: SG.BmGathered(gc=P(self.gc), gv=gv, ebase=P(self.base), rbase=P(self.rbase),  # noqa: E731
                                          cstride=self.cw, vstride=emax, W=W, bits=self.bits)
            self.gview = (mk(None), mk(P(self.gv)))   # (front: columns only; back: columns and values)
            self.B = CSR(m, B_panel.n, rowptr, torch.zeros(0, dtype=torch.int32, device=dev),
                         torch.zeros(0, dtype=torch.float32, device=dev))
        # ---- one eager step (checks every launch and the kernels' error bits:
        # a product the row kernels cannot take, or with units beyond the reload
        # kernel, is not replayed), then the capture ---------------------------
        self._step(None, None)
        if not _agree(comm, int(self.bufs["z"][0]) == 0):
            raise ValueError("RowblockGraph: the bitmap kernels flagged this product on a rank (eager steps)")
        err = None
        # (every rank past its eager launches before any captures, and each capture
        # alone: in-process loopback ranks are threads of one device, and no thread
        # may launch while another's capture is open)
        comm.barrier()
        try:
            with _CAPTURE_LOCK:
                side = torch.cuda.Stream(dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                self.g1, self.g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.g1, stream=side, capture_error_mode="thread_local"):
                    self._front()
                with torch.cuda.graph(self.g2, stream=side, capture_error_mode="thread_local"):
                    self._back()
                torch.cuda.current_stream(dev).wait_stream(side)
        except RuntimeError as e:   # (a capture failure on one rank: every rank takes the eager step)
            err = e
        comm.barrier()
        if not _agree(comm, err is None):
            raise ValueError(f"RowblockGraph: graph capture failed on a rank ({err})")

    def _col_payload(self, panel: CSR, out: torch.Tensor) -> None:
        pack_cols(panel.col, self.bits, out)

    def _val_payload(self, panel: CSR, out: torch.Tensor) -> None:
        n = panel.nnz
        out[:n].copy_(panel.val.view(torch.int32))

    def _unpack(self, gc, gv) -> None:
        unpack_gathered(gc, gv, self.comm.world, self.emax, self.cw, self.bits, self.base, self.emax, self.B.col,
                        self.B.val if gv is not None else None)

    def _front(self) -> None:
        from ..ops import spgemm as SG

        if self.gview is not None:
            self.built = SG.bitmap_front(self.A, self.B, self.plan, self.bufs, values=False, gathered=self.gview[0])
            return
        self._unpack(self.gc, None)
        self.built = SG.bitmap_front(self.A, self.B, self.plan, self.bufs, values=False)

    def _back(self) -> None:
        from ..ops import spgemm as SG

        if self.gview is not None:
            SG.bitmap_back(self.A, self.B, self.plan, self.bufs, self.built, gathered=self.gview[1])
            return
        self._unpack(None, self.gv)
        SG.bitmap_back(self.A, self.B, self.plan, self.bufs, self.built)

    def _step(self, g1, g2) -> dict:
        self._col_payload(self.Bp, self.cb)
        self._val_payload(self.Bp, self.vb)
        rec = None
        if GATHER_STATS.enabled:
            rec = [self.gather_bytes, GATHER_STATS.mark(self.A.device), None]
            GATHER_STATS.calls.append(rec)
        wait_c = self.comm.all_gather_into(self.gc, self.cb)
        wait_v = self.comm.all_gather_into(self.gv, self.vb)
        wait_c()
        g1.replay() if g1 is not None else self._front()
        wait_v()
        if rec is not None:
            rec[2] = GATHER_STATS.mark(self.A.device)
        g2.replay() if g2 is not None else self._back()
        return self.bufs

    def run(self) -> dict:
        """One step: gathers + both graphs, no host synchronisation."""
        return self._step(self.g1, self.g2)

    def result(self, info: Optional[SpgemmInfo] = None) -> Optional[CSR]:
        """This rank's C row panel of the last step (one read-back)."""
        from ..ops import spgemm as SG

        info = info if info is not None else SpgemmInfo()
        C_ = SG._bitmap_finish(self.A, self.B, self.plan, self.bufs, info, True)
        if isinstance(C_, str):
            raise RuntimeError("RowblockGraph: B's window segments no longer fit the packed 16-bit lengths")
        return C_


def sparse_reduce_scatter(partial: CSR, comm: Comm, row_counts: List[int],
                          info: Optional[SpgemmInfo] = None) -> CSR:
    """Sum every rank's full-height ``partial`` (same m x n on all ranks) and
    return this rank's row panel of the sum (panels of ``row_counts`` rows,
    rank order).

    Three all-to-all-v exchanges (RCCL over xGMI, or gloo): per-destination
    nnz, per-row counts (fixed-size, panel r is rows of rank r), then the
    columns and values — partial rows are contiguous in CSR, so the send
    buffers are the partial's own arrays, no packing copy.  The received
    panels are merged on the SpGEMM kernels (``csr_sum``)."""
    if not comm.is_dist:
        return partial
    if sum(row_counts) != partial.m or len(row_counts) != comm.world:
        raise ValueError(f"row_counts {row_counts} do not split {partial.m} rows over {comm.world} ranks")
    W = comm.world
    dev = partial.device
    offs = [0]
    for c in row_counts:
        offs.append(offs[-1] + c)
    bounds = partial.rowptr[torch.tensor(offs, device=dev)]
    nnz_to = bounds[1:] - bounds[:-1]
    nnz_from = comm.all_to_all_v(nnz_to, [1] * W, [1] * W)
    send_n, recv_n = nnz_to.tolist(), nnz_from.tolist()
    mp = row_counts[comm.rank]
    cnt = partial.rowptr[1:] - partial.rowptr[:-1]
    cnt_from = comm.all_to_all_v(cnt, list(row_counts), [mp] * W).view(W, mp)
    col = comm.all_to_all_v(partial.col, send_n, recv_n)
    val = comm.all_to_all_v(partial.val.float(), send_n, recv_n)
    parts, e = [], 0
    for r in range(W):
        rp = torch.zeros(mp + 1, dtype=torch.int64, device=dev)
        torch.cumsum(cnt_from[r], 0, out=rp[1:])
        parts.append(CSR(mp, partial.n, rp, col[e:e + recv_n[r]], val[e:e + recv_n[r]]))
        e += recv_n[r]
    return csr_sum(parts, info)


def innerdim_spgemm(A_colpanel: CSR, B_panel: CSR, comm: Comm, row_counts: List[int],
                    info: Optional[SpgemmInfo] = None) -> CSR:
    """C's row panel of this rank, where rank r holds A[:, K_r] (all rows,
    columns re-indexed from 0) and B[K_r, :]: local full-height partial
    product, then :func:`sparse_reduce_scatter`.  ``info`` counts the local
    product's FLOPs (the merge's additions are not counted)."""
    local = spgemm(A_colpanel, B_panel, info)
    if info is not None:
        info.partial_nnz = local.nnz
    return sparse_reduce_scatter(local, comm, row_counts)


STREAM_MEM_FRACTION = 0.4   # of free device memory for one panel's C bound + staging (16 B / product)


def stream_budget(dev: torch.device) -> int:
    """Intermediate products per streamed row panel: the panel's product-count
    bound C plus an equal staging buffer (the one-pass mode) in a fixed share
    of the free device memory."""
    if dev.type != "cuda":
        return 1 << 28
    free, _ = torch.cuda.mem_get_info(dev)
    free += torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    return max(1 << 24, int(STREAM_MEM_FRACTION * free) // 16)


def stream_panels(nprod: torch.Tensor, budget: int) -> List[Tuple[int, int]]:
    """Contiguous row panels of at most ``budget`` products each (a row with
    more products is a panel of its own)."""
    m = nprod.numel()
    if m == 0:
        return []
    prefix = torch.cumsum(nprod.long(), 0)
    total = int(prefix[-1])
    if total <= budget:
        return [(0, m)]
    panels, lo, done = [], 0, 0
    while lo < m:
        # last row whose prefix stays within done + budget (at least one row)
        hi = int(torch.searchsorted(prefix, torch.tensor([done + budget], device=prefix.device), right=True))
        hi = min(max(hi, lo + 1), m)
        panels.append((lo, hi))
        done = int(prefix[hi - 1])
        lo = hi
    return panels


def streamed_spgemm(A: CSR, B: CSR, consume: Callable[[int, int, CSR], None], budget: Optional[int] = None,
                    info: Optional[SpgemmInfo] = None, overlap: bool = False) -> SpgemmInfo:
    """C = A . B produced in row panels and handed to ``consume(lo, hi,
    C[lo:hi])`` one at a time, so C never has to be resident: R-MAT scale-24
    A.A^T has ~10^12 intermediate products and a C of several TB, more than
    8 x 288 GB of HBM.  Every panel is a complete SpGEMM of A's rows lo..hi
    against all of B (nothing is skipped); only C's lifetime is bounded.  The
    reference bounds its device footprint the same way, with rounds of <= 500
    output tiles copied back to the host (sparse_matrix_mult.cu:181-270).

    ``overlap``: a panel is handed to ``consume`` while its last copies (the
    compaction and the long-row placement, on the side stream) may still be
    writing its column / value arrays -- its row pointer and nnz are final --
    so the next panel's planning and kernels overlap them; a consumer that
    reads C's arrays first calls ``ops.spgemm.wait_ready(C)``.  Every product
    and every write still happens (a device synchronise covers them all)."""
    info = info if info is not None else SpgemmInfo()
    from ..ops.spgemm import row_nprod

    nprod = row_nprod(A, B)
    budget = budget if budget is not None else stream_budget(A.device)
    todo = list(reversed(stream_panels(nprod, budget)))
    while todo:
        lo, hi = todo.pop()
        pi = SpgemmInfo()
        try:
            if overlap:
                from ..ops.spgemm import deferred_placement

                with deferred_placement():
                    C = spgemm(A.row_slice(lo, hi), B, pi)
            else:
                C = spgemm(A.row_slice(lo, hi), B, pi)
        except torch.OutOfMemoryError:
            # the budget was a forecast: split the panel and go on with a
            # smaller budget (a single row that does not fit is a real limit)
            if hi - lo <= 1:
                raise
            if A.device.type == "cuda":   # drain the failed attempt before its blocks are reused
                torch.cuda.synchronize(A.device)
                torch.cuda.empty_cache()
            mid = (lo + hi) // 2
            todo += [(mid, hi), (lo, mid)]
            info.rows_per_bin_num["oom_splits"] = info.rows_per_bin_num.get("oom_splits", 0) + 1
            continue
        info.flops += pi.flops
        info.nnz += pi.nnz
        info.resorted_rows += pi.resorted_rows
        for b, c in pi.rows_per_bin_num.items():
            info.rows_per_bin_num[b] = info.rows_per_bin_num.get(b, 0) + c
        consume(lo, hi, C)
        del C
    info.mean_seg = info.flops / 2 / max(A.nnz, 1)
    return info


@dataclass
class UniformProblem:
    """A, B uniform random n x n at ``density``; this rank's row panels."""

    n: int
    density: float
    seed: int
    rows: Tuple[int, int]
    A: CSR
    B: CSR

    @staticmethod
    def build(n: int, density: float, comm: Comm, seed: int = 1) -> "UniformProblem":
        # any split yields the same global matrices (the generator is chunk-seeded)
        panels = row_panels(n, comm.world)
        lo, hi = panels[comm.rank]
        A = uniform_csr(n, n, density, seed=seed, device=comm.device, rows=(lo, hi))
        B = uniform_csr(n, n, density, seed=seed + 1, device=comm.device, rows=(lo, hi))
        return UniformProblem(n, density, seed, (lo, hi), A, B)

    def inner_operand(self) -> CSR:
        """A's column panel over this rank's inner-dimension slice (the rows
        ``self.rows`` of B), for :func:`innerdim_spgemm`: generated in full
        (chunk-seeded, so identical on every rank) and column-sliced."""
        lo, hi = self.rows
        A = uniform_csr(self.n, self.n, self.density, seed=self.seed, device=self.A.device)
        return A.col_slice(lo, hi)


def shuffle_entries(comm: Comm, rows: torch.Tensor, cols: torch.Tensor, vals: Optional[torch.Tensor],
                    cuts: List[int]):
    """Send every entry (row, col[, val]) to the rank that owns ``row`` (rank r
    owns rows [cuts[r], cuts[r + 1])): one all-to-all-v of the counts, one of
    the packed int64 records (float64 values travel as their bit patterns).
    Returns the (rows, cols, vals) this rank received, in rank order."""
    if not comm.is_dist:
        return rows, cols, vals
    W = comm.world
    dev = rows.device
    inner = torch.tensor(cuts[1:-1], dtype=torch.int64, device=dev)
    dest = torch.searchsorted(inner, rows, right=True)
    order = torch.argsort(dest, stable=True)
    send = torch.bincount(dest, minlength=W)
    fields = [rows[order], cols[order]]
    if vals is not None:
        fields.append(vals.to(torch.float64)[order].view(torch.int64))
    k = len(fields)
    packed = torch.stack(fields, 1).reshape(-1)
    del order, dest, fields
    recv = comm.all_to_all_v(send, [1] * W, [1] * W)
    got = comm.all_to_all_v(packed, (k * send).tolist(), (k * recv).tolist()).view(-1, k)
    return got[:, 0].contiguous(), got[:, 1].contiguous(), (got[:, 2].contiguous().view(torch.float64)
                                                             if vals is not None else None)


def shuffle_pairs(comm: Comm, rows: torch.Tensor, cols: torch.Tensor, cuts: List[int]) -> Tuple[torch.Tensor, torch.Tensor]:
    """:func:`shuffle_entries` of a 0/1 pattern."""
    r, c, _ = shuffle_entries(comm, rows, cols, None, cuts)
    return r, c


def read_mtx_rowblock(path: str, comm: Comm, dtype=torch.float32) -> Tuple[CSR, int, List[int]]:
    """This rank's row panel of a Matrix Market file (row_panels split): every
    rank parses 1/P of the file's text, the entries go to their row owners
    (all-to-all-v) and each owner sums duplicates into its CSR panel — no rank
    reads or holds the whole matrix (reference: rank-local loading of its
    share of the chain, sparse_matrix_mult.cu:437-456).  Returns (panel,
    its first row, the panel cuts of every rank)."""
    from ..ops.csr import from_coo
    from ..utils.mtx import read_mtx_coo

    m, n, ri, ci, v = read_mtx_coo(path, comm.rank, comm.world,
                                   gather_counts=comm.gather_ints if comm.is_dist else None)
    cuts = [lo for lo, _ in row_panels(m, comm.world)] + [m]
    dev = comm.device
    ri, ci, v = shuffle_entries(comm, ri.to(dev), ci.to(dev), v.to(dev), cuts)
    lo, hi = cuts[comm.rank], cuts[comm.rank + 1]
    A = from_coo(ri - lo, ci, v, hi - lo, n, sum_duplicates=True, dtype=dtype)
    return A, lo, cuts


def transpose_rowblock(panel: CSR, row0: int, m_total: int, comm: Comm) -> Tuple[CSR, int]:
    """This rank's row panel of A^T (row_panels split of A's columns) from
    the row panels of A: every entry (i, j, v) goes as (j, i, v) to the owner
    of row j of A^T (all-to-all-v).  Returns (panel, its first row)."""
    from ..ops.csr import from_coo

    tcuts = [lo for lo, _ in row_panels(panel.n, comm.world)] + [panel.n]
    tj, ti, tv = shuffle_entries(comm, panel.col.long(), panel.row_ids() + row0, panel.val, tcuts)
    lo, hi = tcuts[comm.rank], tcuts[comm.rank + 1]
    return from_coo(tj - lo, ti, tv, hi - lo, m_total, sum_duplicates=True, dtype=panel.val.dtype), lo


def write_rows_p2p(path: str, panel: CSR, row0: int, comm: Comm, dst: int = 0, pattern: bool = False) -> None:
    """Write a row-distributed CSR (rank r holds rows row0_r .. in rank order)
    as one Matrix Market file on rank ``dst``: the total nnz and row count
    are summed first (header), then ``dst`` receives the panels point-to-point
    in rank order and appends each as it arrives — C is never all-gathered or
    held whole anywhere (reference: partials sent to rank 0, which writes
    ``matrix``, sparse_matrix_mult.cu:466-607)."""
    from ..utils.mtx import MtxWriter

    tot = torch.tensor([panel.m, panel.nnz], dtype=torch.int64, device=panel.device)
    comm.all_reduce_(tot)
    m_tot, nnz_tot = (int(x) for x in tot.tolist())
    if comm.rank != dst:
        comm.send(torch.tensor([row0, panel.m, panel.nnz], dtype=torch.int64, device=panel.device), dst)
        if panel.m:
            comm.send(panel.rowptr[1:] - panel.rowptr[:-1], dst)
        if panel.nnz:
            comm.send(panel.col, dst)
            if not pattern:
                comm.send(panel.val.float(), dst)
        return
    w = MtxWriter(path, m_tot, panel.n, nnz_tot, pattern)
    try:
        for r in range(comm.world):
            if r == dst:
                w.panel(row0, panel)
                continue
            hdr = comm.recv(torch.empty(3, dtype=torch.int64), r)
            r0, mp, nz = (int(x) for x in hdr.tolist())
            cnt = torch.zeros(mp, dtype=torch.int64)
            col = torch.empty(nz, dtype=torch.int32)
            val = torch.empty(0 if pattern else nz, dtype=torch.float32)
            if mp:
                comm.recv(cnt, r)
            if nz:
                comm.recv(col, r)
                if not pattern:
                    comm.recv(val, r)
            rp = torch.zeros(mp + 1, dtype=torch.int64)
            torch.cumsum(cnt, 0, out=rp[1:])
            w.panel(r0, CSR(mp, panel.n, rp, col, val))
    finally:
        w.close()


def csr_chain(paths: List[str], comm: Comm, out_path: Optional[str] = None,
              log: Optional[Callable[[str], None]] = None, info: Optional[SpgemmInfo] = None) -> Tuple[CSR, int]:
    """Ordered product M_1 . M_2 . ... . M_N of Matrix Market files on the CSR
    engine (fp32), the CSR counterpart of the reference's chain
    (sparse_matrix_mult.cu:402-681): the running product stays distributed in
    row panels, every next factor is read 1/P per rank and all-gathered inside
    the row-block multiply, and the result is streamed to rank 0 for writing.
    ``log`` gets the reference's "multiplying i i+1" line per product (rank 0).
    Returns (this rank's row panel of the product, its first row)."""
    if not paths:
        raise ValueError("empty chain")
    panel, row0, _ = read_mtx_rowblock(paths[0], comm)
    for i, path in enumerate(paths[1:], start=1):
        if log is not None and comm.rank == 0:
            log(f"multiplying {i} {i + 1}")
        Bp, _, bcuts = read_mtx_rowblock(path, comm)
        if bcuts[-1] != panel.n:
            raise ValueError(f"{path}: {bcuts[-1]} rows, the product so far has {panel.n} columns")
        pi = SpgemmInfo()
        panel = rowblock_spgemm(panel, Bp, comm, pi)
        if info is not None:
            info.flops += pi.flops
    if out_path:
        write_rows_p2p(out_path, panel, row0, comm)
    return panel, row0


@dataclass
class RmatProblem:
    """BASELINE config 5 (R-MAT A.A^T) as a 1D row-block problem, built the
    distributed way (reference: the rank-local work split and explicit
    inter-rank transfers of sparse_matrix_mult.cu:437-553):

    1. rank r generates its share of the edge chunks (chunk-seeded: the global
       graph does not depend on P), relabelled by the common permutation;
    2. row panels balanced on intermediate products: column degrees and the
       per-row weight sum_{(i,j)} coldeg(j) (duplicate edges included) are
       summed over ranks (two all-reduces of 2^scale entries);
    3. edges go to their row owner (all-to-all-v), which builds its CSR row
       panel A_r (duplicates merged, unit weights);
    4. distributed transpose: every entry (i, j) of A_r goes as (j, i) to the
       owner of row j of A^T (all-to-all-v), which builds its panel At_r;
    5. each step all-gathers the At_r into the right operand A^T (as
       :func:`rowblock_spgemm`) and multiplies its A_r by it."""

    scale: int
    edge_factor: int
    seed: int
    rows: Tuple[int, int]
    cuts: List[int]
    A: CSR
    At: CSR

    @staticmethod
    def build(scale: int, edge_factor: int, comm: Comm, seed: int = 1, chunk: Optional[int] = None) -> "RmatProblem":
        from ..utils import gen_csr

        chunk = chunk or gen_csr.RMAT_CHUNK_EDGES
        dev = comm.device
        n = 1 << scale
        k0, k1 = row_panels(rmat_nchunks(scale, edge_factor, chunk), comm.world)[comm.rank]
        perm = rmat_perm(scale, seed, dev)
        s, d, _ = rmat_edges(scale, edge_factor, seed=seed, device=dev, chunk=chunk, chunks=(k0, k1), perm=perm)
        del perm
        coldeg = comm.all_reduce_(torch.bincount(d, minlength=n))
        w = comm.all_reduce_(torch.zeros(n, dtype=torch.int64, device=dev).index_add_(0, s, coldeg[d]))
        del coldeg
        panels = weighted_row_panels(torch.cumsum(w, 0), comm.world)
        del w
        cuts = [lo for lo, _ in panels] + [n]
        lo, hi = panels[comm.rank]
        rs, cs = shuffle_pairs(comm, s, d, cuts)
        del s, d
        A = pattern_csr(rs, cs, hi - lo, n, row0=lo)
        del rs, cs
        tj, ti = shuffle_pairs(comm, A.col.long(), A.row_ids() + lo, cuts)   # (j, i) to the owner of j
        At = pattern_csr(tj, ti, hi - lo, n, row0=lo)
        return RmatProblem(scale, edge_factor, seed, (lo, hi), cuts, A, At)

    def right_operand(self, comm: Comm) -> CSR:
        """A^T on every rank: the all-gather of the At_r panels."""
        return allgather_operand(self.At, comm)

    def step(self, comm: Comm, info: Optional[SpgemmInfo] = None,
             consume: Optional[Callable[[int, int, CSR], None]] = None, overlap: bool = False) -> Optional[CSR]:
        """One product: C_r = A_r . A^T with A^T all-gathered inside the step.
        Resident (returns C_r, the gather overlapping the row planning) or,
        with ``consume``, streamed in row panels (returns None; ``overlap``:
        see :func:`streamed_spgemm`)."""
        if consume is None:
            return rowblock_spgemm(self.A, self.At, comm, info)
        streamed_spgemm(self.A, self.right_operand(comm), consume, info=info, overlap=overlap)
        return None


def smoke(dev: torch.device) -> None:
    """Tiny SpGEMM on the GPU vs a dense fp32 PyTorch reference."""
    A = uniform_csr(300, 257, 0.05, seed=3, device=dev)
    B = uniform_csr(257, 311, 0.05, seed=4, device=dev)
    C = spgemm(A, B)
    ref = A.to_dense() @ B.to_dense()
    got = C.to_dense()
    assert C.is_sorted(), "SpGEMM output not column-sorted"
    err = (got - ref).abs().max().item()
    assert err < 1e-4, f"SpGEMM mismatch {err}"
    # structural: every reference non-zero present
    assert int(((ref != 0) & (got == 0)).sum()) == 0
