"""Runtime configuration (replaces the reference's compile-time globals).

Reference constants (sparse_matrix_mult.cu): ``BIG_SIZE = 1e9`` staging
elements (:22), ``small_size = 500`` output tiles per GPU round (:23),
``num_threads(16)`` parser threads (:334), ``CHUNK_KEYS = 262144`` /
``CHUNK_VALS = 4194304`` MPI message chunks (:467-468).  None of those is
needed here (tiles stay in HBM, RCCL chunks internally); what remains
tunable is read from the environment (``SPMM_*``) with these defaults.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field, fields


def _env(name: str, default, cast):
    v = os.environ.get(name)
    return default if v in (None, "") else cast(v)


@dataclass
class Config:
    threads: int = field(default_factory=lambda: _env("SPMM_THREADS", 0, int))          # 0 = all host threads
    device: str = field(default_factory=lambda: _env("SPMM_DEVICE", "auto", str))
    comm: str = field(default_factory=lambda: _env("SPMM_COMM", "auto", str))
    streams: int = field(default_factory=lambda: _env("SPMM_STREAMS", 4, int))           # chain-level concurrency
    spgemm_load: float = field(default_factory=lambda: _env("SPMM_SPGEMM_LOAD", 0.5, float))   # single-pass LDS tables
    # 16K-key (symbolic) / 8K-slot (numeric) tables of long rows: a higher load
    # means fewer column slices, i.e. fewer re-reads of the B rows
    spgemm_load_sliced: float = field(default_factory=lambda: _env("SPMM_SPGEMM_LOAD_SLICED", 0.5, float))
    # SpGEMM without the symbolic phase (product-count staging buffer + compaction):
    # "auto" = when twice the product count fits in 80% of free memory
    spgemm_onepass: str = field(default_factory=lambda: _env("SPMM_SPGEMM_ONEPASS", "auto", str))
    spgemm_esc_min: int = field(default_factory=lambda: _env("SPMM_SPGEMM_ESC_MIN", 2048, int))
    # one-pass over row chunks, compaction overlapped on a side stream: "auto" = when the plain
    # one-pass does not fit in memory, "on" = whenever the product is large enough, "off"
    spgemm_pipeline: str = field(default_factory=lambda: _env("SPMM_SPGEMM_PIPELINE", "auto", str))
    # one-pass numeric writing rows at final offsets (decoupled look-back, no compaction copy)
    spgemm_ordered: str = field(default_factory=lambda: _env("SPMM_SPGEMM_ORDERED", "auto", str))
    # products per ordered unit: 7680 (512-thread workgroups, 2 per CU) or 3840 (256 threads, 4 per CU)
    spgemm_ordered_pcap: int = field(default_factory=lambda: _env("SPMM_SPGEMM_ORDERED_PCAP", 7680, int))
    # bitmap-rank SpGEMM (count kernel + numeric kernel, exact offsets, no look-back):
    # "auto" = when every row's columns look uniform enough for its windows, "on", "off"
    spgemm_bitmap: str = field(default_factory=lambda: _env("SPMM_SPGEMM_BITMAP", "auto", str))
    # its window configuration (csr_spgemm_bitmap.hip kCfgs), -1 = chosen from the row statistics
    spgemm_bitmap_cfg: int = field(default_factory=lambda: _env("SPMM_SPGEMM_BITMAP_CFG", -1, int))
    # row-major numeric kernel of the bitmap path (a row's windows back to back, <= 8 windows):
    # "auto" = for the widest-window configurations (0, 3), "on", "off" (per-unit kernel)
    spgemm_bitmap_rows: str = field(default_factory=lambda: _env("SPMM_SPGEMM_BITMAP_ROWS", "auto", str))
    # B's (column, value) pairs for the numeric kernels (1), or the two arrays (0: per-unit kernels
    # only -- the row kernel reads the padded pairs)
    spgemm_bitmap_cv: int = field(default_factory=lambda: _env("SPMM_SPGEMM_BITMAP_CV", 1, int))
    # ... with every (row, window) segment of those pairs starting on a 128-byte line (1) or packed (0)
    spgemm_bitmap_pad: int = field(default_factory=lambda: _env("SPMM_SPGEMM_BITMAP_PAD", 1, int))
    # fixed fp32 summation order (Gustavson order: bitwise run-to-run reproducible, equal to the CPU
    # engine) on the bitmap-rank path: 0 = off, 1 = on (other GPU paths stay unordered), 2 = strict
    # (a product no deterministic GPU kernel covers runs on the CPU engine)
    # row-major bitmap numeric and count kernels: software-pipelined (the next unit's B gathers
    # issued before this unit's write-out / popcount, buffer-descriptor addressing) = 1; 0 = the
    # per-unit numeric kernel and the flat row count kernel (PERF_LOG rounds 5-6)
    spgemm_bitmap_pipe: int = field(default_factory=lambda: _env("SPMM_SPGEMM_BITMAP_PIPE", 1, int))
    spgemm_deterministic: int = field(default_factory=lambda: _env("SPMM_SPGEMM_DETERMINISTIC", 0, int))
    spgemm_global_ws_gb: float = field(default_factory=lambda: _env("SPMM_GLOBAL_WS_GB", 8.0, float))
    # long-row routing histogram reads a chunk-offset table for the long rows of B (1) or their columns (0)
    spgemm_long_btab: int = field(default_factory=lambda: _env("SPMM_SPGEMM_LONG_BTAB", 1, int))
    # long rows: items of > LR_CAP products read their long B rows' products
    # straight from B (no scratch round trip; needs spgemm_long_btab).  Off by
    # default: R-MAT 24 17.0 s vs 16.1 s (PERF_LOG "direct long-row products")
    spgemm_long_direct: int = field(default_factory=lambda: _env("SPMM_SPGEMM_LONG_DIRECT", 0, int))
    # MFMA panel SpMM when the panel column reuse reaches this.  At reuse 1.03
    # (65536^2 @ 0.1 % x 128 cols, BASELINE config 3, which names the MFMA path)
    # the two kernels are within 5 %: MFMA 149 us, row kernel 142 us (PERF_LOG)
    spmm_mfma_min_reuse: float = field(default_factory=lambda: _env("SPMM_MFMA_MIN_REUSE", 1.0, float))
    # seconds before a pending collective raises / aborts.  torch.distributed's
    # watchdog also counts the wait for a slower peer to arrive (skewed R-MAT
    # panels, rank 0 writing output), so the default leaves room for that; the
    # test suite sets 120 s (tests/conftest.py).  The native a4 separates the
    # two: an MPI arrival handshake first, then a 120 s bound on the RCCL
    # transfer alone (csrc/runtime/comm.cpp RcclComm::arrive)
    # long-row path: each batch's accumulation on the side stream, beside the next batch's routing
    spgemm_long_side: int = field(default_factory=lambda: _env("SPMM_SPGEMM_LONG_SIDE", 1, int))
    comm_timeout_s: float = field(default_factory=lambda: _env("SPMM_COMM_TIMEOUT", 600.0, float))

    def as_dict(self) -> dict:
        return {f.name: getattr(self, f.name) for f in fields(self)}


CONFIG = Config()
