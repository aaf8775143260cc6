"""spmm_amd — an MI355X-native (gfx950 / CDNA4) sparse matrix multiplication framework.

Capabilities of UmeshK2005/Sparse-Matrix-Multiplication-using-OpenMP-MPI-and-CUDA
(block-sparse uint64 chain products, its folder I/O, CLI and output layout),
re-designed for MI355X, plus the north-star CSR SpGEMM / SpMM engines with a
1D row-block multi-GPU decomposition over RCCL.

Layout:
  ops/       device ops (HIP kernels via libspmm_hip.so, CPU via libspmm_host.so)
  models/    workloads: block-sparse chain product, CSR SpGEMM, SpMM
  parallel/  process groups, P2P/collective transport, partitioning
  utils/     I/O (reference format, Matrix Market), generators, timers, config
  apps/      command-line programs (a4 drop-in, spgemm)
"""
__version__ = "0.1.0"
