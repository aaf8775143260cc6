"""Workloads built from the ops: chain product (the reference's), CSR SpGEMM, SpMM."""
