"""Device operators: BSR uint64 products, CSR SpGEMM, SpMM."""
