"""Distribution: process groups over RCCL/gloo, BSR/CSR transport, partitioning."""
