// Helpers and layout constants shared by the bitmap-rank SpGEMM kernels
// (csr_spgemm_bitmap.hip) and the kernels that lay out their right operand
// (csr_bitmap_layout.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace spmm_bitmap {

// 64-lane inclusive prefix sum on the DPP network (VALU only; no LDS
// traffic): row_shr 1/2/4/8 inside 16-lane rows, then row_bcast 15 / 31.
__device__ __forceinline__ int bm_wave_incl(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
  return x;
}

constexpr int kPadLg = 4;    // padded segments: multiples of 2^4 pairs (128 bytes)
constexpr int kPadCLg = 5;   // padded count segments (column groups of a count unit): 2^5 columns (128 bytes)

}  // namespace spmm_bitmap
