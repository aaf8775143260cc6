// CSR x dense SpMM for gfx950:  Y[m][D] = A[m][n] (CSR, bf16 values) . X[n][D] (bf16),
// fp32 accumulation, fp32 or bf16 output.
//
// North-star config 3 ("65536^2 CSR x dense 128-col, bf16, MFMA path").  The
// reference has no SpMM; its one kernel is a per-element dot loop
// (sparse_matrix_mult.cu:44-66).
//
// Two kernels:
//
// spmm_panel_mfma — the MFMA path.  Rows are grouped in panels of 64.  An
//   inspector (ops/spmm.py) lists, per panel, the sorted union of the panel's
//   column indices in chunks of 64 and the panel's entries by chunk.  Per
//   chunk a 256-thread workgroup (4 waves) gathers the 64 X rows of the chunk
//   into LDS once (shared by every row of the panel that touches them),
//   scatters the chunk's entries into a dense 64x64 bf16 A tile in LDS, and
//   issues v_mfma_f32_16x16x32_bf16: wave w owns output rows 16w..16w+15 and
//   all 128 columns (8 accumulator tiles).  The X tile is read as the B
//   operand with ds_read_b64_tr_b16 (hardware transpose of the row-major
//   gathered rows) from an XOR-swizzled image that keeps the 8 rows a 32-lane
//   half reads on distinct banks.
//   Gathered bytes are (union columns) x 256 B per panel instead of
//   nnz x 256 B, so matrices whose rows share columns (banded, clustered,
//   power-law) cut HBM/MALL traffic; the A tile density is irrelevant to the
//   cost because the MFMA rate is ~2.5 PF.
//
// spmm_rowwise — VALU path: one wave per row, each lane owns 2 of every 128
//   output columns, the row's indices read once and 16 gathered X rows in
//   flight per lane.  Best when rows share no columns (uniform random at very
//   low density): no inspector needed.
#include <hip/hip_bf16.h>

#include "common.hpp"

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int PR = 64;      // panel rows
constexpr int CK = 64;      // union columns per chunk (2 MFMA K-steps)
constexpr int DB = 128;     // output columns per workgroup
constexpr int NT = 256;

__device__ __forceinline__ float bf2f(unsigned short b) { return __uint_as_float(((unsigned)b) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  // round-to-nearest-even; NaN kept NaN by the plain cast path below
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<unsigned short*>(&h);
}

// X tile image: 64 rows x 256 B.  Byte (r, c) at r*256 + ((c>>4) ^ s(r))*32 + (c&15)*2,
// s(r) = (r + 4*(r>>3)) & 7: 32-byte chunks of a row are permuted so the 8 rows
// one 32-lane half reads by ds_read_b64_tr_b16 fall on 8 disjoint bank windows.
__device__ __forceinline__ int xswz(int r) { return (r + 4 * (r >> 3)) & 7; }

template <bool OUT_BF16>
__global__ __launch_bounds__(NT) void spmm_panel_mfma(
    const int64_t* __restrict__ panel_chunk_ptr,   // [npanels+1] chunk ranges per panel
    const int32_t* __restrict__ chunk_cols,        // [nchunks*64] X row per union slot, -1 = pad
    const int64_t* __restrict__ chunk_ent_ptr,     // [nchunks+1]
    const int32_t* __restrict__ ent_rc,            // row_in_panel*64 + slot
    const unsigned short* __restrict__ ent_val,    // bf16
    const unsigned short* __restrict__ X, int64_t ldx, int64_t m, void* __restrict__ Yv, int64_t ldy) {
  __shared__ __attribute__((aligned(16))) unsigned short At[PR * CK];      // 8 KB, row-major [row][k]
  __shared__ __attribute__((aligned(16))) unsigned char Xt[CK * DB * 2];    // 16 KB, swizzled rows

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t panel = blockIdx.x;
  const int64_t dcol0 = (int64_t)blockIdx.y * DB;
  v4f acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = v4f{0.f, 0.f, 0.f, 0.f};

  const int64_t c0 = panel_chunk_ptr[panel], c1 = panel_chunk_ptr[panel + 1];
  // gather mapping: thread -> (row gr, 64-byte part gp)
  const int gr = tid >> 2, gp = tid & 3;
  for (int64_t ch = c0; ch < c1; ++ch) {
    // 1. issue the X row gather (registers) early
    const int xr = chunk_cols[ch * CK + gr];
    uint4 xv[4];
    if (xr >= 0) {
      const uint4* src = reinterpret_cast<const uint4*>(X + (int64_t)xr * ldx + dcol0) + gp * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) xv[q] = src[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) xv[q] = make_uint4(0, 0, 0, 0);
    }
    // 2. zero the A tile
    reinterpret_cast<uint4*>(At)[tid * 2 + 0] = make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4*>(At)[tid * 2 + 1] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    // 3. scatter the chunk's entries, store the gathered rows
    for (int64_t e = chunk_ent_ptr[ch] + tid; e < chunk_ent_ptr[ch + 1]; e += NT) {
      At[ent_rc[e]] = ent_val[e];
    }
    {
      const int s = xswz(gr);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cbyte = gp * 64 + q * 16;          // byte within the 256-B row
        const int chunk = cbyte >> 5, within = cbyte & 31;
        *reinterpret_cast<uint4*>(Xt + gr * 256 + ((chunk ^ s) << 5) + within) = xv[q];
      }
    }
    __syncthreads();
    // 4. MFMA: 2 K-steps of 32 over the chunk
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const v8bf a = *reinterpret_cast<const v8bf*>(&At[(16 * w + (lane & 15)) * CK + ks * 32 + 8 * (lane >> 4)]);
      const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
      const int r0 = ks * 32 + 8 * g + q, r1 = r0 + 4;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const unsigned char* p0 = Xt + r0 * 256 + ((t ^ xswz(r0)) << 5) + p * 8;
        const unsigned char* p1 = Xt + r1 * 256 + ((t ^ xswz(r1)) << 5) + p * 8;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p0));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p1));
        // whole-vector shuffle + bitcast: per-element short->__bf16 inserts are
        // miscompiled by hipcc (ROCm 7.2) into duplicated lanes
        const v8s bs = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        const v8bf b = __builtin_bit_cast(v8bf, bs);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // epilogue: C/D map col = lane&15, row = (lane>>4)*4 + i
  const int64_t rbase = panel * PR + 16 * w + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = rbase + i;
    if (row >= m) break;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int64_t col = dcol0 + 16 * t + (lane & 15);
      if (OUT_BF16)
        reinterpret_cast<unsigned short*>(Yv)[row * ldy + col] = f2bf(acc[t][i]);
      else
        reinterpret_cast<float*>(Yv)[row * ldy + col] = acc[t][i];
    }
  }
}

// One wave per row; lane owns columns 2*lane, 2*lane+1 of each 128-column
// block.  The row's column indices and values are read once, coalesced, 64
// per lane-round; each entry's X row address is then a readlane (scalar) and
// RW_DEPTH gathered X rows are in flight per lane: the gather of a row costs
// ~nnz / RW_DEPTH memory latencies instead of two dependent latencies (index,
// then X row) per 4 entries.
constexpr int RW_DEPTH = 16;

template <bool OUT_BF16>
__global__ __launch_bounds__(NT) void spmm_rowwise(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                   const unsigned short* __restrict__ av,
                                                   const unsigned short* __restrict__ X, int64_t ldx, int64_t m,
                                                   int64_t D, void* __restrict__ Yv, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (row >= m) return;   // wave-uniform
  const int64_t e0 = rp[row], e1 = rp[row + 1];
  for (int64_t d0 = 0; d0 < D; d0 += 128) {
    const int64_t col = d0 + 2 * lane;
    const bool live = col < D;
    const unsigned short* Xc = X + (live ? col : 0);
    float s0 = 0.f, s1 = 0.f;
    for (int64_t eb = e0; eb < e1; eb += 64) {   // 64 entries per lane-round
      const int ne = (int)(e1 - eb < 64 ? e1 - eb : 64);
      const int myj = lane < ne ? ci[eb + lane] : 0;
      const float mya = lane < ne ? bf2f(av[eb + lane]) : 0.f;
      for (int k0 = 0; k0 < ne; k0 += RW_DEPTH) {
        unsigned x[RW_DEPTH];
        float a[RW_DEPTH];
#pragma unroll
        for (int u = 0; u < RW_DEPTH; ++u) {
          const int k = k0 + u < ne ? k0 + u : ne - 1;   // (tail: reload the last entry, not accumulated)
          const int j = __builtin_amdgcn_readlane(myj, k);
          a[u] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mya), k));
          x[u] = *reinterpret_cast<const unsigned*>(Xc + (int64_t)j * ldx);
        }
#pragma unroll
        for (int u = 0; u < RW_DEPTH; ++u) {
          if (k0 + u < ne) {   // wave-uniform
            s0 += a[u] * bf2f((unsigned short)(x[u] & 0xFFFF));
            s1 += a[u] * bf2f((unsigned short)(x[u] >> 16));
          }
        }
      }
    }
    if (live) {
      if (OUT_BF16) {
        unsigned short* Y = reinterpret_cast<unsigned short*>(Yv) + row * ldy + col;
        Y[0] = f2bf(s0);
        if (col + 1 < D) Y[1] = f2bf(s1);
      } else {
        float* Y = reinterpret_cast<float*>(Yv) + row * ldy + col;
        Y[0] = s0;
        if (col + 1 < D) Y[1] = s1;
      }
    }
  }
}

}  // namespace

SPMM_EXPORT int spmm_spmm_panel_mfma(const int64_t* panel_chunk_ptr, const int32_t* chunk_cols,
                                     const int64_t* chunk_ent_ptr, const int32_t* ent_rc, const void* ent_val,
                                     const void* X, int64_t ldx, int64_t m, int64_t D, void* Y, int64_t ldy,
                                     int out_bf16, void* stream) {
  if (m <= 0) return 0;
  if (D % DB != 0 || ldx % 8 != 0) return (int)hipErrorInvalidValue;
  const int64_t npanels = (m + PR - 1) / PR;
  dim3 grid((unsigned)npanels, (unsigned)(D / DB));
  if (out_bf16)
    hipLaunchKernelGGL(spmm_panel_mfma<true>, grid, dim3(NT), 0, (hipStream_t)stream, panel_chunk_ptr, chunk_cols,
                       chunk_ent_ptr, ent_rc, (const unsigned short*)ent_val, (const unsigned short*)X, ldx, m, Y,
                       ldy);
  else
    hipLaunchKernelGGL(spmm_panel_mfma<false>, grid, dim3(NT), 0, (hipStream_t)stream, panel_chunk_ptr, chunk_cols,
                       chunk_ent_ptr, ent_rc, (const unsigned short*)ent_val, (const unsigned short*)X, ldx, m, Y,
                       ldy);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spmm_rowwise(const int64_t* rp, const int32_t* ci, const void* av, const void* X, int64_t ldx,
                                  int64_t m, int64_t D, void* Y, int64_t ldy, int out_bf16, void* stream) {
  if (m <= 0) return 0;
  if (D % 2 != 0 || ldx % 2 != 0) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((m + 3) / 4));
  if (out_bf16)
    hipLaunchKernelGGL(spmm_rowwise<true>, grid, dim3(NT), 0, (hipStream_t)stream, rp, ci,
                       (const unsigned short*)av, (const unsigned short*)X, ldx, m, D, Y, ldy);
  else
    hipLaunchKernelGGL(spmm_rowwise<false>, grid, dim3(NT), 0, (hipStream_t)stream, rp, ci,
                       (const unsigned short*)av, (const unsigned short*)X, ldx, m, D, Y, ldy);
  SPMM_LAUNCH_CHECK();
  return 0;
}
