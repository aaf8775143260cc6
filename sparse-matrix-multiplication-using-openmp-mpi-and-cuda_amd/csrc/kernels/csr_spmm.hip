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

#include <cstdlib>

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

// spmm_panel_mfma_db — the panel kernel software-pipelined over chunks
// ("issue chunk c+1's X-row gather before chunk c's MFMAs, 2
// barriers instead of 3").  Two A tiles and one X tile in LDS (32 KB: four
// to five workgroups per CU); chunk c+1's X rows and entries are gathered
// into registers while chunk c is multiplied:
//   top of c:  At[c & 1] and Xt hold chunk c, chunk c+1's loads in flight
//   zero At[(c+1) & 1] (its last reader, chunk c-1's MFMAs, passed the last
//   barrier); MFMAs of chunk c;                                    barrier
//   store chunk c+1's rows into Xt, scatter its entries into
//   At[(c+1) & 1], issue chunk c+2's gathers;                      barrier
struct ChunkRegs {
  uint4 xv[4];
  int rc[2];
  unsigned short val[2];
  int nent;
};

template <bool OUT_BF16>
__global__ __launch_bounds__(NT, 4) void spmm_panel_mfma_db(
    const int64_t* __restrict__ panel_chunk_ptr, const int32_t* __restrict__ chunk_cols,
    const int64_t* __restrict__ chunk_ent_ptr, const int32_t* __restrict__ ent_rc,
    const unsigned short* __restrict__ ent_val, const unsigned short* __restrict__ X, int64_t ldx, int64_t m,
    void* __restrict__ Yv, int64_t ldy) {
  __shared__ __attribute__((aligned(16))) unsigned short At[2][PR * CK];   // 2 x 8 KB
  __shared__ __attribute__((aligned(16))) unsigned char Xt[CK * DB * 2];   // 16 KB, swizzled rows

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t panel = blockIdx.x;
  const int64_t dcol0 = (int64_t)blockIdx.y * DB;
  v4f acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = v4f{0.f, 0.f, 0.f, 0.f};
  const int64_t c0 = panel_chunk_ptr[panel], c1 = panel_chunk_ptr[panel + 1];
  const int gr = tid >> 2, gp = tid & 3;
  const int sw = xswz(gr);

  // chunk ch's gathers into registers (a chunk past the panel loads nothing)
  auto issue = [&](int64_t ch, ChunkRegs& r) {
    r.nent = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) r.xv[q] = make_uint4(0, 0, 0, 0);
    if (ch < c1) {
      const int xr = chunk_cols[ch * CK + gr];
      if (xr >= 0) {
        const uint4* src = reinterpret_cast<const uint4*>(X + (int64_t)xr * ldx + dcol0) + gp * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) r.xv[q] = src[q];
      }
      const int64_t e0 = chunk_ent_ptr[ch], e1 = chunk_ent_ptr[ch + 1];
      const int64_t ne = e1 - e0;
      r.nent = (int)(ne > 2 * NT ? 2 * NT : ne);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int64_t e = e0 + tid + k * NT;
        r.rc[k] = e < e1 ? ent_rc[e] : -1;
        r.val[k] = e < e1 ? ent_val[e] : (unsigned short)0;
      }
      // (> 512 entries in one chunk: the remainder is scattered from memory, see store)
    }
  };
  // chunk ch into LDS: X rows into Xt, entries into tile a
  auto store = [&](int64_t ch, const ChunkRegs& r, unsigned short* a) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cbyte = gp * 64 + q * 16;
      const int chunk = cbyte >> 5, within = cbyte & 31;
      *reinterpret_cast<uint4*>(Xt + gr * 256 + ((chunk ^ sw) << 5) + within) = r.xv[q];
    }
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (r.rc[k] >= 0) a[r.rc[k]] = r.val[k];
    if (r.nent == 2 * NT) {   // rare: more than 512 entries in the chunk
      const int64_t e1 = chunk_ent_ptr[ch + 1];
      for (int64_t e = chunk_ent_ptr[ch] + 2 * NT + tid; e < e1; e += NT) a[ent_rc[e]] = ent_val[e];
    }
  };
  auto zero = [&](unsigned short* a) {
    reinterpret_cast<uint4*>(a)[tid * 2 + 0] = make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4*>(a)[tid * 2 + 1] = make_uint4(0, 0, 0, 0);
  };
  auto mfma = [&](const unsigned short* a) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const v8bf av = *reinterpret_cast<const v8bf*>(&a[(16 * w + (lane & 15)) * CK + ks * 32 + 8 * (lane >> 4)]);
      const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
      const int r0 = ks * 32 + 8 * g + q, r1 = r0 + 4;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const unsigned char* p0 = Xt + r0 * 256 + ((t ^ xswz(r0)) << 5) + pp * 8;
        const unsigned char* p1 = Xt + r1 * 256 + ((t ^ xswz(r1)) << 5) + pp * 8;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p0));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p1));
        const v8s bs = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        const v8bf b = __builtin_bit_cast(v8bf, bs);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b, acc[t], 0, 0, 0);
      }
    }
  };

  ChunkRegs r;
  // prologue: chunk c0 into LDS (tile 0), chunk c0 + 1's gathers in flight
  if (c0 < c1) {
    issue(c0, r);
    zero(At[0]);
    __syncthreads();
    store(c0, r, At[0]);
    issue(c0 + 1, r);
    __syncthreads();
  }
  for (int64_t ch = c0; ch < c1; ++ch) {
    const int par = (int)((ch - c0) & 1);
    zero(At[par ^ 1]);
    mfma(At[par]);
    __syncthreads();   // chunk ch's MFMAs done: Xt and tile par free
    if (ch + 1 < c1) {
      store(ch + 1, r, At[par ^ 1]);
      issue(ch + 2, r);   // in flight across the next chunk's MFMAs
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

// spmm_rowwise_v8 — the row kernel with 16-byte gathers (D % 8 == 0, X
// 16-byte aligned).  Lane = (group g = lane / 16, part p = lane % 16): part p
// owns output columns d0 + 8p .. d0 + 8p + 7 of every 128, group g takes the
// row's entries g, g + 4, g + 8, ...  One load instruction gathers four X rows
// (4 x 256 B instead of one), RW8_DEPTH loads in flight per lane cover
// 4 * RW8_DEPTH entries, so a 65-entry row needs ~2 memory latencies instead
// of ~5; the four groups' partial sums meet in two cross-lane adds.
#ifndef SPMM_RW8_DEPTH   // 16-byte gathers in flight per lane (4 X rows each per load instruction)
#define SPMM_RW8_DEPTH 8
#endif
constexpr int RW8_DEPTH = SPMM_RW8_DEPTH;

template <bool OUT_BF16>
__global__ __launch_bounds__(NT) void spmm_rowwise_v8(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                      const unsigned short* __restrict__ av,
                                                      const unsigned short* __restrict__ X, int64_t ldx, int64_t m,
                                                      int64_t D, void* __restrict__ Yv, int64_t ldy) {
  const int lane = threadIdx.x & 63, g = lane >> 4, p = lane & 15;
  const int64_t row = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (row >= m) return;   // wave-uniform
  const int64_t e0 = rp[row], e1 = rp[row + 1];
  for (int64_t d0 = 0; d0 < D; d0 += 128) {
    const int64_t col = d0 + 8 * p;
    const bool live = col < D;
    const unsigned short* Xc = X + (live ? col : 0);
    float s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = 0.f;
    for (int64_t eb = e0; eb < e1; eb += 64) {   // 64 entries per lane-round
      const int ne = (int)(e1 - eb < 64 ? e1 - eb : 64);
      const int myj = lane < ne ? ci[eb + lane] : 0;
      const float mya = lane < ne ? bf2f(av[eb + lane]) : 0.f;
      for (int k0 = 0; k0 < ne; k0 += 4 * RW8_DEPTH) {
        uint4 x[RW8_DEPTH];
        float a[RW8_DEPTH];
#pragma unroll
        for (int u = 0; u < RW8_DEPTH; ++u) {
          const int k = k0 + 4 * u + g;
          const int kk = k < ne ? k : 0;   // (past the row: entry 0 reloaded, not accumulated)
          const int j = __shfl(myj, kk);
          a[u] = __shfl(mya, kk);
          x[u] = *reinterpret_cast<const uint4*>(Xc + (int64_t)j * ldx);
        }
#pragma unroll
        for (int u = 0; u < RW8_DEPTH; ++u) {
          if (k0 + 4 * u < ne && k0 + 4 * u + g < ne) {
            const unsigned w4[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              s[2 * h] += a[u] * bf2f((unsigned short)(w4[h] & 0xFFFF));
              s[2 * h + 1] += a[u] * bf2f((unsigned short)(w4[h] >> 16));
            }
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s[i] += __shfl_xor(s[i], 16);
      s[i] += __shfl_xor(s[i], 32);
    }
    if (g == 0 && live) {
      if (OUT_BF16) {
        uint4 o;
        o.x = (unsigned)f2bf(s[0]) | ((unsigned)f2bf(s[1]) << 16);
        o.y = (unsigned)f2bf(s[2]) | ((unsigned)f2bf(s[3]) << 16);
        o.z = (unsigned)f2bf(s[4]) | ((unsigned)f2bf(s[5]) << 16);
        o.w = (unsigned)f2bf(s[6]) | ((unsigned)f2bf(s[7]) << 16);
        *reinterpret_cast<uint4*>(reinterpret_cast<unsigned short*>(Yv) + row * ldy + col) = o;
      } else {
        float4* Y = reinterpret_cast<float4*>(reinterpret_cast<float*>(Yv) + row * ldy + col);
        Y[0] = make_float4(s[0], s[1], s[2], s[3]);
        Y[1] = make_float4(s[4], s[5], s[6], s[7]);
      }
    }
  }
}

// ---- row-owning sweep: resident waves, grouped 16-byte gathers -------------
// The row kernels launch one wave per row: a wave gathers its row's ~65 X
// rows in two or three dependent rounds and exits, with every wave at its own
// column position, so the X rows an XCD touches span all of X (16.8 MB at
// 65536 x 128 bf16) against a 4 MB L2 (~55 % of gathers miss:
// profiles/r3/spmm_pmc.md, 434 MB fetched per call).  Here the grid is
// resident and every wave owns up to SW_RPW rows (gw, gw + G, ...): it stages
// their entries in LDS once (column-sorted, with each row's offsets at SW_S
// column-slice boundaries), then walks the slices in order, slice s of every
// owned row before slice s + 1, so all waves sweep A's columns together.  A
// 16-lane group owns 4 of the wave's rows (a lane: 8 output columns of each,
// 32 accumulator VGPRs for the whole sweep); every load instruction gathers
// four X rows (one per group, 16 B per lane) and SW_U entries of each of a
// group's rows are in flight per round (16 loads).  Measured (65536^2 @ 0.1 %
// x 128): 0.106 ms per call vs 0.123 ms for the one-row-per-wave kernel; the
// fabric traffic drops ~3.6x with 16 slices but more slices mean more rounds,
// and 1 slice is within 2 % of the best (2): the win is the many independent
// gathers per wave more than the L2 reuse.  The host plans the rows so that
// no wave holds more than SW_CAP entries; a wave that would sets err (its Y
// rows are then zeros and the host reruns the product on the row kernel).
// D = 128 (one column block).
#ifndef SPMM_SW_U   // spmm_sweep: entries of each owned row in flight per round
#define SPMM_SW_U 4
#endif
#ifndef SPMM_SW_S   // spmm_sweep: column slices
#define SPMM_SW_S 2   // 65536^2 x 128: 1 / 2 / 4 / 8 slices = 0.108 / 0.106 / 0.110 / 0.118 ms per call
#endif
constexpr int SW_RPW = 16, SW_S = SPMM_SW_S, SW_CAP = 1280, SW_U = SPMM_SW_U;

template <bool OUT_BF16>
__global__ __launch_bounds__(NT, 4) void spmm_sweep(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                    const unsigned short* __restrict__ av,
                                                    const unsigned short* __restrict__ X, int64_t ldx, int64_t m,
                                                    int lgs, void* __restrict__ Yv, int64_t ldy,
                                                    int32_t* __restrict__ err) {
  constexpr int NWV = NT / 64;
  __shared__ uint32_t ent_all[NWV][SW_CAP];                  // (column - slice base) | bf16 value << 16
  __shared__ uint16_t bnd_all[NWV][SW_RPW][SW_S + 1];        // entry offsets at the slice boundaries
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t G = (int64_t)gridDim.x * NWV;
  const int64_t gw = (int64_t)blockIdx.x * NWV + w;
  uint32_t* const E = ent_all[w];
  uint16_t(*const bnd)[SW_S + 1] = bnd_all[w];
  const uint32_t rel_mask = (1u << lgs) - 1u;

  // ---- stage the owned rows (row k = gw + k G), slice offsets by ballots ----
  int off = 0;
  bool fits = true;
#pragma unroll 1
  for (int k = 0; k < SW_RPW; ++k) {
    const int64_t r = gw + k * G;
    int64_t e0 = 0, e1 = 0;
    if (r < m) {
      e0 = rp[r];
      e1 = rp[r + 1];
    }
    const int nk = (int)(e1 - e0);
    fits = fits && off + nk <= SW_CAP;   // uniform
    int lt = 0;                          // lane s: entries of the row in slices < s
#pragma unroll 1
    for (int i0 = 0; i0 < nk; i0 += 64) {
      const int i = i0 + lane;
      const bool ok = i < nk;
      int c = 0;
      unsigned short v = 0;
      if (ok) {
        c = ci[e0 + i];
        v = av[e0 + i];
      }
      const int sl = c >> lgs;
#pragma unroll
      for (int s = 1; s <= SW_S; ++s) {
        const unsigned long long b = __ballot(ok && sl < s);
        if (lane == s) lt += __popcll(b);
      }
      if (fits && ok) E[off + i] = ((uint32_t)c & rel_mask) | ((uint32_t)v << 16);
    }
    if (lane <= SW_S) bnd[k][lane] = (uint16_t)(fits ? off + lt : 0);
    off += nk;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  if (!fits && lane == 0 && err != nullptr) atomicOr(err, 1);   // (the host's plan rules it out; Y rows: 0)
  // lane = (group g = lane / 16, part p = lane % 16): group g owns rows
  // g, g + 4, g + 8, g + 12 of the wave (slot t = row / 4), part p output
  // columns 8p .. 8p + 7; one load instruction gathers four X rows (one per
  // group, 16 B per lane), SW_U entries of each of a group's rows per round
  const int g = lane >> 4, p = lane & 15;
  float acc[SW_RPW / 4][8];
#pragma unroll
  for (int t = 0; t < SW_RPW / 4; ++t)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[t][i] = 0.f;

  if (fits) {
    // ---- the sweep: slice s of every owned row, then slice s + 1 ----------
#pragma unroll 1
    for (int s = 0; s < SW_S; ++s) {
      const int64_t cbase = (int64_t)s << lgs;
      int bb[SW_RPW / 4], ee[SW_RPW / 4], lm = 0;
#pragma unroll
      for (int t = 0; t < SW_RPW / 4; ++t) {
        bb[t] = bnd[g + 4 * t][s];
        ee[t] = bnd[g + 4 * t][s + 1];
        lm = max(lm, ee[t] - bb[t]);
      }
#pragma unroll
      for (int o = 32; o >= 16; o >>= 1) lm = max(lm, __shfl_xor(lm, o));   // (groups differ; parts agree)
      const int longest = __builtin_amdgcn_readfirstlane(lm);
#pragma unroll 1
      for (int j = 0; j < longest; j += SW_U) {
        uint4 x[SW_RPW / 4][SW_U];
#pragma unroll
        for (int t = 0; t < SW_RPW / 4; ++t)
#pragma unroll
          for (int u = 0; u < SW_U; ++u) {
            const int idx = bb[t] + j + u;
            x[t][u] = make_uint4(0u, 0u, 0u, 0u);
            if (idx < ee[t]) {
              const uint32_t e = E[idx];
              x[t][u] = *reinterpret_cast<const uint4*>(X + (cbase + (int64_t)(e & 0xFFFFu)) * ldx + 8 * p);
            }
          }
#pragma unroll
        for (int t = 0; t < SW_RPW / 4; ++t)
#pragma unroll
          for (int u = 0; u < SW_U; ++u) {
            const int idx = bb[t] + j + u;
            if (idx < ee[t]) {
              const float a = bf2f((unsigned short)(E[idx] >> 16));
              const unsigned w4[4] = {x[t][u].x, x[t][u].y, x[t][u].z, x[t][u].w};
#pragma unroll
              for (int h = 0; h < 4; ++h) {
                acc[t][2 * h] += a * bf2f((unsigned short)(w4[h] & 0xFFFFu));
                acc[t][2 * h + 1] += a * bf2f((unsigned short)(w4[h] >> 16));
              }
            }
          }
      }
    }
  }
  // ---- Y rows: group g writes its rows' columns 8p .. 8p + 7 ---------------
#pragma unroll
  for (int t = 0; t < SW_RPW / 4; ++t) {
    const int64_t r = gw + (int64_t)(g + 4 * t) * G;
    if (r < m) {
      if constexpr (OUT_BF16) {
        uint4 o;
        o.x = (unsigned)f2bf(acc[t][0]) | ((unsigned)f2bf(acc[t][1]) << 16);
        o.y = (unsigned)f2bf(acc[t][2]) | ((unsigned)f2bf(acc[t][3]) << 16);
        o.z = (unsigned)f2bf(acc[t][4]) | ((unsigned)f2bf(acc[t][5]) << 16);
        o.w = (unsigned)f2bf(acc[t][6]) | ((unsigned)f2bf(acc[t][7]) << 16);
        *reinterpret_cast<uint4*>(reinterpret_cast<unsigned short*>(Yv) + r * ldy + 8 * p) = o;
      } else {
        float4* const y = reinterpret_cast<float4*>(reinterpret_cast<float*>(Yv) + r * ldy + 8 * p);
        y[0] = make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
        y[1] = make_float4(acc[t][4], acc[t][5], acc[t][6], acc[t][7]);
      }
    }
  }
}

// ---- row-group MFMA: the sweep's gather scheme, products on the matrix cores ----
// A wave owns 16 consecutive rows; their entries are contiguous in A, taken in
// chunks of RM_K = 32 (rows mixed inside a chunk).  Chunk c is one
// v_mfma_f32_16x16x32_bf16 per 16-column output tile: K = the chunk's
// entries, A operand [row][k] = the entry's value when entry k is in that row
// (else 0: 1/16 useful, the matrix cores are ~30x faster than the gathers),
// B operand [k][col] = the entry's gathered X row.  Lane (kg = lane / 16,
// p = lane % 16) gathers 16 bytes (columns 8p .. 8p + 7) of entries 4i + kg,
// i < 8, like the sweep (one load instruction: four X rows); the rows go
// through an 8 KB per-wave LDS image (the swizzle of spmm_panel_mfma) and
// come back transposed (ds_read_b64_tr_b16) as the B operand.  Software
// pipeline, no workgroup barriers (every LDS byte is wave-private):
//   iteration c: issue chunk c+2's column / value loads (one entry a lane),
//   chunk c+1's gathers (columns landed one iteration ago, spread by
//   ds_bpermute), build chunk c's A operand, then consume chunk c's gathers
//   (issued one iteration ago) -> LDS -> 8 MFMAs.
// D = 128, X 16-byte aligned (as spmm_sweep); fp32 accumulation.
constexpr int RM_K = 32;
#ifndef SPMM_RM_CPI   // row-group MFMA SpMM: chunks (of 32 entries, 8 gathers a lane) in flight per wave
#define SPMM_RM_CPI 3
#endif
#ifndef SPMM_RM_WPC   // ... and the workgroups per CU its registers are sized for
#define SPMM_RM_WPC 2
#endif
constexpr int RM_CPI = SPMM_RM_CPI;

template <bool OUT_BF16>
// (ci / av / X without __restrict__: restrict read-only loads are free to sink
// below the asm barriers that keep the software pipeline's order)
__global__ __launch_bounds__(NT, SPMM_RM_WPC) void spmm_rows_mfma(const int64_t* __restrict__ rp, const int32_t* ci,
                                                        const unsigned short* av,
                                                        const unsigned short* X, int64_t ldx, int64_t m,
                                                        void* __restrict__ Yv, int64_t ldy) {
  __shared__ __attribute__((aligned(16))) unsigned char xs_all[NT / 64][RM_K * 256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = ((int64_t)blockIdx.x * (NT / 64) + w) * 16;
  if (r0 >= m) return;   // (whole wave; nothing below synchronises waves)
  unsigned char* const Xs = xs_all[w];
  const int mr = lane & 15, kg = lane >> 4, p = lane & 15;
  const int64_t lo = rp[min(r0 + mr, m)], hi = rp[min(r0 + mr + 1, m)];   // lane's A-operand row (empty past m)
  const int64_t e0 = __builtin_amdgcn_readfirstlane(rp[r0]);
  const int64_t e1 = __builtin_amdgcn_readfirstlane(rp[min(r0 + 16, m)]);
  v4f acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = v4f{0.f, 0.f, 0.f, 0.f};
  if (e1 > e0) {
    // one entry per lane (lanes 32..63 repeat 0..31): column and value of entry base + lane % 32
    auto ld_ent = [&](int64_t base, int& c, unsigned& v) {
      const int64_t e = base + (lane & 31);
      const int64_t ec = e < e1 ? e : e1 - 1;   // (clamped: in bounds, masked below)
      c = ci[ec];
      const unsigned raw = av[ec];   // (unconditional: a load under a branch costs the loop its vmcnt counts)
      v = e < e1 ? raw : 0u;
    };
    // chunk gathers: entry 4 i + kg of the chunk, 16 bytes at part p; past the
    // entries: row 0 of X, zeroed when staged
    auto gather = [&](int c, uint4 (&x)[8]) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int col = __shfl(c, 4 * i + kg, 64);
        x[i] = *reinterpret_cast<const uint4*>(X + (int64_t)col * ldx + 8 * p);
      }
    };
    // chunk `base`: its gathered X rows xc (landed) and its entries' values vc -> 8 MFMAs
    auto consume = [&](int64_t base, const uint4 (&xc)[8], unsigned vc) {
      // A operand: lane (row mr, k-group kg) holds k = 8 kg .. 8 kg + 7
      uint32_t aw[4];
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const int64_t k0 = base + 8 * kg + j;
        const unsigned v0 = (unsigned)__shfl((int)vc, 8 * kg + j, 64);
        const unsigned v1 = (unsigned)__shfl((int)vc, 8 * kg + j + 1, 64);
        const unsigned m0 = (k0 >= lo && k0 < hi) ? v0 : 0u;
        const unsigned m1 = (k0 + 1 >= lo && k0 + 1 < hi) ? v1 : 0u;
        aw[j / 2] = m0 | (m1 << 16);
      }
      const v8bf a = __builtin_bit_cast(v8bf, make_uint4(aw[0], aw[1], aw[2], aw[3]));
      // the X rows -> the swizzled image (rows past the entries: zeros)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = 4 * i + kg;
        const uint4 v = base + r < e1 ? xc[i] : make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(Xs + r * 256 + (((p >> 1) ^ xswz(r)) << 5) + (p & 1) * 16) = v;
      }
      // (no fence: one wave's LDS instructions execute in order, so the transposing reads
      // below see the stores above, and the next chunk's stores follow these reads)
      const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
      const int r0k = 8 * g + q, r1k = r0k + 4;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const unsigned char* p0 = Xs + r0k * 256 + ((t ^ xswz(r0k)) << 5) + pp * 8;
        const unsigned char* p1 = Xs + r1k * 256 + ((t ^ xswz(r1k)) << 5) + pp * 8;
        v4s blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p0));
        v4s bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p1));
        const v8s bs = __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(v8bf, bs), acc[t], 0, 0, 0);
      }
    };
    // RM_CPI chunks an iteration: their 8 RM_CPI gathers issue together, then
    // the next iteration's entries, then the chunks are consumed in order.  No
    // gather is in flight across the loop's back edge (hipcc copies loop-carried
    // load registers and waits for them there); the other resident waves cover
    // the start of each iteration's gathers, as in spmm_sweep's rounds.
    int cc[RM_CPI];
    unsigned vv[RM_CPI];
#pragma unroll
    for (int q = 0; q < RM_CPI; ++q) ld_ent(e0 + q * RM_K, cc[q], vv[q]);
#pragma unroll 1
    for (int64_t base = e0; base < e1; base += RM_CPI * RM_K) {
      uint4 x[RM_CPI][8];
#pragma unroll
      for (int q = 0; q < RM_CPI; ++q) gather(cc[q], x[q]);
      int cn[RM_CPI];
      unsigned vn[RM_CPI];
#pragma unroll
      for (int q = 0; q < RM_CPI; ++q) ld_ent(base + (RM_CPI + q) * RM_K, cn[q], vn[q]);
      asm volatile("" ::: "memory");   // (every load above issues before the first chunk is consumed)
#pragma unroll
      for (int q = 0; q < RM_CPI; ++q) consume(base + q * RM_K, x[q], vv[q]);   // (past the entries: zero A)
#pragma unroll
      for (int q = 0; q < RM_CPI; ++q) {
        cc[q] = cn[q];
        vv[q] = vn[q];
      }
    }
  }
  // C/D map: col = lane & 15 of tile t, row = 4 (lane / 16) + i
  const int64_t rb = r0 + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = rb + i;
    if (row >= m) break;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int64_t col = 16 * t + (lane & 15);
      if constexpr (OUT_BF16)
        reinterpret_cast<unsigned short*>(Yv)[row * ldy + col] = f2bf(acc[t][i]);
      else
        reinterpret_cast<float*>(Yv)[row * ldy + col] = acc[t][i];
    }
  }
}

// ---- inspector: the panel plan on the device -------------------------------
// (ops/spmm.py plan_panels; was a chain of torch sort / unique / bincount
// launches, ~37 ms for the 65536^2 config.)  Per 64-row panel, one workgroup:
//   count: the size of the panel's column union (an LDS bitmap of a 2^16-
//          column window, popcounts), per window of the columns it touches;
//   fill:  the union's sorted columns in chunks of 64 slots (chunk_cols, -1
//          padding), the entries' (row in panel, slot) grouped by chunk
//          (chunk_ent_ptr: an LDS count + scan per chunk; inside a chunk the
//          order is arbitrary: the MFMA kernel scatters into a tile), and the
//          values as bf16.  A panel's entries keep the index range they have
//          in A (rp[p*64] ..), so no global scan over entries is needed; the
//          chunk ranges come from one scan of the union sizes (host side).
constexpr int PL_LG = 16, PL_W = 1 << PL_LG, PL_WORDS = PL_W / 64;   // 8 KB bitmap window
constexpr int PL_MAXCH = 1024;                                       // chunks per panel (65536 union columns)

// block-wide exclusive scan of one int per thread (256 threads), + total
__device__ __forceinline__ int pl_scan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    pre += i < w ? wsum[i] : 0;
    tot += wsum[i];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

struct PlanArgs {
  const int64_t* rp;
  const int32_t* ci;
  const void* av;          // A values: bf16 or fp32
  int val_f32;
  int64_t m, n;
  int64_t* nunion;         // count: [npanels]
  const int64_t* pcp;      // fill: panel_chunk_ptr [npanels + 1]
  int32_t* chunk_cols;
  int64_t* chunk_ent_ptr;  // [nchunks + 1]
  int32_t* ent_rc;
  unsigned short* ent_val;
  int32_t* err;            // bit 0: a panel has more than PL_MAXCH chunks
};

// One panel per workgroup.  FILL = false: union size only.
template <bool FILL>
__global__ __launch_bounds__(NT) void spmm_plan(PlanArgs a) {
  __shared__ unsigned long long bm[PL_WORDS];
  __shared__ int pre[PL_WORDS];
  __shared__ int64_t srp[PR + 1];
  __shared__ int chcnt[FILL ? PL_MAXCH : 1], chpre[FILL ? PL_MAXCH : 1], chfill[FILL ? PL_MAXCH : 1];
  __shared__ int wsum[NT / 64];
  __shared__ int snext;

  const int tid = threadIdx.x;
  const int64_t panel = blockIdx.x;
  const int64_t r0 = panel * PR;
  const int nrows = (int)(a.m - r0 < PR ? a.m - r0 : PR);
  if (tid <= nrows) srp[tid] = a.rp[r0 + tid];
  __syncthreads();
  const int64_t e0 = srp[0], e1 = srp[nrows];
  const int64_t nwin = (a.n + PL_W - 1) >> PL_LG;
  int64_t chunk0 = 0;
  int nch = 0;
  if constexpr (FILL) {
    chunk0 = a.pcp[panel];
    nch = (int)(a.pcp[panel + 1] - chunk0);
    if (nch > PL_MAXCH) {   // uniform; the host falls back to the torch inspector
      if (tid == 0) atomicOr(a.err, 1);
      return;
    }
    for (int k = tid; k < nch; k += NT) {
      chcnt[k] = 0;
      chfill[k] = 0;
    }
  }
  auto row_of = [&](int64_t e) {   // row in panel of entry e (binary search over the panel's row pointers)
    int lo = 0, hi = nrows - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (srp[mid] <= e) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  // one window: OR its columns, exclusive rank prefix per word (base = union
  // slots before the window); returns the window's union size
  auto window = [&](int64_t w, int base) {
    for (int i = tid; i < PL_WORDS; i += NT) bm[i] = 0ull;
    __syncthreads();
    const int64_t lo = w << PL_LG, hi = lo + PL_W;
    for (int64_t e = e0 + tid; e < e1; e += NT) {
      const int64_t c = a.ci[e];
      if (c >= lo && c < hi) {
        const int cc = (int)(c - lo);
        atomicOr(&bm[cc >> 6], 1ull << (cc & 63));
      }
    }
    __syncthreads();
    constexpr int WPT = PL_WORDS / NT;   // 4 words per thread
    int cnt[WPT], s = 0;
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      cnt[i] = __popcll(bm[tid * WPT + i]);
      s += cnt[i];
    }
    int tot;
    int p = pl_scan(s, wsum, &tot);
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      pre[tid * WPT + i] = base + p;
      p += cnt[i];
    }
    __syncthreads();
    return tot;
  };
  // next window holding a column of the panel at or after window w (or nwin)
  auto next_window = [&](int64_t w) {
    if (tid == 0) snext = 0x7fffffff;
    __syncthreads();
    const int64_t lo = w << PL_LG;
    int best = 0x7fffffff;
    for (int64_t e = e0 + tid; e < e1; e += NT) {
      const int64_t c = a.ci[e];
      if (c >= lo) best = min(best, (int)(c >> PL_LG));
    }
    if (best != 0x7fffffff) atomicMin(&snext, best);
    __syncthreads();
    const int r = snext;
    __syncthreads();
    return r == 0x7fffffff ? nwin : (int64_t)r;
  };
  auto rank = [&](int cc) { return pre[cc >> 6] + __popcll(bm[cc >> 6] & ((1ull << (cc & 63)) - 1ull)); };

  int total = 0, nwt = 0;
  for (int64_t w = next_window(0); w < nwin; w = next_window(w + 1)) {
    const int base = total;
    total += window(w, base);
    ++nwt;
    if constexpr (FILL) {
      // the union's columns of this window in slot order
      constexpr int WPT = PL_WORDS / NT;
      for (int i = 0; i < WPT; ++i) {
        const int wd = tid * WPT + i;
        unsigned long long bits = bm[wd];
        int slot = pre[wd];
        while (bits) {
          const int b = __builtin_ctzll(bits);
          bits &= bits - 1;
          a.chunk_cols[chunk0 * 64 + slot] = (int32_t)((w << PL_LG) + wd * 64 + b);
          ++slot;
        }
      }
      // entries per chunk
      const int64_t lo = w << PL_LG, hi = lo + PL_W;
      for (int64_t e = e0 + tid; e < e1; e += NT) {
        const int64_t c = a.ci[e];
        if (c >= lo && c < hi) atomicAdd(&chcnt[rank((int)(c - lo)) >> 6], 1);
      }
      __syncthreads();
    }
  }
  if constexpr (!FILL) {
    if (tid == 0) a.nunion[panel] = total;
    return;
  } else {
    for (int s = total + tid; s < nch * 64; s += NT) a.chunk_cols[chunk0 * 64 + s] = -1;   // last chunk's padding
    // chunk entry ranges: the panel's entries keep A's index range [e0, e1)
    int run = 0;
    for (int k0 = 0; k0 < nch; k0 += NT) {
      const int k = k0 + tid;
      const int v = k < nch ? chcnt[k] : 0;
      int tot;
      const int p = pl_scan(v, wsum, &tot);
      if (k < nch) {
        chpre[k] = run + p;
        a.chunk_ent_ptr[chunk0 + k] = e0 + run + p;
      }
      run += tot;
    }
    if (panel == (int64_t)gridDim.x - 1 && tid == 0) a.chunk_ent_ptr[chunk0 + nch] = e1;
    __syncthreads();
    // scatter the entries (the bitmap of the last window is still valid when
    // the panel touches one window; otherwise every window is rebuilt)
    int acc = 0;   // rank base of the window: union slots of the windows before it
    for (int64_t w = next_window(0); w < nwin; w = next_window(w + 1)) {
      if (nwt > 1) acc += window(w, acc);
      const int64_t lo = w << PL_LG, hi = lo + PL_W;
      for (int64_t e = e0 + tid; e < e1; e += NT) {
        const int64_t c = a.ci[e];
        if (c >= lo && c < hi) {
          const int slot = rank((int)(c - lo));
          const int k = slot >> 6;
          const int64_t pos = e0 + chpre[k] + atomicAdd(&chfill[k], 1);
          a.ent_rc[pos] = row_of(e) * 64 + (slot & 63);
          a.ent_val[pos] = a.val_f32 ? f2bf(reinterpret_cast<const float*>(a.av)[e])
                                     : reinterpret_cast<const unsigned short*>(a.av)[e];
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace

// Inspector, count pass: nunion[p] = size of panel p's column union.
SPMM_EXPORT int spmm_spmm_plan_count(const int64_t* rp, const int32_t* ci, int64_t m, int64_t n, int64_t* nunion,
                                     void* stream) {
  if (m <= 0) return 0;
  PlanArgs a{rp, ci, nullptr, 0, m, n, nunion, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(spmm_plan<false>, dim3((unsigned)((m + PR - 1) / PR)), dim3(NT), 0, (hipStream_t)stream, a);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Inspector, fill pass (pcp = exclusive scan of ceil(nunion / 64)); err bit 0:
// a panel has more than 1024 chunks (the host uses the torch inspector).
SPMM_EXPORT int spmm_spmm_plan_fill(const int64_t* rp, const int32_t* ci, const void* av, int val_f32, int64_t m,
                                    int64_t n, const int64_t* pcp, int32_t* chunk_cols, int64_t* chunk_ent_ptr,
                                    int32_t* ent_rc, void* ent_val, int32_t* err, void* stream) {
  if (m <= 0) return 0;
  PlanArgs a{rp, ci, av, val_f32, m, n, nullptr, pcp, chunk_cols, chunk_ent_ptr, ent_rc, (unsigned short*)ent_val,
             err};
  hipLaunchKernelGGL(spmm_plan<true>, dim3((unsigned)((m + PR - 1) / PR)), dim3(NT), 0, (hipStream_t)stream, a);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spmm_panel_mfma(const int64_t* panel_chunk_ptr, const int32_t* chunk_cols,
                                     const int64_t* chunk_ent_ptr, const int32_t* ent_rc, const void* ent_val,
                                     const void* X, int64_t ldx, int64_t m, int64_t D, void* Y, int64_t ldy,
                                     int out_bf16, void* stream) {
  if (m <= 0) return 0;
  if (D % DB != 0 || ldx % 8 != 0) return (int)hipErrorInvalidValue;
  const int64_t npanels = (m + PR - 1) / PR;
  dim3 grid((unsigned)npanels, (unsigned)(D / DB));
  static const int db = [] {   // SPMM_SPMM_MFMA_DB=0: the single-buffered kernel (A/B)
    const char* e = getenv("SPMM_SPMM_MFMA_DB");
    return e && *e ? atoi(e) : 1;
  }();
  auto k = db ? (out_bf16 ? spmm_panel_mfma_db<true> : spmm_panel_mfma_db<false>)
              : (out_bf16 ? spmm_panel_mfma<true> : spmm_panel_mfma<false>);
  hipLaunchKernelGGL(k, grid, dim3(NT), 0, (hipStream_t)stream, panel_chunk_ptr, chunk_cols, chunk_ent_ptr, ent_rc,
                     (const unsigned short*)ent_val, (const unsigned short*)X, ldx, m, Y, ldy);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// spmm_spmm_sweep's launch for an m x n operand: *waves = G (row k of wave
// w is w + k G), *rpw = rows per wave (<= SW_RPW), *cap = LDS entries per
// wave; *waves = 0 when it cannot run (too many rows for the resident grid,
// or slices wider than 2^16 columns).  The host checks every wave's entry
// count against *cap once per operand (ops/spmm.py sweep_plan).
SPMM_EXPORT int spmm_spmm_sweep_geometry(int64_t m, int64_t n, int64_t* waves, int* rpw, int* cap) {
  *waves = 0;
  *rpw = SW_RPW;
  *cap = SW_CAP;
  int lgs = 0;
  while (((int64_t)SW_S << lgs) < n) ++lgs;
  if (lgs > 16 || m <= 0) return 0;
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return (int)hipErrorInvalidDevice;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  int per_bf = 0;   // (both output types share one geometry: the smaller residency)
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, spmm_sweep<false>, NT, 0) != hipSuccess || per <= 0) per = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_bf, spmm_sweep<true>, NT, 0) == hipSuccess && per_bf > 0 &&
      per_bf < per)
    per = per_bf;
  int64_t g = (int64_t)per * ncu;
  const int64_t need = (m + (int64_t)(NT / 64) * SW_RPW - 1) / ((int64_t)(NT / 64) * SW_RPW);
  if (need > g) return 0;
  const int64_t one_row = (m + NT / 64 - 1) / (NT / 64);
  if (one_row < g) g = one_row;
  *waves = g * (NT / 64);
  return 0;
}

// Row-owning sweep (spmm_sweep): D == 128, ldx / ldy multiples of 8, 16-byte aligned X
// and Y; the grid is the resident capacity and must hold every row in
// SW_RPW rows per wave (else hipErrorInvalidValue: use spmm_spmm_rowwise).
// n = columns of A: the slices are 2^lgs columns, lgs = ceil(log2(n / SW_S)).  err (may be null):
// set when a wave would overflow its LDS stage (the host plan check rules it out).
SPMM_EXPORT int spmm_spmm_sweep(const int64_t* rp, const int32_t* ci, const void* av, const void* X, int64_t ldx,
                                int64_t m, int64_t n, int64_t D, void* Y, int64_t ldy, int out_bf16, int32_t* err,
                                void* stream) {
  if (m <= 0) return 0;
  if (D != 128 || ldx % 8 != 0 || ldy % 8 != 0 || ((uintptr_t)X & 15) || ((uintptr_t)Y & 15)) return (int)hipErrorInvalidValue;
  int lgs = 0;
  while (((int64_t)SW_S << lgs) < n) ++lgs;   // (<= 16: slice-relative columns are 16-bit; geometry checks)
  auto k = out_bf16 ? spmm_sweep<true> : spmm_sweep<false>;
  int64_t waves = 0;
  int rpw = 0, cap = 0;
  const int rc = spmm_spmm_sweep_geometry(m, n, &waves, &rpw, &cap);
  if (rc) return rc;
  if (waves == 0) return (int)hipErrorInvalidValue;
  const int64_t g = waves / (NT / 64);
  hipLaunchKernelGGL(k, dim3((unsigned)g), dim3(NT), 0, (hipStream_t)stream, rp, ci, (const unsigned short*)av,
                     (const unsigned short*)X, ldx, m, lgs, Y, ldy, err);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Row-group MFMA SpMM (spmm_rows_mfma): D == 128, ldx a multiple of 8 and X
// 16-byte aligned; no inspector.
SPMM_EXPORT int spmm_spmm_rows_mfma(const int64_t* rp, const int32_t* ci, const void* av, const void* X, int64_t ldx,
                                    int64_t m, int64_t D, void* Y, int64_t ldy, int out_bf16, void* stream) {
  if (m <= 0) return 0;
  if (D != 128 || ldx % 8 != 0 || ((uintptr_t)X & 15)) return (int)hipErrorInvalidValue;
  const int64_t wg = (m + 16 * (NT / 64) - 1) / (16 * (NT / 64));
  if (wg > (int64_t)UINT32_MAX) return (int)hipErrorInvalidValue;
  auto k = out_bf16 ? spmm_rows_mfma<true> : spmm_rows_mfma<false>;
  hipLaunchKernelGGL(k, dim3((unsigned)wg), dim3(NT), 0, (hipStream_t)stream, rp, ci, (const unsigned short*)av,
                     (const unsigned short*)X, ldx, m, Y, ldy);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spmm_rowwise(const int64_t* rp, const int32_t* ci, const void* av, const void* X, int64_t ldx,
                                  int64_t m, int64_t D, void* Y, int64_t ldy, int out_bf16, void* stream) {
  if (m <= 0) return 0;
  if (D % 2 != 0 || ldx % 2 != 0) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((m + 3) / 4));
  // 16-byte gathers when every X row and Y row piece is 16-byte aligned
  // (SPMM_SPMM_ROWWISE_V8=0: the 4-byte kernel, for A/B runs)
  static const int v8 = [] {
    const char* e = getenv("SPMM_SPMM_ROWWISE_V8");
    return e && e[0] == '0' ? 0 : 1;
  }();
  const bool al16 = D % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)X & 15) == 0 && ((uintptr_t)Y & 15) == 0 &&
                    ldy % 8 == 0;
  if (v8 && al16) {
    if (out_bf16)
      hipLaunchKernelGGL(spmm_rowwise_v8<true>, grid, dim3(NT), 0, (hipStream_t)stream, rp, ci,
                         (const unsigned short*)av, (const unsigned short*)X, ldx, m, D, Y, ldy);
    else
      hipLaunchKernelGGL(spmm_rowwise_v8<false>, grid, dim3(NT), 0, (hipStream_t)stream, rp, ci,
                         (const unsigned short*)av, (const unsigned short*)X, ldx, m, D, Y, ldy);
    SPMM_LAUNCH_CHECK();
    return 0;
  }
  if (out_bf16)
    hipLaunchKernelGGL(spmm_rowwise<true>, grid, dim3(NT), 0, (hipStream_t)stream, rp, ci,
                       (const unsigned short*)av, (const unsigned short*)X, ldx, m, D, Y, ldy);
  else
    hipLaunchKernelGGL(spmm_rowwise<false>, grid, dim3(NT), 0, (hipStream_t)stream, rp, ci,
                       (const unsigned short*)av, (const unsigned short*)X, ldx, m, D, Y, ldy);
  SPMM_LAUNCH_CHECK();
  return 0;
}
