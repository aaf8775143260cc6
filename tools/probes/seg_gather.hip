// Calibration probe for the bitmap SpGEMM's B gathers: what rate does a
// gather of random contiguous segments reach, by segment length, element
// width and buffer size, and with register vs direct-to-LDS (glds) landing?
//
// Each 64-lane wave owns a list of segments (random starts in a buffer of NB
// bytes); a group of G lanes reads one segment of S elements (G = the
// smallest power of two >= min(S, 64); longer segments take S/G rounds).
// D segment-groups in flight per wave.  Prints useful GB/s and the number of
// distinct 128-byte lines per useful byte (so line-bound rates can be read).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstdlib>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// register landing: D loads in flight per lane, xor-reduced
template <int D, typename T>
__global__ __launch_bounds__(256) void gather_reg(const T* __restrict__ buf, const uint32_t* __restrict__ starts,
                                                  int64_t nseg, int S, int lgG, int* out) {
  const int lane = threadIdx.x & 63;
  const int G = 1 << lgG;
  const int gpw = 64 >> lgG;                       // segments per wave-round
  const int gi = lane >> lgG, gl = lane & (G - 1);
  const int rounds = (S + G - 1) >> lgG;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
  uint32_t acc = 0;
  for (int64_t s0 = wave * D * gpw; s0 < nseg; s0 += nw * D * gpw) {
    for (int r = 0; r < rounds; ++r) {
      T v[D];
#pragma unroll
      for (int u = 0; u < D; ++u) {
        int64_t s = s0 + u * gpw + gi;
        s = s < nseg ? s : nseg - 1;
        const int e = r * G + gl;
        const uint32_t b = starts[s];
        v[u] = e < S ? buf[b + e] : T{};
      }
#pragma unroll
      for (int u = 0; u < D; ++u) {
        if constexpr (sizeof(T) == 8) acc ^= (uint32_t)v[u] ^ (uint32_t)(v[u] >> 32);
        else acc ^= (uint32_t)v[u];
      }
    }
  }
  if (acc == 0x12345678u) out[0] = (int)acc;
}

// direct-to-LDS landing: each lane's element lands at ring[slot][u][lane]; D
// glds per lane in flight, then one wait and a read-back of the ring.
template <int D>
__global__ __launch_bounds__(256) void gather_glds(const uint32_t* __restrict__ buf, const uint32_t* __restrict__ starts,
                                                   int64_t nseg, int S, int lgG, int* out) {
  __shared__ uint32_t ring[4][D][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int G = 1 << lgG;
  const int gpw = 64 >> lgG;
  const int gi = lane >> lgG, gl = lane & (G - 1);
  const int rounds = (S + G - 1) >> lgG;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
  uint32_t acc = 0;
  for (int64_t s0 = wave * D * gpw; s0 < nseg; s0 += nw * D * gpw) {
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        int64_t s = s0 + u * gpw + gi;
        s = s < nseg ? s : nseg - 1;
        int e = r * G + gl;
        e = e < S ? e : S - 1;
        const uint32_t b = starts[s];
        __builtin_amdgcn_global_load_lds(const_cast<uint32_t*>(buf + b + e), &ring[w][u][0], 4, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < D; ++u) acc ^= ring[w][u][lane];
    }
  }
  if (acc == 0x12345678u) out[0] = (int)acc;
}

int main() {
  const int64_t maxbytes = 1400ll << 20;
  void* buf;
  CK(hipMalloc(&buf, maxbytes));
  CK(hipMemset(buf, 1, maxbytes));
  const int64_t nseg_max = 1 << 25;
  uint32_t* starts;
  CK(hipMalloc(&starts, nseg_max * 4));
  int* out;
  CK(hipMalloc(&out, 4));
  std::vector<uint32_t> h(nseg_max);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint64_t x = 88172645463325252ull;
  const int align_mode = getenv("SEG_ALIGN") ? atoi(getenv("SEG_ALIGN")) : 0;   // 1: starts on 128-byte lines
  printf("align=%d\n", align_mode);
  printf("kind,elem_bytes,buf_MB,seg_elems,seg_bytes,D,ms,useful_GBps,lines_per_seg,line_GBps\n");
  const int64_t useful_target = 4ll << 30;   // 4 GB of useful bytes per launch
  for (int64_t sz : {420ll << 20, 840ll << 20, 1280ll << 20}) {
    if (sz > maxbytes) continue;
    for (int eb : {4, 8}) {
      for (int S : {6, 12, 13, 16, 25, 26, 32, 50}) {
        const int64_t nel = sz / eb - 256;
        const int64_t nseg = std::min<int64_t>(nseg_max, useful_target / ((int64_t)S * eb));
        double lines = 0;
        for (int64_t i = 0; i < nseg; ++i) {
          x ^= x << 13; x ^= x >> 7; x ^= x << 17;
          h[i] = (uint32_t)(x % (uint64_t)nel);
          if (align_mode) h[i] &= ~(uint32_t)(128 / eb - 1);
          if (i < 100000) {
            const int64_t b0 = (int64_t)h[i] * eb, b1 = b0 + (int64_t)S * eb - 1;
            lines += (double)(b1 / 128 - b0 / 128 + 1);
          }
        }
        lines /= (double)std::min<int64_t>(nseg, 100000);
        CK(hipMemcpy(starts, h.data(), nseg * 4, hipMemcpyHostToDevice));
        int lgG = 0;
        while ((1 << lgG) < std::min(S, 64)) ++lgG;
        auto run = [&](int kind, int D) -> int {
          float best = 1e30f;
          for (int it = 0; it < 3; ++it) {
            CK(hipEventRecord(e0));
            if (kind == 0) {
              if (eb == 4) {
                if (D == 8) hipLaunchKernelGGL((gather_reg<8, uint32_t>), dim3(256 * 8), dim3(256), 0, 0, (const uint32_t*)buf, starts, nseg, S, lgG, out);
                else hipLaunchKernelGGL((gather_reg<16, uint32_t>), dim3(256 * 8), dim3(256), 0, 0, (const uint32_t*)buf, starts, nseg, S, lgG, out);
              } else {
                if (D == 8) hipLaunchKernelGGL((gather_reg<8, uint64_t>), dim3(256 * 8), dim3(256), 0, 0, (const uint64_t*)buf, starts, nseg, S, lgG, out);
                else hipLaunchKernelGGL((gather_reg<16, uint64_t>), dim3(256 * 8), dim3(256), 0, 0, (const uint64_t*)buf, starts, nseg, S, lgG, out);
              }
            } else {
              if (D == 8) hipLaunchKernelGGL((gather_glds<8>), dim3(256 * 8), dim3(256), 0, 0, (const uint32_t*)buf, starts, nseg, S, lgG, out);
              else hipLaunchKernelGGL((gather_glds<16>), dim3(256 * 8), dim3(256), 0, 0, (const uint32_t*)buf, starts, nseg, S, lgG, out);
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
          }
          const double ub = (double)nseg * S * eb;
          printf("%s,%d,%lld,%d,%d,%d,%.3f,%.1f,%.2f,%.1f\n", kind == 0 ? "reg" : "glds", eb, (long long)(sz >> 20), S,
                 S * eb, D, best, ub / best / 1e6, lines, (double)nseg * lines * 128 / best / 1e6);
          fflush(stdout);
          return 0;
        };
        if (run(0, 8)) return 1;
      }
    }
  }
  return 0;
}
