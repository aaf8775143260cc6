// Segment-gather bandwidth probe: each 64-lane group reads random contiguous
// segments of SEG int32 from a buffer of NB bytes (the SpGEMM B-row access
// pattern) with D segments in flight per wave.  Prints effective GB/s of
// useful bytes for a few buffer sizes / segment lengths.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int D>
__global__ __launch_bounds__(256) void gather(const int* __restrict__ buf, const int64_t* __restrict__ starts,
                                              int64_t nseg, int seg, int* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = (gridDim.x * 256) >> 6;
  int acc = 0;
  for (int64_t s0 = wave * D; s0 < nseg; s0 += nw * D) {
    int v[D];
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int64_t s = s0 + u < nseg ? s0 + u : nseg - 1;
      const int64_t b = starts[s];
      v[u] = lane < seg ? buf[b + lane] : 0;
    }
#pragma unroll
    for (int u = 0; u < D; ++u) acc ^= v[u];
  }
  if (acc == 0x12345678) out[0] = acc;
}

int main() {
  const int64_t maxbytes = 1ll << 30;
  int* buf;
  CK(hipMalloc(&buf, maxbytes));
  CK(hipMemset(buf, 1, maxbytes));
  const int64_t nseg = 1 << 24;
  int64_t* starts;
  CK(hipMalloc(&starts, nseg * 8));
  int* out;
  CK(hipMalloc(&out, 4));
  std::vector<int64_t> h(nseg);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint64_t x = 88172645463325252ull;
  for (int64_t sz : {32ll << 20, 256ll << 20, 440ll << 20, 1ll << 30}) {
    for (int seg : {16, 32, 52, 64}) {
      const int64_t nints = sz / 4 - 64;
      for (auto& s : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; s = (int64_t)(x % (uint64_t)nints); }
      CK(hipMemcpy(starts, h.data(), nseg * 8, hipMemcpyHostToDevice));
      for (int it = 0; it < 2; ++it) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(gather<8>, dim3(256 * 8), dim3(256), 0, 0, buf, starts, nseg, seg, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
      }
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("buf %5lld MB seg %3d: %.3f ms, %.1f GB/s useful, %.2f Gseg/s\n", (long long)(sz >> 20), seg, ms,
             nseg * seg * 4.0 / ms / 1e6, nseg / ms / 1e6);
    }
  }
  return 0;
}
