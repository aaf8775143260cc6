// LDS instruction throughput on gfx950: cycles per wave-instruction for random
// (conflict-prone) addresses, 16 waves per CU, every CU busy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int NT = 1024, SLOTS = 32768, ITERS = 4096;
template <int OP>
__global__ __launch_bounds__(NT) void k(unsigned long long* out, int salt) {
  __shared__ __attribute__((aligned(16))) int t[SLOTS + 4];
  for (int i = threadIdx.x; i < SLOTS; i += NT) t[i] = (OP == 1 ? -1 : 0);
  __syncthreads();
  uint32_t x = threadIdx.x * 2654435761u + salt + blockIdx.x;
  int acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
    x = x * 1664525u + 1013904223u;
    const int a = (x >> 8) & (SLOTS - 1);
    if (OP == 0) acc += t[a];                                                       // ds_read_b32
    if (OP == 1) acc += atomicCAS(&t[a], -1, (int)x);                               // ds_cmpst_rtn_b32
    if (OP == 2) atomicOr(&t[a], 1u << (x & 31));                                   // ds_or_b32 (no rtn)
    if (OP == 3) atomicAdd(reinterpret_cast<float*>(&t[a]), 1.0f);                  // ds_add_f32
    if (OP == 4) acc += atomicAdd(&t[a], 1);                                        // ds_add_rtn_u32
    if (OP == 5) { int4 v = *reinterpret_cast<int4*>(&t[a & ~3]); acc += v.x ^ v.w; } // ds_read_b128
    if (OP == 6) acc += atomicOr(&t[a], 1u << (x & 31));                            // ds_or_rtn_b32
    if (OP == 7) t[a] = (int)x;                                                     // ds_write_b32
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) atomicAdd(out, t1 - t0);
  if (acc == 12345678) out[1] = acc;
}
int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 16);
  const char* names[] = {"ds_read_b32", "ds_cmpst_rtn_b32", "ds_or_b32(no rtn)", "ds_add_f32(no rtn)", "ds_add_rtn_u32", "ds_read_b128", "ds_or_rtn_b32", "ds_write_b32"};
  void (*fns[])(unsigned long long*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>};
  for (int op = 0; op < 8; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipMemset(d, 0, 16);
      hipLaunchKernelGGL(fns[op], dim3(256), dim3(NT), 0, 0, d, rep);
      unsigned long long h[2];
      (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
      if (rep) {
        const double cyc_blk = (double)h[0] / 256.0;
        // per CU: 16 waves x ITERS wave-instructions executed in cyc_blk cycles
        printf("%-20s %8.1f cycles per wave-instruction per CU (%.2f per lane-op)\n", names[op], cyc_blk / (16.0 * ITERS), cyc_blk / (16.0 * ITERS * 64));
      }
    }
  }
  return 0;
}
