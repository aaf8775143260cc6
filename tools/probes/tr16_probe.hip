// Empirical semantics of ds_read_b64_tr_b16 on gfx950: LDS holds element
// index e at 16-bit slot e; lane i points at slot 4*i (8 bytes).  Prints, for
// each lane, the 4 slot indices it receives.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void probe(int* out, int mode) {
  __shared__ short lds[64 * 16];
  for (int i = threadIdx.x; i < 64 * 16; i += 64) lds[i] = (short)i;
  __syncthreads();
  int lane = threadIdx.x;
  int slot = (mode == 0) ? 4 * lane : ((lane & 15) >> 2) * 64 + (lane & 3) * 4 + (lane >> 4) * 256;
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds + slot));
  for (int q = 0; q < 4; ++q) out[lane * 4 + q] = r[q];
}
int main() {
  int* d; hipMalloc(&d, 64 * 4 * sizeof(int));
  int h[256];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("mode %d (lane: slot_of_own_address -> received slots)\n", mode);
    for (int l = 0; l < 64; ++l) {
      int slot = (mode == 0) ? 4 * l : ((l & 15) >> 2) * 64 + (l & 3) * 4 + (l >> 4) * 256;
      printf("  lane %2d addr %4d -> %4d %4d %4d %4d\n", l, slot, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
    }
  }
  hipFree(d);
  return 0;
}
