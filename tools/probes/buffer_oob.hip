// Probe: range check of raw buffer dwordx4 stores / loads that straddle
// num_records (is the check per dword or per access?) at aligned and
// dword-unaligned offsets.  hipcc --offload-arch=gfx950 -O3 buffer_oob.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_store(unsigned* out, int nrec_bytes, int off_bytes) {
  // one lane stores {1,2,3,4} at byte offset off_bytes of a buffer of nrec_bytes
  if (threadIdx.x != 0) return;
  auto r = __builtin_amdgcn_make_buffer_rsrc(out, 0, nrec_bytes, 0x00020000);
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  v4u v = {1u, 2u, 3u, 4u};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off_bytes, 0, 0);
}
__global__ void k_load(const unsigned* in, unsigned* out, int nrec_bytes, int off_bytes) {
  if (threadIdx.x != 0) return;
  auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(in), 0, nrec_bytes, 0x00020000);
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, 0);
  out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
}
int main() {
  unsigned *d, *o, h[16];
  hipMalloc(&d, 64);
  hipMalloc(&o, 64);
  int bad = 0;
  for (int off = 0; off <= 8; off += 4)
    for (int n = 0; n <= 24; n += 4) {
      hipMemset(d, 0, 64);
      k_store<<<1, 64>>>(d, n, off);
      hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
      printf("store off=%2d nrec=%2d :", off, n);
      for (int i = 0; i < 8; ++i) printf(" %u", h[i]);
      // per-dword expectation: dword i (bytes off+4i..) written iff off+4i+4 <= n
      for (int i = 0; i < 4; ++i) {
        unsigned want = (off + 4 * i + 4 <= n) ? (unsigned)(i + 1) : 0u;
        if (h[off / 4 + i] != want) bad |= 1;
      }
      printf("\n");
    }
  unsigned src[16];
  for (int i = 0; i < 16; ++i) src[i] = 100 + i;
  hipMemcpy(d, src, 64, hipMemcpyHostToDevice);
  for (int off = 0; off <= 8; off += 4)
    for (int n = 0; n <= 24; n += 4) {
      k_load<<<1, 64>>>(d, o, n, off);
      hipMemcpy(h, o, 16, hipMemcpyDeviceToHost);
      printf("load  off=%2d nrec=%2d : %u %u %u %u\n", off, n, h[0], h[1], h[2], h[3]);
      for (int i = 0; i < 4; ++i) {
        unsigned want = (off + 4 * i + 4 <= n) ? 100u + off / 4 + i : 0u;
        if (h[i] != want) bad |= 2;
      }
    }
  printf("per-dword range check: stores %s, loads %s\n", (bad & 1) ? "NO" : "yes", (bad & 2) ? "NO" : "yes");
  return 0;
}
