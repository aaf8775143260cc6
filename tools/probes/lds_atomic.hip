// LDS atomic throughput probe (gfx950): cycles per wave-instruction of ds_add_f32 / ds_add_u32 /
// ds_or_b32 / ds_write_b32 under random, lane-consecutive and colliding address patterns, with
// one 1024-thread workgroup per CU holding a 128 KB accumulator (the long-row dense kernel's
// shape).  Build: hipcc --offload-arch=gfx950 -O3 tools/probes/lds_atomic.hip -o /tmp/lds_atomic
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int W = 1 << 15;       // accumulator floats (128 KB)
constexpr int NT = 1024;
constexpr int ITER = 4096;

template <int MODE>
__global__ __launch_bounds__(NT) void probe(float* out, uint32_t seed) {
  __shared__ float acc[W];
  for (int i = threadIdx.x; i < W; i += NT) acc[i] = 0.f;
  __syncthreads();
  uint32_t x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  const int lane = threadIdx.x & 63;
  float v = 1.0f + (threadIdx.x & 7);
#pragma unroll 8
  for (int it = 0; it < ITER; ++it) {
    x = x * 1664525u + 1013904223u;
    uint32_t a;
    if (MODE == 4 || MODE == 8) {          // lane-consecutive run from a wave-uniform random base
      uint32_t b = __builtin_amdgcn_readfirstlane(x);
      a = ((b >> 17) + lane) & (W - 1);
    } else if (MODE == 14 || MODE == 15 || MODE == 16) {   // the whole wave on one address
      a = __builtin_amdgcn_readfirstlane(x) >> 17;
    } else if (MODE == 5 || MODE == 10 || MODE == 13) {                // 4 lanes per address (16 distinct addresses per wave)
      uint32_t b = __builtin_amdgcn_readfirstlane(x);
      a = ((b >> 17) + (lane >> 2) * 37) & (W - 1);
    } else if (MODE == 6) {                // sorted-ish: 64 lanes over a random 256-float span
      uint32_t b = __builtin_amdgcn_readfirstlane(x);
      a = ((b >> 17) + (x >> 24)) & (W - 1);
    } else {
      a = x >> 17;
    }
    if (MODE == 0 || MODE == 4 || MODE == 5 || MODE == 6) atomicAdd(&acc[a], v);
    else if (MODE == 1) atomicAdd(reinterpret_cast<uint32_t*>(acc) + a, 1u);
    else if (MODE == 2) atomicOr(reinterpret_cast<uint32_t*>(acc) + (a >> 5), 1u << (a & 31));
    else if (MODE == 3 || MODE == 8) acc[a] = v;
    else if (MODE == 7) v += atomicAdd(&acc[a], 1.0f) * 1e-9f;   // returning form
    else if (MODE == 11) { if (lane < 8) atomicAdd(&acc[a], v); }
    else if (MODE == 15) atomicAdd(&acc[a], v);
    else if (MODE == 12 || MODE == 13 || MODE == 14) {   // one compare-swap try, losers fall back to ds_add_f32
      uint32_t* q = reinterpret_cast<uint32_t*>(acc) + a;
      const uint32_t old = *q;
      if (atomicCAS(q, old, __float_as_uint(__uint_as_float(old) + v)) != old) atomicAdd(&acc[a], v);
    }
    else if (MODE == 9 || MODE == 10 || MODE == 16) {    // float add as read + compare-swap loop (integer LDS ops)
      uint32_t* q = reinterpret_cast<uint32_t*>(acc) + a;
      uint32_t old = *q;
      while (true) {
        const uint32_t prev = atomicCAS(q, old, __float_as_uint(__uint_as_float(old) + v));
        if (prev == old) break;
        old = prev;
      }
    }
  }
  __syncthreads();
  float s = 0.f;
  for (int i = threadIdx.x; i < W; i += NT) s += acc[i];
  if (s == 12345.f || v == 12345.f) out[blockIdx.x] = s;
}

template <int MODE>
static void run(const char* name, int cus) {
  float* o;
  hipMalloc(&o, 4096 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int grid = cus * 8;
  probe<MODE><<<grid, NT>>>(o, 1);
  hipEventRecord(e0);
  probe<MODE><<<grid, NT>>>(o, 2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double wave_insts = double(grid) * (NT / 64) * ITER;   // per kernel
  double cu_cycles = ms * 1e-3 * 2.4e9 * cus;
  printf("%-44s %8.3f ms  %6.2f CU-cycles per wave-instruction  %.3g lane-ops/s\n", name, ms,
         cu_cycles / wave_insts, wave_insts * 64 / (ms * 1e-3));
  hipFree(o);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount;
  printf("CUs %d\n", cus);
  run<3>("ds_write_b32 random", cus);
  run<8>("ds_write_b32 lane-consecutive", cus);
  run<0>("ds_add_f32 random (no return)", cus);
  run<7>("ds_add_rtn_f32 random", cus);
  run<1>("ds_add_u32 random", cus);
  run<2>("ds_or_b32 random over 1K words", cus);
  run<4>("ds_add_f32 lane-consecutive", cus);
  run<6>("ds_add_f32 64 lanes in a 256-float span", cus);
  run<5>("ds_add_f32 4 lanes per address", cus);
  run<9>("read + ds_cmpst_rtn_b32 loop, random", cus);
  run<10>("read + ds_cmpst_rtn_b32 loop, 4 lanes/address", cus);
  run<11>("ds_add_f32 random, 8 active lanes", cus);
  run<12>("hybrid CAS once + ds_add_f32, random", cus);
  run<13>("hybrid, 4 lanes/address", cus);
  run<14>("hybrid, 64 lanes one address", cus);
  run<15>("ds_add_f32, 64 lanes one address", cus);
  run<16>("CAS loop, 64 lanes one address", cus);
  return 0;
}
