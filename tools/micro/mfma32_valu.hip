// Microbenchmark (round 6): does a v_mfma_f32_32x32x16_f16 chain on one wave overlap another wave's VALU on the
// same SIMD?  The shape of k_bwd32's group: 48 MFMAs in chains of 6 on one accumulator, ~470 VALU fmas.
// Each wave runs ITER iterations of a body; waves/SIMD set by the grid (blocks of 256 threads = one wave per SIMD).
//   A: MFMA only (8 chains of 6)       B: VALU only (NV fmas, 8 independent chains)
//   C: both in one wave, NV/48 VALU between consecutive MFMAs (compiler-interleaved, sched_group_barrier)
//   D: both in one wave, phased: all VALU of the iteration, then the 48 MFMAs
//   E, F: C and D with the MFMA accumulating in VGPRs (inline asm; the compiler puts C and D's accumulator in AGPRs)
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma32_valu tools/micro/mfma32_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int KIND, int NV>
__global__ __launch_bounds__(256) void k(float* out, int iters, float s) {
  f32x16 acc = {};
  f16x8 a8, b8;
  for (int j = 0; j < 8; ++j) {
    a8[j] = (_Float16)(threadIdx.x * 1e-3f + j);
    b8[j] = (_Float16)(s * j);
  }
  float a = threadIdx.x * 1e-3f, b = s;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  for (int it = 0; it < iters; ++it) {
    if constexpr (KIND == 4 || KIND == 5) {
      if constexpr (KIND == 5) {
#pragma unroll
        for (int q = 0; q < NV; ++q) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[q & 7]) : "v"(b), "v"(a));
      }
#pragma unroll
      for (int m = 0; m < 48; ++m) {
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a8), "v"(b8));
        if constexpr (KIND == 4) {
#pragma unroll
          for (int q = 0; q < NV / 48; ++q) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[q & 7]) : "v"(b), "v"(a));
        }
      }
    }
    if constexpr (KIND == 0 || KIND == 2) {
#pragma unroll
      for (int m = 0; m < 48; ++m) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, acc, 0, 0, 0);
        if constexpr (KIND == 2) {
#pragma unroll
          for (int q = 0; q < NV / 48; ++q) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[q & 7]) : "v"(b), "v"(a));
        }
      }
    }
    if constexpr (KIND == 1 || KIND == 3) {
#pragma unroll
      for (int q = 0; q < NV; ++q) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[q & 7]) : "v"(b), "v"(a));
    }
    if constexpr (KIND == 3) {
#pragma unroll
      for (int m = 0; m < 48; ++m)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, acc, 0, 0, 0);
    }
  }
  float r = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) r += acc[j];
#pragma unroll
  for (int j = 0; j < 8; ++j) r += v[j];
  if (r == 12345.678f) out[threadIdx.x] = r;
}

template <int KIND, int NV>
void run(const char* name, int wps) {
  float* d;
  hipMalloc(&d, 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 400;
  const int blocks = 256 * wps;  // 256 CUs x wps blocks of 4 waves = wps waves per SIMD
  hipLaunchKernelGGL((k<KIND, NV>), dim3(blocks), dim3(256), 0, 0, d, 4, 1.0001f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<KIND, NV>), dim3(blocks), dim3(256), 0, 0, d, iters, 1.0001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double ns_per_iter_per_simd = ms * 1e6 / iters / wps;  // per group (iteration) of one wave, SIMD time
  printf("%-34s waves/SIMD %d  %.3f ms  %.1f ns per wave-iteration of SIMD time (%.0f cyc @2.1GHz)\n", name, wps, ms,
         ns_per_iter_per_simd, ns_per_iter_per_simd * 2.1);
  hipFree(d);
}

int main() {
  for (int wps : {1, 2, 3}) {
    run<0, 480>("A mfma32 x48 (chains of 6)", wps);
    run<1, 480>("B valu fma x480", wps);
    run<2, 480>("C interleaved 10 valu / mfma", wps);
    run<3, 480>("D phased valu x480 then mfma x48", wps);
    run<4, 480>("E interleaved, acc in VGPRs", wps);
    run<5, 480>("F phased, acc in VGPRs", wps);
  }
  return 0;
}
