// Microbenchmark: do f32 / bf16 MFMAs overlap with independent VALU work on gfx950?
// Each wave runs ITER iterations of {NM MFMAs on 4 independent accumulators, NV independent VALU fmas}.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_overlap tools/micro/mfma_overlap.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int KIND, int NM, int NV>
__global__ __launch_bounds__(256) void k(float* out, int iters, float s) {
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  float a = threadIdx.x * 1e-3f, b = s;
  bf16x8 ab = {1, 2, 3, 4, 5, 6, 7, 8};
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < NM; m += 4) {
      if constexpr (KIND == 0) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
      } else {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, c3, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < NV / (NM / 4 > 0 ? NM / 4 : 1); ++q)
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[q & 7]) : "v"(b), "v"(a));
    }
    if constexpr (NM == 0) {
#pragma unroll
      for (int q = 0; q < NV; ++q) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[q & 7]) : "v"(b), "v"(a));
    }
  }
  float r = c0[0] + c1[1] + c2[2] + c3[3];
#pragma unroll
  for (int j = 0; j < 8; ++j) r += v[j];
  if (r == 12345.678f) out[threadIdx.x] = r;
}

template <int KIND, int NM, int NV>
void run(const char* name, int blocks) {
  float* d;
  hipMalloc(&d, 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  hipLaunchKernelGGL((k<KIND, NM, NV>), dim3(blocks), dim3(256), 0, 0, d, 10, 1.0001f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<KIND, NM, NV>), dim3(blocks), dim3(256), 0, 0, d, iters, 1.0001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // per SIMD: blocks*4 waves over 1024 SIMDs
  const double waves_per_simd = blocks * 4.0 / 1024.0;
  const double ns_per_iter_per_wave = ms * 1e6 / iters / waves_per_simd;
  printf("%-28s blocks %5d  %.3f ms  %.1f ns/iter/wave-slot (%.1f cyc@2.1GHz)\n", name, blocks, ms, ns_per_iter_per_wave,
         ns_per_iter_per_wave * 2.1);
  hipFree(d);
}

int main() {
  for (int blocks : {256, 1024}) {
    run<0, 16, 0>("f32 mfma x16", blocks);
    run<0, 0, 64>("valu fma x64", blocks);
    run<0, 16, 64>("f32 mfma x16 + valu x64", blocks);
    run<0, 16, 32>("f32 mfma x16 + valu x32", blocks);
    run<1, 16, 0>("bf16 mfma x16", blocks);
    run<1, 16, 64>("bf16 mfma x16 + valu x64", blocks);
    run<1, 16, 32>("bf16 mfma x16 + valu x32", blocks);
  }
  return 0;
}
