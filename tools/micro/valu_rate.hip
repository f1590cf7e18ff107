// Microbenchmark: issue cost of v_fma_f32 vs v_pk_fma_f32 vs v_exp_f32 on gfx950, at 1..4 waves per
// SIMD (blocks of 256 threads = one wave per SIMD per block; grid = CUs x waves).  Prints ns per
// instruction per wave and the implied cycles at the measured clock-free estimate (2.4 GHz nominal).
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate tools/micro/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, int iters, float s) {
  float v[16];
  float a = threadIdx.x * 1e-3f, b = s;
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = a + j;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      if constexpr (KIND == 0) {
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[q]) : "v"(b), "v"(a));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[q + 1]) : "v"(b), "v"(a));
      } else if constexpr (KIND == 1) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 x = {v[q], v[q + 1]};
        f2 bb = {b, b}, aa = {a, a};
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(bb), "v"(aa));
        v[q] = x.x;
        v[q + 1] = x.y;
      } else if constexpr (KIND == 2) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(v[q]));
        asm volatile("v_exp_f32 %0, %0" : "+v"(v[q + 1]));
      } else {
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[q]) : "v"(b));
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[q + 1]) : "v"(b));
      }
    }
  }
  float r = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) r += v[j];
  if (r == 12345.678f) out[threadIdx.x] = r;
}

template <int KIND>
void run(const char* name, int waves) {
  float* d;
  hipMalloc(&d, 4096);
  int cus = 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  hipLaunchKernelGGL(k<KIND>, dim3(cus * waves), dim3(256), 0, 0, d, 10, 0.999f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<KIND>, dim3(cus * waves), dim3(256), 0, 0, d, iters, 0.999f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const int instrs = KIND == 1 ? 8 : 16;  // per iteration per wave
  const double ns = ms * 1e6 / ((double)iters * instrs * waves);
  printf("%-12s waves/SIMD=%d  %.3f ns per instr per SIMD (%.2f cyc @2.4GHz)\n", name, waves, ns, ns * 2.4);
  hipFree(d);
}

int main() {
  for (int w = 1; w <= 4; w *= 2) {
    run<0>("v_fma_f32", w);
    run<1>("v_pk_fma_f32", w);
    run<2>("v_exp_f32", w);
    run<3>("v_mul_f32", w);
  }
  return 0;
}
