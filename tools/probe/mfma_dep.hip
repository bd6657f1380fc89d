// Dependent-accumulator MFMA throughput probe (gfx950): v_mfma_f32_32x32x16_bf16 issued as
//   mode 0: four independent accumulators round-robin (no dependency between neighbours)
//   mode 1: one accumulator (every MFMA depends on the previous one: the S-tile chain)
//   mode 2: four accumulators, three dependent MFMAs on each before switching (the G pattern)
//   mode 3: two accumulators alternating
// 24 MFMAs per iteration in every mode. blocks = 256 -> one wave per SIMD, 512 -> two.
//   hipcc -O3 --offload-arch=gfx950 mfma_dep.hip -o mfma_dep && ./mfma_dep
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define MF(c) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0)

template <int MODE>
__global__ __launch_bounds__(256, 2) void k(int iters, float* out, unsigned long long* clk) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)(0.002f * (threadIdx.x - i));
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  unsigned long long t0 = 0, r0 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int q = 0; q < 6; ++q) { MF(c0); MF(c1); MF(c2); MF(c3); }
    } else if (MODE == 1) {
#pragma unroll
      for (int q = 0; q < 24; ++q) MF(c0);
    } else if (MODE == 2) {
#pragma unroll
      for (int q = 0; q < 2; ++q) { MF(c0); MF(c0); MF(c0); MF(c1); MF(c1); MF(c1); MF(c2); MF(c2); MF(c2); MF(c3); MF(c3); MF(c3); }
    } else {
#pragma unroll
      for (int q = 0; q < 12; ++q) { MF(c0); MF(c1); }
    }
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

template <int MODE>
void run(int blocks, int iters, float* out, unsigned long long* clk) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, iters, out, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2];
    hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    const double per_mfma = (double)h[0] / (24.0 * iters);  // shader cycles per MFMA, one wave
    if (rep == 1)
      printf("{\"mode\": %d, \"blocks\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"ghz\": %.3f, \"cycles_per_mfma_wave\": %.2f}\n",
             MODE, blocks, ms, 2.0 * 32 * 32 * 16 * 24.0 * iters * blocks * 4.0 / (ms * 1e-3) / 1e12, ghz, per_mfma);
  }
}

int main() {
  const int iters = 4000;
  float* out;
  unsigned long long* clk;
  hipMalloc(&out, 1024 * 256 * sizeof(float));
  hipMalloc(&clk, 2 * sizeof(unsigned long long));
  for (int blocks : {256, 512}) {
    run<0>(blocks, iters, out, clk);
    run<1>(blocks, iters, out, clk);
    run<2>(blocks, iters, out, clk);
    run<3>(blocks, iters, out, clk);
  }
  return 0;
}
