// MFMA-only throughput and shader clock probe (MI355X, gfx950): every wave issues ITERS x 4
// independent v_mfma_f32_32x32x16_bf16 chains; wave 0 of block 0 records s_memtime (shader
// clock) and s_memrealtime (100 MHz) at start and end. Prints achieved TF/s and the clock.
//   hipcc -O3 --offload-arch=gfx950 mfma_clock.hip -o mfma_clock && ./mfma_clock [blocks] [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256, 2) void mfma_loop(int iters, float* out, unsigned long long* clk) {
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
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 512;
  const int iters = argc > 2 ? atoi(argv[2]) : 20000;
  float* out;
  unsigned long long* clk;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  hipMalloc(&clk, 2 * sizeof(unsigned long long));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, iters, out, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2];
    hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    const double flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * (blocks * 4.0);
    printf("{\"blocks\": %d, \"iters\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"shader_clock_ghz\": %.3f}\n", blocks,
           iters, ms, flops / (ms * 1e-3) / 1e12, (double)h[0] / ((double)h[1] / 100e6) / 1e9);
  }
  return 0;
}
