// Probe: HBM read+write rate of the weight-stationary GEMM's access pattern (lane (c, h) reads
// row c, 16 B at k = 8i + 4h: 32 rows x 32 B per instruction; float4 stores of 32 B per row)
// against a row-contiguous pattern (64 lanes = 2 rows x 512 B per instruction). Each wave
// moves 32-row x 128-float strips (16 KB in, 16 KB out). Standalone: hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(256, 1) void copy_k(const float* __restrict__ A, float* __restrict__ C, long M) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, c = lane & 31;
  const long nstrips = M / 32;
  for (long s = (long)blockIdx.x * 4 + wave; s < nstrips; s += (long)gridDim.x * 4) {
    float4 b[16];
    if (MODE == 0) {
      const float* src = A + (s * 32 + c) * 128 + 4 * h;
#pragma unroll
      for (int i = 0; i < 16; ++i) b[i] = *reinterpret_cast<const float4*>(src + 8 * i);
      float* dst = C + (s * 32 + c) * 128 + 4 * h;
#pragma unroll
      for (int i = 0; i < 16; ++i) *reinterpret_cast<float4*>(dst + 8 * i) = b[i];
    } else {
      const float* src = A + s * 32 * 128 + lane * 4;
#pragma unroll
      for (int i = 0; i < 16; ++i) b[i] = *reinterpret_cast<const float4*>(src + 256 * i);
      float* dst = C + s * 32 * 128 + lane * 4;
#pragma unroll
      for (int i = 0; i < 16; ++i) *reinterpret_cast<float4*>(dst + 256 * i) = b[i];
    }
  }
}

int main() {
  const long M = 160000, n = M * 128;
  float *A, *C;
  hipMalloc(&A, n * 4);
  hipMalloc(&C, n * 4);
  hipMemset(A, 0, n * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 2; ++mode)
    for (int grid : {256, 512, 1024, 2048}) {
      for (int w = 0; w < 3; ++w) {
        if (mode == 0) hipLaunchKernelGGL(copy_k<0>, dim3(grid), dim3(256), 0, 0, A, C, M);
        else hipLaunchKernelGGL(copy_k<1>, dim3(grid), dim3(256), 0, 0, A, C, M);
      }
      hipEventRecord(e0);
      for (int w = 0; w < 20; ++w) {
        if (mode == 0) hipLaunchKernelGGL(copy_k<0>, dim3(grid), dim3(256), 0, 0, A, C, M);
        else hipLaunchKernelGGL(copy_k<1>, dim3(grid), dim3(256), 0, 0, A, C, M);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 20;
      printf("mode %d grid %d: %.1f us  %.0f GB/s\n", mode, grid, ms * 1e3, 2.0 * n * 4 / ms / 1e6);
    }
  return 0;
}
