// Random-line gather rate probe (MI355X, gfx950): how many random L-byte lines per second the
// chip reads from a table far larger than the Infinity Cache (default 5 GiB, like DeepFM's 39
// packed 10^6-row tables). Each group of L/16 lanes reads one line (16 B per lane), U lines per
// group in flight before first use. Prints lines/s and GB/s of line traffic.
//   hipcc -O3 --offload-arch=gfx950 gather_lines.hip -o gather_lines && ./gather_lines [L] [U] [waves/CU]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <int U>
__global__ __launch_bounds__(256) void gather(const float4* tab, unsigned long long nlines, int lpl, int iters,
                                              unsigned seed, float* out) {
  const int lanes = lpl;  // lanes per line
  const unsigned gid = (blockIdx.x * blockDim.x + threadIdx.x) / lanes;
  const int sub = threadIdx.x % lanes;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int it = 0; it < iters; ++it) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned long long line = (((unsigned long long)hash32(seed ^ (gid * 977u + it * 131071u + u * 7919u)) << 20) ^
                                       hash32(gid + 3u * it + 101u * u + seed)) % nlines;
      v[u] = tab[line * lanes + sub];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

int main(int argc, char** argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 128;
  const int U = argc > 2 ? atoi(argv[2]) : 8;
  const int wpc = argc > 3 ? atoi(argv[3]) : 8;
  const size_t bytes = (size_t)5 << 30;
  const unsigned long long nlines = bytes / L;
  float4* tab;
  float* out;
  if (hipMalloc(&tab, bytes) != hipSuccess) return 1;
  hipMemset(tab, 0, bytes);
  const int blocks = 256 * wpc / 4;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  const int iters = 64;
  auto run = [&](unsigned seed) {
    switch (U) {
      case 1: hipLaunchKernelGGL(gather<1>, dim3(blocks), dim3(256), 0, 0, tab, nlines, L / 16, iters, seed, out); break;
      case 2: hipLaunchKernelGGL(gather<2>, dim3(blocks), dim3(256), 0, 0, tab, nlines, L / 16, iters, seed, out); break;
      case 4: hipLaunchKernelGGL(gather<4>, dim3(blocks), dim3(256), 0, 0, tab, nlines, L / 16, iters, seed, out); break;
      case 8: hipLaunchKernelGGL(gather<8>, dim3(blocks), dim3(256), 0, 0, tab, nlines, L / 16, iters, seed, out); break;
      default: hipLaunchKernelGGL(gather<16>, dim3(blocks), dim3(256), 0, 0, tab, nlines, L / 16, iters, seed, out); break;
    }
  };
  run(1);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) run(100 + r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  const double lines = (double)blocks * 256 / (L / 16) * iters * U;
  printf("{\"line_bytes\": %d, \"in_flight_per_group\": %d, \"waves_per_cu\": %d, \"ms\": %.4f, \"glines_per_s\": %.2f, \"tb_per_s\": %.3f}\n",
         L, U, wpc, ms, lines / ms / 1e6, lines * L / ms / 1e9);
  return 0;
}
