// Random-line gather probe, piece-wise form (MI355X, gfx950): does the memory path merge
// several in-flight loads of ONE 128-B line issued by different instructions? The DeepFM design
// question: a lane (c, h) that needs 32 B of line c (an MFMA fragment's hi and lo halves) issues
// two 16-B loads of the same line from two instructions, plus a third 4-B load (the first-order
// weight in the same line).
//   mode 0: 8 lanes per line, one dwordx4 each (one instruction covers the line)       [baseline]
//   mode 1: 2 lanes per line per instruction, 16 B each; 2 instructions (bytes 0-31, 32-63)
//   mode 2: mode 1 + a third instruction, one lane per line, 4 B at byte 64
//   mode 3: 4 lanes per line, dwordx4 each (bytes 0-63: one instruction, half the line)
//   mode 4: mode 1 + a third instruction, both lanes of the pair load the dword at byte 64
//   mode 5: mode 1 + a third instruction, dwordx4 at byte 64 + 16*sub (bytes 64-95)
// Prints lines/s (distinct 128-B lines touched per second).
//   hipcc -O3 --offload-arch=gfx950 gather_pieces.hip -o gather_pieces && ./gather_pieces <mode> [U] [waves/CU]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__device__ __forceinline__ unsigned long long pick(unsigned seed, unsigned gid, int it, int u, unsigned long long n) {
  return ((((unsigned long long)hash32(seed ^ (gid * 977u + it * 131071u + u * 7919u))) << 20) ^
          hash32(gid + 3u * it + 101u * u + seed)) % n;
}

template <int MODE, int U>
__global__ __launch_bounds__(256) void gather(const float* tab, unsigned long long nlines, int iters, unsigned seed,
                                              float* out) {
  constexpr int LPL = MODE == 0 ? 8 : (MODE == 3 ? 4 : 2);  // lanes per line per instruction
  constexpr bool TWO = MODE == 1 || MODE == 2 || MODE == 4 || MODE == 5;
  const unsigned gid = (blockIdx.x * blockDim.x + threadIdx.x) / LPL;
  const int sub = threadIdx.x % LPL;
  float acc = 0.0f;
  for (int it = 0; it < iters; ++it) {
    float4 v[U], w[U];
    float s[U];
    unsigned long long ln[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ln[u] = pick(seed, gid, it, u, nlines) * 32;  // float offset of the line
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (MODE == 0) v[u] = reinterpret_cast<const float4*>(tab + ln[u])[sub];
      else if (MODE == 3) v[u] = reinterpret_cast<const float4*>(tab + ln[u])[sub];
      else v[u] = reinterpret_cast<const float4*>(tab + ln[u])[sub];          // bytes 16*sub: 0..31
    }
    if (TWO) {
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = reinterpret_cast<const float4*>(tab + ln[u])[2 + sub];  // 32..63
    }
    float4 z[U];
    if (MODE == 2) {
#pragma unroll
      for (int u = 0; u < U; ++u) s[u] = sub == 0 ? tab[ln[u] + 16] : 0.0f;  // byte 64
    }
    if (MODE == 4) {
#pragma unroll
      for (int u = 0; u < U; ++u) s[u] = tab[ln[u] + 16];  // byte 64, both lanes
    }
    if (MODE == 5) {
#pragma unroll
      for (int u = 0; u < U; ++u) z[u] = reinterpret_cast<const float4*>(tab + ln[u])[4 + sub];  // 64..95
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc += v[u].x + v[u].y + v[u].z + v[u].w;
      if (TWO) acc += w[u].x + w[u].y + w[u].z + w[u].w;
      if (MODE == 2 || MODE == 4) acc += s[u];
      if (MODE == 5) acc += z[u].x + z[u].w;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
void launch(int U, int blocks, const float* tab, unsigned long long nlines, int iters, unsigned seed, float* out) {
  switch (U) {
    case 4: hipLaunchKernelGGL((gather<MODE, 4>), dim3(blocks), dim3(256), 0, 0, tab, nlines, iters, seed, out); break;
    case 16: hipLaunchKernelGGL((gather<MODE, 16>), dim3(blocks), dim3(256), 0, 0, tab, nlines, iters, seed, out); break;
    default: hipLaunchKernelGGL((gather<MODE, 8>), dim3(blocks), dim3(256), 0, 0, tab, nlines, iters, seed, out); break;
  }
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int U = argc > 2 ? atoi(argv[2]) : 8;
  const int wpc = argc > 3 ? atoi(argv[3]) : 8;
  const size_t bytes = (size_t)5 << 30;
  const unsigned long long nlines = bytes / 128;
  float* tab;
  float* out;
  if (hipMalloc(&tab, bytes) != hipSuccess) return 1;
  hipMemset(tab, 0, bytes);
  const int blocks = 256 * wpc / 4;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  const int iters = 32;
  auto run = [&](unsigned seed) {
    switch (mode) {
      case 1: launch<1>(U, blocks, tab, nlines, iters, seed, out); break;
      case 2: launch<2>(U, blocks, tab, nlines, iters, seed, out); break;
      case 3: launch<3>(U, blocks, tab, nlines, iters, seed, out); break;
      case 4: launch<4>(U, blocks, tab, nlines, iters, seed, out); break;
      case 5: launch<5>(U, blocks, tab, nlines, iters, seed, out); break;
      default: launch<0>(U, blocks, tab, nlines, iters, seed, out); break;
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
  const int lpl = mode == 0 ? 8 : (mode == 3 ? 4 : 2);
  const double lines = (double)blocks * 256 / lpl * iters * U;
  printf("{\"mode\": %d, \"in_flight_per_group\": %d, \"waves_per_cu\": %d, \"ms\": %.4f, \"glines_per_s\": %.2f}\n", mode, U,
         wpc, ms, lines / ms / 1e6);
  return 0;
}
