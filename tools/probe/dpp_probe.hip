// Probe of the lane-move semantics behind a DPP / permlane wave reduction (round 6): for a wave
// whose lane i holds x[i], record what each move delivers to every lane, and compare the DPP
// butterfly sum with the __shfl_xor butterfly sum bit for bit. Built by tools/probe/dpp_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
}

__device__ float sum_shfl(float v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ float sum_dpp(float v, int width) {
  if (width == 64) {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  if (width >= 32) {
    const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  v += dpp<0x128>(v);
  v += dpp<0x124>(v);
  v += dpp<0x122>(v);
  v += dpp<0x121>(v);
  return v;
}

// moves[k][lane]: 0 p16 sw0, 1 p16 sw1, 2 p32 sw0, 3 p32 sw1, 4 ror8, 5 ror4, 6 ror2, 7 ror1
__global__ void probe_k(const float* x, float* moves, float* sums, int nsets) {
  const int lane = threadIdx.x;
  const float v = (float)lane;
  {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    moves[0 * 64 + lane] = __uint_as_float(a[0]);
    moves[1 * 64 + lane] = __uint_as_float(a[1]);
    moves[2 * 64 + lane] = __uint_as_float(b[0]);
    moves[3 * 64 + lane] = __uint_as_float(b[1]);
    moves[4 * 64 + lane] = dpp<0x128>(v);
    moves[5 * 64 + lane] = dpp<0x124>(v);
    moves[6 * 64 + lane] = dpp<0x122>(v);
    moves[7 * 64 + lane] = dpp<0x121>(v);
  }
  for (int s = 0; s < nsets; ++s) {
    const float xv = x[s * 64 + lane];
    sums[(s * 6 + 0) * 64 + lane] = sum_shfl(xv, 16);
    sums[(s * 6 + 1) * 64 + lane] = sum_dpp(xv, 16);
    sums[(s * 6 + 2) * 64 + lane] = sum_shfl(xv, 32);
    sums[(s * 6 + 3) * 64 + lane] = sum_dpp(xv, 32);
    sums[(s * 6 + 4) * 64 + lane] = sum_shfl(xv, 64);
    sums[(s * 6 + 5) * 64 + lane] = sum_dpp(xv, 64);
  }
}

extern "C" int dpp_probe(const float* x, float* moves, float* sums, int nsets, void* stream) {
  hipLaunchKernelGGL(probe_k, dim3(1), dim3(64), 0, (hipStream_t)stream, x, moves, sums, nsets);
  return (int)hipGetLastError();
}
