// Shared device/host helpers for the recsys_amd C-ABI library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace rsx {

// Thread-local last-error text; read back through rsx_last_error().
void set_error(const char* fmt, ...);

constexpr int kWave = 64;

// Counter-based dropout RNG: murmur3's fmix32 finaliser over the element index mixed with
// the 64-bit seed (32-bit integer ops only: ~10 VALU per element, cheap enough to evaluate
// per attention score). Forward and backward regenerate the identical keep-mask from the
// same (seed, index).
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  uint32_t x = (uint32_t)idx ^ ((uint32_t)(idx >> 32) * 0x9E3779B1u) ^ (uint32_t)seed;
  x ^= (uint32_t)(seed >> 32) * 0x85EBCA77u;
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

struct Dropout {
  uint64_t seed;
  uint32_t thresh;  // keep iff hash >= thresh ; thresh == 0 => no dropout
  float scale;      // 1 / (1 - p)
  __device__ __forceinline__ bool active() const { return thresh != 0u; }
  __device__ __forceinline__ float apply(float v, uint64_t idx) const {
    if (thresh == 0u) return v;
    return hash_u32(seed, idx) >= thresh ? v * scale : 0.0f;
  }
};

inline Dropout make_dropout(float p, uint64_t seed) {
  Dropout d;
  d.seed = seed;
  if (p <= 0.0f) {
    d.thresh = 0u;
    d.scale = 1.0f;
  } else {
    double t = (double)p * 4294967296.0;
    if (t >= 4294967295.0) t = 4294967295.0;
    d.thresh = (uint32_t)t;
    if (d.thresh == 0u) d.thresh = 1u;
    d.scale = 1.0f / (1.0f - p);
  }
  return d;
}

template <typename T>
__device__ __forceinline__ T wave_sum_width(T v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float fmax_nan(float a, float b) { return a > b ? a : b; }

// compute units of the current device (grid sizing, speed only); 256 when the query fails
inline int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

}  // namespace rsx

#define RSX_ARG(cond, msg)                                   \
  do {                                                       \
    if (!(cond)) {                                           \
      rsx::set_error("%s: invalid argument: %s", __func__, msg); \
      return 1;                                              \
    }                                                        \
  } while (0)

#define RSX_LAUNCHED()                                                        \
  do {                                                                        \
    hipError_t e_ = hipGetLastError();                                        \
    if (e_ != hipSuccess) {                                                   \
      rsx::set_error("%s: launch failed: %s", __func__, hipGetErrorString(e_)); \
      return (int)e_;                                                         \
    }                                                                         \
  } while (0)

#define RSX_API extern "C" __attribute__((visibility("default")))
