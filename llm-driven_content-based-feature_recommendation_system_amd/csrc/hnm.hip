// Hard-negative mining for the HNM losses, one fused kernel per call:
//   cos      = u_norm @ i_norm.T                                  v1_refine_usertower.py:646-647, 709
//   ignore   = same target | (i_norm @ i_norm.T > thr & ~diag)    :650-657, 712-719, 781-783
//   mining   = (cos / tau).masked_fill(ignore, -inf)              :662-663, 724-725, 786-787
//   top_k    = torch.topk(mining, k, dim=1)                        :669, 728, 790
//   avail    = (~ignore).sum(dim=1)                                :666
// The reference materialises five N x N tensors (cos, item_sim, three masks) plus the top-k's
// sort. Here a workgroup owns R rows: it streams the N normalised column rows once (L2-resident:
// 2 MB at N = 4096, d = 128), computes both products for its R rows on the VALU, keeps the
// masked cosines of its rows in LDS, and per row runs an exact 4 x 8-bit radix select for the
// k-th largest mining value, an ordered collect (ties at the threshold value go to the lowest
// column index) and a bitonic sort of the k winners in LDS. HBM traffic is the two N x d inputs
// plus the k-wide outputs; the N x N intermediates never leave the CU.
// Output order: mining value descending, then column index ascending (torch.topk leaves tie
// order unspecified; ties need equal fp32 quotients, which random cosines do not produce).
#include "rsx_common.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

template <int D, int R>
__global__ __launch_bounds__(kThreads) void hnm_mine_k(const float* __restrict__ u, const float* __restrict__ it,
                                                      const int64_t* __restrict__ tgt, int64_t N, int k, int kpad,
                                                      float thr, float tau, int64_t* __restrict__ out_idx,
                                                      float* __restrict__ out_cos, int32_t* __restrict__ out_avail) {
  extern __shared__ __attribute__((aligned(16))) float s_dyn[];
  float* s_val = s_dyn;                                                 // [R][N] masked cosines
  float* s_u = s_val + (size_t)R * N;                                   // [R][D]
  float* s_i = s_u + R * D;                                             // [R][D]
  unsigned long long* s_sort = reinterpret_cast<unsigned long long*>(s_i + R * D);  // [kpad]
  __shared__ uint32_t s_hist[256];
  __shared__ int s_cnt[R];
  __shared__ uint32_t s_sel[3];  // prefix, remaining, gt counter
  __shared__ int s_wave_tot[kThreads / 64];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t row0 = (int64_t)blockIdx.x * R;

  for (int e = tid; e < R * D; e += kThreads) {
    const int r = e / D, c = e % D;
    const int64_t row = row0 + r;
    s_u[e] = row < N ? u[row * D + c] : 0.0f;
    s_i[e] = row < N ? it[row * D + c] : 0.0f;
  }
  if (tid < R) s_cnt[tid] = 0;
  __syncthreads();

  int64_t my_tgt[R];
#pragma unroll
  for (int r = 0; r < R; ++r) my_tgt[r] = row0 + r < N ? tgt[row0 + r] : 0;

  // ---- phase 1: both products for R rows x all columns, masked into LDS ----
  int avail[R];
#pragma unroll
  for (int r = 0; r < R; ++r) avail[r] = 0;
  for (int64_t j = tid; j < N; j += kThreads) {
    float ac[R], as[R];
#pragma unroll
    for (int r = 0; r < R; ++r) { ac[r] = 0.0f; as[r] = 0.0f; }
    const float4* xj = reinterpret_cast<const float4*>(it + j * D);
#pragma unroll 4
    for (int q = 0; q < D / 4; ++q) {
      const float4 x = xj[q];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float4 a = reinterpret_cast<const float4*>(s_u + r * D)[q];
        const float4 b = reinterpret_cast<const float4*>(s_i + r * D)[q];
        ac[r] = fmaf(a.x, x.x, ac[r]); ac[r] = fmaf(a.y, x.y, ac[r]);
        ac[r] = fmaf(a.z, x.z, ac[r]); ac[r] = fmaf(a.w, x.w, ac[r]);
        as[r] = fmaf(b.x, x.x, as[r]); as[r] = fmaf(b.y, x.y, as[r]);
        as[r] = fmaf(b.z, x.z, as[r]); as[r] = fmaf(b.w, x.w, as[r]);
      }
    }
    const int64_t tj = tgt[j];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t row = row0 + r;
      const bool ign = (tj == my_tgt[r]) || (as[r] > thr && j != row);
      avail[r] += ign ? 0 : 1;
      s_val[(size_t)r * N + j] = ign ? -INFINITY : ac[r];
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int a = rsx::wave_sum_width(avail[r], 64);
    if (lane == 0) atomicAdd(&s_cnt[r], a);
  }
  __syncthreads();

  // ---- per row: radix select, ordered collect, bitonic sort ----
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + r;
    if (row >= N) break;  // uniform across the block
    const float* v = s_val + (size_t)r * N;
    if (tid == 0) { s_sel[0] = 0u; s_sel[1] = (uint32_t)k; s_sel[2] = 0u; out_avail[row] = s_cnt[r]; }
    uint32_t mask = 0u;
    for (int shift = 24; shift >= 0; shift -= 8) {
      s_hist[tid] = 0u;
      __syncthreads();
      const uint32_t prefix = s_sel[0];
      for (int64_t j = tid; j < N; j += kThreads) {
        const uint32_t key = f2key(v[j] / tau);
        if ((key & mask) == prefix) atomicAdd(&s_hist[(key >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (wid == 0) {
        // lane l holds bins 255-4l .. 252-4l (descending); inclusive scan over lanes
        uint32_t h[4], loc = 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) { h[q] = s_hist[255 - 4 * lane - q]; loc += h[q]; }
        uint32_t inc = loc;
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t t = __shfl_up(inc, o, 64);
          if (lane >= o) inc += t;
        }
        const uint32_t rem = s_sel[1];
        const unsigned long long hit = __ballot(inc >= rem);
        const int first = __ffsll((long long)hit) - 1;  // rem <= N guarantees a hit
        if (lane == first) {
          uint32_t cum = inc - loc;
          int bin = 255 - 4 * lane;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (cum + h[q] >= rem) { bin = 255 - 4 * lane - q; break; }
            cum += h[q];
          }
          s_sel[0] = prefix | ((uint32_t)bin << shift);
          s_sel[1] = rem - cum;
        }
      }
      mask |= 255u << shift;
      __syncthreads();
    }
    const uint32_t T = s_sel[0];
    const uint32_t n_eq = s_sel[1];           // elements equal to T still to take
    const uint32_t n_gt = (uint32_t)k - n_eq;  // elements strictly above T
    for (int t = tid; t < kpad; t += kThreads) s_sort[t] = 0ull;
    __syncthreads();
    uint32_t eq_base = 0u;
    for (int64_t j0 = 0; j0 < N; j0 += kThreads) {
      const int64_t j = j0 + tid;
      uint32_t key = 0u;
      if (j < N) key = f2key(v[j] / tau);
      const unsigned long long code = ((unsigned long long)key << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)j);
      if (j < N && key > T) {
        const uint32_t slot = atomicAdd(&s_sel[2], 1u);
        s_sort[slot] = code;
      }
      const bool eq = j < N && key == T;
      const unsigned long long b = __ballot(eq);
      const uint32_t below = (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
      if (lane == 0) s_wave_tot[wid] = __popcll(b);
      __syncthreads();
      uint32_t off = eq_base;
      for (int w = 0; w < wid; ++w) off += s_wave_tot[w];
      if (eq && off + below < n_eq) s_sort[n_gt + off + below] = code;
      for (int w = 0; w < kThreads / 64; ++w) eq_base += s_wave_tot[w];
      __syncthreads();
    }
    // bitonic sort, descending on (key, -index)
    for (int size = 2; size <= kpad; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int t = tid; t < kpad / 2; t += kThreads) {
          const int lo = 2 * t - (t & (stride - 1));
          const int hi = lo + stride;
          const bool desc = (lo & size) == 0;
          const unsigned long long a = s_sort[lo], b = s_sort[hi];
          if ((a < b) == desc) { s_sort[lo] = b; s_sort[hi] = a; }
        }
        __syncthreads();
      }
    }
    for (int t = tid; t < k; t += kThreads) {
      const uint32_t j = 0xFFFFFFFFu - (uint32_t)(s_sort[t] & 0xFFFFFFFFull);
      out_idx[row * k + t] = (int64_t)j;
      // raw cosine, also for ignored columns picked when fewer than k are available
      // (the reference's torch.gather(cos_sim, 1, top_k_indices), :690, 753, 818)
      const float4* xj = reinterpret_cast<const float4*>(it + (int64_t)j * D);
      const float4* a = reinterpret_cast<const float4*>(s_u + r * D);
      float c = 0.0f;
      for (int q = 0; q < D / 4; ++q) {
        const float4 x = xj[q], y = a[q];
        c = fmaf(y.x, x.x, c); c = fmaf(y.y, x.y, c); c = fmaf(y.z, x.z, c); c = fmaf(y.w, x.w, c);
      }
      out_cos[row * k + t] = v[j] == -INFINITY ? c : v[j];
    }
    __syncthreads();
  }
}

template <int D, int R>
int launch(const float* u, const float* it, const int64_t* tgt, int64_t N, int k, int kpad, float thr, float tau,
           int64_t* out_idx, float* out_cos, int32_t* out_avail, size_t lds, hipStream_t st) {
  static bool attr_set = false;  // idempotent; racing first calls set the same value
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)hnm_mine_k<D, R>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024 - 2048);
    if (e != hipSuccess) {
      rsx::set_error("rsx_hnm_mine: cannot raise the LDS limit: %s", hipGetErrorString(e));
      return (int)e;
    }
    attr_set = true;
  }
  const unsigned g = (unsigned)((N + R - 1) / R);
  hipLaunchKernelGGL((hnm_mine_k<D, R>), dim3(g), dim3(kThreads), lds, st, u, it, tgt, N, k, kpad, thr, tau,
                     out_idx, out_cos, out_avail);
  RSX_LAUNCHED();
  return 0;
}

constexpr size_t kLdsBudget = 160 * 1024 - 2048 - 2048;  // minus the static arrays, with slack

size_t lds_bytes(int R, int64_t N, int D, int kpad) {
  return (size_t)R * N * 4 + (size_t)2 * R * D * 4 + (size_t)kpad * 8;
}

}  // namespace

RSX_API int64_t rsx_hnm_max_rows() {
  // R = 1, D = 128, k <= 1% of N
  int64_t n = 1;
  while (lds_bytes(1, n * 2, 128, 1024) <= kLdsBudget) n *= 2;
  return n;
}

RSX_API int rsx_hnm_mine(const float* u_norm, const float* i_norm, const int64_t* target_ids, int64_t N, int64_t D,
                         int64_t k, float hnm_threshold, float temperature, int64_t* top_idx, float* top_cos,
                         int32_t* avail, void* stream) {
  RSX_ARG(u_norm && i_norm && target_ids && top_idx && top_cos && avail, "null tensor");
  RSX_ARG(D == 64 || D == 128, "D must be 64 or 128");
  RSX_ARG(N >= 1 && k >= 1 && k <= N, "need 1 <= k <= N");
  RSX_ARG(temperature > 0.0f, "temperature must be positive");
  int kpad = 1;
  while (kpad < k) kpad <<= 1;
  RSX_ARG(kpad <= 4096, "k must be <= 4096");
  int R = 8;
  while (R > 1 && lds_bytes(R, N, (int)D, kpad) > kLdsBudget) R >>= 1;
  RSX_ARG(lds_bytes(R, N, (int)D, kpad) <= kLdsBudget, "N too large for one LDS-resident row (see rsx_hnm_max_rows)");
  // fewer rows per workgroup when that is what fills the 256 CUs
  while (R > 1 && (N + R - 1) / R < 1024) R >>= 1;
  const size_t lds = lds_bytes(R, N, (int)D, kpad);
  hipStream_t st = (hipStream_t)stream;
  const int kk = (int)k;
#define RSX_H(DD, RR) \
  if (D == DD && R == RR) return launch<DD, RR>(u_norm, i_norm, target_ids, N, kk, kpad, hnm_threshold, temperature, top_idx, top_cos, avail, lds, st);
  RSX_H(64, 1) RSX_H(64, 2) RSX_H(64, 4) RSX_H(64, 8)
  RSX_H(128, 1) RSX_H(128, 2) RSX_H(128, 4) RSX_H(128, 8)
#undef RSX_H
  rsx::set_error("rsx_hnm_mine: no instance");
  return 1;
}
