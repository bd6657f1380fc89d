// Hard-negative mining for the HNM losses:
//   cos      = u_norm @ i_norm.T                                  v1_refine_usertower.py:646-647, 709
//   ignore   = same target | (i_norm @ i_norm.T > thr & ~diag)    :650-657, 712-719, 781-783
//   mining   = (cos / tau).masked_fill(ignore, -inf)              :662-663, 724-725, 786-787
//   top_k    = torch.topk(mining, k, dim=1)                        :669, 728, 790
//   avail    = (~ignore).sum(dim=1)                                :666
// The reference materialises five N x N tensors (cos, item_sim, three masks) plus the top-k's
// sort. Here two kernels and ONE N x N fp32 workspace:
//   hnm_products_k: 128 rows per workgroup (32 per wave, both u and i rows held in registers),
//     32-column tiles of i_norm (and their targets) staged through LDS, both products on the
//     fp32 MFMA (v_mfma_f32_32x32x2f32), the same-target / item-similarity mask applied to the
//     accumulators, masked cosines stored as float4 rows of the workspace;
//   hnm_select_k: R rows per workgroup read back into LDS (coalesced), per row an exact
//     4 x 8-bit radix select of the k-th largest mining value, an ordered collect (ties at the
//     threshold value go to the lowest column index) and a bitonic sort of the k winners.
// Output order: mining value descending, then column index ascending (torch.topk leaves tie
// order unspecified; ties need equal fp32 quotients, which random cosines do not produce).
#include "rsx_common.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}


typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kRowsPerBlock = 128;
constexpr int kTileCols = 32;

__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

int64_t ws_ld(int64_t N) { return (N + kTileCols - 1) / kTileCols * kTileCols; }

// ws[q, j] = ignore(q, j) ? -inf : u_q . i_j for q < N, j < ws_ld(N) (columns >= N: don't care).
// Lane (c, h) of wave w owns row q = 128 * rb + 32 * w + c and the k-half h of its u and i rows;
// the 32x32x2 MFMA with the tile's item row c as A and the row's registers as B leaves the
// products of row q with items tile_row(r, h), r < 16, in the lane's accumulators.
template <int D>
__global__ __launch_bounds__(256) void hnm_products_k(const float* __restrict__ u, const float* __restrict__ it,
                                                     const int64_t* __restrict__ tgt, int64_t N, int nsplit,
                                                     int64_t span, float thr, float* __restrict__ ws, int64_t ldw) {
  constexpr int KH = D / 2;
  constexpr int LS = D + 4;
  __shared__ __attribute__((aligned(16))) float sI[2][kTileCols][LS];
  __shared__ int64_t sT[2][kTileCols];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int rb = blockIdx.x / nsplit, split = blockIdx.x % nsplit;
  const int64_t q = (int64_t)rb * kRowsPerBlock + wave * 32 + c;
  const bool q_ok = q < N;
  float ur[KH], ir[KH];
#pragma unroll
  for (int t = 0; t < KH / 4; ++t) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (q_ok) {
      a = reinterpret_cast<const float4*>(u + q * D + h * KH)[t];
      b = reinterpret_cast<const float4*>(it + q * D + h * KH)[t];
    }
    ur[4 * t] = a.x; ur[4 * t + 1] = a.y; ur[4 * t + 2] = a.z; ur[4 * t + 3] = a.w;
    ir[4 * t] = b.x; ir[4 * t + 1] = b.y; ir[4 * t + 2] = b.z; ir[4 * t + 3] = b.w;
  }
  const int64_t tq = q_ok ? tgt[q] : -1;
  const int64_t j_begin = (int64_t)split * span;
  int64_t j_end = j_begin + span;
  if (j_end > ldw) j_end = ldw;

  // staging: 256 threads x (D / 8) floats = one 32 x D tile (8 threads per row, float4 loads)
  constexpr int V4 = D / 32;  // float4 per thread: 4 (D = 128) or 2 (D = 64)
  const int srow = tid >> 3, scol = (tid & 7) * (D / 8);
  float4 stg[V4];
  int64_t stg_t = 0;
  auto gload = [&](int64_t j0) {
    const int64_t j = j0 + srow;
    const bool ok = j < N;
#pragma unroll
    for (int t = 0; t < V4; ++t)
      stg[t] = ok ? reinterpret_cast<const float4*>(it + j * D + scol)[t] : make_float4(0.f, 0.f, 0.f, 0.f);
    if ((tid & 7) == 0) stg_t = ok ? tgt[j] : INT64_MIN;
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int t = 0; t < V4; ++t) *reinterpret_cast<float4*>(&sI[buf][srow][scol + 4 * t]) = stg[t];
    if ((tid & 7) == 0) sT[buf][srow] = stg_t;
  };
  if (j_begin >= j_end) return;
  gload(j_begin);
  lstore(0);
  __syncthreads();
  int cur = 0;
  for (int64_t j0 = j_begin; j0 < j_end; j0 += kTileCols) {
    const bool has_next = j0 + kTileCols < j_end;
    if (has_next) gload(j0 + kTileCols);
    f32x16 ac, as;
#pragma unroll
    for (int r = 0; r < 16; ++r) { ac[r] = 0.0f; as[r] = 0.0f; }
    const float* xrow = &sI[cur][c][h * KH];
#pragma unroll
    for (int s = 0; s < KH; s += 4) {
      const float4 bv = *reinterpret_cast<const float4*>(xrow + s);
      ac = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.x, ur[s + 0], ac, 0, 0, 0);
      as = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.x, ir[s + 0], as, 0, 0, 0);
      ac = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.y, ur[s + 1], ac, 0, 0, 0);
      as = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.y, ir[s + 1], as, 0, 0, 0);
      ac = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.z, ur[s + 2], ac, 0, 0, 0);
      as = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.z, ir[s + 2], as, 0, 0, 0);
      ac = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.w, ur[s + 3], ac, 0, 0, 0);
      as = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.w, ir[s + 3], as, 0, 0, 0);
    }
    if (q_ok) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          const int jt = tile_row(r, h);
          const int64_t j = j0 + jt;
          const bool ign = (sT[cur][jt] == tq) || (as[r] > thr && j != q);
          o[e] = ign ? -INFINITY : ac[r];
        }
        *reinterpret_cast<float4*>(ws + q * ldw + j0 + 8 * g + 4 * h) = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
    __syncthreads();
    if (has_next) lstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
}

// Block-wide exclusive prefix of per-thread counts (256 threads); returns the block total.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_wt, uint32_t& excl) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = x;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) s_wt[wid] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (int w = 0; w < kThreads / 64; ++w) {
    if (w < wid) base += s_wt[w];
    tot += s_wt[w];
  }
  excl = base + inc - x;
  __syncthreads();
  return tot;
}

// wave 0: bins 255..0 scanned from the top; the bin where the running count reaches rem.
// Writes s_out[0] = bin, s_out[1] = count strictly above that bin.
__device__ __forceinline__ void find_bin(const uint32_t* s_hist, uint32_t rem, uint32_t* s_out) {
  const int lane = threadIdx.x & 63;
  uint32_t h[4], loc = 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) { h[q] = s_hist[255 - 4 * lane - q]; loc += h[q]; }
  uint32_t inc = loc;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  const unsigned long long hit = __ballot(inc >= rem);
  const int first = __ffsll((long long)hit) - 1;  // rem <= total guarantees a hit
  if (lane == first) {
    uint32_t cum = inc - loc;
    int bin = 255 - 4 * lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (cum + h[q] >= rem) { bin = 255 - 4 * lane - q; break; }
      cum += h[q];
    }
    s_out[0] = (uint32_t)bin;
    s_out[1] = cum;
  }
}

// Per row: the k largest (mining value desc, column asc) of the row's masked cosines.
// Fast path: one pass bins the available values linearly over [row min, row max] into 256
// bins (monotone in the value, so every value of a higher bin is strictly larger), a second
// pass compacts the bins above the k-th value's bin plus that bin's members into a buffer of
// at most BUF codes, which is bitonic-sorted. If the boundary bin holds more than the buffer
// allows (heavy ties / degenerate rows), an exact 4 x 8-bit radix select over the order-
// preserving uint32 keys finds the k-th key and an ordered collect takes the ties at it in
// column order. Codes are (key << 32 | ~column), so one descending sort gives the total order.
template <int D, int R>
__global__ __launch_bounds__(kThreads) void hnm_select_k(const float* __restrict__ u, const float* __restrict__ it,
                                                        const float* __restrict__ ws, int64_t ldw, int64_t N, int k,
                                                        int buf, float tau, int64_t* __restrict__ out_idx,
                                                        float* __restrict__ out_cos, int32_t* __restrict__ out_avail) {
  extern __shared__ __attribute__((aligned(16))) float s_dyn[];
  const int64_t NP = (N + 3) & ~(int64_t)3;
  float* s_val = s_dyn;                                                   // [R][NP] mining values
  float* s_u = s_val + (size_t)R * NP;                                    // [R][D]
  unsigned long long* s_sort = reinterpret_cast<unsigned long long*>(s_u + R * D);  // [buf]
  __shared__ uint32_t s_hist[256];
  __shared__ int s_cnt[R];
  __shared__ uint32_t s_mx[R], s_mn[R];  // order keys of the row max / min available value
  __shared__ uint32_t s_sel[4];
  __shared__ uint32_t s_wt[kThreads / 64];

  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const uint32_t kNegInf = f2key(-INFINITY);

  for (int e = tid; e < R * D; e += kThreads) {
    const int r = e / D, c = e % D;
    const int64_t row = row0 + r;
    s_u[e] = row < N ? u[row * D + c] : 0.0f;
  }
  if (tid < R) { s_cnt[tid] = 0; s_mx[tid] = 0u; s_mn[tid] = 0xFFFFFFFFu; }
  __syncthreads();

  // ---- phase 1: mining values (cos / tau) into LDS; available counts, min and max ----
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int avail = 0;
    uint32_t mx = 0u, mn = 0xFFFFFFFFu;
    if (row0 + r < N) {
      const float* src = ws + (row0 + r) * ldw;
      for (int64_t j = tid; j < N; j += kThreads) {
        const float x = src[j] / tau;
        const uint32_t key = f2key(x);
        if (key != kNegInf) {
          ++avail;
          mx = max(mx, key);
          mn = min(mn, key);
        }
        s_val[(size_t)r * NP + j] = x;
      }
    }
    avail = rsx::wave_sum_width(avail, 64);
    for (int o = 32; o > 0; o >>= 1) {
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
      mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
    }
    if (lane == 0) { atomicAdd(&s_cnt[r], avail); atomicMax(&s_mx[r], mx); atomicMin(&s_mn[r], mn); }
  }
  __syncthreads();

  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + r;
    if (row >= N) break;  // uniform across the block
    const float* v = s_val + (size_t)r * NP;
    const uint32_t n_av = (uint32_t)s_cnt[r];
    if (tid == 0) out_avail[row] = (int32_t)n_av;
    int nsort = 0;  // entries of s_sort to sort (power of two)
    bool done = false;

    if (n_av >= (uint32_t)k) {
      // ---- fast path: linear bins over [min, max] ----
      const float lo = __uint_as_float((s_mn[r] & 0x80000000u) ? (s_mn[r] & 0x7FFFFFFFu) : ~s_mn[r]);
      const float hi = __uint_as_float((s_mx[r] & 0x80000000u) ? (s_mx[r] & 0x7FFFFFFFu) : ~s_mx[r]);
      const float scale = 256.0f / (hi - lo);
      if (hi > lo && isfinite(scale) && scale > 0.0f) {
        s_hist[tid] = 0u;
        __syncthreads();
        for (int64_t j = tid; j < N; j += kThreads) {
          const float x = v[j];
          if (x != -INFINITY) atomicAdd(&s_hist[min(255, (int)((x - lo) * scale))], 1u);
        }
        __syncthreads();
        if ((tid >> 6) == 0) find_bin(s_hist, (uint32_t)k, s_sel);
        __syncthreads();
        const int b = (int)s_sel[0];
        const uint32_t n_take = s_sel[1] + s_hist[b];  // everything above b plus bin b
        if (n_take <= (uint32_t)buf) {
          // insertion order is free (the buffer is sorted next): wave-aggregated slot claims
          if (tid == 0) s_sel[2] = 0u;
          __syncthreads();
          for (int64_t j0 = tid - lane; j0 < N; j0 += kThreads) {  // wave-uniform trip count
            const int64_t j = j0 + lane;
            bool take = false;
            float x = -INFINITY;
            if (j < N) {
              x = v[j];
              take = x != -INFINITY && min(255, (int)((x - lo) * scale)) >= b;
            }
            const unsigned long long m = __ballot(take);
            if (m == 0ull) continue;
            uint32_t slot0 = 0u;
            if (lane == 0) slot0 = atomicAdd(&s_sel[2], (uint32_t)__popcll(m));
            slot0 = (uint32_t)__shfl((int)slot0, 0, 64);
            if (take)
              s_sort[slot0 + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] =
                  ((unsigned long long)f2key(x) << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)j);
          }
          __syncthreads();
          nsort = 1;
          while (nsort < (int)n_take) nsort <<= 1;
          for (int t = (int)n_take + tid; t < nsort; t += kThreads) s_sort[t] = 0ull;
          done = true;
        }
      }
    }
    if (!done) {
      // ---- exact radix select of the k-th key, then ordered collect ----
      __syncthreads();  // the fast path's readers of s_sel are done
      if (tid == 0) { s_sel[0] = 0u; s_sel[1] = (uint32_t)k; }
      uint32_t mask = 0u;
      for (int shift = 24; shift >= 0; shift -= 8) {
        s_hist[tid] = 0u;
        __syncthreads();
        const uint32_t prefix = s_sel[0];
        const uint32_t rem = s_sel[1];
        for (int64_t j = tid; j < N; j += kThreads) {
          const uint32_t key = f2key(v[j]);
          if ((key & mask) == prefix) atomicAdd(&s_hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if ((tid >> 6) == 0) find_bin(s_hist, rem, s_sel + 2);
        __syncthreads();
        if (tid == 0) {
          s_sel[0] = prefix | (s_sel[2] << shift);
          s_sel[1] = rem - s_sel[3];
        }
        mask |= 255u << shift;
        __syncthreads();
      }
      const uint32_t T = s_sel[0];
      const uint32_t n_eq = s_sel[1];           // elements equal to T to take (lowest columns)
      const uint32_t n_gt = (uint32_t)k - n_eq;  // elements strictly above T
      uint32_t gt_base = 0, eq_base = 0;
      for (int64_t j0 = 0; j0 < N; j0 += kThreads) {
        const int64_t j = j0 + tid;
        uint32_t key = 0u;
        if (j < N) key = f2key(v[j]);
        const unsigned long long code = ((unsigned long long)key << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)j);
        const bool gt = j < N && key > T, eq = j < N && key == T;
        uint32_t e_gt, e_eq;
        const uint32_t t_gt = block_excl_scan(gt ? 1u : 0u, s_wt, e_gt);
        const uint32_t t_eq = block_excl_scan(eq ? 1u : 0u, s_wt, e_eq);
        if (gt) s_sort[gt_base + e_gt] = code;
        if (eq && eq_base + e_eq < n_eq) s_sort[n_gt + eq_base + e_eq] = code;
        gt_base += t_gt;
        eq_base += t_eq;
      }
      nsort = 1;
      while (nsort < k) nsort <<= 1;
      for (int t = k + tid; t < nsort; t += kThreads) s_sort[t] = 0ull;
    }
    __syncthreads();
    // bitonic sort of nsort codes, descending
    for (int size = 2; size <= nsort; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int t = tid; t < nsort / 2; t += kThreads) {
          const int lo = 2 * t - (t & (stride - 1));
          const int hi = lo + stride;
          const bool desc = (lo & size) == 0;
          const unsigned long long a = s_sort[lo], b = s_sort[hi];
          if ((a < b) == desc) { s_sort[lo] = b; s_sort[hi] = a; }
        }
        __syncthreads();
      }
    }
    // outputs; the raw cosine is recomputed (also for ignored columns picked when fewer than
    // k are available: the reference's torch.gather(cos_sim, 1, top_k_indices), :690, 753, 818)
    for (int t = tid; t < k; t += kThreads) {
      const uint32_t j = 0xFFFFFFFFu - (uint32_t)(s_sort[t] & 0xFFFFFFFFull);
      out_idx[row * k + t] = (int64_t)j;
      const float4* xj = reinterpret_cast<const float4*>(it + (int64_t)j * D);
      const float4* a = reinterpret_cast<const float4*>(s_u + r * D);
      float c = 0.0f;
      for (int q = 0; q < D / 4; ++q) {
        const float4 x = xj[q], y = a[q];
        c = fmaf(y.x, x.x, c); c = fmaf(y.y, x.y, c); c = fmaf(y.z, x.z, c); c = fmaf(y.w, x.w, c);
      }
      out_cos[row * k + t] = c;
    }
    __syncthreads();
  }
}

constexpr size_t kLdsBudget = 160 * 1024 - 2048 - 2048;  // minus the static arrays, with slack

size_t lds_bytes(int R, int64_t N, int D, int buf) {
  return (size_t)R * ((N + 3) & ~(int64_t)3) * 4 + (size_t)R * D * 4 + (size_t)buf * 8;
}

template <int D, int R>
int launch_select(const float* u, const float* it, const float* ws, int64_t ldw, int64_t N, int k, int buf,
                  float tau, int64_t* out_idx, float* out_cos, int32_t* out_avail, size_t lds, hipStream_t st) {
  static bool attr_set = false;  // idempotent; racing first calls set the same value
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)hnm_select_k<D, R>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024 - 2048);
    if (e != hipSuccess) {
      rsx::set_error("rsx_hnm_mine: cannot raise the LDS limit: %s", hipGetErrorString(e));
      return (int)e;
    }
    attr_set = true;
  }
  const unsigned g = (unsigned)((N + R - 1) / R);
  hipLaunchKernelGGL((hnm_select_k<D, R>), dim3(g), dim3(kThreads), lds, st, u, it, ws, ldw, N, k, buf, tau,
                     out_idx, out_cos, out_avail);
  RSX_LAUNCHED();
  return 0;
}

}  // namespace

RSX_API int64_t rsx_hnm_max_rows() {
  // R = 1, D = 128, k <= 4096
  int64_t n = 1;
  while (lds_bytes(1, n * 2, 128, 8192) <= kLdsBudget) n *= 2;
  return n;
}

RSX_API int64_t rsx_hnm_workspace_bytes(int64_t N) { return N * ws_ld(N) * (int64_t)sizeof(float); }

RSX_API int rsx_hnm_mine(const float* u_norm, const float* i_norm, const int64_t* target_ids, int64_t N, int64_t D,
                         int64_t k, float hnm_threshold, float temperature, void* ws, size_t ws_bytes,
                         int64_t* top_idx, float* top_cos, int32_t* avail, void* stream) {
  RSX_ARG(u_norm && i_norm && target_ids && ws && top_idx && top_cos && avail, "null tensor");
  RSX_ARG(D == 64 || D == 128, "D must be 64 or 128");
  RSX_ARG(N >= 1 && k >= 1 && k <= N, "need 1 <= k <= N");
  RSX_ARG(temperature > 0.0f, "temperature must be positive");
  RSX_ARG((int64_t)ws_bytes >= rsx_hnm_workspace_bytes(N), "workspace smaller than rsx_hnm_workspace_bytes(N)");
  RSX_ARG(((uintptr_t)ws & 15) == 0, "workspace must be 16-byte aligned");
  int kpad = 1;
  while (kpad < k) kpad <<= 1;
  RSX_ARG(kpad <= 4096, "k must be <= 4096");
  // sort buffer: the k winners, or (fast path) everything from the k-th value's bin upward
  const int buf = kpad * 2 > 1024 ? kpad * 2 : 1024;
  int R = 8;
  while (R > 1 && lds_bytes(R, N, (int)D, buf) > kLdsBudget) R >>= 1;
  RSX_ARG(lds_bytes(R, N, (int)D, buf) <= kLdsBudget, "N too large for one LDS-resident row (see rsx_hnm_max_rows)");
  // keep several workgroups per CU resident (the select is latency-bound)
  while (R > 1 && lds_bytes(R, N, (int)D, buf) > 40 * 1024) R >>= 1;
  // fewer rows per workgroup when that is what fills the 256 CUs
  while (R > 1 && (N + R - 1) / R < 2048) R >>= 1;
  const size_t lds = lds_bytes(R, N, (int)D, buf);
  hipStream_t st = (hipStream_t)stream;
  float* w = (float*)ws;
  const int64_t ldw = ws_ld(N);

  // products: row blocks x column splits, >= ~1024 workgroups, spans whole 32-column tiles
  const int64_t nrb = (N + kRowsPerBlock - 1) / kRowsPerBlock;
  const int64_t ntiles = ldw / kTileCols;
  int64_t nsplit = (1024 + nrb - 1) / nrb;
  if (nsplit > ntiles) nsplit = ntiles;
  if (nsplit < 1) nsplit = 1;
  const int64_t span = (ntiles + nsplit - 1) / nsplit * kTileCols;
  nsplit = (ldw + span - 1) / span;
  const unsigned gp = (unsigned)(nrb * nsplit);
  if (D == 128)
    hipLaunchKernelGGL(hnm_products_k<128>, dim3(gp), dim3(256), 0, st, u_norm, i_norm, target_ids, N, (int)nsplit,
                       span, hnm_threshold, w, ldw);
  else
    hipLaunchKernelGGL(hnm_products_k<64>, dim3(gp), dim3(256), 0, st, u_norm, i_norm, target_ids, N, (int)nsplit,
                       span, hnm_threshold, w, ldw);
  RSX_LAUNCHED();

  const int kk = (int)k;
#define RSX_H(DD, RR) \
  if (D == DD && R == RR) return launch_select<DD, RR>(u_norm, i_norm, w, ldw, N, kk, buf, temperature, top_idx, top_cos, avail, lds, st);
  RSX_H(64, 1) RSX_H(64, 2) RSX_H(64, 4) RSX_H(64, 8)
  RSX_H(128, 1) RSX_H(128, 2) RSX_H(128, 4) RSX_H(128, 8)
#undef RSX_H
  rsx::set_error("rsx_hnm_mine: no instance");
  return 1;
}
