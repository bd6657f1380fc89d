// Row-wise gather / scatter / L2-normalise kernels used around the towers and losses:
//   * pretrained_lookup[item_ids]                    v1_usertower_train.py:760
//   * F.normalize(x, p=2, dim=-1) (eps 1e-12)        v1_refine_usertower.py:504, 584-585;
//                                                    v1_usertower_train.py:807, 811; item_tower.py:286
//   * normalize(item_matrix)[target_ids]             v1_usertower_train.py:810-811 +
//                                                    v1_refine_usertower.py:833 (row-wise, so only
//                                                    the gathered rows are normalised)
//   * output[valid_mask] / output[b, last_idx]       v1_usertower_train.py:797, 833-835
// Every row is D fp32 owned by D/4 lanes (one float4 each): 16-B coalesced accesses.
#include "rsx_common.h"

namespace {

template <int D>
struct RowGeo {
  static constexpr int LPR = D / 4;
  static constexpr int RPW = 64 / LPR;
};

// out[r] = src[idx[r]] (idx nullptr => identity), optionally L2-normalised.
template <int D, bool NORM>
__global__ __launch_bounds__(256) void gather_rows_k(const float* __restrict__ src, int64_t ld_src,
                                                    const int64_t* __restrict__ idx, int64_t n, float eps,
                                                    float* __restrict__ out, float* __restrict__ nrm_out) {
  constexpr int LPR = RowGeo<D>::LPR, RPW = RowGeo<D>::RPW;
  const int lane = threadIdx.x & 63, sub = lane / LPR, c = lane % LPR;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r0 = wave_g * RPW; r0 < n; r0 += nw * RPW) {
    const int64_t r = r0 + sub;
    const bool ok = r < n;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) {
      const int64_t s = idx ? idx[r] : r;
      x = reinterpret_cast<const float4*>(src + s * ld_src)[c];
    }
    if (NORM) {
      float ss = x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
      ss = rsx::wave_sum_width(ss, LPR);
      const float nv = sqrtf(ss);
      const float dn = fmaxf(nv, eps);
      x.x = x.x / dn; x.y = x.y / dn; x.z = x.z / dn; x.w = x.w / dn;
      if (ok && c == 0 && nrm_out) nrm_out[r] = nv;
    }
    if (ok) reinterpret_cast<float4*>(out + r * D)[c] = x;
  }
}

// Backward of y = x / max(|x|, eps):  dx = (dy - y <y,dy>) / |x|   (|x| > eps)
//                                      dx = dy / eps                 (|x| <= eps)
// dst row = idx[r] (nullptr => r); ATOMIC scatter-adds (duplicate indices allowed).
template <int D, bool NORM, bool ATOMIC>
__global__ __launch_bounds__(256) void scatter_rows_k(const float* __restrict__ dy, const float* __restrict__ y,
                                                     const float* __restrict__ nrm, const int64_t* __restrict__ idx,
                                                     int64_t n, float eps, float* __restrict__ dst, int64_t ld_dst,
                                                     int accumulate, int64_t skip_idx) {
  constexpr int LPR = RowGeo<D>::LPR, RPW = RowGeo<D>::RPW;
  __shared__ __attribute__((aligned(16))) float s_xr[ATOMIC ? 4 : 1][ATOMIC ? RPW : 1][ATOMIC ? D : 4];
  const int lane = threadIdx.x & 63, sub = lane / LPR, c = lane % LPR;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r0 = wave_g * RPW; r0 < n; r0 += nw * RPW) {
    const int64_t r = r0 + sub;
    const bool ok = r < n;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) g = reinterpret_cast<const float4*>(dy + r * D)[c];
    if (NORM) {
      float4 yv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok) yv = reinterpret_cast<const float4*>(y + r * D)[c];
      float dot = yv.x * g.x + yv.y * g.y + yv.z * g.z + yv.w * g.w;
      dot = rsx::wave_sum_width(dot, LPR);
      const float nv = ok ? nrm[r] : 1.0f;
      if (nv > eps) {
        g.x = (g.x - yv.x * dot) / nv; g.y = (g.y - yv.y * dot) / nv;
        g.z = (g.z - yv.z * dot) / nv; g.w = (g.w - yv.w * dot) / nv;
      } else {
        g.x = g.x / eps; g.y = g.y / eps; g.z = g.z / eps; g.w = g.w / eps;
      }
    }
    if (ATOMIC) {
      // lane-strided order for the atomics (lane c adds elements c + LPR*k): one line per row
      // per instruction instead of four (see seq_embed.hip); exchanged through a per-wave row
      float* xr = &s_xr[threadIdx.x >> 6][sub][0];
      reinterpret_cast<float4*>(xr)[c] = g;
      __builtin_amdgcn_wave_barrier();
      float xs[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) xs[k] = xr[c + LPR * k];
      __builtin_amdgcn_wave_barrier();
      if (!ok) continue;
      const int64_t d = idx ? idx[r] : r;
      if (d == skip_idx) continue;
      float* q = dst + d * ld_dst + c;
#pragma unroll
      for (int k = 0; k < 4; ++k) atomicAdd(q + LPR * k, xs[k]);
      continue;
    }
    if (!ok) continue;
    const int64_t d = idx ? idx[r] : r;
    if (d == skip_idx) continue;
    float* p = dst + d * ld_dst + 4 * c;
    if (accumulate) {
      float4 o = *reinterpret_cast<float4*>(p);
      o.x += g.x; o.y += g.y; o.z += g.z; o.w += g.w;
      *reinterpret_cast<float4*>(p) = o;
    } else {
      *reinterpret_cast<float4*>(p) = g;
    }
  }
}

unsigned grid_for(int64_t n, int D) {
  const int64_t rows_per_block = 4 * (64 / (D / 4));
  int64_t b = (n + rows_per_block - 1) / rows_per_block;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (unsigned)b;
}

// Segmented row sums: dst[rows[u]] (+)= scale * sum_{k in [seg[u], seg[u+1])} src[perm[k]].
// The deterministic, atomic-free form of a scatter-add with repeated indices when the sort by
// destination row is known (the embedding-table gradient of the user tower's item ids, whose
// Zipf-hot rows made the atomic form contend): one row group of lanes per segment, summed in
// segment order. rows[u] == skip (padding_idx) is left untouched; scale: device scalar.
template <int D>
__global__ __launch_bounds__(256) void segsum_rows_k(const float* __restrict__ src, int64_t ld_src,
                                                    const int64_t* __restrict__ perm,
                                                    const int64_t* __restrict__ seg,
                                                    const int64_t* __restrict__ rows, int64_t nseg,
                                                    const float* __restrict__ scale, int64_t skip,
                                                    float* __restrict__ dst, int64_t ld_dst, int accumulate) {
  constexpr int LPR = RowGeo<D>::LPR, RPW = RowGeo<D>::RPW;
  const int lane = threadIdx.x & 63, sub = lane / LPR, c = lane % LPR;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const float sc = scale ? scale[0] : 1.0f;
  for (int64_t u0 = wave_g * RPW; u0 < nseg; u0 += nw * RPW) {
    const int64_t u = u0 + sub;
    if (u >= nseg) continue;
    const int64_t row = rows ? rows[u] : u;
    if (row == skip) continue;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t k1 = seg[u + 1];
    int64_t k = seg[u];
    // sixteen index loads, then sixteen row loads in flight before the first add (the loop is a
    // dependent perm -> row chain per row otherwise); the adds keep the segment order
    for (; k + 16 <= k1; k += 16) {
      int64_t p[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) p[i] = perm ? perm[k + i] : k + i;
      float4 x[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = reinterpret_cast<const float4*>(src + p[i] * ld_src)[c];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        acc.x += x[i].x; acc.y += x[i].y; acc.z += x[i].z; acc.w += x[i].w;
      }
    }
    if (k < k1) {  // the last < 16 rows, also all in flight at once
      const int n = (int)(k1 - k);
      int64_t p[15];
#pragma unroll
      for (int i = 0; i < 15; ++i) p[i] = i < n ? (perm ? perm[k + i] : k + i) : 0;
      float4 x[15];
#pragma unroll
      for (int i = 0; i < 15; ++i)
        x[i] = i < n ? reinterpret_cast<const float4*>(src + p[i] * ld_src)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < 15; ++i)
        if (i < n) { acc.x += x[i].x; acc.y += x[i].y; acc.z += x[i].z; acc.w += x[i].w; }
    }
    float4* d = reinterpret_cast<float4*>(dst + row * ld_dst) + c;
    float4 v = make_float4(sc * acc.x, sc * acc.y, sc * acc.z, sc * acc.w);
    if (accumulate) {
      const float4 o = *d;
      v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
    }
    *d = v;
  }
}

// out[i] = ids[i] if lo <= ids[i] < hi else 0; *flag |= 1 for any id outside [lo, hi)
__global__ __launch_bounds__(256) void ids_check_k(const int64_t* __restrict__ ids, int64_t n, int64_t lo, int64_t hi,
                                                   int64_t* __restrict__ out, int* flag) {
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t v = ids[i];
    const bool ok = v >= lo && v < hi;
    out[i] = ok ? v : 0;
    bad |= !ok;
  }
  if (__builtin_amdgcn_ballot_w64(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// The contrastive step's objective from its device loss sums (train_user_tower_all_time,
// tower_code/v1_usertower_train.py:814-845, per rank of the global batch: dist.py): main = s_main /
// n, cl = s_un / b + lambda_sup * s_sup / max(cnt, 1), total = main + lambda_cl * cl.
// total[0] = total; logs = {total, main, cl} (separate storage: detached copies for logging).
__global__ void loss_combine_k(const float* s_main, const float* s_un, const float* s_sup, const float* cnt,
                               float inv_n, float inv_b, float lsup, float lcl, float* total, float* logs) {
  if (threadIdx.x != 0) return;
  const float m = s_main ? s_main[0] * inv_n : 0.0f;
  float cl = s_un[0] * inv_b;
  if (s_sup) cl += lsup * (s_sup[0] / fmaxf(cnt[0], 1.0f));
  const float t = m + lcl * cl;
  total[0] = t;
  logs[0] = t; logs[1] = m; logs[2] = cl;
}

// its backward: g3 = {d/d s_main, d/d s_un, d/d s_sup} of g * total
__global__ void loss_combine_bwd_k(const float* g, const float* cnt, float inv_n, float inv_b, float lsup, float lcl,
                                   float* g3) {
  if (threadIdx.x != 0) return;
  const float gv = g[0];
  g3[0] = gv * inv_n;
  g3[1] = gv * lcl * inv_b;
  g3[2] = cnt ? gv * lcl * lsup / fmaxf(cnt[0], 1.0f) : 0.0f;
}

}  // namespace

RSX_API int rsx_loss_combine(const float* s_main, const float* s_un, const float* s_sup, const float* cnt,
                             float inv_n, float inv_b, float lambda_sup, float lambda_cl, float* total, float* logs,
                             void* stream) {
  RSX_ARG(s_un && total && logs && (!s_sup || cnt), "null tensor");
  hipLaunchKernelGGL(loss_combine_k, dim3(1), dim3(64), 0, (hipStream_t)stream, s_main, s_un, s_sup, cnt, inv_n,
                     inv_b, lambda_sup, lambda_cl, total, logs);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_loss_combine_bwd(const float* g, const float* cnt, float inv_n, float inv_b, float lambda_sup,
                                 float lambda_cl, float* g3, void* stream) {
  RSX_ARG(g && g3, "null tensor");
  hipLaunchKernelGGL(loss_combine_bwd_k, dim3(1), dim3(64), 0, (hipStream_t)stream, g, cnt, inv_n, inv_b,
                     lambda_sup, lambda_cl, g3);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_gather_rows(const float* src, int64_t ld_src, const int64_t* idx, int64_t n, int64_t D, int normalize,
                            float eps, float* out, float* nrm_out, void* stream) {
  RSX_ARG(src && out, "null tensor");
  RSX_ARG(D == 64 || D == 128 || D == 256, "D must be 64, 128 or 256");
  RSX_ARG(ld_src >= D && ld_src % 4 == 0, "bad ld_src");
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = grid_for(n, (int)D);
#define RSX_G(DD)                                                                                     \
  if (D == DD) {                                                                                      \
    if (normalize) hipLaunchKernelGGL((gather_rows_k<DD, true>), dim3(g), dim3(256), 0, st, src, ld_src, idx, n, eps, out, nrm_out); \
    else hipLaunchKernelGGL((gather_rows_k<DD, false>), dim3(g), dim3(256), 0, st, src, ld_src, idx, n, eps, out, nrm_out); \
  }
  RSX_G(64) RSX_G(128) RSX_G(256)
#undef RSX_G
  RSX_LAUNCHED();
  return 0;
}

// mode: 0 = plain store, 1 = accumulate (+=, indices must be unique), 2 = atomic scatter-add
RSX_API int rsx_scatter_rows(const float* dy, const float* y, const float* nrm, const int64_t* idx, int64_t n,
                             int64_t D, int normalize, float eps, int mode, int64_t skip_idx, float* dst,
                             int64_t ld_dst, void* stream) {
  RSX_ARG(dy && dst, "null tensor");
  RSX_ARG(!normalize || (y && nrm), "normalize backward needs y and norms");
  RSX_ARG(D == 64 || D == 128 || D == 256, "D must be 64, 128 or 256");
  RSX_ARG(mode >= 0 && mode <= 2, "mode must be 0,1,2");
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = grid_for(n, (int)D);
#define RSX_S(DD, NN, AA)                                                                           \
  hipLaunchKernelGGL((scatter_rows_k<DD, NN, AA>), dim3(g), dim3(256), 0, st, dy, y, nrm, idx, n, eps, dst, ld_dst, \
                     mode == 1 ? 1 : 0, skip_idx)
#define RSX_SD(DD)                                          \
  if (D == DD) {                                            \
    if (normalize) {                                        \
      if (mode == 2) RSX_S(DD, true, true); else RSX_S(DD, true, false);   \
    } else {                                                \
      if (mode == 2) RSX_S(DD, false, true); else RSX_S(DD, false, false); \
    }                                                       \
  }
  RSX_SD(64) RSX_SD(128) RSX_SD(256)
#undef RSX_SD
#undef RSX_S
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_segment_sum_rows(const float* src, int64_t ld_src, const int64_t* perm, const int64_t* seg_off,
                                 const int64_t* rows, int64_t nseg, int64_t D, const float* scale, int64_t skip_row,
                                 float* dst, int64_t ld_dst, int accumulate, void* stream) {
  RSX_ARG(src && seg_off && dst, "null tensor");  // perm NULL: identity; rows NULL: row u
  RSX_ARG(D == 64 || D == 128 || D == 256, "D must be 64, 128 or 256");
  RSX_ARG(ld_src >= D && ld_dst >= D && ld_src % 4 == 0 && ld_dst % 4 == 0, "bad leading dimensions");
  if (nseg == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = grid_for(nseg, (int)D);
#define RSX_SS(DD)                                                                                            \
  if (D == DD)                                                                                                \
    hipLaunchKernelGGL(segsum_rows_k<DD>, dim3(g), dim3(256), 0, st, src, ld_src, perm, seg_off, rows, nseg, \
                       scale, skip_row, dst, ld_dst, accumulate);
  RSX_SS(64) RSX_SS(128) RSX_SS(256)
#undef RSX_SS
  RSX_LAUNCHED();
  return 0;
}

// Range check of an id tensor on the device, with no host synchronisation: out = ids with every
// id outside [lo, hi) replaced by 0 (so a following gather never reads out of bounds), *flag set
// to 1 if any id was out of range, else left as the caller initialised it.
RSX_API int rsx_ids_check(const int64_t* ids, int64_t n, int64_t lo, int64_t hi, int64_t* out, int* flag,
                          void* stream) {
  RSX_ARG(ids && out && flag, "null tensor");
  RSX_ARG(lo <= 0 && 0 < hi, "the replacement id 0 must lie in [lo, hi)");
  if (n == 0) return 0;
  int64_t g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(ids_check_k, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, ids, n, lo, hi, out, flag);
  RSX_LAUNCHED();
  return 0;
}
