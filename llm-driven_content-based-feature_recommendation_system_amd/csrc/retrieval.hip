// Retrieval: top-k items by inner product, without materialising the [Q, I] score matrix.
// Two exact paths: the list-based scan below (small corpora, and the gated fallback), and the
// candidate -> threshold -> collect path further down (large corpora: two MFMA scans, no
// per-insertion list maintenance).
// Reference: evaluate_model (tower_code/v1_usertower_train.py:672-675: scores = U W_n^T;
// topk(max_k)) and ReRankingSystem.recommend (temp_model/ranker_skelet.py:193-196).
//
// Pass 1 (topk_scan_k): every workgroup owns 128 query rows (32 per wave, in registers as
// in the InfoNCE kernels) and one item split; 32-item tiles stream through LDS and the
// fp32-input MFMA produces a 32x32 score tile per wave. Each lane sees 16 of the tile's
// items for its query and keeps the best KMAX of its stream in a private list (L1/L2
// resident, replacement of the current minimum + rescan; after the first KMAX items an
// insertion is rare, ~K ln(n/K) per stream).
// Pass 2 (topk_merge_k): per query, the 2 * nsplit lists are bitonic-sorted in LDS by
// (score desc, index asc) and the first k are written. Ties therefore resolve to the lower
// item index (documented tie-break; torch.topk leaves tie order unspecified).
#include "rsx_common.h"
#include <math.h>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kD = 128;
constexpr int kTile = 32;
constexpr int kOwnRows = 128;
constexpr int kLdsStride = kD + 4;

__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

struct ScanArgs {
  const int* gate;  // nullptr, or: run only if *gate != 0 (the exact fallback of the fast path)
  const int* qmap;  // nullptr, or: logical row r is query qmap[r], for r < *qcount (per-query fallback)
  const int* qcount;
  const float* U;  // [Q, ldu]
  const float* I;  // [NI, ldi]
  int64_t Q, NI, ldu, ldi;
  int nsplit;
  int64_t span;
  int K;          // k (<= KMAX)
  float* cs;      // [Q][nsplit][2][KMAX] scores
  int* ci;        // [Q][nsplit][2][KMAX] indices
};

// (a beats b) <=> a.score > b.score or (equal and a.idx < b.idx)
__device__ __forceinline__ bool better(float sa, int ia, float sb, int ib) {
  return sa > sb || (sa == sb && ia < ib);
}

template <int KMAX>
__global__ __launch_bounds__(256, 2) void topk_scan_k(ScanArgs a) {
  if (a.gate && *a.gate == 0) return;
  const int64_t nq = a.qcount ? (int64_t)*a.qcount : a.Q;
  __shared__ __attribute__((aligned(16))) float sI[2][kTile][kLdsStride];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int b = blockIdx.x;
  const int nsub = a.nsplit >> 3;
  const int split = (b & 7) + 8 * ((b >> 3) % nsub);
  const int rb = (b >> 3) / nsub;
  if ((int64_t)rb * kOwnRows >= nq) return;  // whole workgroup: no logical rows here
  const int64_t ql = (int64_t)rb * kOwnRows + wave * 32 + c;  // logical row (workspace index)
  const bool q_ok = ql < nq;
  const int64_t q = (q_ok && a.qmap) ? (int64_t)a.qmap[ql] : ql;
  float u[64];
  if (q_ok) {
    const float4* src = reinterpret_cast<const float4*>(a.U + q * a.ldu + h * 64);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float4 v = src[t];
      u[4 * t] = v.x; u[4 * t + 1] = v.y; u[4 * t + 2] = v.z; u[4 * t + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < 64; ++t) u[t] = 0.0f;
  }
  const int64_t j_begin = (int64_t)split * a.span;
  int64_t j_end = j_begin + a.span;
  if (j_end > a.NI) j_end = a.NI;

  const int64_t lbase = ((q_ok ? ql : 0) * a.nsplit + split) * 2 + h;
  float* ls = a.cs + lbase * KMAX;
  int* li = a.ci + lbase * KMAX;
  const int K = a.K;
  int cnt = 0, minslot = 0;
  float thr = -INFINITY;
  int thr_i = 0x7fffffff;

  auto rescan = [&]() {
    float ms = ls[0];
    int mi = li[0], mslot = 0;
    for (int t = 1; t < K; ++t) {
      const float s = ls[t];
      const int ii = li[t];
      if (better(ms, mi, s, ii)) { ms = s; mi = ii; mslot = t; }
    }
    thr = ms; thr_i = mi; minslot = mslot;
  };

  const int srow = tid >> 3, scol = (tid & 7) * 16;
  float4 stg[4];
  auto gload = [&](int64_t j0) {
    const int64_t j = j0 + srow;
    if (j < j_end) {
      const float4* src = reinterpret_cast<const float4*>(a.I + j * a.ldi + scol);
#pragma unroll
      for (int t = 0; t < 4; ++t) stg[t] = src[t];
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) stg[t] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int t = 0; t < 4; ++t) *reinterpret_cast<float4*>(&sI[buf][srow][scol + 4 * t]) = stg[t];
  };

  if (j_begin < j_end) {
    gload(j_begin);
    lstore(0);
    __syncthreads();
    int cur = 0;
    for (int64_t j0 = j_begin; j0 < j_end; j0 += kTile) {
      const bool has_next = j0 + kTile < j_end;
      if (has_next) gload(j0 + kTile);
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
      const float* xrow = &sI[cur][c][h * 64];
#pragma unroll
      for (int s = 0; s < 64; s += 4) {
        const float4 bv = *reinterpret_cast<const float4*>(xrow + s);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.x, u[s + 0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.y, u[s + 1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.z, u[s + 2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.w, u[s + 3], acc, 0, 0, 0);
      }
      if (q_ok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t j = j0 + tile_row(r, h);
          const float s = acc[r];
          if (j < j_end) {
            if (cnt < K) {
              ls[cnt] = s;
              li[cnt] = (int)j;
              ++cnt;
              if (cnt == K) rescan();
            } else if (better(s, (int)j, thr, thr_i)) {
              ls[minslot] = s;
              li[minslot] = (int)j;
              rescan();
            }
          }
        }
      }
      __syncthreads();
      if (has_next) lstore(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }
  if (q_ok) {
    for (int t = cnt; t < KMAX; ++t) {
      ls[t] = -INFINITY;
      li[t] = 0x7fffffff;
    }
  }
}

// One workgroup per query: bitonic sort of NC = 2*nsplit*KMAX candidates, descending.
template <int NC>
__global__ __launch_bounds__(256) void topk_merge_k(const float* cs, const int* ci, int64_t Q, int ncand, int K,
                                                    float* out_s, int64_t* out_i, const int* gate, const int* qmap,
                                                    const int* qcount) {
  if (gate && *gate == 0) return;
  __shared__ float ss[NC];
  __shared__ int si[NC];
  const int64_t ql = blockIdx.x;
  if (qcount && ql >= *qcount) return;
  const int64_t q = qmap ? (int64_t)qmap[ql] : ql;
  const float* s = cs + ql * ncand;
  const int* ii = ci + ql * ncand;
  for (int t = threadIdx.x; t < NC; t += blockDim.x) {
    if (t < ncand) {
      ss[t] = s[t];
      si[t] = ii[t];
    } else {
      ss[t] = -INFINITY;
      si[t] = 0x7fffffff;
    }
  }
  __syncthreads();
  for (int size = 2; size <= NC; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < NC / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);  // descending runs first => overall descending
        const float a0 = ss[lo], a1 = ss[hi];
        const int b0 = si[lo], b1 = si[hi];
        const bool swap = desc ? better(a1, b1, a0, b0) : better(a0, b0, a1, b1);
        if (swap) {
          ss[lo] = a1; ss[hi] = a0;
          si[lo] = b1; si[hi] = b0;
        }
      }
      __syncthreads();
    }
  }
  for (int t = threadIdx.x; t < K; t += blockDim.x) {
    out_s[q * K + t] = ss[t];
    out_i[q * K + t] = (si[t] == 0x7fffffff) ? -1 : (int64_t)si[t];
  }
}

// ---- fast exact path (large corpora): candidates -> threshold -> collect -> final sort -----
// K1 (MODE 0): the scan above, but each lane keeps only the best T of its stream in registers.
// K2: per query, the k-th best of the 2*nsplit*T candidates is a lower bound t_q of the true
//     k-th best score (the candidates are real items).
// K3 (MODE 1): the scan again; every item with score >= t_q is appended to the query's buffer
//     (a superset of the true top-k, ties included; typically ~k entries).
// K4: per query, sort the buffer by (score desc, index asc) and write the first k.
// If a buffer overflows (massive exact ties at t_q), K4 raises a device flag and the exact
// list-based kernels above re-run for the whole batch, gated on that flag (no host sync).
struct FastArgs {
  const float* U;
  const float* I;
  int64_t Q, NI, ldu, ldi;
  int nsplit;
  int64_t span;
  int K, cap;
  float* cand_s;        // [Q][nsplit][2][T]
  int* cand_i;
  const float* thresh;  // [Q]
  int* count;           // [Q]
  float* buf_s;         // [Q][cap]
  int* buf_i;
};

template <int MODE, int T>
__global__ __launch_bounds__(256, 2) void topk_fast_scan_k(FastArgs a) {
  __shared__ __attribute__((aligned(16))) float sI[2][kTile][kLdsStride];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int b = blockIdx.x;
  const int nsub = a.nsplit >> 3;
  const int split = (b & 7) + 8 * ((b >> 3) % nsub);
  const int rb = (b >> 3) / nsub;
  const int64_t q = (int64_t)rb * kOwnRows + wave * 32 + c;
  const bool q_ok = q < a.Q;
  float u[64];
  if (q_ok) {
    const float4* src = reinterpret_cast<const float4*>(a.U + q * a.ldu + h * 64);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float4 v = src[t];
      u[4 * t] = v.x; u[4 * t + 1] = v.y; u[4 * t + 2] = v.z; u[4 * t + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < 64; ++t) u[t] = 0.0f;
  }
  const int64_t j_begin = (int64_t)split * a.span;
  int64_t j_end = j_begin + a.span;
  if (j_end > a.NI) j_end = a.NI;

  float ts[T];
  int ti[T];
#pragma unroll
  for (int t = 0; t < T; ++t) { ts[t] = -INFINITY; ti[t] = 0x7fffffff; }
  const float th = (MODE == 1 && q_ok) ? a.thresh[q] : INFINITY;

  const int srow = tid >> 3, scol = (tid & 7) * 16;
  float4 stg[4];
  auto gload = [&](int64_t j0) {
    const int64_t j = j0 + srow;
    if (j < j_end) {
      const float4* src = reinterpret_cast<const float4*>(a.I + j * a.ldi + scol);
#pragma unroll
      for (int t = 0; t < 4; ++t) stg[t] = src[t];
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) stg[t] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int t = 0; t < 4; ++t) *reinterpret_cast<float4*>(&sI[buf][srow][scol + 4 * t]) = stg[t];
  };
  if (j_begin < j_end) {
    gload(j_begin);
    lstore(0);
    __syncthreads();
    int cur = 0;
    for (int64_t j0 = j_begin; j0 < j_end; j0 += kTile) {
      const bool has_next = j0 + kTile < j_end;
      if (has_next) gload(j0 + kTile);
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
      const float* xrow = &sI[cur][c][h * 64];
#pragma unroll
      for (int s4 = 0; s4 < 64; s4 += 4) {
        const float4 bv = *reinterpret_cast<const float4*>(xrow + s4);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.x, u[s4 + 0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.y, u[s4 + 1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.z, u[s4 + 2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.w, u[s4 + 3], acc, 0, 0, 0);
      }
      if (q_ok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t j = j0 + tile_row(r, h);
          const float sc = acc[r];
          if (j >= j_end) continue;
          if (MODE == 0) {
            if (better(sc, (int)j, ts[T - 1], ti[T - 1])) {  // rare after the first T items
              ts[T - 1] = sc;
              ti[T - 1] = (int)j;
#pragma unroll
              for (int t = T - 1; t > 0; --t) {
                if (better(ts[t], ti[t], ts[t - 1], ti[t - 1])) {
                  const float fs = ts[t]; ts[t] = ts[t - 1]; ts[t - 1] = fs;
                  const int fi = ti[t]; ti[t] = ti[t - 1]; ti[t - 1] = fi;
                }
              }
            }
          } else if (sc >= th) {
            const int pos = atomicAdd(a.count + q, 1);
            if (pos < a.cap) {
              a.buf_s[q * a.cap + pos] = sc;
              a.buf_i[q * a.cap + pos] = (int)j;
            }
          }
        }
      }
      if (has_next) lstore(cur ^ 1);  // cur^1 was read in the previous tile, fenced by its barrier
      __syncthreads();
      cur ^= 1;
    }
  }
  if (MODE == 0 && q_ok) {
    const int64_t base = ((q * a.nsplit + split) * 2 + h) * T;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      a.cand_s[base + t] = ts[t];
      a.cand_i[base + t] = ti[t];
    }
  }
}

// bitonic sort of NC (score, idx) pairs in LDS by (score desc, idx asc)
template <int NC>
__device__ __forceinline__ void bitonic_desc(float* ss, int* si) {
  for (int size = 2; size <= NC; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < NC / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const float a0 = ss[lo], a1 = ss[hi];
        const int b0 = si[lo], b1 = si[hi];
        const bool swap = desc ? better(a1, b1, a0, b0) : better(a0, b0, a1, b1);
        if (swap) {
          ss[lo] = a1; ss[hi] = a0;
          si[lo] = b1; si[hi] = b0;
        }
      }
      __syncthreads();
    }
  }
}

// K2: t_q = k-th best candidate (or -inf if fewer valid candidates than k); count[q] = 0
template <int NC>
__global__ __launch_bounds__(256) void topk_thresh_k(const float* cs, const int* ci, int ncand, int K, float* thresh,
                                                     int* count) {
  __shared__ float ss[NC];
  __shared__ int si[NC];
  const int64_t q = blockIdx.x;
  for (int t = threadIdx.x; t < NC; t += blockDim.x) {
    const bool ok = t < ncand;
    ss[t] = ok ? cs[q * ncand + t] : -INFINITY;
    si[t] = ok ? ci[q * ncand + t] : 0x7fffffff;
  }
  __syncthreads();
  bitonic_desc<NC>(ss, si);
  if (threadIdx.x == 0) {
    const bool valid = si[K - 1] != 0x7fffffff;
    thresh[q] = valid ? ss[K - 1] : -INFINITY;
    count[q] = 0;
  }
}

// K4: sort the collected entries and write the top k; overflow -> flag for the fallback
template <int NC>
__global__ __launch_bounds__(256) void topk_final_k(const float* bs, const int* bi, const int* count, int cap, int K,
                                                    float* out_s, int64_t* out_i, int* overflow) {
  __shared__ float ss[NC];
  __shared__ int si[NC];
  const int64_t q = blockIdx.x;
  const int n = count[q];
  if (n > cap) {
    if (threadIdx.x == 0) atomicOr(overflow, 1);
    return;
  }
  for (int t = threadIdx.x; t < NC; t += blockDim.x) {
    const bool ok = t < n;
    ss[t] = ok ? bs[q * cap + t] : -INFINITY;
    si[t] = ok ? bi[q * cap + t] : 0x7fffffff;
  }
  __syncthreads();
  bitonic_desc<NC>(ss, si);
  for (int t = threadIdx.x; t < K; t += blockDim.x) {
    out_s[q * K + t] = ss[t];
    out_i[q * K + t] = (si[t] == 0x7fffffff) ? -1 : (int64_t)si[t];
  }
}


// ---- bf16 path (large corpora): one full scan at bf16 MFMA rate, exact fp32 rescoring ----------
// P0 (topk_bf16_prep_k): the corpus as a bf16 image (RNE) and max_j ||w_j||.
// Rounding bound (query_delta): |a - e| <= delta_q between the bf16 score a (bf16 RNE operands,
//     fp32 accumulation) and the fp32 score e of the rescoring: with u = u' + du, w = w' + dw (u',
//     w' the bf16 operands), u.w - u'.w' = u'.dw + du.w' + du.dw, so by Cauchy-Schwarz
//     delta_q = ||u|| D + ||du|| W + 3 ||du|| D + 2^-12 ||u|| W, D = max_j ||dw_j||, W = max_j ||w_j||
//     (the last term covers both fp32 accumulations, each < 2^-16 relative). Round 4 used the
//     elementwise worst case (2^-7 + 2^-12) ||u|| W; the residual norms are ~0.58 of it on spread
//     data, so the band of scores above t_q (the appends of P3) and the margin set of P4 narrow.
// P1 (topk_bf16_scan_k<MODE 0>): a strided sample of the corpus (every S-th 32-item tile of each
//     split, S ~ 8 nsplit / k so that ~4 collected entries per stream are expected in P3) over
//     ns0 <= nsplit splits (sample_nsplit); each lane keeps its best T0 sample scores in registers
//     (T0 = 1 where 2 ns0 >= 2k: a compare and two selects per score, no sorted insert).
// P2 (topk_bf16_thresh_k): per query, c_k = k-th best of the sampled candidates. The k sampled
//     items with a >= c_k have e >= c_k - delta, so the true k-th best exact score e_k >= c_k -
//     delta, and every true top-k item has a >= e_k - delta >= c_k - 2 delta =: t_q.
// P3 (topk_bf16_scan_k<MODE 1>): the one full scan; every (a, j) with a >= t_q is appended to
//     its lane's stream buffer (cap kStreamCap; ~0.25 % of the items on spread data).
// P4 (topk_bf16_select_k): per query, gather the appended entries, sort by a; a_k = k-th; every
//     entry with a >= a_k - 2 delta (the only ones that can reach the exact k-th) is rescored in
//     fp32 and sorted by (e desc, index asc); the first k are written. A stream buffer overflow or
//     more than kSelMax entries sends the query to the exact list-based kernels above (a device
//     list of query ids; their grid exits past its count: no host sync).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kImgStride = 272;   // bytes per staged item row: 256 + 16 (conflict-free ds_read_b128)
constexpr int kStreamCap = 32;    // P3 entries per lane stream
constexpr int kSelMax = 8192;     // P4 entries per query (LDS sort)

// 16 threads per row, 8 floats each; 4 rows per wave per step. hdr[0] = max_j ||w_j||, hdr[1] =
// max_j ||w_j - bf16(w_j)|| (float bits; both inflated against their own fp32 rounding)
__global__ __launch_bounds__(256) void topk_bf16_prep_k(const float* __restrict__ I, int64_t ldi, int64_t NI,
                                                        __bf16* __restrict__ img, unsigned* hdr) {
  const int lane = threadIdx.x & 63, sub = lane >> 4, c = lane & 15;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  float mx = 0.0f, md = 0.0f;
  for (int64_t j0 = wave_g * 8; j0 < NI; j0 += nw * 8) {
    float4 v[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t j = j0 + 4 * u + sub;
      if (j < NI) {
        const float4* src = reinterpret_cast<const float4*>(I + j * ldi) + 2 * c;
        v[u][0] = src[0];
        v[u][1] = src[1];
      } else {
        v[u][0] = make_float4(0.f, 0.f, 0.f, 0.f);
        v[u][1] = v[u][0];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t j = j0 + 4 * u + sub;
      const float4 a = v[u][0], b = v[u][1];
      const float ss = rsx::wave_sum_width(a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w +
                                           b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w, 16);
      mx = fmaxf(mx, sqrtf(ss));
      bf16x8 h;
      h[0] = (__bf16)a.x; h[1] = (__bf16)a.y; h[2] = (__bf16)a.z; h[3] = (__bf16)a.w;
      h[4] = (__bf16)b.x; h[5] = (__bf16)b.y; h[6] = (__bf16)b.z; h[7] = (__bf16)b.w;
      const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      float dd = 0.0f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float r = f[e] - (float)h[e];  // exact (Sterbenz)
        dd = fmaf(r, r, dd);
      }
      md = fmaxf(md, sqrtf(rsx::wave_sum_width(dd, 16)));
      if (j < NI) *reinterpret_cast<bf16x8*>(img + j * kD + 8 * c) = h;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    md = fmaxf(md, __shfl_xor(md, o, 64));
  }
  // non-negative floats order like their bit patterns
  if (lane == 0 && mx > 0.0f) atomicMax(hdr, __float_as_uint(mx * 1.0000001f));
  if (lane == 0 && md > 0.0f) atomicMax(hdr + 1, __float_as_uint(md * 1.0001f));
}

struct BfArgs {
  const __bf16* img;   // [NI][128]
  const float* U;      // [Q, ldu]
  int64_t Q, NI, ldu;
  int nsplit, nqb, sample;
  int64_t span;
  float* cand_s;       // MODE 0: [Q][nsplit][2][T], each stream's list sorted desc
  int* cand_i;
  const float* thr;    // MODE 1: [Q] collection threshold t_q
  // MODE 1: [Q][nsplit][2][kStreamCap] entries (score, item id as float bits): one 8-B store per
  // append (two separate 4-B arrays made two write requests of a partial line each)
  float2* buf_e;
  int* buf_n;          // MODE 1: [Q][nsplit][2] appended count (may exceed the cap: overflow)
};

template <int G, int T, int MODE>
__global__ __launch_bounds__(256, 2) void topk_bf16_scan_k(BfArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char sI[2][kTile * kImgStride];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  // XCD-aware order: the nqb query blocks of one split sit 8 block ids apart, i.e. on one XCD
  const int b = blockIdx.x, x = b & 7, y = b >> 3;
  const int qb = y % a.nqb;
  const int split = (y / a.nqb) * 8 + x;
  const int64_t q0 = (int64_t)qb * (128 * G) + wave * (32 * G) + c;
  bf16x8 ub[G][8];
  bool q_ok[G];
  float thr[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t q = q0 + 32 * g;
    q_ok[g] = q < a.Q;
    thr[g] = (MODE == 1 && q_ok[g]) ? a.thr[q] : INFINITY;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
      if (q_ok[g]) {
        const float4* src = reinterpret_cast<const float4*>(a.U + q * a.ldu + 16 * ks + 8 * h);
        v0 = src[0];
        v1 = src[1];
      }
      ub[g][ks][0] = (__bf16)v0.x; ub[g][ks][1] = (__bf16)v0.y; ub[g][ks][2] = (__bf16)v0.z; ub[g][ks][3] = (__bf16)v0.w;
      ub[g][ks][4] = (__bf16)v1.x; ub[g][ks][5] = (__bf16)v1.y; ub[g][ks][6] = (__bf16)v1.z; ub[g][ks][7] = (__bf16)v1.w;
    }
  }
  const int64_t j_begin = (int64_t)split * a.span;
  int64_t j_end = j_begin + a.span;
  if (j_end > a.NI) j_end = a.NI;
  const int64_t step = MODE == 0 ? (int64_t)kTile * a.sample : kTile;

  float ts[G][T];
  int ti[G][T];
  int cnt[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    cnt[g] = 0;
#pragma unroll
    for (int t = 0; t < T; ++t) { ts[g][t] = -INFINITY; ti[g][t] = 0x7fffffff; }
  }
  int64_t sbase[G];
#pragma unroll
  for (int g = 0; g < G; ++g) sbase[g] = ((q0 + 32 * g) * a.nsplit + split) * 2 + h;
  float2* bep[G];
#pragma unroll
  for (int g = 0; g < G; ++g)  // MODE 1 stream buffers of this lane's queries
    bep[g] = MODE == 1 ? a.buf_e + sbase[g] * kStreamCap : nullptr;

  // staging: 8 threads per item row, each moving 16-B piece (tid & 7) of both 128-B halves (the
  // 8 threads of a row write 128 contiguous bytes per store: no bank conflicts, as in
  // topk_bf16_collect_k; the previous 32 B per thread was 2-way)
  const int srow = tid >> 3, sb = (tid & 7) * 16;
  u32x4 stg[2];
  auto gload = [&](int64_t j0) {
    const int64_t j = j0 + srow;
    if (j < j_end) {
      const unsigned char* src = reinterpret_cast<const unsigned char*>(a.img + j * kD);
      stg[0] = *reinterpret_cast<const u32x4*>(src + sb);
      stg[1] = *reinterpret_cast<const u32x4*>(src + 128 + sb);
    } else {
      stg[0] = u32x4{0u, 0u, 0u, 0u};
      stg[1] = stg[0];
    }
  };
  auto lstore = [&](int buf) {
    unsigned char* dst = &sI[buf][srow * kImgStride];
    *reinterpret_cast<u32x4*>(dst + sb) = stg[0];
    *reinterpret_cast<u32x4*>(dst + 128 + sb) = stg[1];
  };
  if (j_begin < j_end) {
    gload(j_begin);
    lstore(0);
    __syncthreads();
    int cur = 0;
    for (int64_t j0 = j_begin; j0 < j_end; j0 += step) {
      const bool has_next = j0 + step < j_end;
      if (has_next) gload(j0 + step);
      f32x16 acc[G];
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[g][r] = 0.0f;
      const unsigned char* xrow = &sI[cur][c * kImgStride + 16 * h];
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(xrow + 32 * ks);
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, ub[g][ks], acc[g], 0, 0, 0);
      }
      // item ids in 32 bits (NI < 2^31, host-checked) and the split-end check only on the split's
      // last tile. MODE 0 first compares a lane's tile max (v_max3) with its list minimum: the
      // sorted insert is then skipped by most lanes once the lists have filled. (In MODE 1 about
      // 0.25 % of the scores pass t_q, but some lane of a wave passes on ~90 % of the tiles, so a
      // per-lane gate would not skip work there.)
      const int jt0 = (int)j0;
      const bool full_tile = j0 + kTile <= j_end;
      const int jend = (int)j_end;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (!q_ok[g]) continue;
        if (MODE == 0) {
          float mx = fmaxf(acc[g][0], acc[g][1]);
#pragma unroll
          for (int r = 2; r < 16; r += 2) mx = fmaxf(mx, fmaxf(acc[g][r], acc[g][r + 1]));
          if (!(mx > ts[g][T - 1])) continue;  // no score of this lane enters its list
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = jt0 + tile_row(r, h);
          const float sc = acc[g][r];
          if (MODE == 0) {
            if (sc > ts[g][T - 1] && (full_tile || j < jend)) {
              ts[g][T - 1] = sc;
              ti[g][T - 1] = j;
#pragma unroll
              for (int t = T - 1; t > 0; --t) {
                if (ts[g][t] > ts[g][t - 1]) {
                  const float fs = ts[g][t]; ts[g][t] = ts[g][t - 1]; ts[g][t - 1] = fs;
                  const int fi = ti[g][t]; ti[g][t] = ti[g][t - 1]; ti[g][t - 1] = fi;
                }
              }
            }
          } else if (sc >= thr[g] && (full_tile || j < jend)) {
            if (cnt[g] < kStreamCap) bep[g][cnt[g]] = make_float2(sc, __int_as_float(j));
            ++cnt[g];
          }
        }
      }
      if (has_next) lstore(cur ^ 1);  // cur^1 was read in the previous tile, fenced by its barrier
      __syncthreads();
      cur ^= 1;
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (!q_ok[g]) continue;
    if (MODE == 0) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        a.cand_s[sbase[g] * T + t] = ts[g][t];
        a.cand_i[sbase[g] * T + t] = ti[g][t];
      }
    } else {
      a.buf_n[sbase[g]] = cnt[g];
    }
  }
}

// P3 as its own kernel (round 4): the one full scan, with every (a, j), a >= t_q, appended to its
// lane's stream buffer. Against round 3's topk_bf16_scan_k<G, 8, 1> (a compare-and-append branch
// per score: ~3 VALU + 5 SALU for each of a lane's 32 scores per tile):
//   * a max gate: each lane takes the max of its 16 scores of a query group (v_max3) and only
//     lanes whose max reaches t_q go on (one divergent branch per query group and tile);
//   * behind the gate, one compare per score on tiles wholly inside the split (the split-end
//     check only on its last tile) and the append as one 8-B (score, id) store -- t_q lets ~0.25 %
//     of the scores through, so some lane of a wave passes on ~90 % of the (tile, group) pairs and
//     the appends, not the MFMAs, set the kernel's time (the same kernel with the gate but no
//     appends runs 0.83 ms, the MFMA floor is ~0.5 ms). EXTRACT (RSX_TOPK_COLLECT=1) appends
//     max-first instead (the lane's max, knocked out, repeated while the new max passes);
//   * a clamped slot instead of a capacity branch: a stream that overflows keeps counting and its
//     query goes to the exact kernels (P4), so what lands in its last slot is never read;
//   * staging stores without bank conflicts: the 8 threads of an item row write its two 128-B
//     halves as 8 contiguous 16-B pieces each.
// 4096 x 1M, k = 100 (rocprof): with 4-B score and id stores, 1.70 ms per-score, 1.56 ms max-first;
// with 8-B entries 1.49 max-first, 1.47 per-score with the whole-tile compare (the default);
// round 3's form 1.66-1.76. Measured and not kept (profiles/r04_retrieval_collect_ab.json): a
// two-level gate (groups of four scores, 1.54 ms),
// a loader wave filling a 4-slot LDS ring by LDS-DMA (3.24 ms: 2 compute waves per SIMD instead of
// 3), a per-wave LDS event queue drained one event per lane (1.60 / 1.91 ms), the appends placed
// after the next tile's staging store (1.67 ms), a second accumulator set pipelining the compares
// under the next tile's MFMAs (2.49 ms). The entries of a stream are the same set in every form;
// their order within the stream differs with EXTRACT, which P4 never sees (its margin set and
// final sort use the total order (score desc, index asc)).
template <int G, bool EXTRACT, bool BALLOT = false>
__global__ __launch_bounds__(256, 2) void topk_bf16_collect_k(BfArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char sI[2][kTile * kImgStride];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int b = blockIdx.x, x = b & 7, y = b >> 3;
  const int qb = y % a.nqb;
  const int split = (y / a.nqb) * 8 + x;
  const int64_t q0 = (int64_t)qb * (128 * G) + wave * (32 * G) + c;
  bf16x8 ub[G][8];
  float thr[G];
  int cnt[G];
  float2* bep[G];
  int64_t sbase[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t q = q0 + 32 * g;
    const bool ok = q < a.Q;
    thr[g] = ok ? a.thr[q] : INFINITY;  // no finite score reaches +inf: rows past Q collect nothing
    cnt[g] = 0;
    sbase[g] = ((ok ? q : 0) * a.nsplit + split) * 2 + h;
    bep[g] = a.buf_e + sbase[g] * kStreamCap;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
      if (ok) {
        const float4* src = reinterpret_cast<const float4*>(a.U + q * a.ldu + 16 * ks + 8 * h);
        v0 = src[0];
        v1 = src[1];
      }
      ub[g][ks][0] = (__bf16)v0.x; ub[g][ks][1] = (__bf16)v0.y; ub[g][ks][2] = (__bf16)v0.z; ub[g][ks][3] = (__bf16)v0.w;
      ub[g][ks][4] = (__bf16)v1.x; ub[g][ks][5] = (__bf16)v1.y; ub[g][ks][6] = (__bf16)v1.z; ub[g][ks][7] = (__bf16)v1.w;
    }
  }
  const int64_t j_begin = (int64_t)split * a.span;
  int64_t j_end = j_begin + a.span;
  if (j_end > a.NI) j_end = a.NI;
  const int jend = (int)j_end;

  const int srow = tid >> 3, sb = (tid & 7) * 16;
  u32x4 stg[2];
  auto gload = [&](int64_t j0) {
    const int64_t j = j0 + srow;
    if (j < j_end) {
      const unsigned char* src = reinterpret_cast<const unsigned char*>(a.img + j * kD);
      stg[0] = *reinterpret_cast<const u32x4*>(src + sb);
      stg[1] = *reinterpret_cast<const u32x4*>(src + 128 + sb);
    } else {
      stg[0] = u32x4{0u, 0u, 0u, 0u};
      stg[1] = stg[0];
    }
  };
  auto lstore = [&](int buf) {
    unsigned char* dst = &sI[buf][srow * kImgStride];
    *reinterpret_cast<u32x4*>(dst + sb) = stg[0];
    *reinterpret_cast<u32x4*>(dst + 128 + sb) = stg[1];
  };
  auto append = [&](int g, float sc, int j) {
    const int slot = cnt[g] < kStreamCap ? cnt[g] : kStreamCap - 1;
    bep[g][slot] = make_float2(sc, __int_as_float(j));
    ++cnt[g];
  };
  auto collect = [&](const f32x16 (&acc)[G], int jt0) {
    const bool full = jt0 + kTile <= jend;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float m0 = fmaxf(fmaxf(acc[g][0], acc[g][1]), acc[g][2]);
      float m1 = fmaxf(fmaxf(acc[g][3], acc[g][4]), acc[g][5]);
      float m2 = fmaxf(fmaxf(acc[g][6], acc[g][7]), acc[g][8]);
      float m3 = fmaxf(fmaxf(acc[g][9], acc[g][10]), acc[g][11]);
      float m4 = fmaxf(fmaxf(acc[g][12], acc[g][13]), acc[g][14]);
      const float mx = fmaxf(fmaxf(fmaxf(m0, m1), fmaxf(m2, m3)), fmaxf(m4, acc[g][15]));
      // wave-uniform gate: skip the group unless some lane's max reaches its threshold
      if (BALLOT && !__builtin_amdgcn_ballot_w64(mx >= thr[g])) continue;
      if (!(mx >= thr[g])) continue;  // most lanes: no collected item of this query in the tile
      if (EXTRACT) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[g][r];
        float m = mx;
        // at most 16 rounds (t_q = -inf lets every score through)
        for (int it = 0; it < 16 && m >= thr[g]; ++it) {
          int rs = 15;
#pragma unroll
          for (int r = 14; r >= 0; --r) rs = v[r] == m ? r : rs;  // lowest position holding the max
          const int j = jt0 + tile_row(rs, h);
          if (full || j < jend) append(g, m, j);
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = r == rs ? -INFINITY : v[r];
          const float n0 = fmaxf(fmaxf(v[0], v[1]), v[2]);
          const float n1 = fmaxf(fmaxf(v[3], v[4]), v[5]);
          const float n2 = fmaxf(fmaxf(v[6], v[7]), v[8]);
          const float n3 = fmaxf(fmaxf(v[9], v[10]), v[11]);
          const float n4 = fmaxf(fmaxf(v[12], v[13]), v[14]);
          m = fmaxf(fmaxf(fmaxf(n0, n1), fmaxf(n2, n3)), fmaxf(n4, v[15]));
        }
      } else if (full) {  // whole tile inside the split: one compare per score
        // BALLOT (A/B, RSX_TOPK_COLLECT=3): each append behind a wave-uniform branch on the ballot of
        // its compare. The compiler already skips empty append bodies (s_cbranch_execnz to
        // out-of-line blocks); the ballots only add SALU (4096 x 1M: 1.69 vs 1.50 ms)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool pass = acc[g][r] >= thr[g];
          if (!BALLOT || __builtin_amdgcn_ballot_w64(pass)) {
            if (pass) append(g, acc[g][r], jt0 + tile_row(r, h));
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = jt0 + tile_row(r, h);
          const bool pass = acc[g][r] >= thr[g] && (full || j < jend);
          if (!BALLOT || __builtin_amdgcn_ballot_w64(pass)) {
            if (pass) append(g, acc[g][r], j);
          }
        }
      }
    }
  };
  if (j_begin < j_end) {
    gload(j_begin);
    lstore(0);
    __syncthreads();
    int cur = 0;
    for (int64_t j0 = j_begin; j0 < j_end; j0 += kTile) {
      const bool has_next = j0 + kTile < j_end;
      if (has_next) gload(j0 + kTile);
      f32x16 acc[G];
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[g][r] = 0.0f;
      const unsigned char* xrow = &sI[cur][c * kImgStride + 16 * h];
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(xrow + 32 * ks);
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, ub[g][ks], acc[g], 0, 0, 0);
      }
      collect(acc, (int)j0);
      if (has_next) lstore(cur ^ 1);  // cur^1 was read in the previous tile, fenced by its barrier
      __syncthreads();
      cur ^= 1;
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g)
    if (q0 + 32 * g < a.Q) a.buf_n[sbase[g]] = cnt[g];
}

// bitonic sort of the first P (power of two) entries, (score desc, idx asc)
__device__ __forceinline__ void bitonic_desc_n(float* ss, int* si, int P) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < P / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const float a0 = ss[lo], a1 = ss[hi];
        const int b0 = si[lo], b1 = si[hi];
        const bool swap = desc ? better(a1, b1, a0, b0) : better(a0, b0, a1, b1);
        if (swap) {
          ss[lo] = a1; ss[hi] = a0;
          si[lo] = b1; si[hi] = b0;
        }
      }
      __syncthreads();
    }
  }
}

// delta_q (see the bf16 path's header): ||u|| and ||u - bf16(u)|| by fixed-order wave reductions
// (every wave computes them), hdr = the corpus header of topk_bf16_prep_k
__device__ __forceinline__ float query_delta(const float* U, int64_t ldu, int64_t q, const unsigned* hdr) {
  const float2 uv = reinterpret_cast<const float2*>(U + q * ldu)[threadIdx.x & 63];
  const float dx = uv.x - (float)(__bf16)uv.x, dy = uv.y - (float)(__bf16)uv.y;
  const float nu = sqrtf(rsx::wave_sum_width(uv.x * uv.x + uv.y * uv.y, 64)) * 1.0000001f;
  const float nd = sqrtf(rsx::wave_sum_width(dx * dx + dy * dy, 64)) * 1.0001f;
  const float W = __uint_as_float(hdr[0]), D = __uint_as_float(hdr[1]);
  return (nu * D + nd * W + 3.0f * nd * D + 0.000244140625f * nu * W) * 1.00001f + 1e-30f;
}

// Order-preserving uint key of a float (larger float <=> larger key).
__device__ __forceinline__ unsigned okey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float from_okey(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// K-th largest (1 <= K <= n) of v[0, n) in LDS, by an 8-bit radix select over okey (integer LDS
// histograms; wave 0 finds each pass's digit with a 64-lane scan over 4 bins per lane). Replaces a
// full bitonic sort where only the K-th value is needed. The passes start at the highest bit in
// which the keys differ (block min / max first): scores of one query share their sign and top
// exponent bits, and a pass over a constant digit put every key's LDS atomic on one address (the
// round-3 form's first pass). Every thread returns the value. red: >= 8 ints of LDS scratch.
__device__ float block_kth_largest(const float* v, int n, int K, int* hist, int* sel, unsigned* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned kmin = 0xffffffffu, kmax = 0u;
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const unsigned k = okey(v[t]);
    kmin = min(kmin, k);
    kmax = max(kmax, k);
  }
  for (int o = 32; o > 0; o >>= 1) {
    kmin = min(kmin, (unsigned)__shfl_xor((int)kmin, o, 64));
    kmax = max(kmax, (unsigned)__shfl_xor((int)kmax, o, 64));
  }
  if (lane == 0) {
    red[wave] = kmin;
    red[4 + wave] = kmax;
  }
  __syncthreads();
  kmin = red[0];
  kmax = red[4];
  for (int w = 1; w < nw; ++w) {
    kmin = min(kmin, red[w]);
    kmax = max(kmax, red[4 + w]);
  }
  const unsigned diff = kmin ^ kmax;
  if (diff == 0u) return from_okey(kmin);  // block-uniform: every key equal
  const int hb = 31 - __clz((int)diff);
  unsigned mask = ~((2u << hb) - 1u);       // hb = 31: 2u << 31 wraps to 0, mask 0
  unsigned prefix = kmin & mask;
  int krem = K;
  for (int top = hb; top >= 0; top -= 8) {
    const int lo = top >= 7 ? top - 7 : 0;
    const unsigned dm = (2u << (top - lo)) - 1u;  // digit mask, top - lo + 1 bits
    for (int t = threadIdx.x; t < 256; t += blockDim.x) hist[t] = 0;
    __syncthreads();
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
      const unsigned k = okey(v[t]);
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> lo) & dm], 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // lane l owns digits 255-4l .. 252-4l (descending)
      const int l = threadIdx.x;
      int c[4], sum = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = hist[255 - 4 * l - j];
        sum += c[j];
      }
      int incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (l >= o) incl += y;
      }
      const int excl = incl - sum;
      if (excl < krem && krem <= incl) {
        int acc = excl;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (acc + c[j] >= krem) {
            sel[0] = 255 - 4 * l - j;
            sel[1] = krem - acc;
            break;
          }
          acc += c[j];
        }
      }
    }
    __syncthreads();
    prefix |= (unsigned)sel[0] << lo;
    mask |= dm << lo;
    krem = sel[1];
    __syncthreads();  // sel / hist are rewritten by the next pass
  }
  return from_okey(prefix);
}

// P2: t_q = c_r - 2 delta_q (c_r: r-th best sampled candidate, r <= k (thr_rank); -inf if fewer
// than r valid ones). r = k guarantees >= k collected items at or above c_k; r < k admits fewer
// items and P4 checks, per query, that its k-th best collected score still clears c_r (else the
// query goes to the exact kernels).
template <int NC>
__global__ __launch_bounds__(256) void topk_bf16_thresh_k(const float* __restrict__ cs, const int* __restrict__ ci,
                                                          int ncand, const float* __restrict__ U, int64_t ldu, int K,
                                                          const unsigned* wmax_bits, float* thr) {
  __shared__ float ss[NC];
  __shared__ int hist[256], sel[2], nval_s;
  __shared__ unsigned red[8];
  const int64_t q = blockIdx.x;
  if (threadIdx.x == 0) nval_s = 0;
  __syncthreads();
  int nv = 0;
  for (int t = threadIdx.x; t < ncand; t += 256) {
    const bool ok = ci[q * ncand + t] != 0x7fffffff;
    ss[t] = ok ? cs[q * ncand + t] : -INFINITY;
    nv += ok ? 1 : 0;
  }
  nv = rsx::wave_sum_width(nv, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(&nval_s, nv);
  const float delta = query_delta(U, ldu, q, wmax_bits);
  __syncthreads();
  if (nval_s < K) {  // block-uniform
    if (threadIdx.x == 0) thr[q] = -INFINITY;
    return;
  }
  const float ck = block_kth_largest(ss, ncand, K, hist, sel, red);
  if (threadIdx.x == 0) thr[q] = ck - 2.0f * delta;
}

// P4: gather the query's appended entries; a_k = their k-th best (radix select); compact the
// margin set {a >= a_k - 2 delta}, rescore it exactly in fp32, sort it by (e desc, idx asc) and
// write the first k. (The margin set's order before the final sort does not matter: (e, idx)
// pairs are distinct, so the output is deterministic.)
constexpr int kMarginMax = 2048;
__global__ __launch_bounds__(256) void topk_bf16_select_k(const float2* __restrict__ be,
                                                          const int* __restrict__ bn, int nstreams,
                                                          const float* __restrict__ U, int64_t ldu,
                                                          const float* __restrict__ I, int64_t ldi, int K,
                                                          const unsigned* wmax_bits, const float* __restrict__ thr_q,
                                                          int check, float* out_s, int64_t* out_i, int* qcount,
                                                          int* qmap, int* qtotal) {
  // LDS: the appended scores only (their item ids are read back from global for the margin set),
  // so three workgroups fit per CU
  __shared__ __attribute__((aligned(16))) float ss[kSelMax];
  __shared__ __attribute__((aligned(16))) float ms[kMarginMax];
  __shared__ __attribute__((aligned(16))) int mi[kMarginMax];
  __shared__ int off[513];
  __shared__ int hist[256], sel[2];
  __shared__ unsigned red[8];
  __shared__ int bad_s, nsel_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t q = blockIdx.x;
  const float delta = query_delta(U, ldu, q, wmax_bits);
  if (tid == 0) { bad_s = 0; nsel_s = 0; }
  __syncthreads();
  // counts (nstreams <= 512) -> exclusive prefix in LDS: wave 0, eight streams per lane
  if (wave == 0) {
    int c8[8], sum = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = 8 * lane + u;
      const int n = t < nstreams ? bn[q * nstreams + t] : 0;
      if (n > kStreamCap) bad_s = 1;
      c8[u] = n < kStreamCap ? n : kStreamCap;
      sum += c8[u];
    }
    int incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    int run = incl - sum;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      off[8 * lane + u] = run;
      run += c8[u];
    }
    if (lane == 63) off[512] = incl;
  }
  __syncthreads();
  const int total = off[512];
  if (bad_s || total > kSelMax) {
    if (tid == 0) {
      qmap[atomicAdd(qcount, 1)] = (int)q;
      atomicAdd(qtotal, 1);
    }
    return;
  }
  // 32 threads per stream, 8 streams per pass; 32 passes' loads are issued before their LDS
  // stores (one memory latency per 256 streams instead of per 8)
  for (int s0 = 0; s0 < nstreams; s0 += 256) {
    float v[32];
    int dst[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int st = s0 + 8 * u + (tid >> 5), e = tid & 31;
      dst[u] = -1;
      if (st < nstreams) {
        const int n = off[st + 1] - off[st];
        if (e < n) {
          dst[u] = off[st] + e;
          v[u] = be[(q * nstreams + st) * kStreamCap + e].x;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (dst[u] >= 0) ss[dst[u]] = v[u];
  }
  __syncthreads();
  const float ak = (total >= K) ? block_kth_largest(ss, total, K, hist, sel, red) : -INFINITY;
  // threshold rank r < k (check): the collected set holds every true top-k item iff its k-th best
  // bf16 score a_k satisfies a_k - 2 delta >= t_q (k items with a >= a_k have exact scores >= a_k -
  // delta, so every top-k item has a >= a_k - 2 delta); delta inflated by 1e-5 against the
  // subtraction's rounding. Otherwise (or with fewer than k collected) the exact kernels run it.
  if (check && thr_q[q] > -INFINITY && (total < K || ak - 2.0f * (delta * 1.00001f) < thr_q[q])) {
    if (tid == 0) {
      qmap[atomicAdd(qcount, 1)] = (int)q;
      atomicAdd(qtotal, 1);
    }
    return;
  }
  const float thr = (total >= K) ? ak - 2.0f * delta : -INFINITY;
  // margin set: one thread per stream walks that stream's entries (~5 on spread data) and notes
  // the buffer slot of each selected one; every selected item id is then loaded from global at
  // once (one memory latency). (Round 3 walked 8 streams per step with 32 threads each: 64
  // dependent LDS steps per query.)
  for (int st = tid; st < nstreams; st += 256) {
    const int o = off[st], cn = off[st + 1] - o;
    for (int e = 0; e < cn; ++e) {
      if (ss[o + e] >= thr) {
        const int slot = atomicAdd(&nsel_s, 1);
        if (slot < kMarginMax) mi[slot] = st * kStreamCap + e;
      }
    }
  }
  __syncthreads();
  const int n = nsel_s;
  if (n > kMarginMax) {  // block-uniform: the exact kernels take this query
    if (tid == 0) {
      qmap[atomicAdd(qcount, 1)] = (int)q;
      atomicAdd(qtotal, 1);
    }
    return;
  }
  {
    int ids[kMarginMax / 256];
#pragma unroll
    for (int u = 0; u < kMarginMax / 256; ++u) {
      const int t = tid + 256 * u;
      ids[u] = t < n ? __float_as_int(be[q * nstreams * kStreamCap + mi[t]].y) : 0;
    }
    __syncthreads();  // every slot read before any is overwritten
#pragma unroll
    for (int u = 0; u < kMarginMax / 256; ++u) {
      const int t = tid + 256 * u;
      if (t < n) mi[t] = ids[u];
    }
    __syncthreads();
  }
  // exact fp32 rescoring: 32 lanes per item, float4 per lane, fixed-order shuffle reduction
  const int sub = lane >> 5, c = lane & 31;
  const float4 u4 = reinterpret_cast<const float4*>(U + q * ldu)[c];
  for (int t0 = 0; t0 < n; t0 += 64) {  // eight items per half-wave in flight
    float4 w4[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 + 8 * u + wave * 2 + sub;
      w4[u] = t < n ? reinterpret_cast<const float4*>(I + (int64_t)mi[t] * ldi)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 + 8 * u + wave * 2 + sub;
      float e = u4.x * w4[u].x + u4.y * w4[u].y + u4.z * w4[u].z + u4.w * w4[u].w;
      for (int o = 16; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
      if (t < n && c == 0) ms[t] = e;
    }
  }
  // rank-sort keys (n <= 512): okey(e) << 32 | ~id, so "beats" is one unsigned 64-bit compare
  // (e desc, then id asc); padded to a multiple of two with 0 (beats nothing). ss is free now.
  unsigned long long* rk = reinterpret_cast<unsigned long long*>(ss);
  __syncthreads();  // every rescored ms[t] written
  if (n <= 512)
    for (int t = tid; t < ((n + 1) & ~1); t += 256)
      rk[t] = t < n ? ((unsigned long long)okey(ms[t]) << 32) | (unsigned)(~mi[t]) : 0ull;
  __syncthreads();
  if (n <= 512) {
    // rank sort: an entry's output position is the number of entries that beat it under (e desc,
    // index asc) -- distinct item ids make the ranks a permutation; all threads read entry j at
    // once (LDS broadcast), no barrier per step as in the bitonic network below
    for (int t = tid; t < K; t += 256) {
      if (t >= n) {
        out_s[q * K + t] = -INFINITY;
        out_i[q * K + t] = -1;
      }
    }
    const int n2 = (n + 1) >> 1;
    const ulonglong2* rk2 = reinterpret_cast<const ulonglong2*>(rk);
    for (int t = tid; t < n; t += 256) {
      const float e = ms[t];
      const int id = mi[t];
      const unsigned long long kt = rk[t];
      int r = 0;
#pragma unroll 4
      for (int j = 0; j < n2; ++j) {
        const ulonglong2 kj = rk2[j];
        r += (kj.x > kt) ? 1 : 0;
        r += (kj.y > kt) ? 1 : 0;
      }
      if (r < K) {
        out_s[q * K + r] = e;
        out_i[q * K + r] = (int64_t)id;
      }
    }
  } else {
    int P2 = 1;
    while (P2 < n) P2 <<= 1;
    for (int t = n + tid; t < P2; t += 256) {
      ms[t] = -INFINITY;
      mi[t] = 0x7fffffff;
    }
    __syncthreads();
    bitonic_desc_n(ms, mi, P2);
    for (int t = tid; t < K; t += 256) {
      const bool ok = t < n;
      out_s[q * K + t] = ok ? ms[t] : -INFINITY;
      out_i[q * K + t] = ok ? (int64_t)mi[t] : -1;
    }
  }
}

constexpr int kFastCap = 2048;

struct FastPlan {
  bool use;
  int T, nsplit;
};

FastPlan fast_plan(int64_t Q, int64_t NI, int64_t k) {
  FastPlan p;
  p.T = k <= 128 ? 8 : 16;
  p.use = NI > 16384 && k <= 512;
  // enough candidates for a tight threshold (2*ns*T >= 4k), enough workgroups, <= 8192 candidates
  const int64_t rbs = (Q + kOwnRows - 1) / kOwnRows;
  int ns = 8;
  while (ns < 256 && (2 * ns * p.T < 4 * k || rbs * ns < 1024) && NI / (ns * 2) >= 1024 && 2 * ns * 2 * p.T <= 8192)
    ns *= 2;
  p.nsplit = ns;
  if (2 * ns * p.T < k) p.use = false;  // too few candidates for a threshold
  return p;
}


struct BfPlan {
  bool use;
  int G, T, nsplit, nqb, sample;
};

BfPlan bf_plan(int64_t Q, int64_t NI, int64_t k) {
  BfPlan p;
  p.T = 8;
  p.G = Q >= 512 ? 2 : 1;
  p.nqb = (int)((Q + 128 * p.G - 1) / (128 * p.G));
  // at most 256 splits (<= 512 streams per query); >= 512 items per stream where possible
  int ns = 8;
  while (ns < 256 && NI / (2 * (int64_t)ns * 2) >= 512) ns *= 2;
  p.nsplit = ns;
  // sample one tile in S: about k S / (2 nsplit) <= 4 items per stream reach the P3 threshold
  int S = 1;
  while (S < 16 && k * (int64_t)S * 2 <= 8 * (int64_t)ns) S *= 2;
  p.sample = S;
  // the sample's candidates must hold k items: 2 nsplit T >= 2 k
  p.use = NI > 16384 && k <= 512 && 2 * ns * p.T >= 2 * k;
  static const bool off = getenv("RSX_TOPK_BF16") != nullptr && getenv("RSX_TOPK_BF16")[0] == '0';
  if (off) p.use = false;
  return p;
}

// splits of the P1 sample scan: nsplit / 4 (>= 8, a multiple of 8 like nsplit) unless
// RSX_TOPK_SAMPLE_DIV names another divisor (1 = the full split count, the round-3 form); at
// least k / T splits, so the 2 ns0 T candidates hold 2k (bf_plan's condition for nsplit)
int sample_nsplit(int nsplit, int64_t k, int T) {
  static const int div = [] {
    const char* e = getenv("RSX_TOPK_SAMPLE_DIV");
    const int v = e ? atoi(e) : 4;
    return (v == 1 || v == 2 || v == 4 || v == 8) ? v : 4;
  }();
  int ns0 = nsplit / div;
  if (ns0 < 8) ns0 = 8;
  while (ns0 < nsplit && 2 * (int64_t)ns0 * T < 2 * k) ns0 *= 2;
  if (ns0 > nsplit) ns0 = nsplit;
  return ns0;
}

// Rank r of the sampled candidate that sets t_q. The candidates are stream maxima of 1/S of the
// corpus, so about S r corpus items score above c_r and the collect pass appends a multiple of
// that: at 4096 x 1M, k = 100 (S = 8), r = k admits ~0.25 % of the scores and the appends set the
// collect kernel's time. r < k is exact only while the k-th best collected score clears c_r (P4
// checks it per query; a query that fails runs on the exact kernels, whose latency is that of a
// whole batch). r = clamp(ceil(3 k / S), 32, k) keeps S r >= 3k with r >= 32 candidates behind the
// estimate (tools/retrieval_micro.py, 4096 spread queries: no fallback down to r = 25 at k = 100,
// 2 at r = 17; k = 10 at r = 3: 88); RSX_TOPK_RANK_DIV=d forces r = ceil(k / d) (A/B).
int thr_rank(int k, int S) {
  static const int div = [] {
    const char* e = getenv("RSX_TOPK_RANK_DIV");
    const int v = e ? atoi(e) : 0;
    return v >= 1 && v <= 16 ? v : 0;
  }();
  int r = div ? (k + div - 1) / div : (3 * k + S - 1) / S;
  if (!div && r < 32) r = 32;
  if (r > k) r = k;
  return r < 1 ? 1 : r;
}

// RSX_TOPK_SAMPLE_T1=0: the sample scan keeps T best per lane stream (A/B)
bool sample_t1() {
  static const bool on = [] {
    const char* e = getenv("RSX_TOPK_SAMPLE_T1");
    return !(e && e[0] == '0');
  }();
  return on;
}

int choose_nsplit(int64_t Q, int64_t NI, int kmax) {
  // >= ~1024 workgroups when there are enough items; each split keeps >= 2048 items; the
  // merge sorts at most 8192 candidates per query in LDS (2 * nsplit * kmax <= 8192)
  const int64_t rbs = (Q + kOwnRows - 1) / kOwnRows;
  const int ns_max = 8192 / (2 * kmax);
  int ns = 8;
  while (ns < ns_max && rbs * ns < 1024 && NI / (ns * 2) >= 2048) ns *= 2;
  return ns;
}

}  // namespace

namespace {
int64_t old_ws_bytes(int64_t Q, int64_t NI, int64_t k) {
  const int kmax = k <= 128 ? 128 : 512;
  const int ns = choose_nsplit(Q, NI, kmax);
  return Q * ns * 2 * (int64_t)kmax * 8;
}
int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }
struct FastLayout {
  int64_t thresh, count, cand_s, cand_i, buf_s, buf_i, fallback, total;
};
FastLayout fast_layout(int64_t Q, int64_t NI, int64_t k, const FastPlan& p) {
  FastLayout L;
  L.thresh = 256;
  L.count = L.thresh + align256(Q * 4);
  L.cand_s = L.count + align256(Q * 4);
  const int64_t nc = Q * p.nsplit * 2 * (int64_t)p.T;
  L.cand_i = L.cand_s + align256(nc * 4);
  L.buf_s = L.cand_i + align256(nc * 4);
  L.buf_i = L.buf_s + align256(Q * (int64_t)kFastCap * 4);
  const int64_t fast_end = L.buf_i + align256(Q * (int64_t)kFastCap * 4);
  L.fallback = L.cand_s;  // the exact fallback reuses the candidate/buffer region after K4
  const int64_t fb_end = L.fallback + old_ws_bytes(Q, NI, k);
  L.total = (fast_end > fb_end ? fast_end : fb_end) + 256;
  return L;
}


// Every workspace starts with a 256-byte header (zeroed by each call):
//   int32 [0] queries the bf16 path sent to the exact kernels (all chunks), [1] path id
//   (rsx_topk_path), [2] the fast path's whole-batch fallback flag, [3] the current chunk's
//   fallback-query count (indexes qmap).
// The bf16 path's corpus image (rsx_topk_prepare_corpus: a 256-byte header holding the bits of
// max ||w|| and max ||w - bf16(w)||,
// then the [NI][128] bf16 image) either lives in the caller's cached buffer or is built into the
// workspace per call. Queries run in chunks of at most kQChunk (workspace bounded in Q).
constexpr int64_t kHeader = 256;
constexpr int64_t kQChunk = 4096;
int64_t corpus_bytes(int64_t NI) { return kHeader + align256(NI * kD * 2); }

struct BfLayout {
  int64_t corpus, thr, qmap, cand_s, cand_i, buf_e, buf_n, fallback, total;
};
BfLayout bf_layout(int64_t Qc, int64_t NI, int64_t k, const BfPlan& p, bool own_corpus) {
  BfLayout L;
  L.corpus = kHeader;
  const int64_t nstream = Qc * p.nsplit * 2;
  L.thr = L.corpus + (own_corpus ? corpus_bytes(NI) : 0);
  L.qmap = L.thr + align256(Qc * 4);
  L.cand_s = L.qmap + align256(Qc * 4);
  L.cand_i = L.cand_s + align256(nstream * p.T * 4);
  L.buf_e = L.cand_i + align256(nstream * p.T * 4);
  L.buf_n = L.buf_e + align256(nstream * kStreamCap * 8);
  const int64_t end = L.buf_n + align256(nstream * 4);
  // the exact kernels for the chunk's listed queries run after its P4: they reuse the
  // candidate / stream-buffer region (never the corpus image, which later chunks still read)
  L.fallback = L.cand_s;
  const int64_t fb_end = L.fallback + old_ws_bytes(Qc, NI, k);
  L.total = (end > fb_end ? end : fb_end) + 256;
  return L;
}

int launch_old(const float* U, int64_t ldu, const float* I, int64_t ldi, int64_t Q, int64_t NI, int64_t k,
               char* ws, float* out_scores, int64_t* out_idx, const int* gate, hipStream_t st,
               const int* qmap = nullptr, const int* qcount = nullptr) {
  const int kmax = k <= 128 ? 128 : 512;
  ScanArgs a;
  a.gate = gate;
  a.qmap = qmap;
  a.qcount = qcount;
  a.U = U; a.I = I; a.Q = Q; a.NI = NI; a.ldu = ldu; a.ldi = ldi;
  a.nsplit = choose_nsplit(Q, NI, kmax);
  a.span = ((NI + a.nsplit - 1) / a.nsplit + kTile - 1) / kTile * kTile;
  if (a.span < kTile) a.span = kTile;
  a.K = (int)k;
  a.cs = reinterpret_cast<float*>(ws);
  a.ci = reinterpret_cast<int*>(ws + Q * a.nsplit * 2 * (int64_t)kmax * 4);
  const int blocks = (int)(((Q + kOwnRows - 1) / kOwnRows) * a.nsplit);
  if (kmax == 128) hipLaunchKernelGGL(topk_scan_k<128>, dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(topk_scan_k<512>, dim3(blocks), dim3(256), 0, st, a);
  RSX_LAUNCHED();
  const int ncand = a.nsplit * 2 * kmax;
  if (ncand <= 2048)
    hipLaunchKernelGGL(topk_merge_k<2048>, dim3((unsigned)Q), dim3(256), 0, st, a.cs, a.ci, Q, ncand, (int)k,
                       out_scores, out_idx, gate, qmap, qcount);
  else
    hipLaunchKernelGGL(topk_merge_k<8192>, dim3((unsigned)Q), dim3(256), 0, st, a.cs, a.ci, Q, ncand, (int)k,
                       out_scores, out_idx, gate, qmap, qcount);
  RSX_LAUNCHED();
  return 0;
}

template <int T>
void launch_fast_scans(FastArgs f, int blocks, int mode, hipStream_t st) {
  if (mode == 0) hipLaunchKernelGGL((topk_fast_scan_k<0, T>), dim3(blocks), dim3(256), 0, st, f);
  else hipLaunchKernelGGL((topk_fast_scan_k<1, T>), dim3(blocks), dim3(256), 0, st, f);
}
}  // namespace

namespace {
int topk_path(int64_t Q, int64_t NI, int64_t k) {
  if (bf_plan(Q < kQChunk ? Q : kQChunk, NI, k).use) return 2;
  return fast_plan(Q, NI, k).use ? 1 : 0;
}

void launch_prep(const float* I, int64_t ldi, int64_t NI, char* corpus, hipStream_t st) {
  (void)hipMemsetAsync(corpus, 0, 8, st);  // max ||w||, max ||w - bf16(w)||
  int64_t pb = (NI + 31) / 32;
  if (pb > 4096) pb = 4096;
  hipLaunchKernelGGL(topk_bf16_prep_k, dim3((unsigned)pb), dim3(256), 0, st, I, ldi, NI,
                     reinterpret_cast<__bf16*>(corpus + kHeader), reinterpret_cast<unsigned*>(corpus));
}

// P1-P4 (+ the exact kernels for listed queries) over queries [0, Q) of U / out (one chunk)
int run_bf16_chunk(const BfPlan& bp, const BfLayout& L, const float* U, int64_t ldu, const float* I, int64_t ldi,
                   int64_t Q, int64_t NI, int64_t k, const char* corpus, char* w, float* out_scores,
                   int64_t* out_idx, hipStream_t st) {
  int* qtotal = reinterpret_cast<int*>(w);
  int* qcount = reinterpret_cast<int*>(w + 12);
  int* qmap = reinterpret_cast<int*>(w + L.qmap);
  const unsigned* wmax = reinterpret_cast<const unsigned*>(corpus);
  (void)hipMemsetAsync(qcount, 0, 4, st);
  BfArgs b;
  b.img = reinterpret_cast<const __bf16*>(corpus + kHeader);
  b.U = U; b.Q = Q; b.NI = NI; b.ldu = ldu;
  b.nsplit = bp.nsplit; b.nqb = bp.nqb; b.sample = bp.sample;
  b.span = ((NI + bp.nsplit - 1) / bp.nsplit + kTile - 1) / kTile * kTile;
  b.cand_s = reinterpret_cast<float*>(w + L.cand_s);
  b.cand_i = reinterpret_cast<int*>(w + L.cand_i);
  b.thr = reinterpret_cast<const float*>(w + L.thr);
  b.buf_e = reinterpret_cast<float2*>(w + L.buf_e);
  b.buf_n = reinterpret_cast<int*>(w + L.buf_n);
  const dim3 grid((unsigned)(bp.nqb * bp.nsplit));
  // P1 over ns0 <= nsplit splits: each workgroup samples nsplit / ns0 times the items (same
  // sampled fraction), so the query-fragment prologue is amortised over more tiles; any subset's
  // k-th best gives a valid t_q (P2), so the split count only moves the threshold's tightness
  // T0 = 1 (each lane stream keeps only its best sample: a compare and two selects per score
  // instead of a sorted insert) where 2 nsplit streams can hold 2k candidates, T0 = 2 (one
  // compare-swap) where 4 nsplit can (k = 500 at 1M items: 3.19 -> 2.52 ms per 4096-query call
  // against T0 = T = 8), else T0 = T
  BfArgs b0 = b;
  const int T0 = !sample_t1() ? bp.T : bp.nsplit >= k ? 1 : 2 * bp.nsplit >= k ? 2 : bp.T;
  const int ns0 = sample_nsplit(bp.nsplit, k, T0);
  b0.nsplit = ns0;
  b0.span = ((NI + ns0 - 1) / ns0 + kTile - 1) / kTile * kTile;
  const dim3 grid0((unsigned)(bp.nqb * ns0));
  if (T0 == 1) {
    if (bp.G == 2) hipLaunchKernelGGL((topk_bf16_scan_k<2, 1, 0>), grid0, dim3(256), 0, st, b0);
    else hipLaunchKernelGGL((topk_bf16_scan_k<1, 1, 0>), grid0, dim3(256), 0, st, b0);
  } else if (T0 == 2) {
    if (bp.G == 2) hipLaunchKernelGGL((topk_bf16_scan_k<2, 2, 0>), grid0, dim3(256), 0, st, b0);
    else hipLaunchKernelGGL((topk_bf16_scan_k<1, 2, 0>), grid0, dim3(256), 0, st, b0);
  } else {
    if (bp.G == 2) hipLaunchKernelGGL((topk_bf16_scan_k<2, 8, 0>), grid0, dim3(256), 0, st, b0);
    else hipLaunchKernelGGL((topk_bf16_scan_k<1, 8, 0>), grid0, dim3(256), 0, st, b0);
  }
  RSX_LAUNCHED();
  const int ncand = ns0 * 2 * T0;
  float* thr = reinterpret_cast<float*>(w + L.thr);
  const int r = thr_rank((int)k, bp.sample);
  if (ncand <= 1024)
    hipLaunchKernelGGL(topk_bf16_thresh_k<1024>, dim3((unsigned)Q), dim3(256), 0, st, b.cand_s, b.cand_i, ncand, U,
                       ldu, r, wmax, thr);
  else if (ncand <= 2048)
    hipLaunchKernelGGL(topk_bf16_thresh_k<2048>, dim3((unsigned)Q), dim3(256), 0, st, b.cand_s, b.cand_i, ncand, U,
                       ldu, r, wmax, thr);
  else
    hipLaunchKernelGGL(topk_bf16_thresh_k<4096>, dim3((unsigned)Q), dim3(256), 0, st, b.cand_s, b.cand_i, ncand, U,
                       ldu, r, wmax, thr);
  RSX_LAUNCHED();
  // RSX_TOPK_COLLECT (A/B): 2 (default) topk_bf16_collect_k, per-score appends behind the max gate;
  // 1 its max-first extraction; 0 topk_bf16_scan_k<G, 8, 1> (round 3's full scan)
  static const int collect_k = [] {
    const char* e = getenv("RSX_TOPK_COLLECT");
    return e ? atoi(e) : 2;
  }();
  if (collect_k == 1) {
    if (bp.G == 2) hipLaunchKernelGGL((topk_bf16_collect_k<2, true>), grid, dim3(256), 0, st, b);
    else hipLaunchKernelGGL((topk_bf16_collect_k<1, true>), grid, dim3(256), 0, st, b);
  } else if (collect_k == 0) {
    if (bp.G == 2) hipLaunchKernelGGL((topk_bf16_scan_k<2, 8, 1>), grid, dim3(256), 0, st, b);
    else hipLaunchKernelGGL((topk_bf16_scan_k<1, 8, 1>), grid, dim3(256), 0, st, b);
  } else if (collect_k == 3) {  // A/B: each append behind a wave-uniform ballot branch (slower: 1.69 vs 1.50 ms)
    if (bp.G == 2) hipLaunchKernelGGL((topk_bf16_collect_k<2, false, true>), grid, dim3(256), 0, st, b);
    else hipLaunchKernelGGL((topk_bf16_collect_k<1, false, true>), grid, dim3(256), 0, st, b);
  } else {
    if (bp.G == 2) hipLaunchKernelGGL((topk_bf16_collect_k<2, false>), grid, dim3(256), 0, st, b);
    else hipLaunchKernelGGL((topk_bf16_collect_k<1, false>), grid, dim3(256), 0, st, b);
  }
  RSX_LAUNCHED();
  hipLaunchKernelGGL(topk_bf16_select_k, dim3((unsigned)Q), dim3(256), 0, st, b.buf_e, b.buf_n,
                     bp.nsplit * 2, U, ldu, I, ldi, (int)k, wmax, thr, r < k ? 1 : 0, out_scores, out_idx, qcount,
                     qmap, qtotal);
  RSX_LAUNCHED();
  // exact list-based kernels for the queries P4 listed (none on spread data)
  return launch_old(U, ldu, I, ldi, Q, NI, k, w + L.fallback, out_scores, out_idx, nullptr, st, qmap, qcount);
}

int64_t ws_bytes(int64_t Q, int64_t NI, int64_t k, bool own_corpus) {
  const int path = topk_path(Q, NI, k);
  if (path == 2) {
    const int64_t Qc = Q < kQChunk ? Q : kQChunk;
    return bf_layout(Qc, NI, k, bf_plan(Qc, NI, k), own_corpus).total;
  }
  if (path == 1) return fast_layout(Q, NI, k, fast_plan(Q, NI, k)).total;
  return kHeader + old_ws_bytes(Q, NI, k) + 256;
}

int retrieve(const float* U, int64_t ldu, const float* I, int64_t ldi, const void* corpus_in, int64_t Q, int64_t NI,
             int64_t k, void* ws, float* out_scores, int64_t* out_idx, void* stream) {
  RSX_ARG(U && I && ws && out_scores && out_idx, "null tensor");
  RSX_ARG(k >= 1 && k <= 512, "k must be in [1,512]");
  RSX_ARG(ldu >= kD && ldi >= kD && ldu % 4 == 0 && ldi % 4 == 0, "D must be 128 (row strides >= 128)");
  RSX_ARG(NI < 0x7fffffff, "item count must fit int32");
  hipStream_t st = (hipStream_t)stream;
  char* w = reinterpret_cast<char*>(ws);
  const int path = topk_path(Q, NI, k);
  (void)hipMemsetAsync(w, 0, 16, st);
  (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(w + 4), path, 1, st);
  if (Q == 0) return 0;
  if (path == 2) {
    const int64_t Qc = Q < kQChunk ? Q : kQChunk;
    const BfPlan bp = bf_plan(Qc, NI, k);
    const BfLayout L = bf_layout(Qc, NI, k, bp, corpus_in == nullptr);
    const char* corpus = reinterpret_cast<const char*>(corpus_in);
    if (!corpus) {
      launch_prep(I, ldi, NI, w + L.corpus, st);
      RSX_LAUNCHED();
      corpus = w + L.corpus;
    }
    for (int64_t q0 = 0; q0 < Q; q0 += Qc) {
      const int64_t qn = Q - q0 < Qc ? Q - q0 : Qc;
      const BfPlan bc = qn == Qc ? bp : bf_plan(qn, NI, k);
      const int rc = run_bf16_chunk(bc, L, U + q0 * ldu, ldu, I, ldi, qn, NI, k, corpus, w, out_scores + q0 * k,
                                    out_idx + q0 * k, st);
      if (rc) return rc;
    }
    return 0;
  }
  if (path == 0) return launch_old(U, ldu, I, ldi, Q, NI, k, w + kHeader, out_scores, out_idx, nullptr, st);
  const FastPlan p = fast_plan(Q, NI, k);
  const FastLayout L = fast_layout(Q, NI, k, p);
  int* flag = reinterpret_cast<int*>(w + 8);
  FastArgs f;
  f.U = U; f.I = I; f.Q = Q; f.NI = NI; f.ldu = ldu; f.ldi = ldi;
  f.nsplit = p.nsplit;
  f.span = ((NI + p.nsplit - 1) / p.nsplit + kTile - 1) / kTile * kTile;
  if (f.span < kTile) f.span = kTile;
  f.K = (int)k;
  f.cap = kFastCap;
  f.cand_s = reinterpret_cast<float*>(w + L.cand_s);
  f.cand_i = reinterpret_cast<int*>(w + L.cand_i);
  f.thresh = reinterpret_cast<const float*>(w + L.thresh);
  f.count = reinterpret_cast<int*>(w + L.count);
  f.buf_s = reinterpret_cast<float*>(w + L.buf_s);
  f.buf_i = reinterpret_cast<int*>(w + L.buf_i);
  const int blocks = (int)(((Q + kOwnRows - 1) / kOwnRows) * p.nsplit);
  if (p.T == 8) launch_fast_scans<8>(f, blocks, 0, st);
  else launch_fast_scans<16>(f, blocks, 0, st);
  RSX_LAUNCHED();
  const int ncand = p.nsplit * 2 * p.T;
  float* th = reinterpret_cast<float*>(w + L.thresh);
  if (ncand <= 2048)
    hipLaunchKernelGGL(topk_thresh_k<2048>, dim3((unsigned)Q), dim3(256), 0, st, f.cand_s, f.cand_i, ncand, (int)k,
                       th, f.count);
  else
    hipLaunchKernelGGL(topk_thresh_k<8192>, dim3((unsigned)Q), dim3(256), 0, st, f.cand_s, f.cand_i, ncand, (int)k,
                       th, f.count);
  RSX_LAUNCHED();
  if (p.T == 8) launch_fast_scans<8>(f, blocks, 1, st);
  else launch_fast_scans<16>(f, blocks, 1, st);
  RSX_LAUNCHED();
  hipLaunchKernelGGL(topk_final_k<kFastCap>, dim3((unsigned)Q), dim3(256), 0, st, f.buf_s, f.buf_i, f.count,
                     kFastCap, (int)k, out_scores, out_idx, flag);
  RSX_LAUNCHED();
  // exact fallback for the whole batch, a no-op unless some query overflowed its buffer
  return launch_old(U, ldu, I, ldi, Q, NI, k, w + L.fallback, out_scores, out_idx, flag, st);
}
}  // namespace

RSX_API int rsx_topk_path(int64_t Q, int64_t NI, int64_t k) { return topk_path(Q, NI, k); }

RSX_API int64_t rsx_topk_workspace_bytes(int64_t Q, int64_t NI, int64_t k) { return ws_bytes(Q, NI, k, true); }

RSX_API int64_t rsx_topk_workspace_bytes_corpus(int64_t Q, int64_t NI, int64_t k) {
  return ws_bytes(Q, NI, k, false);
}

RSX_API int64_t rsx_topk_corpus_bytes(int64_t NI) { return corpus_bytes(NI); }

RSX_API int rsx_topk_prepare_corpus(const float* I, int64_t ldi, int64_t NI, void* corpus, void* stream) {
  RSX_ARG(I && corpus, "null tensor");
  RSX_ARG(ldi >= kD && ldi % 4 == 0, "D must be 128 (row stride >= 128)");
  RSX_ARG(NI >= 1 && NI < 0x7fffffff, "item count must be in [1, 2^31)");
  launch_prep(I, ldi, NI, reinterpret_cast<char*>(corpus), (hipStream_t)stream);
  RSX_LAUNCHED();
  return 0;
}

// scores [Q, k] (desc), idx [Q, k] int64 (-1 where fewer than k items exist).
RSX_API int rsx_retrieve_topk(const float* U, int64_t ldu, const float* I, int64_t ldi, int64_t Q, int64_t NI,
                              int64_t k, void* ws, float* out_scores, int64_t* out_idx, void* stream) {
  return retrieve(U, ldu, I, ldi, nullptr, Q, NI, k, ws, out_scores, out_idx, stream);
}

RSX_API int rsx_retrieve_topk_corpus(const float* U, int64_t ldu, const float* I, int64_t ldi, const void* corpus,
                                     int64_t Q, int64_t NI, int64_t k, void* ws, float* out_scores,
                                     int64_t* out_idx, void* stream) {
  RSX_ARG(corpus, "null corpus image");
  return retrieve(U, ldu, I, ldi, corpus, Q, NI, k, ws, out_scores, out_idx, stream);
}
