// Token-axis GEMMs of the user tower in bf16x3 split precision.
//
//   C[M, N] = epi(A[M, K] . B[N, K]^T + bias)        (both operands K-contiguous, "NT")
//
// Reference: every nn.Linear / F.linear applied per token in the training step
// (tower_code/v1_refine_usertower.py:447-510: item_proj, the encoder layers' in_proj /
// out_proj / linear1 / linear2, output_proj) — autograd's forward GEMM and its input-gradient
// GEMM (dX = dY . W, called here with B = W^T). M = tokens (~160k for the two dropout views
// at batch 4096) is huge and N, K <= 512 are small, so the GEMMs are bandwidth-bound once the
// products leave the fp32 MFMA: each fp32 operand x is split x = hi + lo (hi = bf16(x),
// lo = bf16(x - hi)) while it is staged into LDS, and a product is hi*hi' + hi*lo' + lo*hi'
// on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (the arithmetic of infonce.hip's
// bf16x3 loss: ~2^-17 relative error per product, 5.3x fewer MFMA cycles than the fp32 MFMA).
//
// Epilogues (fusing the FFN's elementwise work into its two GEMMs):
//   EPI_BIAS       C = acc + bias
//   EPI_GELU_DROP  z = acc + bias; C = dropout_p(gelu_erf(z)) (keep-mask = hash(seed, m*N + n));
//                  aux = gelu_erf'(z), the backward's multiplier (saved instead of z)
//   EPI_DGELU_DROP C = acc * keep(m, n) / (1 - p) * aux[m][n]   (backward of the above:
//                  acc = dAct = dY2 . W2)
//   EPI_ADDLN      (weight-stationary, N = 128) the residual add + LayerNorm after the
//                  attention out-projection: C = s = aux + dropout_p(acc + bias),
//                  y = LayerNorm(s) * ln_w + ln_b, with the row's mean / rstd saved
//
// Tiling: 128 x 128 output tile per 256-thread workgroup (four waves of 64 x 64 = 2 x 2
// MFMA tiles), K staged 16 at a time, double-buffered in LDS with register prefetch and one
// barrier per stage. LDS rows are 16 bf16 + 8 pad (48 B): the fragment reads (ds_read_b128,
// 32 rows x 16 B per lane half) are bank-conflict free, and 48 KB per workgroup leaves room
// for three workgroups per CU (the GEMMs are latency-bound at two). XCD-aware order: the N tiles of one
// M block run back to back on one XCD, so A's rows are re-read from that XCD's L2.
#include "rsx_common.h"
#include <stdlib.h>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#ifndef RSX_GEMM_BK
#define RSX_GEMM_BK 16  // measured (tools/gemm_micro.py): 16 beats 32 by 10-15 % (48 KB LDS: 3 workgroups/CU)
#endif
constexpr int kBM = 128, kBN = 128, kBK = RSX_GEMM_BK;
constexpr int kRow = kBK + 8;  // bf16 per LDS row (80 B at BK 32, 48 B at BK 16: conflict-free b128 reads)
constexpr int kF4 = kBK / 8;   // float4 loads per thread and operand per stage (two threads per row)
constexpr int EPI_BIAS = 0, EPI_GELU_DROP = 1, EPI_DGELU_DROP = 2, EPI_ROWADD = 3, EPI_ADDLN = 4;
#ifndef RSX_GEMM_BLOCKS
#define RSX_GEMM_BLOCKS (1 << 30)  // workgroup budget of the multi-tile stream: at BK 16 one tile each measured best
#endif

__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// gelu(x) = x Phi(x) and gelu'(x) = Phi(x) + x phi(x), branch-free for the weight-stationary
// epilogue: Phi from erfc(z) ~ t P(t) e^{-z^2}, t = 1 / (1 + p z), z = |x| / sqrt 2 (Abramowitz &
// Stegun 7.1.26, |erf error| <= 1.5e-7), and e^{-z^2} = e^{-x^2/2} is also phi's exponential: one
// exp, one rcp and six fma per element instead of erff's two-range polynomial plus an exp.
// Max |error| over [-12, 12] against float64: 4.2e-7 (gelu), 3.2e-7 (gelu'); torch's fp32 gelu
// itself is 1.2e-6 off there.
__device__ __forceinline__ void gelu_pair(float x, float& g, float& d) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __expf(-0.5f * x * x);
  const float q = 0.5f * (p * t) * e;  // 0.5 erfc(z) = Phi(-|x|)
  const float cdf = x >= 0.0f ? 1.0f - q : q;
  g = x * cdf;
  d = fmaf(x * 0.3989422804014327f, e, cdf);
}

// rsx::hash_u32(seed, idx) for idx < 2^32 (the high-word terms vanish), in 32-bit ops
__device__ __forceinline__ bool keep(const rsx::Dropout& d, uint32_t idx) {
  uint32_t x = idx ^ (uint32_t)d.seed;
  x ^= (uint32_t)(d.seed >> 32) * 0x85EBCA77u;
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x >= d.thresh;
}

template <int BK>
struct ImgT {
  __bf16 hi[kBM * (BK + 8)];
  __bf16 lo[kBM * (BK + 8)];
};
using Img = ImgT<kBK>;

struct GArgs {
  const float* A;     // [M, lda]
  const float* B;     // [N, ldb]
  const float* bias;  // [N] (nullable)
  float* C;           // [M, ldc]
  float* aux;         // [M, ldaux]: gelu'(pre) (written by EPI_GELU_DROP, read by EPI_DGELU_DROP);
                      // EPI_ROWADD: the row table R [*, ldaux]
  const int64_t* ridx;  // EPI_ROWADD: C[m] += R[ridx[m]]
  float* y;             // EPI_ADDLN: LayerNorm output [M, ldy]; aux = the residual x [M, ldaux]
  const float* ln_w;    // EPI_ADDLN: LayerNorm weight / bias [N]
  const float* ln_b;
  float* mean;          // EPI_ADDLN: [M] row statistics for the backward
  float* rstd;
  float eps;
  int64_t ldy;
  int64_t lda, ldb, ldc, ldaux, M;
  int N, K, epi, tiles_n, tiles, per;
  int ksplit;    // split-K (> 1): workgroup (split, tile), K range [split * kspan, + kspan), raw sums to part
  int kspan;
  float* part;   // [ksplit][M][N] partial sums (split-K only)
  int transb;  // weight-stationary path only: B given as Bt [K, ldb] (B[n][k] = Bt[k * ldb + n])
  rsx::Dropout drop;
};

// 8 fp32 -> 8 hi + 8 lo bf16 (one 16-B chunk each)
__device__ __forceinline__ void split8(const float4& x, const float4& y, u32x4& hi, u32x4& lo) {
  const float f[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
  bf16x8 h, l;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const __bf16 hk = (__bf16)f[k];
    h[k] = hk;
    l[k] = (__bf16)(f[k] - (float)hk);
  }
  hi = __builtin_bit_cast(u32x4, h);
  lo = __builtin_bit_cast(u32x4, l);
}

template <int EPI>
__device__ __forceinline__ void epilogue(const GArgs& a, f32x16 (&acc)[2][2], int64_t m0, int n0, int wm, int wn,
                                         int h, int c) {
  // row m0 + wm*64 + 32i + tile_row(r,h), column n0 + wn*64 + 32j + c. EPI_DGELU_DROP loads
  // the tile's saved GELU derivatives 16 at a time (rows past M read row M-1), so the loads
  // overlap instead of each waiting in turn.
  if (EPI == EPI_DGELU_DROP) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float z[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int64_t m = m0 + wm * 64 + 32 * i + tile_row(r, h);
          if (m >= a.M) m = a.M - 1;
          z[r] = a.aux[m * a.ldaux + n0 + wn * 64 + 32 * j + c];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] *= z[r];
      }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + 32 * j + c;
    const float bn = a.bias ? a.bias[n] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm * 64 + 32 * i + tile_row(r, h);
        float v = acc[i][j][r];
        acc[i][j][r] = 0.0f;
        if (m >= a.M) continue;
        if (EPI == EPI_BIAS) {
          v += bn;
        } else if (EPI == EPI_GELU_DROP) {
          v += bn;
          const float cdf = 0.5f * (1.0f + erff(v * 0.70710678118654752f));
          if (a.aux) a.aux[m * a.ldaux + n] = cdf + v * 0.3989422804014327f * __expf(-0.5f * v * v);  // gelu'(v)
          v *= cdf;  // gelu(v)
          if (a.drop.active()) v = keep(a.drop, (uint32_t)m * (uint32_t)a.N + (uint32_t)n) ? v * a.drop.scale : 0.0f;
        } else if (a.drop.active()) {
          v = keep(a.drop, (uint32_t)m * (uint32_t)a.N + (uint32_t)n) ? v * a.drop.scale : 0.0f;
        }
        a.C[m * a.ldc + n] = v;
      }
  }
}

// Each workgroup walks `per` consecutive output tiles (same XCD; consecutive tiles share the
// M block) as one continuous stream of K stages: the prefetch of the next stage (possibly
// the next tile's first) overlaps the current stage's MFMAs and the finished tile's epilogue,
// so the load pipeline never drains between tiles.
// Q = stages of A / B kept in flight in registers (Q = 1: the next stage only). With few output tiles
// (M of a few thousand tokens and N <= 768: fewer tiles than CUs, one workgroup per CU, e.g. the text
// BERT's GEMMs) a workgroup's single 16-KB stage in flight leaves it waiting on memory latency for
// most of each stage; Q = 4 keeps four (64 KB) in flight at 16 VGPRs per stage. Same products and
// order (bit-identical results).
template <int EPI, int Q = 1, int BK = kBK>
__global__ __launch_bounds__(256, 2) void gemm_x3_nt_k(GArgs a) {
  constexpr int kRowK = BK + 8, kF4K = BK / 8;
  __shared__ __attribute__((aligned(16))) ImgT<BK> sA[2];
  __shared__ __attribute__((aligned(16))) ImgT<BK> sB[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware block order (the grid is padded to a multiple of 8)
  const int bflat = (blockIdx.x & 7) * ((int)gridDim.x >> 3) + (blockIdx.x >> 3);
  const int split = a.ksplit > 1 ? bflat / a.tiles : 0;
  const int t_begin = a.ksplit > 1 ? bflat % a.tiles : bflat * a.per;
  int t_end = a.ksplit > 1 ? t_begin + 1 : t_begin + a.per;
  if (t_end > a.tiles) t_end = a.tiles;
  if (t_begin >= t_end || split >= (a.ksplit > 1 ? a.ksplit : 1)) return;
  const int nk = (a.ksplit > 1 ? a.kspan : a.K) / BK;
  const int kbase = split * (a.ksplit > 1 ? a.kspan : 0);
  const int nstage = (t_end - t_begin) * nk;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // staging: thread -> row tid>>1 of both tiles, 16 floats at column (tid&1)*16 of the stage.
  // Rows past M load row m0 instead (unconditional loads: a predicated load would make the
  // compiler wait on each one); their C rows are never stored and no other row depends on them.
  const int srow = tid >> 1, scol = (tid & 1) * (BK / 2);
  float4 pa[Q][kF4K], pb[Q][kF4K];
  auto gload_s = [&](int slot, int st) {
    if (st >= nstage) st = nstage - 1;  // unconditional (clamped): the same outstanding loads on every path
    const int t = t_begin + st / nk, k0 = kbase + (st % nk) * BK;
    const int64_t m0 = (int64_t)(t / a.tiles_n) * kBM;
    const int n0 = (t % a.tiles_n) * kBN;
    const float* a_src = a.A + (m0 + srow < a.M ? m0 + srow : m0) * a.lda + scol + k0;
    const float* b_src = a.B + (int64_t)(n0 + srow) * a.ldb + scol + k0;
#pragma unroll
    for (int q = 0; q < kF4K; ++q) {
      pa[slot][q] = *reinterpret_cast<const float4*>(a_src + 4 * q);
      pb[slot][q] = *reinterpret_cast<const float4*>(b_src + 4 * q);
    }
  };
  auto lstore_s = [&](int slot, int buf) {
    const int o = srow * kRowK + scol;
#pragma unroll
    for (int q = 0; q < kF4K / 2; ++q) {
      u32x4 hi, lo;
      split8(pa[slot][2 * q], pa[slot][2 * q + 1], hi, lo);
      *reinterpret_cast<u32x4*>(&sA[buf].hi[o + 8 * q]) = hi;
      *reinterpret_cast<u32x4*>(&sA[buf].lo[o + 8 * q]) = lo;
      split8(pb[slot][2 * q], pb[slot][2 * q + 1], hi, lo);
      *reinterpret_cast<u32x4*>(&sB[buf].hi[o + 8 * q]) = hi;
      *reinterpret_cast<u32x4*>(&sB[buf].lo[o + 8 * q]) = lo;
    }
  };
  auto compute = [&](int cur, int st, bool epi_in_loop) {
    const ImgT<BK>& ta = sA[cur];
    const ImgT<BK>& tb = sB[cur];
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int oa = (wm * 64 + 32 * i + c) * kRowK + 16 * ks + 8 * h;
        const int ob = (wn * 64 + 32 * i + c) * kRowK + 16 * ks + 8 * h;
        ah[i] = *reinterpret_cast<const bf16x8*>(&ta.hi[oa]);
        al[i] = *reinterpret_cast<const bf16x8*>(&ta.lo[oa]);
        bh[i] = *reinterpret_cast<const bf16x8*>(&tb.hi[ob]);
        bl[i] = *reinterpret_cast<const bf16x8*>(&tb.lo[ob]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    if (epi_in_loop && st % nk == nk - 1) {  // tile finished: epilogue (resets acc) while the next stage loads
      const int t = t_begin + st / nk;
      epilogue<EPI>(a, acc, (int64_t)(t / a.tiles_n) * kBM, (t % a.tiles_n) * kBN, wm, wn, h, c);
    }
  };

  if constexpr (Q == 1) {
    gload_s(0, 0);
    lstore_s(0, 0);
    __syncthreads();
    int cur = 0;
    for (int st = 0; st < nstage; ++st) {
      const bool has_next = st + 1 < nstage;
      if (has_next) gload_s(0, st + 1);
      compute(cur, st, true);
      if (has_next) lstore_s(0, cur ^ 1);  // cur^1 was read in the previous stage, fenced by its barrier
      __syncthreads();
      cur ^= 1;
    }
  } else {
    // stage s lives in register slot s % Q; stages st+1 .. st+Q are in flight while stage st computes.
    // One tile per workgroup (the host launches this form only with per == 1): the epilogue runs after
    // the loop, so no branch inside it drains the loads in flight
    gload_s(0, 0);
    lstore_s(0, 0);
#pragma unroll
    for (int k = 1; k <= Q; ++k) gload_s(k % Q, k);
    __syncthreads();
    int cur = 0;
    for (int st0 = 0; st0 < nstage; st0 += Q) {
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        const int st = st0 + k;
        if (st >= nstage) break;
        compute(cur, st, false);
        if (st + 1 < nstage) lstore_s((k + 1) % Q, cur ^ 1);
        __syncthreads();
        gload_s((k + 1) % Q, st + 1 + Q);  // the slot just stored: stage st + 1 + Q (clamped)
        cur ^= 1;
      }
    }
    const int64_t m0 = (int64_t)(t_begin / a.tiles_n) * kBM;
    const int n0 = (t_begin % a.tiles_n) * kBN;
    if (a.ksplit > 1) {  // raw partial sums; gemm_splitk_reduce_k adds the splits in order and applies EPI
      float* P = a.part + (int64_t)split * a.M * a.N;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int64_t m = m0 + wm * 64 + 32 * i + tile_row(r, h);
            if (m < a.M) P[m * a.N + n0 + wn * 64 + 32 * j + c] = acc[i][j][r];
          }
    } else {
      epilogue<EPI>(a, acc, m0, n0, wm, wn, h, c);
    }
  }
}

// C = EPI(sum over the splits of part, in split order) with epilogue<EPI>'s arithmetic per element
template <int EPI>
__global__ __launch_bounds__(256) void gemm_splitk_reduce_k(GArgs a) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= a.M * (int64_t)a.N) return;
  const int64_t m = e / a.N;
  const int n = (int)(e % a.N);
  float v = 0.0f;
  for (int s = 0; s < a.ksplit; ++s) v += a.part[(int64_t)s * a.M * a.N + e];
  if (EPI == EPI_DGELU_DROP) v *= a.aux[m * a.ldaux + n];
  const float bn = a.bias ? a.bias[n] : 0.0f;
  if (EPI == EPI_BIAS) {
    v += bn;
  } else if (EPI == EPI_GELU_DROP) {
    v += bn;
    const float cdf = 0.5f * (1.0f + erff(v * 0.70710678118654752f));
    if (a.aux) a.aux[m * a.ldaux + n] = cdf + v * 0.3989422804014327f * __expf(-0.5f * v * v);
    v *= cdf;
    if (a.drop.active()) v = keep(a.drop, (uint32_t)m * (uint32_t)a.N + (uint32_t)n) ? v * a.drop.scale : 0.0f;
  } else if (a.drop.active()) {
    v = keep(a.drop, (uint32_t)m * (uint32_t)a.N + (uint32_t)n) ? v * a.drop.scale : 0.0f;
  }
  a.C[m * a.ldc + n] = v;
}

// ---------------------------------------------------------------------------------------
// Weight-stationary form (used whenever K is 128, 256 or 384 and N a multiple of the column
// block): the GEMMs here have M ~ 160k and tiny N, K, so the whole column block of B (N_blk x
// K, hi and lo) is split ONCE per workgroup into LDS in MFMA-fragment order, and the
// activations never touch LDS: each wave streams 32-row strips of A straight from HBM into
// registers (a 128-k chunk per strip = 64 fp32 per lane: lane (c, h) reads row c, 16 B at a
// time at k = 8i + 4h), double-buffered across strips so one chunk is always in flight per
// wave (~128 KB per CU with eight waves; the two-stage LDS pipeline above kept ~24 KB of A in
// flight per CU and was latency-bound at 2-3.4 TB/s).
// The summation order over k is a fixed permutation (k-step s of a chunk takes k = 16s + 4h
// + {0..3} and 16s + 8 + 4h + {0..3}); B's fragments use the same permutation, so each
// product is the plain sum over k. Same epilogues and dropout hash as gemm_x3_nt_k.
// WV = 4: one wave per SIMD with the whole 512-register file, three A chunks per wave (one being
// computed, two in flight); WV = 8: two waves per SIMD (256 registers each), two chunks per wave
// (the other wave's loads and stores in flight while one computes).

struct WsArgs {
  GArgs g;
  int nblk;     // column blocks
  int groups;   // workgroups per column block
};

// PF (WV = 4): the next 16-k step's B fragments are read from LDS while this step's MFMAs run (one wave
// per SIMD has no other wave to cover an LDS round trip; without PF hipcc re-reads each fragment right
// before its MFMA and waits for it), with two A chunks per wave instead of three for the registers.
template <int KC, int NBW, int EPI, int WV, bool PF = false>
__global__ __launch_bounds__(64 * WV, 1) void gemm_ws_k(WsArgs w) {
  constexpr int kWsThreads = 64 * WV, kWsWaves = WV;
  constexpr int NT = NBW / 32;
  __shared__ __attribute__((aligned(16))) u32x4 sW[KC * 8 * NT * 2 * 64];
  const GArgs& a = w.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int bflat = (blockIdx.x & 7) * ((int)gridDim.x >> 3) + (blockIdx.x >> 3);
  const int nb = bflat % w.nblk, grp = bflat / w.nblk;
  if (grp >= w.groups) return;  // whole workgroup: no barrier is skipped by part of it
  const int n0 = nb * NBW;

  // B column block -> LDS fragments: slot (step st = 16-k step over all chunks, tile j, lane l)
  // holds B[n0 + 32j + (l & 31)][k-set(st, l >> 5)] as 8 hi and 8 lo bf16.
  for (int slot = tid; slot < KC * 8 * NT * 64; slot += kWsThreads) {
    const int l = slot & 63, rest = slot >> 6;
    const int j = rest % NT, st = rest / NT;
    const int n = n0 + 32 * j + (l & 31), k0 = (st >> 3) * 128 + 16 * (st & 7) + 4 * (l >> 5);
    float4 x0, x1;
    if (a.transb) {  // dX = dY W with W [K, N] as stored: column n of W (lanes read consecutive n)
      const float* src = a.B + (int64_t)k0 * a.ldb + n;
      x0 = make_float4(src[0], src[a.ldb], src[2 * a.ldb], src[3 * a.ldb]);
      src += 8 * a.ldb;
      x1 = make_float4(src[0], src[a.ldb], src[2 * a.ldb], src[3 * a.ldb]);
    } else {
      const float* src = a.B + (int64_t)n * a.ldb + k0;
      x0 = *reinterpret_cast<const float4*>(src);
      x1 = *reinterpret_cast<const float4*>(src + 8);
    }
    u32x4 hi, lo;
    split8(x0, x1, hi, lo);
    sW[(rest * 2 + 0) * 64 + l] = hi;
    sW[(rest * 2 + 1) * 64 + l] = lo;
  }
  __shared__ __attribute__((aligned(16))) float sBias[NBW];
  for (int n = tid; n < NBW; n += kWsThreads) sBias[n] = (EPI != EPI_DGELU_DROP && a.bias) ? a.bias[n0 + n] : 0.0f;
  __shared__ __attribute__((aligned(16))) float sLn[EPI == EPI_ADDLN ? 2 * NBW : 4];
  if (EPI == EPI_ADDLN)
    for (int n = tid; n < NBW; n += kWsThreads) {
      sLn[n] = a.ln_w ? a.ln_w[n] : 1.0f;
      sLn[NBW + n] = a.ln_b ? a.ln_b[n] : 0.0f;
    }
  __syncthreads();

  // this wave's strips: (grp + groups * it) * kWsWaves + wave, it = 0, 1, ...
  const int64_t nstrips = (a.M + 31) >> 5;
  const int64_t s_first = (int64_t)grp * kWsWaves + wave, s_step = (int64_t)w.groups * kWsWaves;
  const int nmine = s_first < nstrips ? (int)((nstrips - 1 - s_first) / s_step + 1) : 0;
  const int nitems = nmine * KC;

  f32x16 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;

  auto load = [&](int t, float4 (&buf)[16]) {
    const int64_t strip = s_first + (int64_t)(t / KC) * s_step;
    int64_t row = strip * 32 + c;
    if (row >= a.M) row = a.M - 1;  // tail rows re-read the last row; never stored
    const float* src = a.A + row * a.lda + (t % KC) * 128 + 4 * h;
#pragma unroll
    for (int i = 0; i < 16; ++i) buf[i] = *reinterpret_cast<const float4*>(src + 8 * i);
  };

  // acc[j] = B_j . A^T (the B fragment is the MFMA's A operand): lane (c, h), register
  // 4g + e holds C[strip*32 + c][n0 + 32j + 8g + 4h + e], so the epilogue moves float4s.
  auto compute = [&](int t, const float4 (&buf)[16]) {
    const int q = t % KC;
    int64_t m = (s_first + (int64_t)(t / KC) * s_step) * 32 + c;
    if (m >= a.M) m = a.M - 1;
    float* crow = a.C + m * a.ldc + n0 + 4 * h;
    float* xrow = (EPI == EPI_GELU_DROP || EPI == EPI_DGELU_DROP) ? a.aux + m * a.ldaux + n0 + 4 * h : nullptr;
    // EPI_DGELU_DROP / EPI_ROWADD: the strip's saved GELU derivatives / added table rows are
    // loaded before its MFMAs (vmcnt retires in order, so a load issued at the epilogue
    // would drain the prefetched strips)
    if (EPI == EPI_ROWADD) xrow = a.aux + a.ridx[m] * a.ldaux + n0 + 4 * h;
    if (EPI == EPI_ADDLN) xrow = a.aux + m * a.ldaux + 4 * h;
    float4 z[NT][4];
    if ((EPI == EPI_DGELU_DROP || EPI == EPI_ROWADD || EPI == EPI_ADDLN) && q == KC - 1) {
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) z[j][g] = *reinterpret_cast<const float4*>(xrow + 32 * j + 8 * g);
    }
    if constexpr (PF) {
      u32x4 wf[2][NT][2];
      auto wload = [&](int s, u32x4 (&wd)[NT][2]) {
        const u32x4* wp = sW + ((q * 8 + s) * NT) * 128 + lane;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          wd[j][0] = wp[j * 128];
          wd[j][1] = wp[j * 128 + 64];
        }
      };
      wload(0, wf[0]);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        if (s + 1 < 8) wload(s + 1, wf[(s + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);  // keep the reads here: hipcc otherwise sinks each to its MFMA
        u32x4 hi, lo;
        split8(buf[2 * s], buf[2 * s + 1], hi, lo);
        const bf16x8 xh = __builtin_bit_cast(bf16x8, hi), xl = __builtin_bit_cast(bf16x8, lo);
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const bf16x8 wh = __builtin_bit_cast(bf16x8, wf[s & 1][j][0]);
          const bf16x8 wl = __builtin_bit_cast(bf16x8, wf[s & 1][j][1]);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh, acc[j], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u32x4 hi, lo;
      split8(buf[2 * s], buf[2 * s + 1], hi, lo);
      const bf16x8 xh = __builtin_bit_cast(bf16x8, hi), xl = __builtin_bit_cast(bf16x8, lo);
      const u32x4* wp = sW + ((q * 8 + s) * NT) * 128 + lane;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const bf16x8 wh = __builtin_bit_cast(bf16x8, wp[j * 128]);
        const bf16x8 wl = __builtin_bit_cast(bf16x8, wp[j * 128 + 64]);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh, acc[j], 0, 0, 0);
      }
    }
    }
    if (q != KC - 1) return;
    // epilogue. Rows past M loaded A row M-1 and computed exactly row M-1's values; they are
    // written to row M-1 again (same values, dropout hashed on the clamped row), so the stores
    // need no branch.
    const uint32_t e0 = (uint32_t)m * (uint32_t)a.N + (uint32_t)(n0 + 4 * h);
    if constexpr (EPI == EPI_ADDLN) {
      // lane (c, h) holds 64 of row m's 128 sums; lane c + 32 the other 64 (one xor-32 swap
      // per statistic). Two-pass variance over the registers, as ln_fwd_k.
      float sum = 0.0f;
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int o = 32 * j + 8 * g;
          const float4 bb = *reinterpret_cast<const float4*>(&sBias[o + 4 * h]);
          const float zz[4] = {z[j][g].x, z[j][g].y, z[j][g].z, z[j][g].w};
          const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[j][4 * g + e] + bv[e];
            if (a.drop.active()) v = keep(a.drop, e0 + o + e) ? v * a.drop.scale : 0.0f;
            v += zz[e];
            acc[j][4 * g + e] = v;
            sum += v;
          }
        }
      sum += __shfl_xor(sum, 32, 64);
      const float mu = sum * (1.0f / NBW);
      float sq = 0.0f;
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[j][r] - mu;
          sq += d * d;
        }
      sq += __shfl_xor(sq, 32, 64);
      const float rs = 1.0f / sqrtf(sq * (1.0f / NBW) + a.eps);
      float* yrow = a.y + m * a.ldy + 4 * h;
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int o = 32 * j + 8 * g;
          const float4 ww = *reinterpret_cast<const float4*>(&sLn[o + 4 * h]);
          const float4 lb = *reinterpret_cast<const float4*>(&sLn[NBW + o + 4 * h]);
          const float s0 = acc[j][4 * g], s1 = acc[j][4 * g + 1], s2 = acc[j][4 * g + 2], s3 = acc[j][4 * g + 3];
          *reinterpret_cast<float4*>(crow + o) = make_float4(s0, s1, s2, s3);
          *reinterpret_cast<float4*>(yrow + o) =
              make_float4((s0 - mu) * rs * ww.x + lb.x, (s1 - mu) * rs * ww.y + lb.y, (s2 - mu) * rs * ww.z + lb.z,
                          (s3 - mu) * rs * ww.w + lb.w);
        }
      if (h == 0) {
        a.mean[m] = mu;
        a.rstd[m] = rs;
      }
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
      return;
    }
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int o = 32 * j + 8 * g;
        float v[4] = {acc[j][4 * g], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]};
        if (EPI == EPI_DGELU_DROP) {
          v[0] *= z[j][g].x; v[1] *= z[j][g].y; v[2] *= z[j][g].z; v[3] *= z[j][g].w;
        } else {
          const float4 bb = *reinterpret_cast<const float4*>(&sBias[o + 4 * h]);
          v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
          if (EPI == EPI_ROWADD) {
            v[0] += z[j][g].x; v[1] += z[j][g].y; v[2] += z[j][g].z; v[3] += z[j][g].w;
          }
        }
        if (EPI == EPI_GELU_DROP) {
          float d[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            gelu_pair(v[e], v[e], d[e]);
          }
          if (a.aux) *reinterpret_cast<float4*>(xrow + o) = make_float4(d[0], d[1], d[2], d[3]);
        }
        if ((EPI == EPI_GELU_DROP || EPI == EPI_DGELU_DROP) && a.drop.active()) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = keep(a.drop, e0 + o + e) ? v[e] * a.drop.scale : 0.0f;
        }
        *reinterpret_cast<float4*>(crow + o) = make_float4(v[0], v[1], v[2], v[3]);
      }
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
  };

  // sched_barrier fences keep the compiler from hoisting one buffer's conversions into another
  // phase (which raised the register demand past the file and forced early vmcnt waits).
#define WS_FENCE __builtin_amdgcn_sched_barrier(0)
  if (nitems == 0) return;  // wave-uniform; no barrier follows
  // every load is unconditional (item index clamped to the last item): all paths into the
  // loop then carry the same outstanding-load pattern, so the compiler's vmcnt waits stay
  // per buffer instead of draining the prefetches. The trailing re-loads are never used.
  const int last = nitems - 1;
  if constexpr (WV == 8 || PF) {
    float4 b0[16], b1[16];
    load(0, b0);
    load(last < 1 ? last : 1, b1);
    for (int t = 0;; t += 2) {
      WS_FENCE;
      compute(t, b0);
      WS_FENCE;
      load(t + 2 < last ? t + 2 : last, b0);
      if (t + 1 > last) break;
      WS_FENCE;
      compute(t + 1, b1);
      WS_FENCE;
      load(t + 3 < last ? t + 3 : last, b1);
      if (t + 2 > last) break;
    }
    return;
  }
  float4 b0[16], b1[16], b2[16];
  load(0, b0);
  load(last < 1 ? last : 1, b1);
  load(last < 2 ? last : 2, b2);
  for (int t = 0;; t += 3) {
    WS_FENCE;
    compute(t, b0);
    WS_FENCE;
    load(t + 3 < last ? t + 3 : last, b0);
    if (t + 1 > last) break;
    WS_FENCE;
    compute(t + 1, b1);
    WS_FENCE;
    load(t + 4 < last ? t + 4 : last, b1);
    if (t + 2 > last) break;
    WS_FENCE;
    compute(t + 2, b2);
    WS_FENCE;
    load(t + 5 < last ? t + 5 : last, b2);
    if (t + 3 > last) break;
  }
#undef WS_FENCE
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                 hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

bool ws_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("RSX_GEMM_WS");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  return on == 1;
}

template <int KC, int NBW, int WV, bool PF = false>
void launch_ws_w(const GArgs& g, hipStream_t st) {
  constexpr int kWsThreads = 64 * WV, kWsWaves = WV;
  WsArgs w;
  w.g = g;
  w.nblk = g.N / NBW;
  const int64_t strips = (g.M + 31) / 32;
  const int64_t blocks_rows = (strips + kWsWaves - 1) / kWsWaves;  // strips per workgroup round
  int groups = num_cus() / w.nblk;
  if (groups < 1) groups = 1;
  if (groups > blocks_rows) groups = (int)blocks_rows;
  w.groups = groups;
  const int grid = (w.nblk * groups + 7) / 8 * 8;
  if (g.epi == EPI_BIAS) hipLaunchKernelGGL((gemm_ws_k<KC, NBW, EPI_BIAS, WV, PF>), dim3(grid), dim3(kWsThreads), 0, st, w);
  else if (g.epi == EPI_ROWADD)
    hipLaunchKernelGGL((gemm_ws_k<KC, NBW, EPI_ROWADD, WV, PF>), dim3(grid), dim3(kWsThreads), 0, st, w);
  else if (g.epi == EPI_ADDLN)
    hipLaunchKernelGGL((gemm_ws_k<KC, NBW, EPI_ADDLN, WV, PF>), dim3(grid), dim3(kWsThreads), 0, st, w);
  else if (g.epi == EPI_GELU_DROP)
    hipLaunchKernelGGL((gemm_ws_k<KC, NBW, EPI_GELU_DROP, WV, PF>), dim3(grid), dim3(kWsThreads), 0, st, w);
  else hipLaunchKernelGGL((gemm_ws_k<KC, NBW, EPI_DGELU_DROP, WV, PF>), dim3(grid), dim3(kWsThreads), 0, st, w);
}

// RSX_GEMM_WS_WAVES = 4 | 8 (A/B): waves per weight-stationary workgroup
int ws_waves() {
  static int v = 0;
  if (v == 0) {
    const char* e = getenv("RSX_GEMM_WS_WAVES");
    v = (e && e[0] == '8') ? 8 : 4;
  }
  return v;
}

// RSX_GEMM_DEEP = 0 | 1 (A/B): the LDS-staged GEMM with four stages in flight when its tiles fit the chip
bool deep_prefetch() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RSX_GEMM_DEEP");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}
bool a_nk_long(int K) { return K / kBK >= 16; }
// the few-tile forms stage 32 of K per barrier (one workgroup per CU: half the barriers and stage
// overheads; 80 KB of LDS) when K allows it; RSX_GEMM_FEW_BK=16 keeps 16 (A/B)
int few_bk(int K) {
  static int v = 0;
  if (v == 0) {
    const char* e = getenv("RSX_GEMM_FEW_BK");
    v = (e && atoi(e) == 16) ? 16 : 32;
  }
  return (v == 32 && K % 32 == 0) ? 32 : 16;
}

// RSX_GEMM_WS_PF = 0 | 1 (A/B): four waves with the B-fragment prefetch (PF) or without
bool ws_pf() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RSX_GEMM_WS_PF");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

template <int KC, int NBW>
void launch_ws(const GArgs& g, hipStream_t st) {
  if (ws_waves() == 8) launch_ws_w<KC, NBW, 8>(g, st);
  else if (ws_pf()) launch_ws_w<KC, NBW, 4, true>(g, st);
  else launch_ws_w<KC, NBW, 4>(g, st);
}

// split-K plan of the LDS-staged path: with fewer output tiles than CUs (one workgroup per CU at most,
// e.g. the text BERT's 768-wide GEMMs at a few thousand tokens) and a long K, S K-ranges of >= 256 per
// tile (S in {8, 4, 3, 2}, tiles * S <= 4 * CUs); M = 3,000 (tools/gemm_bert_micro.py): 768 x 3072 0.135 ->
// 0.101 ms, 768 x 2304 0.105 -> 0.083 ms. 1 = no split. RSX_GEMM_SPLITK=0 disables it.
int split_plan(int64_t M, int N, int K) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("RSX_GEMM_SPLITK");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  if (!on || N % kBN || K % kBK || (K == 128 || K == 256 || K == 384)) return 1;
  const int64_t tiles = ((M + kBM - 1) / kBM) * (N / kBN);
  const int cus = num_cus();
  if (tiles >= cus) return 1;
  for (int S : {8, 4, 3, 2})  // K ranges of >= 256: at 192 (K = 768, S = 4) 0.046 vs 0.042 ms unsplit
    if (K % (S * 32) == 0 && K / S >= 256 && tiles * S <= 4LL * cus) return S;
  return 1;
}
}  // namespace

RSX_API int64_t rsx_gemm_x3_split_floats(int64_t M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int S = split_plan(M, N, K);
  return S > 1 ? (int64_t)S * M * N : 0;
}

static int gemm_x3_impl(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, int64_t M,
                        int N, int K, int epi, float* aux, int64_t ldaux, float p_drop, uint64_t seed, float* C,
                        int64_t ldc, float* ws, int64_t ws_floats, void* stream) {
  RSX_ARG(A && B && C, "null tensor");
  RSX_ARG(M >= 0 && N > 0 && K > 0 && N % kBN == 0 && K % kBK == 0, "N must be a multiple of 128, K of 32");
  static_assert(kBK == 16 || kBK == 32, "stage depth 16 or 32");
  RSX_ARG(lda >= K && ldb >= K && ldc >= N && lda % 4 == 0 && ldb % 4 == 0, "bad leading dimensions");
  RSX_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0, "A/B must be 16-byte aligned");
  RSX_ARG(epi == EPI_BIAS || epi == EPI_GELU_DROP || epi == EPI_DGELU_DROP, "epi must be 0, 1 or 2");
  RSX_ARG(epi == EPI_BIAS || (epi == EPI_GELU_DROP && !aux) || (aux && ldaux >= N),
          "the GELU epilogues need aux [M, >=N] (EPI_GELU_DROP: aux may be null for inference)");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0, 1)");
  RSX_ARG(M * (int64_t)N < (1LL << 32), "M * N must be < 2^32 (dropout element index)");
  if (M == 0) return 0;
  GArgs g = {};
  g.A = A; g.B = B; g.bias = bias; g.C = C; g.aux = aux; g.ridx = nullptr;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldaux = ldaux; g.M = M;
  g.N = N; g.K = K; g.epi = epi;
  g.tiles_n = N / kBN;
  const int64_t tiles = ((M + kBM - 1) / kBM) * g.tiles_n;
  RSX_ARG(tiles < (1LL << 30), "too many tiles");
  g.tiles = (int)tiles;
  g.drop = rsx::make_dropout(epi == EPI_BIAS ? 0.0f : p_drop, seed);
  hipStream_t st = (hipStream_t)stream;
  if (ws_enabled() && ldb % 4 == 0) {
    if (K == 128) { launch_ws<1, 128>(g, st); RSX_LAUNCHED(); return 0; }
    if (K == 256) { launch_ws<2, 128>(g, st); RSX_LAUNCHED(); return 0; }
    if (K == 384) { launch_ws<3, 64>(g, st); RSX_LAUNCHED(); return 0; }
  }
  const int S = split_plan(M, N, K);
  if (S > 1 && ws && ws_floats >= (int64_t)S * M * N && ldc >= N) {
    // split-K: (split, tile) workgroups write raw partial sums, then one pass adds them in split order
    // and applies the epilogue (the epilogue form is not instantiated in the partial kernel)
    g.per = 1;
    g.ksplit = S;
    g.kspan = K / S;
    g.part = ws;
    const int64_t blocks = tiles * S;
    const int grid = (int)((blocks + 7) / 8 * 8);
    if (few_bk(g.kspan) == 32) hipLaunchKernelGGL((gemm_x3_nt_k<EPI_BIAS, 4, 32>), dim3(grid), dim3(256), 0, st, g);
    else hipLaunchKernelGGL((gemm_x3_nt_k<EPI_BIAS, 4>), dim3(grid), dim3(256), 0, st, g);
    RSX_LAUNCHED();
    const unsigned rb = (unsigned)((M * (int64_t)N + 255) / 256);
    if (epi == EPI_BIAS) hipLaunchKernelGGL(gemm_splitk_reduce_k<EPI_BIAS>, dim3(rb), dim3(256), 0, st, g);
    else if (epi == EPI_GELU_DROP) hipLaunchKernelGGL(gemm_splitk_reduce_k<EPI_GELU_DROP>, dim3(rb), dim3(256), 0, st, g);
    else hipLaunchKernelGGL(gemm_splitk_reduce_k<EPI_DGELU_DROP>, dim3(rb), dim3(256), 0, st, g);
    RSX_LAUNCHED();
    return 0;
  }
  // tiles per workgroup: enough workgroups for two per CU, each a continuous stage stream
  g.per = (int)((tiles + RSX_GEMM_BLOCKS - 1) / RSX_GEMM_BLOCKS);
  const int64_t blocks = (tiles + g.per - 1) / g.per;
  const int grid = (int)((blocks + 7) / 8 * 8);
  // few tiles for the chip (one workgroup per CU at most) and a long K: four stages in flight per workgroup
  if (deep_prefetch() && g.per == 1 && blocks <= num_cus() && a_nk_long(K)) {
    const bool b32 = few_bk(K) == 32;
    if (epi == EPI_BIAS && b32) hipLaunchKernelGGL((gemm_x3_nt_k<EPI_BIAS, 4, 32>), dim3(grid), dim3(256), 0, st, g);
    else if (epi == EPI_BIAS) hipLaunchKernelGGL((gemm_x3_nt_k<EPI_BIAS, 4>), dim3(grid), dim3(256), 0, st, g);
    else if (epi == EPI_GELU_DROP && b32)
      hipLaunchKernelGGL((gemm_x3_nt_k<EPI_GELU_DROP, 4, 32>), dim3(grid), dim3(256), 0, st, g);
    else if (epi == EPI_GELU_DROP) hipLaunchKernelGGL((gemm_x3_nt_k<EPI_GELU_DROP, 4>), dim3(grid), dim3(256), 0, st, g);
    else hipLaunchKernelGGL(gemm_x3_nt_k<EPI_DGELU_DROP>, dim3(grid), dim3(256), 0, st, g);  // Q = 4 spills here
  } else if (epi == EPI_BIAS) hipLaunchKernelGGL(gemm_x3_nt_k<EPI_BIAS>, dim3(grid), dim3(256), 0, st, g);
  else if (epi == EPI_GELU_DROP) hipLaunchKernelGGL(gemm_x3_nt_k<EPI_GELU_DROP>, dim3(grid), dim3(256), 0, st, g);
  else hipLaunchKernelGGL(gemm_x3_nt_k<EPI_DGELU_DROP>, dim3(grid), dim3(256), 0, st, g);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_gemm_x3(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, int64_t M,
                        int N, int K, int epi, float* aux, int64_t ldaux, float p_drop, uint64_t seed, float* C,
                        int64_t ldc, void* stream) {
  return gemm_x3_impl(A, lda, B, ldb, bias, M, N, K, epi, aux, ldaux, p_drop, seed, C, ldc, nullptr, 0, stream);
}

RSX_API int rsx_gemm_x3_ws(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, int64_t M,
                           int N, int K, int epi, float* aux, int64_t ldaux, float p_drop, uint64_t seed, float* C,
                           int64_t ldc, float* ws, int64_t ws_floats, void* stream) {
  return gemm_x3_impl(A, lda, B, ldb, bias, M, N, K, epi, aux, ldaux, p_drop, seed, C, ldc, ws, ws_floats, stream);
}

// C = epi(A . Bt + bias) with the right operand as stored, Bt [K, N] (row stride ldbt >= N): the
// input gradient dX = dY . W of a token linear straight from its weight W [out, in] (K = out,
// N = in), without a transposed copy of W per call; epi as rsx_gemm_x3 (EPI_DGELU_DROP: the
// feed-forward's dPre = (dF . W2) * keep / (1 - p) * gelu'). Weight-stationary path: K in
// {128, 256, 384}, N % 128 == 0 (the staging reads W's columns; it runs once per workgroup).
RSX_API int rsx_gemm_x3_tn(const float* A, int64_t lda, const float* Bt, int64_t ldbt, const float* bias, int64_t M,
                           int N, int K, int epi, float* aux, int64_t ldaux, float p_drop, uint64_t seed, float* C,
                           int64_t ldc, void* stream) {
  RSX_ARG(A && Bt && C, "null tensor");
  RSX_ARG(M >= 0 && N > 0 && N % 128 == 0 && (K == 128 || K == 256 || K == 384),
          "N must be a multiple of 128, K 128, 256 or 384");
  RSX_ARG(lda >= K && ldbt >= N && ldc >= N && lda % 4 == 0 && ldc % 4 == 0, "bad leading dimensions");
  RSX_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)C % 16) == 0, "A/C must be 16-byte aligned");
  RSX_ARG(epi == EPI_BIAS || epi == EPI_GELU_DROP || epi == EPI_DGELU_DROP, "epi must be 0, 1 or 2");
  RSX_ARG(epi == EPI_BIAS || (epi == EPI_GELU_DROP && !aux) || (aux && ldaux >= N),
          "the GELU epilogues need aux [M, >=N] (EPI_GELU_DROP: aux may be null for inference)");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0, 1)");
  RSX_ARG(M * (int64_t)N < (1LL << 32), "M * N must be < 2^32 (dropout element index)");
  if (M == 0) return 0;
  GArgs g = {};
  g.A = A; g.B = Bt; g.bias = bias; g.C = C; g.aux = aux; g.ridx = nullptr;
  g.lda = lda; g.ldb = ldbt; g.ldc = ldc; g.ldaux = ldaux; g.M = M;
  g.N = N; g.K = K; g.epi = epi; g.transb = 1;
  g.drop = rsx::make_dropout(epi == EPI_BIAS ? 0.0f : p_drop, seed);
  hipStream_t st = (hipStream_t)stream;
  if (K == 128) launch_ws<1, 128>(g, st);
  else if (K == 256) launch_ws<2, 128>(g, st);
  else launch_ws<3, 64>(g, st);
  RSX_LAUNCHED();
  return 0;
}

// C[m] = A[m] . B^T + bias + R[ridx[m]]  (a per-row table added in the epilogue: the user
// tower's output_proj[0] over the packed tokens plus its per-user profile half,
// v1_refine_usertower.py:498-505). K in {128, 256} (weight-stationary path), N % 128 == 0.
RSX_API int rsx_gemm_x3_rowadd(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
                               int64_t M, int N, int K, const float* R, int64_t ldr, const int64_t* ridx, float* C,
                               int64_t ldc, void* stream) {
  RSX_ARG(A && B && C && R && ridx, "null tensor");
  RSX_ARG(M >= 0 && N > 0 && N % 128 == 0 && (K == 128 || K == 256), "N must be a multiple of 128, K 128 or 256");
  RSX_ARG(lda >= K && ldb >= K && ldc >= N && ldr >= N && lda % 4 == 0 && ldb % 4 == 0 && ldr % 4 == 0 &&
              ldc % 4 == 0, "bad leading dimensions");
  RSX_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0 && ((uintptr_t)R % 16) == 0 &&
              ((uintptr_t)C % 16) == 0, "A/B/R/C must be 16-byte aligned");
  if (M == 0) return 0;
  GArgs g = {};
  g.A = A; g.B = B; g.bias = bias; g.C = C; g.aux = const_cast<float*>(R); g.ridx = ridx;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldaux = ldr; g.M = M;
  g.N = N; g.K = K; g.epi = EPI_ROWADD;
  g.drop = rsx::make_dropout(0.0f, 0);
  hipStream_t st = (hipStream_t)stream;
  if (K == 128) launch_ws<1, 128>(g, st);
  else launch_ws<2, 128>(g, st);
  RSX_LAUNCHED();
  return 0;
}

// s = X + dropout_p(A . B^T + bias), y = LayerNorm(s) (ln_w, ln_b, eps), mean / rstd per row:
// the attention out-projection of a norm_first encoder layer fused with the residual add and the
// LayerNorm after it (v1_refine_usertower.py:343-352: x = x + drop(out_proj(mha(...)));
// norm2(x)). N = 128 (one column block holds the whole row), K in {128, 256}. The dropout mask
// is rsx_ln_fwd's (hash of m * N + n), so rsx_ln_bwd's backward of the add + LayerNorm applies.
RSX_API int rsx_gemm_x3_addln(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
                              int64_t M, int N, int K, const float* X, int64_t ldx, float p_drop, uint64_t seed,
                              const float* ln_w, const float* ln_b, float eps, float* S, int64_t lds, float* Y,
                              int64_t ldy, float* mean, float* rstd, void* stream) {
  RSX_ARG(A && B && X && S && Y && mean && rstd, "null tensor");
  RSX_ARG(M >= 0 && N == 128 && (K == 128 || K == 256), "N must be 128, K 128 or 256");
  RSX_ARG(lda >= K && ldb >= K && ldx >= N && lds >= N && ldy >= N && lda % 4 == 0 && ldb % 4 == 0 &&
              ldx % 4 == 0 && lds % 4 == 0 && ldy % 4 == 0, "bad leading dimensions");
  RSX_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0 && ((uintptr_t)X % 16) == 0 &&
              ((uintptr_t)S % 16) == 0 && ((uintptr_t)Y % 16) == 0, "A/B/X/S/Y must be 16-byte aligned");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0, 1)");
  RSX_ARG(M * (int64_t)N < (1LL << 32), "M * N must be < 2^32 (dropout element index)");
  RSX_ARG(eps > 0.0f, "eps must be positive");
  if (M == 0) return 0;
  GArgs g = {};
  g.A = A; g.B = B; g.bias = bias; g.C = S; g.aux = const_cast<float*>(X); g.ridx = nullptr;
  g.y = Y; g.ln_w = ln_w; g.ln_b = ln_b; g.mean = mean; g.rstd = rstd; g.eps = eps; g.ldy = ldy;
  g.lda = lda; g.ldb = ldb; g.ldc = lds; g.ldaux = ldx; g.M = M;
  g.N = N; g.K = K; g.epi = EPI_ADDLN;
  g.drop = rsx::make_dropout(p_drop, seed);
  hipStream_t st = (hipStream_t)stream;
  if (K == 128) launch_ws<1, 128>(g, st);
  else launch_ws<2, 128>(g, st);
  RSX_LAUNCHED();
  return 0;
}
