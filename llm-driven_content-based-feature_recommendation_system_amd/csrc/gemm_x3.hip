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
//
// Tiling: 128 x 128 output tile per 256-thread workgroup (four waves of 64 x 64 = 2 x 2
// MFMA tiles), K staged 16 at a time, double-buffered in LDS with register prefetch and one
// barrier per stage. LDS rows are 16 bf16 + 8 pad (48 B): the fragment reads (ds_read_b128,
// 32 rows x 16 B per lane half) are bank-conflict free, and 48 KB per workgroup leaves room
// for three workgroups per CU (the GEMMs are latency-bound at two). XCD-aware order: the N tiles of one
// M block run back to back on one XCD, so A's rows are re-read from that XCD's L2.
#include "rsx_common.h"

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
constexpr int EPI_BIAS = 0, EPI_GELU_DROP = 1, EPI_DGELU_DROP = 2;
#ifndef RSX_GEMM_BLOCKS
#define RSX_GEMM_BLOCKS (1 << 30)  // workgroup budget of the multi-tile stream: at BK 16 one tile each measured best
#endif

__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

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

struct Img {
  __bf16 hi[kBM * kRow];
  __bf16 lo[kBM * kRow];
};

struct GArgs {
  const float* A;     // [M, lda]
  const float* B;     // [N, ldb]
  const float* bias;  // [N] (nullable)
  float* C;           // [M, ldc]
  float* aux;         // [M, ldaux]: gelu'(pre) (written by EPI_GELU_DROP, read by EPI_DGELU_DROP)
  int64_t lda, ldb, ldc, ldaux, M;
  int N, K, epi, tiles_n, tiles, per;
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
          a.aux[m * a.ldaux + n] = cdf + v * 0.3989422804014327f * __expf(-0.5f * v * v);  // gelu'(v)
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
template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_x3_nt_k(GArgs a) {
  __shared__ __attribute__((aligned(16))) Img sA[2];
  __shared__ __attribute__((aligned(16))) Img sB[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware block order (the grid is padded to a multiple of 8)
  const int bflat = (blockIdx.x & 7) * ((int)gridDim.x >> 3) + (blockIdx.x >> 3);
  const int t_begin = bflat * a.per;
  int t_end = t_begin + a.per;
  if (t_end > a.tiles) t_end = a.tiles;
  if (t_begin >= t_end) return;
  const int nk = a.K / kBK;
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
  const int srow = tid >> 1, scol = (tid & 1) * (kBK / 2);
  float4 pa[kF4], pb[kF4];
  auto gload = [&](int st) {
    const int t = t_begin + st / nk, k0 = (st % nk) * kBK;
    const int64_t m0 = (int64_t)(t / a.tiles_n) * kBM;
    const int n0 = (t % a.tiles_n) * kBN;
    const float* a_src = a.A + (m0 + srow < a.M ? m0 + srow : m0) * a.lda + scol + k0;
    const float* b_src = a.B + (int64_t)(n0 + srow) * a.ldb + scol + k0;
#pragma unroll
    for (int q = 0; q < kF4; ++q) {
      pa[q] = *reinterpret_cast<const float4*>(a_src + 4 * q);
      pb[q] = *reinterpret_cast<const float4*>(b_src + 4 * q);
    }
  };
  auto lstore = [&](int buf) {
    const int o = srow * kRow + scol;
#pragma unroll
    for (int q = 0; q < kF4 / 2; ++q) {
      u32x4 hi, lo;
      split8(pa[2 * q], pa[2 * q + 1], hi, lo);
      *reinterpret_cast<u32x4*>(&sA[buf].hi[o + 8 * q]) = hi;
      *reinterpret_cast<u32x4*>(&sA[buf].lo[o + 8 * q]) = lo;
      split8(pb[2 * q], pb[2 * q + 1], hi, lo);
      *reinterpret_cast<u32x4*>(&sB[buf].hi[o + 8 * q]) = hi;
      *reinterpret_cast<u32x4*>(&sB[buf].lo[o + 8 * q]) = lo;
    }
  };

  gload(0);
  lstore(0);
  __syncthreads();
  int cur = 0;
  for (int st = 0; st < nstage; ++st) {
    const bool has_next = st + 1 < nstage;
    if (has_next) gload(st + 1);
    const Img& ta = sA[cur];
    const Img& tb = sB[cur];
#pragma unroll
    for (int ks = 0; ks < kBK / 16; ++ks) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int oa = (wm * 64 + 32 * i + c) * kRow + 16 * ks + 8 * h;
        const int ob = (wn * 64 + 32 * i + c) * kRow + 16 * ks + 8 * h;
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
    if (st % nk == nk - 1) {  // tile finished: epilogue (resets acc) while the next stage loads
      const int t = t_begin + st / nk;
      epilogue<EPI>(a, acc, (int64_t)(t / a.tiles_n) * kBM, (t % a.tiles_n) * kBN, wm, wn, h, c);
    }
    if (has_next) lstore(cur ^ 1);  // cur^1 was read in the previous stage, fenced by its barrier
    __syncthreads();
    cur ^= 1;
  }
}

}  // namespace

RSX_API int rsx_gemm_x3(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, int64_t M,
                        int N, int K, int epi, float* aux, int64_t ldaux, float p_drop, uint64_t seed, float* C,
                        int64_t ldc, void* stream) {
  RSX_ARG(A && B && C, "null tensor");
  RSX_ARG(M >= 0 && N > 0 && K > 0 && N % kBN == 0 && K % kBK == 0, "N must be a multiple of 128, K of 32");
  static_assert(kBK == 16 || kBK == 32, "stage depth 16 or 32");
  RSX_ARG(lda >= K && ldb >= K && ldc >= N && lda % 4 == 0 && ldb % 4 == 0, "bad leading dimensions");
  RSX_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0, "A/B must be 16-byte aligned");
  RSX_ARG(epi == EPI_BIAS || epi == EPI_GELU_DROP || epi == EPI_DGELU_DROP, "epi must be 0, 1 or 2");
  RSX_ARG(epi == EPI_BIAS || (aux && ldaux >= N), "the GELU epilogues need aux [M, >=N]");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0, 1)");
  RSX_ARG(M * (int64_t)N < (1LL << 32), "M * N must be < 2^32 (dropout element index)");
  if (M == 0) return 0;
  GArgs g;
  g.A = A; g.B = B; g.bias = bias; g.C = C; g.aux = aux;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldaux = ldaux; g.M = M;
  g.N = N; g.K = K; g.epi = epi;
  g.tiles_n = N / kBN;
  const int64_t tiles = ((M + kBM - 1) / kBM) * g.tiles_n;
  RSX_ARG(tiles < (1LL << 30), "too many tiles");
  g.tiles = (int)tiles;
  g.drop = rsx::make_dropout(epi == EPI_BIAS ? 0.0f : p_drop, seed);
  // tiles per workgroup: enough workgroups for two per CU, each a continuous stage stream
  g.per = (int)((tiles + RSX_GEMM_BLOCKS - 1) / RSX_GEMM_BLOCKS);
  const int64_t blocks = (tiles + g.per - 1) / g.per;
  const int grid = (int)((blocks + 7) / 8 * 8);
  hipStream_t st = (hipStream_t)stream;
  if (epi == EPI_BIAS) hipLaunchKernelGGL(gemm_x3_nt_k<EPI_BIAS>, dim3(grid), dim3(256), 0, st, g);
  else if (epi == EPI_GELU_DROP) hipLaunchKernelGGL(gemm_x3_nt_k<EPI_GELU_DROP>, dim3(grid), dim3(256), 0, st, g);
  else hipLaunchKernelGGL(gemm_x3_nt_k<EPI_DGELU_DROP>, dim3(grid), dim3(256), 0, st, g);
  RSX_LAUNCHED();
  return 0;
}
