// Weight / bias gradient of a token-level linear layer Y = X W^T + b:
//
//   dW[n][k] = sum_t dY[t][n] * X[t][k]        db[n] = sum_t dY[t][n]
//
// Reference: every nn.Linear / F.linear applied per token in the user tower's training step
// (tower_code/v1_refine_usertower.py:447-510: item_proj, the encoder layers' in_proj /
// out_proj / linear1 / linear2, output_proj) — autograd's weight-gradient GEMM. T (tokens,
// ~80k per view at batch 4096) is the reduction axis and N x K (<= 384 x 256) is tiny, which
// library GEMMs tile with only a few dozen workgroups. Here the reduction is split over
// tokens (split-K) into >= 512 workgroups; each writes its 128x128 partial and a second
// kernel sums the partials in a fixed order (deterministic, no atomics).
//
// Compute: fp32-input MFMA (v_mfma_f32_32x32x2_f32, exact fp32 products) — the same
// arithmetic as the fp32 GEMM it replaces. Each wave owns a 64x64 block of the 128x128 tile
// (4 accumulators; one A and one B fragment feed two MFMAs each). 32-token stages of dY and
// X are staged through LDS, double-buffered with register prefetch, one barrier per stage.
// The A operand of token pair (2s, 2s+1) is dY[2s+h][n] on lane (n, h): a plain row read of
// the token-major LDS tile, so no transpose is needed anywhere.
#include "rsx_common.h"
#include <stdlib.h>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kTile = 128;   // output tile (n and k)
constexpr int kStage = 32;   // tokens per LDS stage

__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

struct WArgs {
  const float* dY;  // [T, ldy], columns 0..N-1
  const float* X;   // [T, ldx], columns 0..K-1
  int64_t ldy, ldx, T;
  int N, K, tiles_n, tiles_k, nsplit;
  int64_t span;     // tokens per split (multiple of kStage)
  float* part;      // [nsplit][N*K + N]: dW partial, then db partial
  bool with_db;
};

__global__ __launch_bounds__(256, 2) void wgrad_k(WArgs a) {
  __shared__ __attribute__((aligned(16))) float sY[2][kStage][kTile];
  __shared__ __attribute__((aligned(16))) float sX[2][kStage][kTile];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  // XCD-aware order: the tiles of one split (same token rows) run on one XCD (b % 8)
  const int total = a.tiles_n * a.tiles_k * a.nsplit;
  const int flat = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  const int tiles = a.tiles_n * a.tiles_k;
  const int split = flat / tiles, tile = flat % tiles;
  const int n0 = (tile / a.tiles_k) * kTile, k0 = (tile % a.tiles_k) * kTile;
  const int64_t t_begin = (int64_t)split * a.span;
  int64_t t_end = t_begin + a.span;
  if (t_end > a.T) t_end = a.T;
  const int wn = wave >> 1, wk = wave & 1;
  const bool live = (n0 + wn * 64 < a.N) && (k0 + wk * 64 < a.K);  // wave-uniform
  const bool do_db = a.with_db && k0 == 0;
  const int64_t pstride = (int64_t)a.N * a.K + a.N;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  float dbsum = 0.0f;

  // staging: thread tid -> token row tid>>3, 16 columns from (tid&7)*16, for dY and X
  const int srow = tid >> 3, scol = (tid & 7) * 16;
  float4 py[4], px[4];
  auto gload = [&](int64_t t0) {
    const int64_t t = t0 + srow;
    const bool ok = t < t_end;
    const bool oky = ok && n0 + scol < a.N;
    const bool okx = ok && k0 + scol < a.K;
    const float4* ys = reinterpret_cast<const float4*>(a.dY + (oky ? t : 0) * a.ldy + n0 + scol);
    const float4* xs = reinterpret_cast<const float4*>(a.X + (okx ? t : 0) * a.ldx + k0 + scol);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      py[q] = oky ? ys[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      px[q] = okx ? xs[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      *reinterpret_cast<float4*>(&sY[buf][srow][scol + 4 * q]) = py[q];
      *reinterpret_cast<float4*>(&sX[buf][srow][scol + 4 * q]) = px[q];
    }
  };

  if (t_begin < t_end) {
    gload(t_begin);
    lstore(0);
    __syncthreads();
    int cur = 0;
    for (int64_t t0 = t_begin; t0 < t_end; t0 += kStage) {
      const bool has_next = t0 + kStage < t_end;
      if (has_next) gload(t0 + kStage);
      if (live) {
        const float* yrow = &sY[cur][h][wn * 64 + c];
        const float* xrow = &sX[cur][h][wk * 64 + c];
#pragma unroll
        for (int s = 0; s < kStage / 2; ++s) {
          const float a0 = yrow[2 * s * kTile], a1 = yrow[2 * s * kTile + 32];
          const float b0 = xrow[2 * s * kTile], b1 = xrow[2 * s * kTile + 32];
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
      }
      if (do_db && tid < kTile) {
#pragma unroll 8
        for (int t = 0; t < kStage; ++t) dbsum += sY[cur][t][tid];
      }
      if (has_next) lstore(cur ^ 1);  // cur^1 was read in the previous stage, fenced by its barrier
      __syncthreads();
      cur ^= 1;
    }
  }
  if (live) {
    float* dst = a.part + split * pstride;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = k0 + wk * 64 + j * 32 + c;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int n = n0 + wn * 64 + i * 32 + tile_row(r, h);
          if (n < a.N && k < a.K) dst[(int64_t)n * a.K + k] = acc[i][j][r];
        }
      }
  }
  if (do_db && tid < kTile && n0 + tid < a.N) a.part[split * pstride + (int64_t)a.N * a.K + n0 + tid] = dbsum;
}

// bf16x3 form (rsx_linear_wgrad_x3): the staged dY / X stages are split into hi/lo bf16
// images (x = hi + lo) as they are written to LDS, and every product is hi*hi' + hi*lo' +
// lo*hi' on v_mfma_f32_32x32x16_bf16 (fp32 accumulate; the arithmetic of infonce.hip's
// bf16x3 loss). Both MFMA operands have the token axis as their k index, so both come from
// ds_read_b64_tr_b16 transposed reads of the token-major images: lane (c, h) element j of
// k-step ks is token 16ks + 8(j>>2) + 4h + (j&3), column c of the 32-wide block. Image
// layout (as infonce.hip): 320-B rows + a 16-B skew per 8 rows, conflict-free for the
// transposed reads. db is summed in fp32 from the staged registers.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kImgRow = 160;
__device__ __forceinline__ int img_off(int row, int col) { return row * kImgRow + 8 * (row >> 3) + col; }
// One staged operand: STAGE tokens x 128 columns as bf16 hi/lo images (row stride 160 + 8 per 8 rows).
template <int STAGE>
struct X3Img {
  static constexpr int kElems = STAGE * kImgRow;  // covers img_off(STAGE - 1, 127)
  static_assert((STAGE - 1) * kImgRow + 8 * ((STAGE - 1) >> 3) + 128 <= kElems, "image size");
  __bf16 hi[kElems];
  __bf16 lo[kElems];
};

__device__ __forceinline__ void split8(const float4& a, const float4& b, u32x4& hi, u32x4& lo) {
  const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
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

// STAGE = tokens per LDS stage: 32 (80 KB LDS, two workgroups per CU) or 16 (40 KB, three).
template <int STAGE>
__global__ __launch_bounds__(256, 2) void wgrad_x3_k(WArgs a) {
  constexpr int kStageX3 = STAGE;
  constexpr int kFpt = STAGE / 2;  // floats per thread and operand per stage (256 threads, 128 columns)
  __shared__ __attribute__((aligned(16))) X3Img<STAGE> sY[2];
  __shared__ __attribute__((aligned(16))) X3Img<STAGE> sX[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int total = a.tiles_n * a.tiles_k * a.nsplit;
  const int flat = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  const int tiles = a.tiles_n * a.tiles_k;
  const int split = flat / tiles, tile = flat % tiles;
  const int n0 = (tile / a.tiles_k) * kTile, k0 = (tile % a.tiles_k) * kTile;
  const int64_t t_begin = (int64_t)split * a.span;
  int64_t t_end = t_begin + a.span;
  if (t_end > a.T) t_end = a.T;
  const int wn = wave >> 1, wk = wave & 1;
  const bool live = (n0 + wn * 64 < a.N) && (k0 + wk * 64 < a.K);  // wave-uniform
  const bool do_db = a.with_db && k0 == 0;
  const int64_t pstride = (int64_t)a.N * a.K + a.N;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  float dbp[kFpt];
#pragma unroll
  for (int q = 0; q < kFpt; ++q) dbp[q] = 0.0f;

  const int srow = tid / (kTile / kFpt), scol = (tid % (kTile / kFpt)) * kFpt;
  // two register sets: stage s + 2 is in flight while stage s is multiplied and stage s + 1
  // is converted into LDS (one stage in flight left each workgroup waiting on HBM latency)
  float4 py0[kFpt / 4], px0[kFpt / 4], py1[kFpt / 4], px1[kFpt / 4];
  auto gload = [&](int64_t t0, float4 (&py)[kFpt / 4], float4 (&px)[kFpt / 4]) {
    const int64_t t = t0 + srow;
    const bool ok = t < t_end;
    const bool oky = ok && n0 + scol < a.N;
    const bool okx = ok && k0 + scol < a.K;
    const float4* ys = reinterpret_cast<const float4*>(a.dY + (oky ? t : 0) * a.ldy + n0 + scol);
    const float4* xs = reinterpret_cast<const float4*>(a.X + (okx ? t : 0) * a.ldx + k0 + scol);
    // unconditional loads (from row 0 when out of range), zeroed by a select afterwards: a
    // predicated load is a branch per load
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < kFpt / 4; ++q) {
      const float4 vy = ys[q], vx = xs[q];
      py[q] = oky ? vy : z;
      px[q] = okx ? vx : z;
    }
  };
  auto lstore = [&](int buf, const float4 (&py)[kFpt / 4], const float4 (&px)[kFpt / 4]) {
#pragma unroll
    for (int q = 0; q < kFpt / 8; ++q) {
      const int o = img_off(srow, scol + 8 * q);
      u32x4 hi, lo;
      split8(py[2 * q], py[2 * q + 1], hi, lo);
      *reinterpret_cast<u32x4*>(&sY[buf].hi[o]) = hi;
      *reinterpret_cast<u32x4*>(&sY[buf].lo[o]) = lo;
      split8(px[2 * q], px[2 * q + 1], hi, lo);
      *reinterpret_cast<u32x4*>(&sX[buf].hi[o]) = hi;
      *reinterpret_cast<u32x4*>(&sX[buf].lo[o]) = lo;
    }
    if (do_db) {
#pragma unroll
      for (int q = 0; q < kFpt / 4; ++q) {
        dbp[4 * q] += py[q].x;
        dbp[4 * q + 1] += py[q].y;
        dbp[4 * q + 2] += py[q].z;
        dbp[4 * q + 3] += py[q].w;
      }
    }
  };
  // transposed fragment reads: lane (c, h) gets column 32nb + c of tokens 16ks + 8(j>>2) + 4h + (j&3)
  const int q4 = (lane >> 2) & 3, p4 = lane & 3, cb = (lane >> 4) & 1;
  const int tbase = img_off(4 * h + q4, 16 * cb + 4 * p4);
  auto rd = [&](const __bf16* img, int ks, int nb) -> bf16x8 {
    const int o0 = tbase + img_off(16 * ks, 32 * nb), o1 = tbase + img_off(16 * ks + 8, 32 * nb);
    const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(&img[o0]));
    const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(&img[o1]));
    return __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto compute = [&](int cur) {
    if (!live) return;
#pragma unroll
    for (int ks = 0; ks < kStageX3 / 16; ++ks) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = rd(sY[cur].hi, ks, 2 * wn + i);
        al[i] = rd(sY[cur].lo, ks, 2 * wn + i);
        bh[i] = rd(sX[cur].hi, ks, 2 * wk + i);
        bl[i] = rd(sX[cur].lo, ks, 2 * wk + i);
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
  };

  if (t_begin < t_end) {
    // stage s lives in LDS buffer s & 1; even stages load into set 0, odd into set 1. Loads past
    // t_end read row 0 and are zeroed (never stored: the loop ends first).
    const int nst = (int)((t_end - t_begin + kStageX3 - 1) / kStageX3);
    gload(t_begin, py0, px0);
    gload(t_begin + kStageX3, py1, px1);
    lstore(0, py0, px0);
    __syncthreads();
    for (int st = 0;; st += 2) {
      gload(t_begin + (int64_t)(st + 2) * kStageX3, py0, px0);
      compute(0);
      if (st + 1 >= nst) break;
      lstore(1, py1, px1);
      __syncthreads();
      gload(t_begin + (int64_t)(st + 3) * kStageX3, py1, px1);
      compute(1);
      if (st + 2 >= nst) break;
      lstore(0, py0, px0);
      __syncthreads();
    }
  }
  // the loop leaves after a compute without a barrier: the db reduction below reuses sY[0]
  __syncthreads();
  if (live) {
    float* dst = a.part + split * pstride;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = k0 + wk * 64 + j * 32 + c;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int n = n0 + wn * 64 + i * 32 + tile_row(r, h);
          if (n < a.N && k < a.K) dst[(int64_t)n * a.K + k] = acc[i][j][r];
        }
      }
  }
  if (do_db) {
    // column sums of the 32 token rows: threads with equal tid&7 hold the same 16 columns
    float* red = reinterpret_cast<float*>(&sY[0]);  // free after the loop's last barrier (>= kStageX3 x 128 floats)
#pragma unroll
    for (int q = 0; q < kFpt; ++q) red[srow * kTile + scol + q] = dbp[q];
    __syncthreads();
    if (tid < kTile) {
      float s = 0.0f;
#pragma unroll 8
      for (int t = 0; t < kStageX3; ++t) s += red[t * kTile + tid];
      if (n0 + tid < a.N) a.part[split * pstride + (int64_t)a.N * a.K + n0 + tid] = s;
    }
  }
}

// Deterministic split reduction. A workgroup owns 16 consecutive float4 granules of the
// per-split vector [dW (N*K) | db (N)]; its 16 thread groups each sum the splits g, g+16, ...
// (many independent loads in flight per thread), then group 0 adds the 16 group sums in
// order. Output granule e < N*K/4 goes to dW (row stride ldw), the rest to db.
__global__ __launch_bounds__(256) void wgrad_reduce_k(const float* part, int nsplit, int64_t n4, int64_t pstride4,
                                                      int N, int K, float* dW, int64_t ldw, float* db,
                                                      int accumulate) {
  __shared__ float4 red[16][16];
  const int o = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + o;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    const float4* p = reinterpret_cast<const float4*>(part) + i;
#pragma unroll 4
    for (int k = g; k < nsplit; k += 16) {
      const float4 v = p[k * pstride4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[g][o] = s;
  __syncthreads();
  if (g != 0 || i >= n4) return;
#pragma unroll
  for (int k = 1; k < 16; ++k) {
    const float4 v = red[k][o];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const int64_t e = i * 4, nk = (int64_t)N * K;
  float4* dst;
  if (e < nk) {
    dst = reinterpret_cast<float4*>(dW + (e / K) * ldw + e % K);
  } else {
    if (!db) return;
    dst = reinterpret_cast<float4*>(db + (e - nk));
  }
  if (accumulate) {
    const float4 v = *dst;
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  *dst = s;
}

int choose_nsplit(int64_t T, int tiles) {
  int ns = (512 + tiles - 1) / tiles;
  const int64_t max_ns = T / (2 * kStage);  // at least two stages per split
  if (ns > max_ns) ns = (int)max_ns;
  ns = (ns + 7) / 8 * 8;
  return ns < 8 ? 8 : ns;
}

}  // namespace

RSX_API int64_t rsx_linear_wgrad_workspace_floats(int64_t T, int64_t N, int64_t K) {
  const int tiles = (int)(((N + kTile - 1) / kTile) * ((K + kTile - 1) / kTile));
  const int ns = choose_nsplit(T, tiles);
  return (int64_t)ns * (N * K + N) + 64;
}

namespace {
int wgrad_launch(bool x3, const float* dY, int64_t ldy, const float* X, int64_t ldx, int64_t T, int64_t N,
                             int64_t K, float* dW, int64_t ldw, float* db, int accumulate, float* ws,
                             int64_t ws_floats, void* stream) {
  RSX_ARG(((dY && X) || T == 0) && dW && ws, "null tensor");
  RSX_ARG(T >= 0, "T must be >= 0");
  RSX_ARG(N > 0 && K > 0 && N % 16 == 0 && K % 16 == 0 && N <= 4096 && K <= 4096,
          "N and K must be positive multiples of 16 (<= 4096)");
  RSX_ARG(ldy >= N && ldx >= K && ldw >= K && ldy % 4 == 0 && ldx % 4 == 0 && ldw % 4 == 0,
          "row strides must cover the row and be multiples of 4");
  RSX_ARG(((uintptr_t)dY % 16) == 0 && ((uintptr_t)X % 16) == 0 && ((uintptr_t)dW % 16) == 0,
          "dY/X/dW must be 16-byte aligned");
  RSX_ARG(ws_floats >= rsx_linear_wgrad_workspace_floats(T, N, K), "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  WArgs a;
  a.dY = dY; a.X = X; a.ldy = ldy; a.ldx = ldx; a.T = T;
  a.N = (int)N; a.K = (int)K;
  a.tiles_n = (int)((N + kTile - 1) / kTile);
  a.tiles_k = (int)((K + kTile - 1) / kTile);
  a.nsplit = choose_nsplit(T, a.tiles_n * a.tiles_k);
  a.span = ((T + a.nsplit - 1) / a.nsplit + kStage - 1) / kStage * kStage;
  if (a.span < kStage) a.span = kStage;
  a.part = ws;
  a.with_db = db != nullptr;
  const int blocks = a.tiles_n * a.tiles_k * a.nsplit;
  // 16-token stages measured faster for three or more output row tiles (tools/gemm_micro.py wgrad_384x128:
  // 0.119 vs 0.146 ms) and slower for fewer (wgrad_128x256: 0.075 vs 0.068 ms).
  static const int stage16_min_tiles = [] {  // RSX_WGRAD_STAGE16_TILES: A/B of the stage choice
    const char* e = getenv("RSX_WGRAD_STAGE16_TILES");
    return e ? atoi(e) : 3;
  }();
  if (x3 && a.tiles_n >= stage16_min_tiles) hipLaunchKernelGGL(wgrad_x3_k<16>, dim3(blocks), dim3(256), 0, st, a);
  else if (x3) hipLaunchKernelGGL(wgrad_x3_k<32>, dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(wgrad_k, dim3(blocks), dim3(256), 0, st, a);
  RSX_LAUNCHED();
  const int64_t pstride4 = (N * K + N) / 4;
  const int64_t n4 = db ? pstride4 : N * K / 4;
  hipLaunchKernelGGL(wgrad_reduce_k, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, st, a.part, a.nsplit, n4,
                     pstride4, (int)N, (int)K, dW, ldw, db, accumulate);
  RSX_LAUNCHED();
  return 0;
}
}  // namespace

RSX_API int rsx_linear_wgrad(const float* dY, int64_t ldy, const float* X, int64_t ldx, int64_t T, int64_t N,
                             int64_t K, float* dW, int64_t ldw, float* db, int accumulate, float* ws,
                             int64_t ws_floats, void* stream) {
  return wgrad_launch(false, dY, ldy, X, ldx, T, N, K, dW, ldw, db, accumulate, ws, ws_floats, stream);
}

RSX_API int rsx_linear_wgrad_x3(const float* dY, int64_t ldy, const float* X, int64_t ldx, int64_t T, int64_t N,
                                int64_t K, float* dW, int64_t ldw, float* db, int accumulate, float* ws,
                                int64_t ws_floats, void* stream) {
  return wgrad_launch(true, dY, ldy, X, ldx, T, N, K, dW, ldw, db, accumulate, ws, ws_floats, stream);
}
