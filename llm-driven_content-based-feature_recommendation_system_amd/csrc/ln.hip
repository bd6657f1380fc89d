// LayerNorm over the last dim of token rows, fused with the residual add + dropout that
// precedes it and the GELU that may follow it:
//
//   s = x + dropout(res)         (res nullable: s = x)
//   y = act(LN(s) * w + b)       act: 0 none, 2 GELU (erf form, torch default)
//
// Reference: the norm_first nn.TransformerEncoderLayer of the user tower
// (tower_code/v1_refine_usertower.py:40-50: x + dropout(sa(norm1(x))), norm2, ...) and the
// output head Linear -> LayerNorm -> GELU (:68-72, 499-510). The backward returns the
// gradient of s (plus an optional incoming residual-path gradient), the dropout-masked
// gradient of res, and dw/db through per-block partials summed in a fixed order.
//
// A row of D fp32 is owned by D/4 lanes (one float4 each); row statistics are two-pass
// (mean, then centred variance) in fp32. Dropout keeps element (row, col) iff the counter
// hash of (seed, row*D + col) passes (rsx_common.h): the same mask in forward and backward.
#include "rsx_common.h"
#include <math.h>

namespace {

template <int D>
struct Geo {
  static constexpr int LPR = D / 4;
  static constexpr int RPW = 64 / LPR;
};

__device__ __forceinline__ float gelu_erf(float z) { return 0.5f * z * (1.0f + erff(z * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float z) {
  const float cdf = 0.5f * (1.0f + erff(z * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * z * z);
  return cdf + z * pdf;
}

struct FArgs {
  const float* x;
  const float* res;
  const float* w;
  const float* b;
  float* sum_out;
  float* y;
  float* mean;
  float* rstd;
  int64_t T;
  float eps;
  int act;
  rsx::Dropout drop;
};

template <int D>
__global__ __launch_bounds__(256) void ln_fwd_k(FArgs a) {
  constexpr int LPR = Geo<D>::LPR, RPW = Geo<D>::RPW;
  const int lane = threadIdx.x & 63, sub = lane / LPR, c = lane % LPR;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const float4 w = a.w ? reinterpret_cast<const float4*>(a.w)[c] : make_float4(1.f, 1.f, 1.f, 1.f);
  const float4 b = a.b ? reinterpret_cast<const float4*>(a.b)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t r0 = wave_g * RPW; r0 < a.T; r0 += nw * RPW) {
    const int64_t r = r0 + sub;
    if (r >= a.T) continue;  // row groups are lane-aligned: the shuffles below stay in the group
    float4 s = reinterpret_cast<const float4*>(a.x + r * D)[c];
    if (a.res) {
      float4 q = reinterpret_cast<const float4*>(a.res + r * D)[c];
      const uint64_t bi = (uint64_t)r * D + 4 * c;
      q.x = a.drop.apply(q.x, bi + 0);
      q.y = a.drop.apply(q.y, bi + 1);
      q.z = a.drop.apply(q.z, bi + 2);
      q.w = a.drop.apply(q.w, bi + 3);
      s.x += q.x; s.y += q.y; s.z += q.z; s.w += q.w;
      if (a.sum_out) reinterpret_cast<float4*>(a.sum_out + r * D)[c] = s;
    }
    if (!a.y) continue;  // residual add + dropout only (the encoder's last residual)
    const float mu = rsx::wave_sum_width((s.x + s.y) + (s.z + s.w), LPR) * (1.0f / D);
    const float4 d = make_float4(s.x - mu, s.y - mu, s.z - mu, s.w - mu);
    const float var = rsx::wave_sum_width(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w, LPR) * (1.0f / D);
    const float rs = 1.0f / sqrtf(var + a.eps);
    float4 z = make_float4(d.x * rs * w.x + b.x, d.y * rs * w.y + b.y, d.z * rs * w.z + b.z, d.w * rs * w.w + b.w);
    if (a.act == 2) z = make_float4(gelu_erf(z.x), gelu_erf(z.y), gelu_erf(z.z), gelu_erf(z.w));
    reinterpret_cast<float4*>(a.y + r * D)[c] = z;
    if (c == 0) {
      if (a.mean) a.mean[r] = mu;
      if (a.rstd) a.rstd[r] = rs;
    }
  }
}

// Forward for wide rows (D = 256 NV: 512, 768, 1024 — the BERT hidden sizes of the item
// tower's text encoder — and 2048, the 16d LayerNorm of the item head's SE blocks at d = 128,
// item_tower.py:41-75): one wave per row, NV float4 per lane, same formulas as ln_fwd_k.
template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_wide_k(FArgs a) {
  constexpr int D = 256 * NV;
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  float4 w[NV], b[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = lane + 64 * v;
    w[v] = a.w ? reinterpret_cast<const float4*>(a.w)[c] : make_float4(1.f, 1.f, 1.f, 1.f);
    b[v] = a.b ? reinterpret_cast<const float4*>(a.b)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int64_t r = wave_g; r < a.T; r += nw) {
    float4 s[NV];
    float sum = 0.0f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = lane + 64 * v;
      s[v] = reinterpret_cast<const float4*>(a.x + r * D)[c];
      if (a.res) {
        float4 q = reinterpret_cast<const float4*>(a.res + r * D)[c];
        const uint64_t bi = (uint64_t)r * D + 4 * c;
        q.x = a.drop.apply(q.x, bi + 0);
        q.y = a.drop.apply(q.y, bi + 1);
        q.z = a.drop.apply(q.z, bi + 2);
        q.w = a.drop.apply(q.w, bi + 3);
        s[v].x += q.x; s[v].y += q.y; s[v].z += q.z; s[v].w += q.w;
        if (a.sum_out) reinterpret_cast<float4*>(a.sum_out + r * D)[c] = s[v];
      }
      sum += (s[v].x + s[v].y) + (s[v].z + s[v].w);
    }
    if (!a.y) continue;
    const float mu = rsx::wave_sum_width(sum, 64) * (1.0f / D);
    float sq = 0.0f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      s[v] = make_float4(s[v].x - mu, s[v].y - mu, s[v].z - mu, s[v].w - mu);
      sq += s[v].x * s[v].x + s[v].y * s[v].y + s[v].z * s[v].z + s[v].w * s[v].w;
    }
    const float rs = 1.0f / sqrtf(rsx::wave_sum_width(sq, 64) * (1.0f / D) + a.eps);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const float4 d = s[v];
      float4 z = make_float4(d.x * rs * w[v].x + b[v].x, d.y * rs * w[v].y + b[v].y, d.z * rs * w[v].z + b[v].z,
                             d.w * rs * w[v].w + b[v].w);
      if (a.act == 2) z = make_float4(gelu_erf(z.x), gelu_erf(z.y), gelu_erf(z.z), gelu_erf(z.w));
      reinterpret_cast<float4*>(a.y + r * D)[lane + 64 * v] = z;
    }
    if (lane == 0) {
      if (a.mean) a.mean[r] = mu;
      if (a.rstd) a.rstd[r] = rs;
    }
  }
}

struct BArgs {
  const float* s;
  const float* mean;
  const float* rstd;
  const float* w;
  const float* b;
  const float* dy;
  const float* ds_in;
  float* ds_out;
  float* dres;
  float* part;  // [nblocks][2][D] (dw, db partials) or nullptr
  int64_t T, rows_per_block;
  int act;
  rsx::Dropout drop;
};

template <int D>
__global__ __launch_bounds__(256) void ln_bwd_k(BArgs a) {
  constexpr int LPR = Geo<D>::LPR, RPW = Geo<D>::RPW;
  __shared__ __attribute__((aligned(16))) float s_red[4][2][D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, sub = lane / LPR, c = lane % LPR;
  const float4 w = a.w ? reinterpret_cast<const float4*>(a.w)[c] : make_float4(1.f, 1.f, 1.f, 1.f);
  const float4 b = a.b ? reinterpret_cast<const float4*>(a.b)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc_w = make_float4(0.f, 0.f, 0.f, 0.f), acc_b = acc_w;
  const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_block;
  int64_t r_end = r_begin + a.rows_per_block;
  if (r_end > a.T) r_end = a.T;
  for (int64_t r0 = r_begin; r0 < r_end; r0 += 4 * RPW) {
    const int64_t r = r0 + wave * RPW + sub;
    if (r >= r_end) continue;
    const float4 s = reinterpret_cast<const float4*>(a.s + r * D)[c];
    float4 g = reinterpret_cast<const float4*>(a.dy + r * D)[c];
    const float mu = a.mean[r], rs = a.rstd[r];
    const float4 xh = make_float4((s.x - mu) * rs, (s.y - mu) * rs, (s.z - mu) * rs, (s.w - mu) * rs);
    if (a.act == 2) {
      g.x *= gelu_erf_grad(xh.x * w.x + b.x);
      g.y *= gelu_erf_grad(xh.y * w.y + b.y);
      g.z *= gelu_erf_grad(xh.z * w.z + b.z);
      g.w *= gelu_erf_grad(xh.w * w.w + b.w);
    }
    acc_w.x += g.x * xh.x; acc_w.y += g.y * xh.y; acc_w.z += g.z * xh.z; acc_w.w += g.w * xh.w;
    acc_b.x += g.x; acc_b.y += g.y; acc_b.z += g.z; acc_b.w += g.w;
    const float4 dh = make_float4(g.x * w.x, g.y * w.y, g.z * w.z, g.w * w.w);
    const float c1 = rsx::wave_sum_width((dh.x + dh.y) + (dh.z + dh.w), LPR) * (1.0f / D);
    const float c2 =
        rsx::wave_sum_width(dh.x * xh.x + dh.y * xh.y + dh.z * xh.z + dh.w * xh.w, LPR) * (1.0f / D);
    float4 dx = make_float4((dh.x - c1 - xh.x * c2) * rs, (dh.y - c1 - xh.y * c2) * rs,
                            (dh.z - c1 - xh.z * c2) * rs, (dh.w - c1 - xh.w * c2) * rs);
    if (a.ds_in) {
      const float4 e = reinterpret_cast<const float4*>(a.ds_in + r * D)[c];
      dx.x += e.x; dx.y += e.y; dx.z += e.z; dx.w += e.w;
    }
    if (a.ds_out) reinterpret_cast<float4*>(a.ds_out + r * D)[c] = dx;
    if (a.dres) {
      const uint64_t bi = (uint64_t)r * D + 4 * c;
      float4 q;
      q.x = a.drop.apply(dx.x, bi + 0);
      q.y = a.drop.apply(dx.y, bi + 1);
      q.z = a.drop.apply(dx.z, bi + 2);
      q.w = a.drop.apply(dx.w, bi + 3);
      reinterpret_cast<float4*>(a.dres + r * D)[c] = q;
    }
  }
  if (!a.part) return;
#pragma unroll
  for (int o = LPR; o < 64; o <<= 1) {
    acc_w.x += __shfl_xor(acc_w.x, o, 64); acc_w.y += __shfl_xor(acc_w.y, o, 64);
    acc_w.z += __shfl_xor(acc_w.z, o, 64); acc_w.w += __shfl_xor(acc_w.w, o, 64);
    acc_b.x += __shfl_xor(acc_b.x, o, 64); acc_b.y += __shfl_xor(acc_b.y, o, 64);
    acc_b.z += __shfl_xor(acc_b.z, o, 64); acc_b.w += __shfl_xor(acc_b.w, o, 64);
  }
  if (sub == 0) {
    reinterpret_cast<float4*>(&s_red[wave][0][0])[c] = acc_w;
    reinterpret_cast<float4*>(&s_red[wave][1][0])[c] = acc_b;
  }
  __syncthreads();
  for (int i = tid; i < 2 * D; i += blockDim.x) {
    const float v = (s_red[0][0][i] + s_red[1][0][i]) + (s_red[2][0][i] + s_red[3][0][i]);
    a.part[(int64_t)blockIdx.x * 2 * D + i] = v;
  }
}

// Backward for wide rows (D = 256 NV): one wave per row, NV float4 per lane; the same
// formulas as ln_bwd_k. dw/db partials: each wave accumulates its rows in registers, the
// block's four waves are summed through LDS in a fixed order (deterministic).
template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_wide_k(BArgs a) {
  constexpr int D = 256 * NV;
  __shared__ __attribute__((aligned(16))) float s_red[2][2][D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float4 w[NV], b[NV], acc_w[NV], acc_b[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = lane + 64 * v;
    w[v] = a.w ? reinterpret_cast<const float4*>(a.w)[c] : make_float4(1.f, 1.f, 1.f, 1.f);
    b[v] = a.b ? reinterpret_cast<const float4*>(a.b)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    acc_w[v] = make_float4(0.f, 0.f, 0.f, 0.f);
    acc_b[v] = acc_w[v];
  }
  const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_block;
  int64_t r_end = r_begin + a.rows_per_block;
  if (r_end > a.T) r_end = a.T;
  for (int64_t r = r_begin + wave; r < r_end; r += 4) {
    const float mu = a.mean[r], rs = a.rstd[r];
    float4 xh[NV], g[NV];
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = lane + 64 * v;
      const float4 s = reinterpret_cast<const float4*>(a.s + r * D)[c];
      g[v] = reinterpret_cast<const float4*>(a.dy + r * D)[c];
      xh[v] = make_float4((s.x - mu) * rs, (s.y - mu) * rs, (s.z - mu) * rs, (s.w - mu) * rs);
      if (a.act == 2) {
        g[v].x *= gelu_erf_grad(xh[v].x * w[v].x + b[v].x);
        g[v].y *= gelu_erf_grad(xh[v].y * w[v].y + b[v].y);
        g[v].z *= gelu_erf_grad(xh[v].z * w[v].z + b[v].z);
        g[v].w *= gelu_erf_grad(xh[v].w * w[v].w + b[v].w);
      }
      acc_w[v].x += g[v].x * xh[v].x; acc_w[v].y += g[v].y * xh[v].y;
      acc_w[v].z += g[v].z * xh[v].z; acc_w[v].w += g[v].w * xh[v].w;
      acc_b[v].x += g[v].x; acc_b[v].y += g[v].y; acc_b[v].z += g[v].z; acc_b[v].w += g[v].w;
      const float4 dh = make_float4(g[v].x * w[v].x, g[v].y * w[v].y, g[v].z * w[v].z, g[v].w * w[v].w);
      g[v] = dh;
      s1 += (dh.x + dh.y) + (dh.z + dh.w);
      s2 += dh.x * xh[v].x + dh.y * xh[v].y + dh.z * xh[v].z + dh.w * xh[v].w;
    }
    const float c1 = rsx::wave_sum_width(s1, 64) * (1.0f / D);
    const float c2 = rsx::wave_sum_width(s2, 64) * (1.0f / D);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = lane + 64 * v;
      const float4 dh = g[v];
      float4 dx = make_float4((dh.x - c1 - xh[v].x * c2) * rs, (dh.y - c1 - xh[v].y * c2) * rs,
                              (dh.z - c1 - xh[v].z * c2) * rs, (dh.w - c1 - xh[v].w * c2) * rs);
      if (a.ds_in) {
        const float4 e = reinterpret_cast<const float4*>(a.ds_in + r * D)[c];
        dx.x += e.x; dx.y += e.y; dx.z += e.z; dx.w += e.w;
      }
      if (a.ds_out) reinterpret_cast<float4*>(a.ds_out + r * D)[c] = dx;
      if (a.dres) {
        const uint64_t bi = (uint64_t)r * D + 4 * c;
        float4 q;
        q.x = a.drop.apply(dx.x, bi + 0);
        q.y = a.drop.apply(dx.y, bi + 1);
        q.z = a.drop.apply(dx.z, bi + 2);
        q.w = a.drop.apply(dx.w, bi + 3);
        reinterpret_cast<float4*>(a.dres + r * D)[c] = q;
      }
    }
  }
  if (!a.part) return;
  // waves 2, 3 store; waves 0, 1 add theirs; then wave 1's sums are added to wave 0's
  if (wave >= 2) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      reinterpret_cast<float4*>(&s_red[wave - 2][0][0])[lane + 64 * v] = acc_w[v];
      reinterpret_cast<float4*>(&s_red[wave - 2][1][0])[lane + 64 * v] = acc_b[v];
    }
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      float4* pw = reinterpret_cast<float4*>(&s_red[wave][0][0]) + lane + 64 * v;
      float4* pb = reinterpret_cast<float4*>(&s_red[wave][1][0]) + lane + 64 * v;
      float4 x = *pw, y = *pb;
      x.x += acc_w[v].x; x.y += acc_w[v].y; x.z += acc_w[v].z; x.w += acc_w[v].w;
      y.x += acc_b[v].x; y.y += acc_b[v].y; y.z += acc_b[v].z; y.w += acc_b[v].w;
      *pw = x;
      *pb = y;
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * D; i += blockDim.x) {
    const float v = s_red[0][0][i] + s_red[1][0][i];
    a.part[(int64_t)blockIdx.x * 2 * D + i] = v;
  }
}

// out[i] = sum_k part[k][i] over nblk rows of width n (fixed order, 16 groups per output)
__global__ __launch_bounds__(256) void colsum_k(const float* part, int nblk, int n, float* out0, float* out1,
                                                int split) {
  __shared__ float red[16][16];
  const int o = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + o;
  float s = 0.0f;
  // unrolled: eight partial loads in flight per thread (the sum order, and so the result, is
  // unchanged); one load at a time left these 16-workgroup launches waiting out the latency
  if (i < n) {
#pragma unroll 8
    for (int k = g; k < nblk; k += 16) s += part[(int64_t)k * n + i];
  }
  red[g][o] = s;
  __syncthreads();
  if (g != 0 || i >= n) return;
  for (int k = 1; k < 16; ++k) s += red[k][o];
  if (i < split) {
    if (out0) out0[i] = s;
  } else if (out1) {
    out1[i - split] = s;
  }
}

constexpr int kMaxBlocks = 1024;

int64_t bwd_blocks(int64_t T, int64_t D, int64_t& rpb) {
  const int64_t quantum = D > 256 ? 4 : 4 * (64 / (D / 4));  // rows per block-iteration
  rpb = (T + kMaxBlocks - 1) / kMaxBlocks;
  rpb = (rpb + quantum - 1) / quantum * quantum;
  if (rpb < quantum) rpb = quantum;
  return (T + rpb - 1) / rpb;
}

// dres = dropout mask (the forward's hash of (seed, i)) applied to ds, flat over T x D
__global__ __launch_bounds__(256) void dropout_bwd_k(const float* __restrict__ ds, int64_t n4, rsx::Dropout drop,
                                                     float* __restrict__ dres) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 g = reinterpret_cast<const float4*>(ds)[i];
    const uint64_t bi = (uint64_t)i * 4;
    g.x = drop.apply(g.x, bi + 0);
    g.y = drop.apply(g.y, bi + 1);
    g.z = drop.apply(g.z, bi + 2);
    g.w = drop.apply(g.w, bi + 3);
    reinterpret_cast<float4*>(dres)[i] = g;
  }
}

}  // namespace

RSX_API int rsx_ln_fwd(const float* x, const float* res, float p_drop, uint64_t seed, const float* w, const float* b,
                       float eps, int act, int64_t T, int64_t D, float* sum_out, float* y, float* mean, float* rstd,
                       void* stream) {
  RSX_ARG(x && (y || (res && sum_out)), "null tensor (y may be null only for the add-only form)");
  RSX_ARG(D == 64 || D == 128 || D == 256 || D == 512 || D == 768 || D == 1024 || D == 2048,
          "D must be 64, 128, 256, 512, 768, 1024 or 2048");
  RSX_ARG(act == 0 || act == 2, "act must be 0 (none) or 2 (gelu)");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0,1)");
  if (T == 0) return 0;
  FArgs a;
  a.x = x; a.res = res; a.w = w; a.b = b; a.sum_out = sum_out; a.y = y; a.mean = mean; a.rstd = rstd;
  a.T = T; a.eps = eps; a.act = act;
  a.drop = rsx::make_dropout(res ? p_drop : 0.0f, seed);
  const int64_t rows_per_block = D > 256 ? 4 : 4 * (64 / (D / 4));  // wide: one row per wave
  int64_t blocks = (T + rows_per_block - 1) / rows_per_block;
  if (blocks > 8192) blocks = 8192;
  hipStream_t st = (hipStream_t)stream;
  if (D == 512) hipLaunchKernelGGL(ln_fwd_wide_k<2>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 768) hipLaunchKernelGGL(ln_fwd_wide_k<3>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 1024) hipLaunchKernelGGL(ln_fwd_wide_k<4>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 2048) hipLaunchKernelGGL(ln_fwd_wide_k<8>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 64) hipLaunchKernelGGL(ln_fwd_k<64>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 128) hipLaunchKernelGGL(ln_fwd_k<128>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ln_fwd_k<256>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  RSX_LAUNCHED();
  return 0;
}

// An upper bound of bwd_blocks(T', D) for every T' <= T (bwd_blocks itself is not monotonic in T:
// rounding rows-per-block up to the quantum can leave a larger T with fewer blocks), so a caller may
// size one workspace by its largest row count and use it for smaller ones (the tower backward's
// tail rows R < T: rsx_tower_bwd).
RSX_API int64_t rsx_ln_bwd_workspace_floats(int64_t T, int64_t D) {
  // the row widths rsx_ln_bwd accepts; anything else is an error (-1), never a division by D / 4 = 0
  if (!(D == 64 || D == 128 || D == 256 || D == 512 || D == 768 || D == 1024 || D == 2048)) return -1;
  if (T <= 0) return 64;
  const int64_t quantum = D > 256 ? 4 : 4 * (64 / (D / 4));
  const int64_t b = (T + quantum - 1) / quantum;
  return (b < kMaxBlocks ? b : kMaxBlocks) * 2 * D + 64;
}

RSX_API int rsx_ln_bwd(const float* s, const float* mean, const float* rstd, const float* w, const float* b, int act,
                       const float* dy, const float* ds_in, float p_drop, uint64_t seed, int64_t T, int64_t D,
                       float* ds_out, float* dres, float* dw, float* db, float* ws, int64_t ws_floats, void* stream) {
  RSX_ARG(s && mean && rstd && dy, "null tensor");
  RSX_ARG(D == 64 || D == 128 || D == 256 || D == 512 || D == 768 || D == 1024 || D == 2048,
          "D must be 64, 128, 256, 512, 768, 1024 or 2048");
  RSX_ARG(act == 0 || act == 2, "act must be 0 (none) or 2 (gelu)");
  RSX_ARG(!(dw || db) || (ws && ws_floats >= rsx_ln_bwd_workspace_floats(T, D)), "workspace too small");
  RSX_ARG(act == 0 || w, "gelu needs the LayerNorm weight");
  hipStream_t st = (hipStream_t)stream;
  if (T == 0) {
    if (dw) (void)hipMemsetAsync(dw, 0, D * sizeof(float), st);
    if (db) (void)hipMemsetAsync(db, 0, D * sizeof(float), st);
    RSX_LAUNCHED();
    return 0;
  }
  BArgs a;
  a.s = s; a.mean = mean; a.rstd = rstd; a.w = w; a.b = b; a.dy = dy; a.ds_in = ds_in; a.ds_out = ds_out;
  a.dres = dres; a.part = (dw || db) ? ws : nullptr; a.T = T; a.act = act;
  a.drop = rsx::make_dropout(p_drop, seed);
  const int64_t blocks = bwd_blocks(T, D, a.rows_per_block);
  if (D == 64) hipLaunchKernelGGL(ln_bwd_k<64>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 128) hipLaunchKernelGGL(ln_bwd_k<128>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 256) hipLaunchKernelGGL(ln_bwd_k<256>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 512) hipLaunchKernelGGL(ln_bwd_wide_k<2>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 768) hipLaunchKernelGGL(ln_bwd_wide_k<3>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (D == 1024) hipLaunchKernelGGL(ln_bwd_wide_k<4>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ln_bwd_wide_k<8>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  RSX_LAUNCHED();
  if (dw || db) {
    const int n = (int)(2 * D);
    hipLaunchKernelGGL(colsum_k, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, st, ws, (int)blocks, n, dw, db,
                       (int)D);
    RSX_LAUNCHED();
  }
  return 0;
}

// Backward of s = x + dropout(res) (rsx_ln_fwd with y = NULL): dres = mask(ds) with the same
// (seed, row*D + col) hash; ds itself is dx. Replaces the autograd of
// `x + F.dropout(f, p)` after the encoder's last layer (v1_refine_usertower.py:343-352).
RSX_API int rsx_dropout_bwd(const float* ds, int64_t T, int64_t D, float p_drop, uint64_t seed, float* dres,
                            void* stream) {
  RSX_ARG(ds && dres, "null tensor");
  RSX_ARG(D % 4 == 0, "D must be a multiple of 4");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0,1)");
  if (T == 0) return 0;
  const int64_t n4 = T * D / 4;
  int64_t blocks = (n4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(dropout_bwd_k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, ds, n4,
                     rsx::make_dropout(p_drop, seed), dres);
  RSX_LAUNCHED();
  return 0;
}
