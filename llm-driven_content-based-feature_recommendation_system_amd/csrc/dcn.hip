// DCN-V2 cross network of the reference's second neural reranker (temp_model/ranker_skelet.py:
// 239-272, RankingModel :274-357) fused with the cross half of its final head:
//
//   x_{l+1}[d] = x_0[d] * (<x_l, k_l> + b_l[d]) + x_l[d]      l = 0 .. L-1   (kernel k_l [D, 1])
//   head_part  = <x_L, w_head[0:D]>                            (final_head on cat(cross, deep))
//
// One wave per row: the row stays in registers (D/4 float4 over 64 lanes, D <= 512), every
// <x_l, k_l> is a wave reduction, and only head_part (and optionally x_L) is written. The
// deep half (two Linear + LayerNorm + GELU) runs on the token GEMMs and the LayerNorm kernel.
#include "rsx_common.h"

namespace {

constexpr int kMaxLayers = 8;

struct CArgs {
  const float* x;         // [B, ldx]
  int64_t ldx, B;
  int D, L;
  const float* k[kMaxLayers];
  const float* b[kMaxLayers];
  const float* w_head;    // [D] or nullptr
  float* x_out;           // [B, D] or nullptr
  float* head_part;       // [B] or nullptr
};

template <int NC>  // float4 chunks per lane: D <= 256 * NC
__global__ __launch_bounds__(256) void crossnet_k(CArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int n4 = a.D / 4;
  for (int64_t r = wave_g; r < a.B; r += nw) {
    const float4* xr = reinterpret_cast<const float4*>(a.x + r * a.ldx);
    float4 x0[NC], xl[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int c = j * 64 + lane;
      x0[j] = c < n4 ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
      xl[j] = x0[j];
    }
    for (int l = 0; l < a.L; ++l) {
      const float4* kk = reinterpret_cast<const float4*>(a.k[l]);
      const float4* bb = reinterpret_cast<const float4*>(a.b[l]);
      float s = 0.0f;
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int c = j * 64 + lane;
        if (c < n4) {
          const float4 kv = kk[c];
          s += (xl[j].x * kv.x + xl[j].y * kv.y) + (xl[j].z * kv.z + xl[j].w * kv.w);
        }
      }
      s = rsx::wave_sum_width(s, 64);
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int c = j * 64 + lane;
        if (c < n4) {
          const float4 bv = bb[c];
          xl[j].x = fmaf(x0[j].x, s + bv.x, xl[j].x);
          xl[j].y = fmaf(x0[j].y, s + bv.y, xl[j].y);
          xl[j].z = fmaf(x0[j].z, s + bv.z, xl[j].z);
          xl[j].w = fmaf(x0[j].w, s + bv.w, xl[j].w);
        }
      }
    }
    float h = 0.0f;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int c = j * 64 + lane;
      if (c < n4) {
        if (a.x_out) reinterpret_cast<float4*>(a.x_out + r * a.D)[c] = xl[j];
        if (a.w_head) {
          const float4 wv = reinterpret_cast<const float4*>(a.w_head)[c];
          h += (xl[j].x * wv.x + xl[j].y * wv.y) + (xl[j].z * wv.z + xl[j].w * wv.w);
        }
      }
    }
    if (a.head_part) {
      h = rsx::wave_sum_width(h, 64);
      if (lane == 0) a.head_part[r] = h;
    }
  }
}

}  // namespace

RSX_API int rsx_crossnet(const float* x, int64_t ldx, int64_t B, int D, int L, const float* const* kernels,
                         const float* const* biases, const float* w_head, float* x_out, float* head_part,
                         void* stream) {
  RSX_ARG(x && kernels && biases && (x_out || head_part), "null tensor");
  RSX_ARG(D % 4 == 0 && D >= 4 && D <= 512, "D must be a multiple of 4 in [4, 512]");
  RSX_ARG(L >= 0 && L <= kMaxLayers, "L must be in [0, 8]");
  RSX_ARG(ldx >= D && ldx % 4 == 0, "bad ldx");
  RSX_ARG(!head_part || w_head, "head_part needs w_head");
  if (B == 0) return 0;
  CArgs a;
  a.x = x; a.ldx = ldx; a.B = B; a.D = D; a.L = L;
  for (int l = 0; l < kMaxLayers; ++l) {
    a.k[l] = l < L ? kernels[l] : nullptr;
    a.b[l] = l < L ? biases[l] : nullptr;
  }
  for (int l = 0; l < L; ++l) RSX_ARG(a.k[l] && a.b[l], "null layer kernel/bias");
  a.w_head = w_head; a.x_out = x_out; a.head_part = head_part;
  int64_t blocks = (B + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  hipStream_t st = (hipStream_t)stream;
  if (D <= 256) hipLaunchKernelGGL(crossnet_k<1>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(crossnet_k<2>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  RSX_LAUNCHED();
  return 0;
}
