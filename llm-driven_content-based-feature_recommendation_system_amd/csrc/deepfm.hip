// DeepFM rerank forward (BASELINE configs[2]). The reference pins
// deepctr-torch==0.2.9 (requirements.txt:41) for this model but never imports it; the
// semantics follow that library's published DeepFM:
//   logit = bias + sum_f w_f[x_f]                                  (linear part, emb dim 1)
//         + 1/2 sum_k [ (sum_f v_{f,k})^2 - sum_f v_{f,k}^2 ]        (FM second order)
//         + w_o . relu(W2 relu(W1 concat_f v_f + b1) + b2)          (DNN, no bias on w_o)
//   prob  = sigmoid(logit)
//
// Kernels:
//   deepfm_embed_k  one pass over the 39 x (16 + 1) gathered values per row: first-order
//                   sum, FM term and the concatenated DNN input row (HBM-bound gather).
//   linear_nt_k     Y = act(X W^T + b) on the fp32-input MFMA (v_mfma_f32_32x32x2_f32);
//                   64 rows x up to 256 output columns per workgroup, K streamed through
//                   LDS in 32-wide chunks; optional fused final dot + add + sigmoid.
#include "rsx_common.h"
#include <math.h>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kMaxFields = 64;

struct EmbedArgs {
  const int64_t* x;               // [R, F]
  const float* V[kMaxFields];     // per-field [vocab_f, E]
  const float* W[kMaxFields];     // per-field [vocab_f] first-order weights (nullable)
  int64_t R;
  int F;
  float bias;
  float* emb;                     // [R, F*E] (nullable)
  float* lin;                     // [R] bias + first order + FM
};

// E = 16: a row is owned by 4 lanes (one float4 of every field each). The fields are walked
// in batches of kFB: all ids of a batch first, then all its embedding rows and first-order
// weights, then the sums and the DNN-row stores, so every lane keeps kFB independent random
// row reads in flight instead of one id -> row dependency chain per field.
constexpr int kFB = 13;  // 39 fields = 3 batches
__global__ __launch_bounds__(256) void deepfm_embed_k(EmbedArgs a) {
  const int64_t r = (int64_t)blockIdx.x * 64 + (threadIdx.x >> 2);
  const int q = threadIdx.x & 3;
  if (r >= a.R) return;
  const int64_t* __restrict__ xr = a.x + r * a.F;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), ss = make_float4(0.f, 0.f, 0.f, 0.f);
  float first = 0.0f;
  float* __restrict__ er = a.emb ? a.emb + r * (int64_t)a.F * 16 : nullptr;
  for (int f0 = 0; f0 < a.F; f0 += kFB) {
    int64_t id[kFB];
    float4 v[kFB];
    float w[kFB];
#pragma unroll
    for (int j = 0; j < kFB; ++j) id[j] = (f0 + j < a.F) ? __builtin_nontemporal_load(xr + f0 + j) : 0;
#pragma unroll
    for (int j = 0; j < kFB; ++j) {
      const int f = f0 + j;
      v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      w[j] = 0.0f;
      if (f < a.F) {
        v[j] = reinterpret_cast<const float4*>(a.V[f] + id[j] * 16)[q];
        if (q == (f & 3) && a.W[f]) w[j] = a.W[f][id[j]];
      }
    }
#pragma unroll
    for (int j = 0; j < kFB; ++j) {
      const int f = f0 + j;
      if (f < a.F) {
        s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w;
        ss.x += v[j].x * v[j].x; ss.y += v[j].y * v[j].y; ss.z += v[j].z * v[j].z; ss.w += v[j].w * v[j].w;
        if (er) reinterpret_cast<float4*>(er + f * 16)[q] = v[j];
        first += w[j];
      }
    }
  }
  float fm = (s.x * s.x - ss.x) + (s.y * s.y - ss.y) + (s.z * s.z - ss.z) + (s.w * s.w - ss.w);
  fm += __shfl_xor(fm, 1, 64);
  fm += __shfl_xor(fm, 2, 64);
  first += __shfl_xor(first, 1, 64);
  first += __shfl_xor(first, 2, 64);
  if (q == 0) a.lin[r] = a.bias + first + 0.5f * fm;
}

// ---------------------------------------------------------------------------------------
constexpr int kBM = 64;       // rows per workgroup
constexpr int kBK = 32;       // K chunk
constexpr int kLdsK = kBK + 4;

struct LinArgs {
  const float* X;   // [M, K] (row stride ldx)
  const float* W;   // [N, K] (torch Linear weight layout)
  const float* b;   // [N] or nullptr
  int64_t M, N, K, ldx;
  int act;          // 0 none, 1 relu, 2 gelu(erf)
  float* Y;         // [M, N] or nullptr (fused-dot mode)
  const float* wo;  // [N] final dot weights (fused mode) or nullptr
  const float* add; // [M] added to the dot (fused mode) or nullptr
  float* logit;     // [M] (fused mode)
  float* prob;      // [M] sigmoid(logit) (fused mode, nullable)
};

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) return v > 0.0f ? v : 0.0f;
  if (act == 2) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
  return v;
}

// Wave w owns output columns [w*NW, (w+1)*NW) (NW = N/4, a multiple of 32) for all 64 rows:
// (2 x NW/32) accumulator tiles of 32x32.
template <int NT>  // column tiles per wave (NW = 32*NT), N = 128*NT
__global__ __launch_bounds__(256) void linear_nt_k(LinArgs a) {
  constexpr int NW = 32 * NT;
  constexpr int NFULL = 4 * NW;
  __shared__ __attribute__((aligned(16))) float sX[kBM][kLdsK];
  __shared__ __attribute__((aligned(16))) float sW[NFULL][kLdsK];
  __shared__ float sRow[4][kBM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int64_t m0 = (int64_t)blockIdx.x * kBM;

  f32x16 acc[2][NT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // staging maps: X chunk 64x32 = 512 float4 (2 per thread); W chunk NFULL x 32 (NFULL/32 per thread)
  constexpr int WV = NFULL * kBK / 4 / 256;  // float4 per thread for W
  float4 sx[2], sw[WV];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int idx = tid + t * 256;
      const int row = idx >> 3, c4 = idx & 7;
      const int64_t m = m0 + row, k = k0 + c4 * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < a.M) {
        const float* p = a.X + m * a.ldx + k;
        if (k + 3 < a.K) v = *reinterpret_cast<const float4*>(p);
        else {
          if (k + 0 < a.K) v.x = p[0];
          if (k + 1 < a.K) v.y = p[1];
          if (k + 2 < a.K) v.z = p[2];
        }
      }
      sx[t] = v;
    }
#pragma unroll
    for (int t = 0; t < WV; ++t) {
      const int idx = tid + t * 256;
      const int n = idx >> 3, c4 = idx & 7;
      const int64_t k = k0 + c4 * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n < a.N) {
        const float* p = a.W + (int64_t)n * a.K + k;
        if (k + 3 < a.K) v = *reinterpret_cast<const float4*>(p);
        else {
          if (k + 0 < a.K) v.x = p[0];
          if (k + 1 < a.K) v.y = p[1];
          if (k + 2 < a.K) v.z = p[2];
        }
      }
      sw[t] = v;
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int idx = tid + t * 256;
      *reinterpret_cast<float4*>(&sX[idx >> 3][(idx & 7) * 4]) = sx[t];
    }
#pragma unroll
    for (int t = 0; t < WV; ++t) {
      const int idx = tid + t * 256;
      *reinterpret_cast<float4*>(&sW[idx >> 3][(idx & 7) * 4]) = sw[t];
    }
  };

  // k permutation inside a chunk: lane half h takes k = 16h + s (s = 0..15); A and B use the
  // same permutation, so each product term is paired correctly.
  gload(0);
  for (int64_t k0 = 0; k0 < a.K; k0 += kBK) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (k0 + kBK < a.K) gload(k0 + kBK);
#pragma unroll
    for (int s4 = 0; s4 < 16; s4 += 4) {
      float4 xa[2], wb[NT];
#pragma unroll
      for (int i = 0; i < 2; ++i) xa[i] = *reinterpret_cast<const float4*>(&sX[i * 32 + c][16 * h + s4]);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        wb[j] = *reinterpret_cast<const float4*>(&sW[wave * NW + j * 32 + c][16 * h + s4]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const float av = e == 0 ? xa[i].x : e == 1 ? xa[i].y : e == 2 ? xa[i].z : xa[i].w;
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            const float bv = e == 0 ? wb[j].x : e == 1 ? wb[j].y : e == 2 ? wb[j].z : wb[j].w;
            // D[row][col]: A = X rows (i*32 + lane c), B = W rows as columns
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
          }
        }
      }
    }
  }

  // epilogue. C layout: col = c -> n = wave*NW + j*32 + c ; row = tile_row(r,h) -> m = i*32 + row
  if (a.wo == nullptr) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int64_t n = wave * NW + j * 32 + c;
      if (n >= a.N) continue;
      const float bn = a.b ? a.b[n] : 0.0f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t m = m0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (m < a.M) a.Y[m * a.N + n] = act_fn(acc[i][j][r] + bn, a.act);
        }
    }
  } else {
    // fused final layer: logit_m = sum_n act(acc + b_n) * wo_n + add_m
    float part[2][16];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) part[i][r] = 0.0f;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int64_t n = wave * NW + j * 32 + c;
      const bool ok = n < a.N;
      const float bn = (ok && a.b) ? a.b[n] : 0.0f;
      const float wn = ok ? a.wo[n] : 0.0f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) part[i][r] += act_fn(acc[i][j][r] + bn, a.act) * wn;
    }
    // reduce over the 32 columns held by lanes c (same h)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = part[i][r];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        v += __shfl_xor(v, 16, 64);
        part[i][r] = v;
      }
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) sRow[wave][i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h] = part[i][r];
    }
    __syncthreads();
    if (tid < kBM) {
      const int64_t m = m0 + tid;
      if (m < a.M) {
        float v = sRow[0][tid] + sRow[1][tid] + sRow[2][tid] + sRow[3][tid];
        if (a.add) v += a.add[m];
        a.logit[m] = v;
        if (a.prob) a.prob[m] = 1.0f / (1.0f + expf(-v));
      }
    }
  }
}

int launch_linear(const LinArgs& a, hipStream_t st) {
  const unsigned blocks = (unsigned)((a.M + kBM - 1) / kBM);
  if (a.N <= 128) hipLaunchKernelGGL(linear_nt_k<1>, dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(linear_nt_k<2>, dim3(blocks), dim3(256), 0, st, a);
  return 0;
}

}  // namespace

RSX_API int rsx_deepfm_embed(const int64_t* x, int64_t R, int F, int E, const float* const* V,
                             const float* const* W, float bias, float* emb_out, float* lin_out, void* stream) {
  RSX_ARG(x && V && lin_out, "null tensor");
  RSX_ARG(F >= 1 && F <= kMaxFields, "F must be in [1,64]");
  RSX_ARG(E == 16, "embedding dim must be 16");
  if (R == 0) return 0;
  EmbedArgs a;
  a.x = x;
  for (int f = 0; f < kMaxFields; ++f) {
    a.V[f] = f < F ? V[f] : nullptr;
    a.W[f] = (f < F && W) ? W[f] : nullptr;
  }
  for (int f = 0; f < F; ++f) RSX_ARG(a.V[f] != nullptr, "null field table");
  a.R = R;
  a.F = F;
  a.bias = bias;
  a.emb = emb_out;
  a.lin = lin_out;
  hipLaunchKernelGGL(deepfm_embed_k, dim3((unsigned)((R + 63) / 64)), dim3(256), 0, (hipStream_t)stream, a);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_linear_fwd(const float* X, int64_t ldx, const float* W, const float* b, int64_t M, int64_t N,
                           int64_t K, int act, float* Y, void* stream) {
  RSX_ARG(X && W && Y, "null tensor");
  RSX_ARG(N >= 1 && N <= 256, "N must be in [1,256]");
  RSX_ARG(K >= 1 && ldx >= K, "bad K / ldx");
  RSX_ARG(K % 4 == 0 && ldx % 4 == 0, "K and ldx must be multiples of 4");
  RSX_ARG(act >= 0 && act <= 2, "act must be 0 (none), 1 (relu) or 2 (gelu)");
  if (M == 0) return 0;
  LinArgs a = {};
  a.X = X; a.W = W; a.b = b; a.M = M; a.N = N; a.K = K; a.ldx = ldx; a.act = act; a.Y = Y;
  launch_linear(a, (hipStream_t)stream);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_linear_dot_fwd(const float* X, int64_t ldx, const float* W, const float* b, int64_t M, int64_t N,
                               int64_t K, int act, const float* wo, const float* add, float* logit, float* prob,
                               void* stream) {
  RSX_ARG(X && W && wo && logit, "null tensor");
  RSX_ARG(N >= 1 && N <= 256, "N must be in [1,256]");
  RSX_ARG(K >= 1 && ldx >= K, "bad K / ldx");
  RSX_ARG(K % 4 == 0 && ldx % 4 == 0, "K and ldx must be multiples of 4");
  RSX_ARG(act >= 0 && act <= 2, "act must be 0 (none), 1 (relu) or 2 (gelu)");
  if (M == 0) return 0;
  LinArgs a = {};
  a.X = X; a.W = W; a.b = b; a.M = M; a.N = N; a.K = K; a.ldx = ldx; a.act = act;
  a.wo = wo; a.add = add; a.logit = logit; a.prob = prob;
  launch_linear(a, (hipStream_t)stream);
  RSX_LAUNCHED();
  return 0;
}
