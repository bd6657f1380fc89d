// Gradient clipping + AdamW as two launches (the tail of the contrastive step:
// torch.nn.utils.clip_grad_norm_(model.parameters(), 5.0) then optimizer.step() of
// torch.optim.AdamW, tower_code/v1_usertower_train.py:852-853 / :495-496).
//
// clip_sumsq_k: every workgroup squares and sums one tile of one clipped gradient and writes
//   one partial (fixed slot: no atomics, bit-reproducible).
// adamw_apply_k: every workgroup first reduces ALL partials in the same fixed order (so each
//   one derives the identical norm and clip coefficient: no grid-wide sync), then updates one
//   tile of one parameter: grad *= coef (written back, as clip_grad_norm_ does), the decoupled
//   weight decay, both moments and the bias-corrected step. The per-element arithmetic follows
//   torch's fused AdamW (double-precision scalars, float state), so the update agrees with
//   torch.optim.AdamW(fused=True) to the last bit or two.
// HBM traffic per element: 4 B (norm) + 28 B read/write (p, g, m, v; g written only when the
// coefficient is < 1): memory-bound, ~50 us for the 12.5M parameters of the headline step.
#include "rsx_common.h"
#include "recsys_amd.h"

#include <math.h>
#include <vector>

namespace {

constexpr int kThreads = 256;
constexpr int kTile = 8192;   // elements per workgroup: 256 threads x 8 float4
constexpr int kChunk = 24;    // tensors per launch (kernel argument block ~2.5 KB)

struct OptTensor {
  float* p;
  float* g;
  float* m;
  float* v;
  const float* step_dev;  // device step count (already incremented), or null: use step
  int64_t n;
  double lr, wd, b1, b2, eps;  // torch keeps these as Python floats (double)
  float step;
  int clip;               // 1: the gradient is part of the clipped norm and gets scaled
  int vec;                // 1: every pointer 16-B aligned and n % 4 == 0
};

struct OptChunk {
  OptTensor t[kChunk];
  int blk0[kChunk + 1];  // workgroup prefix over this launch's tensors
  int nt;
  int part0;             // first partial slot of this launch (norm pass)
};

__device__ __forceinline__ int find_tensor(const OptChunk& c, int b) {
  int i = 0;
  while (i + 1 < c.nt && b >= c.blk0[i + 1]) ++i;
  return i;
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  v = rsx::wave_sum_width(v, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  T s = red[0];
#pragma unroll
  for (int k = 1; k < kThreads / 64; ++k) s += red[k];
  return s;
}

__global__ __launch_bounds__(kThreads) void clip_sumsq_k(OptChunk c, float* __restrict__ partials) {
  __shared__ float red[kThreads / 64];
  const int ti = find_tensor(c, blockIdx.x);
  const OptTensor& t = c.t[ti];
  const int64_t base = (int64_t)(blockIdx.x - c.blk0[ti]) * kTile;
  const int64_t len = min((int64_t)kTile, t.n - base);
  const float* g = t.g + base;
  float s = 0.0f;
  if (t.vec) {
    for (int64_t i = threadIdx.x * 4; i < len; i += kThreads * 4) {
      const float4 x = *reinterpret_cast<const float4*>(g + i);
      s += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
    }
  } else {
    for (int64_t i = threadIdx.x; i < len; i += kThreads) s += g[i] * g[i];
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partials[c.part0 + blockIdx.x] = s;
}

__device__ __forceinline__ void adam_elem(float& p, float& g, float& m, float& v, float coef, double lr, double wd,
                                          double b1, double b2, double eps, double step_size, double bc2_sqrt) {
  g = g * coef;
  if (wd != 0.0) p = (float)(p - lr * wd * p);
  m = (float)(b1 * m + (1.0 - b1) * g);
  v = (float)(b2 * v + (1.0 - b2) * g * g);
  const float denom = (float)(sqrtf(v) / bc2_sqrt + eps);
  p -= (float)step_size * m / denom;
}

__global__ __launch_bounds__(kThreads) void adamw_apply_k(OptChunk c, const float* __restrict__ partials, int n_part,
                                                          float max_norm, float* __restrict__ norm_out) {
  __shared__ double red[kThreads / 64];
  const int ti = find_tensor(c, blockIdx.x);
  const OptTensor& t = c.t[ti];
  float coef = 1.0f;
  if (t.clip || (norm_out && blockIdx.x == 0)) {
    double s = 0.0;
    for (int i = threadIdx.x; i < n_part; i += kThreads) s += (double)partials[i];
    s = block_sum(s, red);
    const float tn = (float)sqrt(s);
    if (norm_out && blockIdx.x == 0 && threadIdx.x == 0) norm_out[0] = tn;
    if (t.clip) {
      const float cc = max_norm / (tn + 1e-6f);
      coef = cc > 1.0f ? 1.0f : cc;  // torch.clamp(max=1): a NaN coefficient stays NaN
    }
  }
  const float step = t.step_dev ? *t.step_dev : t.step;
  const double b1 = t.b1, b2 = t.b2, lr = t.lr, wd = t.wd, eps = t.eps;
  const double bc1 = 1.0 - pow(b1, (double)step);
  const double bc2_sqrt = sqrt(1.0 - pow(b2, (double)step));
  const double step_size = lr / bc1;
  const bool write_g = t.clip && coef != 1.0f;
  const int64_t base = (int64_t)(blockIdx.x - c.blk0[ti]) * kTile;
  const int64_t len = min((int64_t)kTile, t.n - base);
  float* P = t.p + base;
  float* G = t.g + base;
  float* M = t.m + base;
  float* V = t.v + base;
  if (t.vec) {
    for (int64_t i = threadIdx.x * 4; i < len; i += kThreads * 4) {
      float4 p = *reinterpret_cast<const float4*>(P + i), g = *reinterpret_cast<const float4*>(G + i);
      float4 m = *reinterpret_cast<const float4*>(M + i), v = *reinterpret_cast<const float4*>(V + i);
      adam_elem(p.x, g.x, m.x, v.x, coef, lr, wd, b1, b2, eps, step_size, bc2_sqrt);
      adam_elem(p.y, g.y, m.y, v.y, coef, lr, wd, b1, b2, eps, step_size, bc2_sqrt);
      adam_elem(p.z, g.z, m.z, v.z, coef, lr, wd, b1, b2, eps, step_size, bc2_sqrt);
      adam_elem(p.w, g.w, m.w, v.w, coef, lr, wd, b1, b2, eps, step_size, bc2_sqrt);
      *reinterpret_cast<float4*>(P + i) = p;
      *reinterpret_cast<float4*>(M + i) = m;
      *reinterpret_cast<float4*>(V + i) = v;
      if (write_g) *reinterpret_cast<float4*>(G + i) = g;
    }
  } else {
    for (int64_t i = threadIdx.x; i < len; i += kThreads) {
      float p = P[i], g = G[i], m = M[i], v = V[i];
      adam_elem(p, g, m, v, coef, lr, wd, b1, b2, eps, step_size, bc2_sqrt);
      P[i] = p;
      M[i] = m;
      V[i] = v;
      if (write_g) G[i] = g;
    }
  }
}

int64_t tiles_of(int64_t n) { return (n + kTile - 1) / kTile; }

}  // namespace

RSX_API int64_t rsx_clip_adamw_workspace_bytes(int n, const int64_t* numel, const int* clip) {
  if (n < 0 || (n > 0 && (!numel || !clip))) return -1;
  int64_t parts = 0;
  for (int i = 0; i < n; ++i)
    if (clip[i]) parts += tiles_of(numel[i]);
  return (parts + 1) * (int64_t)sizeof(float);
}

RSX_API int rsx_clip_adamw(int n, float* const* params, float* const* grads, float* const* exp_avg,
                           float* const* exp_avg_sq, const int64_t* numel, const int* clip, const float* step,
                           const float* const* step_dev, const double* lr, const double* weight_decay,
                           const double* beta1, const double* beta2, const double* eps, float max_norm, void* ws,
                           int64_t ws_bytes, float* norm_out, void* stream) {
  RSX_ARG(n >= 0, "n < 0");
  if (n == 0) return 0;
  RSX_ARG(params && grads && exp_avg && exp_avg_sq && numel && clip && step && lr && weight_decay && beta1 && beta2 &&
              eps,
          "null array");
  const int64_t need = rsx_clip_adamw_workspace_bytes(n, numel, clip);
  RSX_ARG(ws && ws_bytes >= need, "workspace too small (rsx_clip_adamw_workspace_bytes)");
  hipStream_t st = (hipStream_t)stream;
  float* partials = (float*)ws;
  std::vector<OptTensor> all;
  all.reserve(n);
  for (int i = 0; i < n; ++i) {
    RSX_ARG(numel[i] >= 0, "negative numel");
    if (numel[i] == 0) continue;
    RSX_ARG(params[i] && grads[i] && exp_avg[i] && exp_avg_sq[i], "null tensor");
    RSX_ARG(tiles_of(numel[i]) < (1 << 24), "tensor too large");
    OptTensor t;
    t.p = params[i];
    t.g = grads[i];
    t.m = exp_avg[i];
    t.v = exp_avg_sq[i];
    t.step_dev = step_dev ? step_dev[i] : nullptr;
    t.n = numel[i];
    t.step = step[i];
    t.lr = lr[i];
    t.wd = weight_decay[i];
    t.b1 = beta1[i];
    t.b2 = beta2[i];
    t.eps = eps[i];
    t.clip = clip[i] ? 1 : 0;
    const uintptr_t a = (uintptr_t)t.p | (uintptr_t)t.g | (uintptr_t)t.m | (uintptr_t)t.v;
    t.vec = (a % 16 == 0) && (t.n % 4 == 0);
    all.push_back(t);
  }
  // pass 1: partial sums of squares of the clipped gradients
  int n_part = 0;
  {
    OptChunk c;
    c.nt = 0;
    c.blk0[0] = 0;
    c.part0 = 0;
    auto flush = [&]() -> int {
      if (c.nt == 0) return 0;
      hipLaunchKernelGGL(clip_sumsq_k, dim3(c.blk0[c.nt]), dim3(kThreads), 0, st, c, partials);
      RSX_LAUNCHED();
      c.part0 += c.blk0[c.nt];
      c.nt = 0;
      return 0;
    };
    for (const OptTensor& t : all) {
      if (!t.clip) continue;
      c.t[c.nt] = t;
      c.blk0[c.nt + 1] = c.blk0[c.nt] + (int)tiles_of(t.n);
      if (++c.nt == kChunk || c.blk0[c.nt] > (1 << 30)) {
        if (int e = flush()) return e;
      }
    }
    if (int e = flush()) return e;
    n_part = c.part0;
  }
  // pass 2: the clipped AdamW update of every tensor
  {
    OptChunk c;
    c.nt = 0;
    c.blk0[0] = 0;
    c.part0 = 0;
    bool first = true;
    auto flush = [&]() -> int {
      if (c.nt == 0) return 0;
      hipLaunchKernelGGL(adamw_apply_k, dim3(c.blk0[c.nt]), dim3(kThreads), 0, st, c, partials, n_part, max_norm,
                         first ? norm_out : nullptr);
      RSX_LAUNCHED();
      first = false;
      c.nt = 0;
      return 0;
    };
    for (const OptTensor& t : all) {
      c.t[c.nt] = t;
      c.blk0[c.nt + 1] = c.blk0[c.nt] + (int)tiles_of(t.n);
      if (++c.nt == kChunk || c.blk0[c.nt] > (1 << 30)) {
        if (int e = flush()) return e;
      }
    }
    if (int e = flush()) return e;
  }
  return 0;
}
