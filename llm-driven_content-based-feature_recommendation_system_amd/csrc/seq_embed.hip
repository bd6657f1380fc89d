// Fused sequence-embedding stage of SASRecUserTower (reference:
// tower_code/v1_refine_usertower.py:434-459):
//   x   = base + sum_j E_j[ids_j] * gate_j + pos[l]        (fp32, same op order)
//   out = dropout(LayerNorm(x))
// and its backward (LN grads, gate grads, position grads, table scatter-add).
//
// Layout: one token row = D contiguous fp32 (D in {64,128,256}); a row is owned
// by D/4 lanes, each holding one float4, so every global access is 16 B/lane.
// HBM-bound: per token the live bytes are base row + gathered rows + output row.
#include "rsx_common.h"

namespace {

constexpr int kMaxTab = 6;

struct FwdArgs {
  const float* base;
  const int64_t* ids[kMaxTab];
  const float* tab[kMaxTab];
  const float* gate;  // [ntab] on device, nullptr => 1.0
  const float* pos;   // [L,D] or nullptr
  const int64_t* tok_pos;  // [T] position of each token (packed layouts) or nullptr => r % L
  const float* ln_w;  // [D]  (nullptr => no LayerNorm, out = x)
  const float* ln_b;  // [D]
  float* out;
  float* mean;
  float* rstd;
  int64_t T;
  int L;
  int ntab;
  float eps;
  rsx::Dropout drop;
};

__device__ __forceinline__ float4 f4_axpy_rn(float4 x, float4 e, float g) {
  // seq_emb += E[id] * g  -- product rounded, then sum rounded (no FMA contraction),
  // matching the reference's separate `* s_g[j]` and `+=` tensor ops.
#pragma clang fp contract(off)
  x.x = x.x + e.x * g;
  x.y = x.y + e.y * g;
  x.z = x.z + e.z * g;
  x.w = x.w + e.w * g;
  return x;
}

__device__ __forceinline__ float4 f4_add_rn(float4 x, float4 p) {
#pragma clang fp contract(off)
  x.x = x.x + p.x;
  x.y = x.y + p.y;
  x.z = x.z + p.z;
  x.w = x.w + p.w;
  return x;
}

template <int D>
__device__ __forceinline__ float4 build_row(const FwdArgs& a, int64_t r, int c, const float* g) {
  float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.base) x = reinterpret_cast<const float4*>(a.base + r * D)[c];
#pragma unroll
  for (int j = 0; j < kMaxTab; ++j) {
    if (j < a.ntab && g[j] != 0.0f) {
      const int64_t id = a.ids[j][r];
      const float4 e = reinterpret_cast<const float4*>(a.tab[j] + id * D)[c];
      x = f4_axpy_rn(x, e, g[j]);
    }
  }
  if (a.pos) {
    const int l = a.tok_pos ? (int)a.tok_pos[r] : (int)(r % a.L);
    x = f4_add_rn(x, reinterpret_cast<const float4*>(a.pos + (int64_t)l * D)[c]);
  }
  return x;
}

template <int D>
__global__ __launch_bounds__(256) void seq_embed_fwd_k(FwdArgs a) {
  constexpr int LPR = D / 4;
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, c = lane % LPR;
  const int64_t wave_g = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  float g[kMaxTab];
#pragma unroll
  for (int j = 0; j < kMaxTab; ++j) g[j] = (j < a.ntab) ? (a.gate ? a.gate[j] : 1.0f) : 0.0f;
  const bool do_ln = a.ln_w != nullptr;
  float4 w = make_float4(1.f, 1.f, 1.f, 1.f), bb = make_float4(0.f, 0.f, 0.f, 0.f);
  if (do_ln) {
    w = reinterpret_cast<const float4*>(a.ln_w)[c];
    bb = reinterpret_cast<const float4*>(a.ln_b)[c];
  }
  for (int64_t r0 = wave_g * RPW; r0 < a.T; r0 += nwaves * RPW) {
    const int64_t r = r0 + sub;
    const bool ok = r < a.T;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) x = build_row<D>(a, r, c, g);
    float4 y = x;
    if (do_ln) {
      float s = (x.x + x.y) + (x.z + x.w);
      s = rsx::wave_sum_width(s, LPR);
      const float mu = s / (float)D;
      const float4 d = make_float4(x.x - mu, x.y - mu, x.z - mu, x.w - mu);
      float v = d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w;
      v = rsx::wave_sum_width(v, LPR);
      const float rs = 1.0f / sqrtf(v / (float)D + a.eps);
      y.x = d.x * rs * w.x + bb.x;
      y.y = d.y * rs * w.y + bb.y;
      y.z = d.z * rs * w.z + bb.z;
      y.w = d.w * rs * w.w + bb.w;
      if (ok && c == 0) {
        if (a.mean) a.mean[r] = mu;
        if (a.rstd) a.rstd[r] = rs;
      }
    }
    if (ok) {
      if (a.drop.active()) {
        const uint64_t base_idx = (uint64_t)r * D + 4 * c;
        y.x = a.drop.apply(y.x, base_idx + 0);
        y.y = a.drop.apply(y.y, base_idx + 1);
        y.z = a.drop.apply(y.z, base_idx + 2);
        y.w = a.drop.apply(y.w, base_idx + 3);
      }
      reinterpret_cast<float4*>(a.out + r * D)[c] = y;
    }
  }
}

struct BwdArgs {
  FwdArgs f;              // forward operands (for recompute) + saved mean/rstd
  const float* dout;      // [T,D]
  float* dbase;           // [T,D] (written) or nullptr
  float* dtab[kMaxTab];   // accumulated (caller zeroes) or nullptr
  int64_t pad_idx[kMaxTab];
  int small_off[kMaxTab]; // LDS float offset for block-local accumulation, -1 => global atomics
  int small_rows[kMaxTab];
  float* dgate;           // [ntab] accumulated or nullptr
  float* dpos;            // [L,D] accumulated or nullptr
  float* dln_w;           // [D] accumulated or nullptr
  float* dln_b;
  int64_t rows_per_block;
  int small_total;        // floats of LDS for small tables
};

constexpr int kSmallMax = 8192;  // floats (32 KiB)

// One workgroup per contiguous chunk of tokens (~2 per CU). Position and small-table
// gradients accumulate in LDS (ds_add_f32) and are flushed once per workgroup; LN and gate
// gradients fold in registers; big-table rows are scatter-added with global float atomics.
// The LDS and global scatter paths are kept apart so no flat (address-space-generic)
// atomics are emitted.
template <int D>
__global__ __launch_bounds__(256) void seq_embed_bwd_k(BwdArgs a) {
  constexpr int LPR = D / 4;
  constexpr int RPW = 64 / LPR;
  constexpr int NW = 4;
  extern __shared__ __attribute__((aligned(16))) float s_dyn[];  // [L*D] positions + small tables
  __shared__ __attribute__((aligned(16))) float s_red[NW][2][D];
  __shared__ __attribute__((aligned(16))) float s_xr[NW][RPW][D];  // per-wave dx rows (layout change)
  __shared__ float s_gate[NW][kMaxTab];

  const FwdArgs& f = a.f;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int sub = lane / LPR, c = lane % LPR;
  float* s_pos = s_dyn;
  float* s_small = s_dyn + (int64_t)f.L * D;
  const int lds_total = f.L * D + a.small_total;
  for (int i = tid; i < lds_total; i += blockDim.x) s_dyn[i] = 0.0f;
  __syncthreads();

  float g[kMaxTab];
#pragma unroll
  for (int j = 0; j < kMaxTab; ++j) g[j] = (j < f.ntab) ? (f.gate ? f.gate[j] : 1.0f) : 0.0f;
  const bool do_ln = f.ln_w != nullptr;
  float4 w = make_float4(1.f, 1.f, 1.f, 1.f);
  if (do_ln) w = reinterpret_cast<const float4*>(f.ln_w)[c];

  float4 acc_w = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc_b = make_float4(0.f, 0.f, 0.f, 0.f);
  float acc_g[kMaxTab];
#pragma unroll
  for (int j = 0; j < kMaxTab; ++j) acc_g[j] = 0.0f;

  const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_block;
  int64_t r_end = r_begin + a.rows_per_block;
  if (r_end > f.T) r_end = f.T;
  for (int64_t r0 = r_begin; r0 < r_end; r0 += NW * RPW) {
    const int64_t r = r0 + wave * RPW + sub;
    const bool ok = r < r_end;
    if (!ok) continue;  // row groups are lane-aligned: shuffles below stay inside active groups
    float4 dy = reinterpret_cast<const float4*>(a.dout + r * D)[c];
    if (f.drop.active()) {
      const uint64_t bi = (uint64_t)r * D + 4 * c;
      dy.x = f.drop.apply(dy.x, bi + 0);
      dy.y = f.drop.apply(dy.y, bi + 1);
      dy.z = f.drop.apply(dy.z, bi + 2);
      dy.w = f.drop.apply(dy.w, bi + 3);
    }
    float4 dx = dy;
    if (do_ln) {
      const float4 x = build_row<D>(f, r, c, g);
      const float mu = f.mean[r], rs = f.rstd[r];
      const float4 xh = make_float4((x.x - mu) * rs, (x.y - mu) * rs, (x.z - mu) * rs, (x.w - mu) * rs);
      acc_w.x += dy.x * xh.x; acc_w.y += dy.y * xh.y; acc_w.z += dy.z * xh.z; acc_w.w += dy.w * xh.w;
      acc_b.x += dy.x; acc_b.y += dy.y; acc_b.z += dy.z; acc_b.w += dy.w;
      const float4 dh = make_float4(dy.x * w.x, dy.y * w.y, dy.z * w.z, dy.w * w.w);
      float c1 = (dh.x + dh.y) + (dh.z + dh.w);
      float c2 = dh.x * xh.x + dh.y * xh.y + dh.z * xh.z + dh.w * xh.w;
      c1 = rsx::wave_sum_width(c1, LPR) / (float)D;
      c2 = rsx::wave_sum_width(c2, LPR) / (float)D;
      dx.x = (dh.x - c1 - xh.x * c2) * rs;
      dx.y = (dh.y - c1 - xh.y * c2) * rs;
      dx.z = (dh.z - c1 - xh.z * c2) * rs;
      dx.w = (dh.w - c1 - xh.w * c2) * rs;
    }
    if (a.dbase) reinterpret_cast<float4*>(a.dbase + r * D)[c] = dx;
    // Scatter-adds take the row in lane-strided order (lane c holds elements c + LPR*k): each
    // atomic instruction then covers LPR consecutive floats (one 128-B line per row at D=128)
    // instead of LPR 16-B pieces over four lines — 4x fewer lines per L2 atomic and
    // conflict-free LDS adds. The exchange goes through a per-wave LDS row (same wave: LDS
    // operations complete in order, no barrier).
    float xs[4];
    {
      float* xr = &s_xr[wave][sub][0];
      reinterpret_cast<float4*>(xr)[c] = dx;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < 4; ++k) xs[k] = xr[c + LPR * k];
      __builtin_amdgcn_wave_barrier();
    }
    if (a.dpos) {
      const int l = f.tok_pos ? (int)f.tok_pos[r] : (int)(r % f.L);
      float* dst = s_pos + l * D + c;
#pragma unroll
      for (int k = 0; k < 4; ++k) atomicAdd(dst + LPR * k, xs[k]);
    }
#pragma unroll
    for (int j = 0; j < kMaxTab; ++j) {
      if (j < f.ntab && g[j] != 0.0f) {
        const int64_t id = f.ids[j][r];
        if (a.dgate) {
          const float4 e = reinterpret_cast<const float4*>(f.tab[j] + id * D)[c];
          acc_g[j] += dx.x * e.x + dx.y * e.y + dx.z * e.z + dx.w * e.w;
        }
        if (a.dtab[j] && id != a.pad_idx[j]) {
          if (a.small_off[j] >= 0) {
            float* dst = s_small + a.small_off[j] + id * D + c;
#pragma unroll
            for (int k = 0; k < 4; ++k)
              __hip_atomic_fetch_add(dst + LPR * k, xs[k] * g[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else {
            float* dst = a.dtab[j] + id * D + c;
#pragma unroll
            for (int k = 0; k < 4; ++k) atomicAdd(dst + LPR * k, xs[k] * g[j]);
          }
        }
      }
    }
  }

  // ---- block reductions: fold the RPW row slots of each wave, then the waves ----
#pragma unroll
  for (int o = LPR; o < 64; o <<= 1) {
    acc_w.x += __shfl_xor(acc_w.x, o, 64); acc_w.y += __shfl_xor(acc_w.y, o, 64);
    acc_w.z += __shfl_xor(acc_w.z, o, 64); acc_w.w += __shfl_xor(acc_w.w, o, 64);
    acc_b.x += __shfl_xor(acc_b.x, o, 64); acc_b.y += __shfl_xor(acc_b.y, o, 64);
    acc_b.z += __shfl_xor(acc_b.z, o, 64); acc_b.w += __shfl_xor(acc_b.w, o, 64);
  }
#pragma unroll
  for (int j = 0; j < kMaxTab; ++j) {
    float v = acc_g[j];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    acc_g[j] = v;
  }
  if (sub == 0) {
    reinterpret_cast<float4*>(&s_red[wave][0][0])[c] = acc_w;
    reinterpret_cast<float4*>(&s_red[wave][1][0])[c] = acc_b;
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < kMaxTab; ++j) s_gate[wave][j] = acc_g[j];
  }
  __syncthreads();
  if (do_ln) {
    for (int i = tid; i < 2 * D; i += blockDim.x) {
      const int which = i / D, col = i % D;
      float v = 0.0f;
#pragma unroll
      for (int wv = 0; wv < NW; ++wv) v += s_red[wv][which][col];
      float* dst = which == 0 ? a.dln_w : a.dln_b;
      if (dst) atomicAdd(dst + col, v);
    }
  }
  if (tid < f.ntab && a.dgate) {
    float v = 0.0f;
#pragma unroll
    for (int wv = 0; wv < NW; ++wv) v += s_gate[wv][tid];
    atomicAdd(a.dgate + tid, v);
  }
  if (a.dpos) {
    for (int i = tid; i < f.L * D; i += blockDim.x) {
      const float v = s_pos[i];
      if (v != 0.0f) atomicAdd(a.dpos + i, v);
    }
  }
  for (int j = 0; j < f.ntab; ++j) {
    if (a.small_off[j] < 0 || !a.dtab[j]) continue;
    const int n = a.small_rows[j] * D;
    for (int i = tid; i < n; i += blockDim.x) {
      const float v = s_small[a.small_off[j] + i];
      if (v != 0.0f) atomicAdd(a.dtab[j] + i, v);
    }
  }
}

template <int D>
int launch_fwd(const FwdArgs& a, hipStream_t st) {
  const int64_t rows_per_block = 4 * (64 / (D / 4));
  int64_t blocks = (a.T + rows_per_block - 1) / rows_per_block;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(seq_embed_fwd_k<D>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return 0;
}

template <int D>
int launch_bwd(const BwdArgs& a, hipStream_t st) {
  const int64_t blocks = (a.f.T + a.rows_per_block - 1) / a.rows_per_block;
  const size_t lds = (size_t)(a.f.L * D + a.small_total) * sizeof(float);
  hipLaunchKernelGGL(seq_embed_bwd_k<D>, dim3((unsigned)blocks), dim3(256), lds, st, a);
  return 0;
}

int64_t bwd_rows_per_block(int64_t T, int64_t D) {
  // ~2 workgroups per CU, each owning a contiguous token chunk
  int64_t rpb = (T + 511) / 512;
  const int64_t quantum = 4 * (64 / (D / 4));
  rpb = (rpb + quantum - 1) / quantum * quantum;
  if (rpb < quantum) rpb = quantum;
  return rpb;
}

int small_layout(const int64_t* table_rows, int ntab, int64_t D, bool has_grad_j[kMaxTab], int off[kMaxTab],
                 int rows[kMaxTab]) {
  int o = 0;
  for (int j = 0; j < kMaxTab; ++j) {
    off[j] = -1;
    rows[j] = 0;
    if (j < ntab && has_grad_j[j] && table_rows && table_rows[j] * D <= 4096 && o + table_rows[j] * D <= kSmallMax) {
      off[j] = o;
      rows[j] = (int)table_rows[j];
      o += (int)(table_rows[j] * D);
    }
  }
  return o;
}

bool fill_fwd(FwdArgs& a, const float* base, const int64_t* const* ids, const float* const* tabs, int ntab,
              const float* gate, const float* pos, const int64_t* tok_pos, const float* ln_w, const float* ln_b,
              float eps, int64_t T, int64_t L, float* out, float* mean, float* rstd, float p_drop, uint64_t seed) {
  if (ntab < 0 || ntab > kMaxTab) return false;
  a.base = base;
  for (int j = 0; j < kMaxTab; ++j) {
    a.ids[j] = (j < ntab) ? ids[j] : nullptr;
    a.tab[j] = (j < ntab) ? tabs[j] : nullptr;
  }
  a.gate = gate;
  a.pos = pos;
  a.tok_pos = tok_pos;
  a.ln_w = ln_w;
  a.ln_b = ln_b;
  a.out = out;
  a.mean = mean;
  a.rstd = rstd;
  a.T = T;
  a.L = (int)L;
  a.ntab = ntab;
  a.eps = eps;
  a.drop = rsx::make_dropout(p_drop, seed);
  return true;
}

}  // namespace

RSX_API int rsx_seq_embed_fwd(const float* base, const int64_t* const* ids, const float* const* tables, int ntab,
                              const float* gate, const float* pos, const int64_t* tok_pos, const float* ln_w,
                              const float* ln_b, float eps, int64_t T, int64_t L, int64_t D, float p_drop,
                              uint64_t seed, float* out, float* mean, float* rstd, void* stream) {
  RSX_ARG(out != nullptr, "out is null");
  RSX_ARG(T >= 0 && L > 0 && L <= 64, "need T >= 0 and 0 < L <= 64");
  RSX_ARG(D == 64 || D == 128 || D == 256, "D must be 64, 128 or 256");
  RSX_ARG(ntab >= 0 && ntab <= kMaxTab, "ntab must be in [0,6]");
  RSX_ARG(ln_w == nullptr || (ln_b != nullptr), "ln_b required with ln_w");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0,1)");
  for (int j = 0; j < ntab; ++j) RSX_ARG(ids[j] != nullptr && tables[j] != nullptr, "null table/ids");
  if (T == 0) return 0;
  FwdArgs a;
  fill_fwd(a, base, ids, tables, ntab, gate, pos, tok_pos, ln_w, ln_b, eps, T, L, out, mean, rstd, p_drop, seed);
  hipStream_t st = (hipStream_t)stream;
  if (D == 64) launch_fwd<64>(a, st);
  else if (D == 128) launch_fwd<128>(a, st);
  else launch_fwd<256>(a, st);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_seq_embed_bwd(const float* base, const int64_t* const* ids, const float* const* tables,
                              const int64_t* table_rows, const int64_t* padding_idx, int ntab, const float* gate,
                              const float* pos, const int64_t* tok_pos, const float* ln_w, const float* mean,
                              const float* rstd, float eps, int64_t T, int64_t L, int64_t D, float p_drop,
                              uint64_t seed, const float* dout, float* dbase, float* const* dtables, float* dgate,
                              float* dpos, float* dln_w, float* dln_b, void* stream) {
  RSX_ARG(dout != nullptr, "dout is null");
  RSX_ARG(D == 64 || D == 128 || D == 256, "D must be 64, 128 or 256");
  RSX_ARG(ntab >= 0 && ntab <= kMaxTab, "ntab must be in [0,6]");
  RSX_ARG(ln_w == nullptr || (mean != nullptr && rstd != nullptr), "mean/rstd required with ln_w");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0,1)");
  RSX_ARG(L > 0 && L <= 64, "need 0 < L <= 64");
  if (T == 0) return 0;
  BwdArgs a;
  fill_fwd(a.f, base, ids, tables, ntab, gate, pos, tok_pos, ln_w, nullptr, eps, T, L, nullptr,
           const_cast<float*>(mean), const_cast<float*>(rstd), p_drop, seed);
  a.dout = dout;
  a.dbase = dbase;
  bool has_grad[kMaxTab];
  for (int j = 0; j < kMaxTab; ++j) {
    a.dtab[j] = (j < ntab && dtables) ? dtables[j] : nullptr;
    a.pad_idx[j] = (j < ntab && padding_idx) ? padding_idx[j] : -1;
    has_grad[j] = a.dtab[j] != nullptr;
  }
  a.small_total = small_layout(table_rows, ntab, D, has_grad, a.small_off, a.small_rows);
  a.dgate = dgate;
  a.dpos = dpos;
  a.dln_w = dln_w;
  a.dln_b = dln_b;
  a.rows_per_block = bwd_rows_per_block(T, D);
  hipStream_t st = (hipStream_t)stream;
  if (D == 64) launch_bwd<64>(a, st);
  else if (D == 128) launch_bwd<128>(a, st);
  else launch_bwd<256>(a, st);
  RSX_LAUNCHED();
  return 0;
}

