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
#include <mutex>
#include <utility>
#include <vector>

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

// Loads through pointers taken from the per-table pointer arrays (ids_l / tab_l, BwdLive): hipcc
// cannot prove those point to global memory and emits flat loads, which count in lgkmcnt as well as
// vmcnt -- so every LDS shuffle of the row reductions (ds_bpermute + lgkmcnt(0)) also waited for all
// outstanding row loads. Casting to the global address space gives global loads (vmcnt only).
// (through a native vector type: a float4 struct load through an address-space-1 pointer still
// came out as a flat load)
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4v gf4v;
typedef __attribute__((address_space(1))) const int64_t gint64;
__device__ __forceinline__ float4 ldg4(const float* p) {
  const f4v v = *(gf4v*)(p);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int64_t ldg8(const int64_t* p) { return *(gint64*)(p); }

// Row sums of the LayerNorm statistics on VALU lane moves (round 6): the xor butterfly of
// rsx::wave_sum_width in the same order, its partners delivered by v_permlane32_swap / v_permlane16_swap
// (o = 32, 16) and DPP row_ror (o = 8, 4, 2, 1; after the larger steps a lane's partial depends only on its
// index mod 2o, and row_ror:o reaches a lane with the same index mod 2o as lane ^ o) instead of
// ds_bpermute + lgkmcnt waits. The sums equal the shuffle form's bit for bit (tools/probe/dpp_probe.hip on
// the GPU); hipcc generates the neighbouring LayerNorm arithmetic differently around them, so the kernel's
// outputs can differ from the shuffle-form build in the last bit (DESIGN.md, round 6 second session).
template <int W>
__device__ __forceinline__ float lane_sum(float v) {
  if constexpr (W != 16 && W != 32 && W != 64) {
    return rsx::wave_sum_width(v, W);
  } else {
    if constexpr (W == 64) {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
      v = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    if constexpr (W >= 32) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
      v = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    v += __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x128, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x124, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x122, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x121, 0xF, 0xF, false));
    return v;
  }
}

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
  if (a.base) x = ldg4(a.base + r * D + 4 * c);
#pragma unroll
  for (int j = 0; j < kMaxTab; ++j) {
    if (j < a.ntab && g[j] != 0.0f) {
      const int64_t id = ldg8(a.ids[j] + r);
      const float4 e = ldg4(a.tab[j] + id * D + 4 * c);
      x = f4_axpy_rn(x, e, g[j]);
    }
  }
  if (a.pos) {
    const int l = a.tok_pos ? (int)ldg8(a.tok_pos + r) : (int)(r % a.L);
    x = f4_add_rn(x, ldg4(a.pos + (int64_t)l * D + 4 * c));
  }
  return x;
}

// Forward. The gather is latency-bound (each row is an id load followed by a dependent row
// load), so each wave owns U row groups (RPW rows each) per iteration and issues every id load,
// then every row load of all U groups before the first use: U independent id -> row chains per
// lane in flight. Tables whose gate is exactly 0 contribute exactly nothing (x + e*0 == x), so
// the wave first compacts the live tables (gate != 0; the reference's s_mask leaves item-id and
// time live) into NL <= 2 slots, which keeps the register budget at U x 2 rows; more than two
// live tables take the one-row-at-a-time path. Per element the op order is unchanged: base,
// + E_j[id_j] * g_j for the live j in increasing order, + pos, then LayerNorm and dropout.
template <int D>
__device__ __forceinline__ void ln_drop_store(const FwdArgs& a, float4 x, int64_t r, bool ok, int c, float4 w,
                                              float4 bb, bool do_ln) {
  constexpr int LPR = D / 4;
  float4 y = x;
  if (do_ln) {
    float s = (x.x + x.y) + (x.z + x.w);
    s = lane_sum<LPR>(s);
    const float mu = s / (float)D;
    const float4 d = make_float4(x.x - mu, x.y - mu, x.z - mu, x.w - mu);
    float v = d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w;
    v = lane_sum<LPR>(v);
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

// FULL: the packed tower's configuration (base rows, a position table indexed by tok_pos, LayerNorm)
// with every operand's presence known at compile time. With the presence tests as run-time branches
// hipcc closed each of their blocks with a vmcnt(0), so the id -> row chains of one iteration ran
// one after another instead of all in flight (same loads, same op order, same results).
template <int D, int U, int NL, bool FULL = false>
__device__ __forceinline__ void fwd_groups(const FwdArgs& a, const int64_t* const* ids_l, const float* const* tab_l,
                                           const float* g_l, int64_t r0, int sub, int c, float4 w, float4 bb,
                                           bool do_ln) {
  constexpr int RPW = 64 / (D / 4);
  const bool has_pos = FULL || a.pos, has_base = FULL || a.base;
  int64_t rr[U];
  int64_t id[U][NL > 0 ? NL : 1];
  int lp[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t r = r0 + u * RPW + sub;
    rr[u] = r < a.T ? r : a.T - 1;  // clamped: out-of-range slots recompute the last row, store nothing
#pragma unroll
    for (int k = 0; k < NL; ++k) id[u][k] = ldg8(ids_l[k] + rr[u]);
    if (FULL) lp[u] = (int)ldg8(a.tok_pos + rr[u]);
    else lp[u] = a.pos ? (a.tok_pos ? (int)a.tok_pos[rr[u]] : (int)(rr[u] % a.L)) : 0;
  }
  float4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    x[u] = has_base ? ldg4(a.base + rr[u] * D + 4 * c) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 e[U][NL > 0 ? NL : 1];
#pragma unroll
  for (int k = 0; k < NL; ++k)
#pragma unroll
    for (int u = 0; u < U; ++u) e[u][k] = ldg4(tab_l[k] + id[u][k] * D + 4 * c);
  float4 pv[U];
  if (FULL) {
#pragma unroll
    for (int u = 0; u < U; ++u) pv[u] = ldg4(a.pos + (int64_t)lp[u] * D + 4 * c);
  }
#pragma unroll
  for (int k = 0; k < NL; ++k)
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = f4_axpy_rn(x[u], e[u][k], g_l[k]);
  if (has_pos) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      x[u] = f4_add_rn(x[u], FULL ? pv[u] : ldg4(a.pos + (int64_t)lp[u] * D + 4 * c));
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t r = r0 + u * RPW + sub;
    ln_drop_store<D>(a, x[u], r, r < a.T, c, w, bb, FULL || do_ln);
  }
}

template <int D, int U>
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
  // compact the live tables (wave-uniform selects over the kernarg pointers: no dynamic indexing)
  const int64_t* ids_l[2] = {nullptr, nullptr};
  const float* tab_l[2] = {nullptr, nullptr};
  float g_l[2] = {0.0f, 0.0f};
  int nl = 0;
#pragma unroll
  for (int j = 0; j < kMaxTab; ++j) {
    if (g[j] != 0.0f) {
      if (nl == 0) { ids_l[0] = a.ids[j]; tab_l[0] = a.tab[j]; g_l[0] = g[j]; }
      else if (nl == 1) { ids_l[1] = a.ids[j]; tab_l[1] = a.tab[j]; g_l[1] = g[j]; }
      ++nl;
    }
  }
  const bool do_ln = a.ln_w != nullptr;
  float4 w = make_float4(1.f, 1.f, 1.f, 1.f), bb = make_float4(0.f, 0.f, 0.f, 0.f);
  if (do_ln) {
    w = reinterpret_cast<const float4*>(a.ln_w)[c];
    bb = reinterpret_cast<const float4*>(a.ln_b)[c];
  }
  if (nl > 2) {  // generic: one row group per iteration, every table
    for (int64_t r0 = wave_g * RPW; r0 < a.T; r0 += nwaves * RPW) {
      const int64_t r = r0 + sub;
      const bool ok = r < a.T;
      const float4 x = build_row<D>(a, ok ? r : a.T - 1, c, g);
      ln_drop_store<D>(a, x, r, ok, c, w, bb, do_ln);
    }
    return;
  }
  if (nl == 2 && a.base && a.pos && a.tok_pos && do_ln) {  // the packed tower's configuration
    for (int64_t r0 = wave_g * (RPW * U); r0 < a.T; r0 += nwaves * (RPW * U))
      fwd_groups<D, U, 2, true>(a, ids_l, tab_l, g_l, r0, sub, c, w, bb, true);
    return;
  }
  for (int64_t r0 = wave_g * (RPW * U); r0 < a.T; r0 += nwaves * (RPW * U)) {
    if (nl == 2) fwd_groups<D, U, 2>(a, ids_l, tab_l, g_l, r0, sub, c, w, bb, do_ln);
    else if (nl == 1) fwd_groups<D, U, 1>(a, ids_l, tab_l, g_l, r0, sub, c, w, bb, do_ln);
    else fwd_groups<D, U, 0>(a, ids_l, tab_l, g_l, r0, sub, c, w, bb, do_ln);
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
  float* partials;        // [blocks][part_w] per-block sums (then seq_embed_bwd_reduce_k), or nullptr => atomics
  int part_w;             // L*D + small_total + 2*D + kMaxTab
};

struct BwdLive {
  const int64_t* ids[kMaxTab];
  const float* tab[kMaxTab];
  float* dtab[kMaxTab];
  float g[kMaxTab];
  int64_t pad[kMaxTab];
  int soff[kMaxTab];
  int j[kMaxTab];
  int n;
};

struct BwdCtx {
  float* xr;        // this row slot's LDS exchange row
  float* s_pos;
  float* s_small;
  int64_t r_begin, r_end;
  int wave, sub, c;
  float4 w;
  bool do_ln;
};

// U row groups of one wave: every independent load of all U groups is issued before the first
// use — token position and live-table ids, then dout / mean / rstd / base and the dependent
// position and table rows (the LN recompute and the gate dot reuse the same table rows) — so a
// lane has U x (1 + NL) id -> row chains in flight instead of one at a time. NL = kMaxTab is the
// generic more-than-two-live-tables form (slots guarded by lv.n).
template <int D, int U, int NL, int ABL, bool SC>
__device__ __forceinline__ void bwd_groups(const BwdArgs& a, const BwdLive& lv, const BwdCtx& cx, int64_t r00,
                                           float4& acc_w, float4& acc_b, float* acc_l) {
  constexpr int LPR = D / 4;
  constexpr int RPW = 64 / LPR;
  constexpr int NW = 4;
  constexpr int NS = NL > 0 ? NL : 1;
  const FwdArgs& f = a.f;
  const int c = cx.c;
  const bool need_e = cx.do_ln || a.dgate;
  const bool need_l = (f.pos && cx.do_ln) || a.dpos;
  int64_t rc[U];
  int lp[U];
  int64_t id[U][NS];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t ru = r00 + (u * NW + cx.wave) * RPW + cx.sub;
    rc[u] = ru < cx.r_end ? ru : cx.r_begin;  // out-of-range slots re-read a valid row, store nothing
    lp[u] = need_l ? (f.tok_pos ? (int)f.tok_pos[rc[u]] : (int)(rc[u] % f.L)) : 0;
#pragma unroll
    for (int k = 0; k < NS; ++k)
      id[u][k] = (NL > 0 && (NL != kMaxTab || k < lv.n)) ? ldg8(lv.ids[k] + rc[u]) : 0;
  }
  float4 dyv[U], xv[U];
  float muv[U], rsv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    dyv[u] = ldg4(a.dout + rc[u] * D + 4 * c);
    xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    muv[u] = 0.0f; rsv[u] = 0.0f;
    if (cx.do_ln) {
      if (f.base) xv[u] = ldg4(f.base + rc[u] * D + 4 * c);
      muv[u] = f.mean[rc[u]];
      rsv[u] = f.rstd[rc[u]];
    }
  }
  float4 ev[U][NS];
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ev[u][k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (NL > 0 && (NL != kMaxTab || k < lv.n) && need_e && !(ABL & 2))
        ev[u][k] = ldg4(lv.tab[k] + id[u][k] * D + 4 * c);
    }
  if (cx.do_ln) {  // recompute x in the forward's op order: base, + E_j[id] * g_j (j ascending), + pos
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (NL > 0 && (NL != kMaxTab || k < lv.n)) xv[u] = f4_axpy_rn(xv[u], ev[u][k], lv.g[k]);
    if (f.pos) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        xv[u] = f4_add_rn(xv[u], ldg4(f.pos + (int64_t)lp[u] * D + 4 * c));
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t r = r00 + (u * NW + cx.wave) * RPW + cx.sub;
    if (r >= cx.r_end) continue;  // row groups are lane-aligned: shuffles below stay inside active groups
    float4 dy = dyv[u];
    if (f.drop.active()) {
      const uint64_t bi = (uint64_t)r * D + 4 * c;
      dy.x = f.drop.apply(dy.x, bi + 0);
      dy.y = f.drop.apply(dy.y, bi + 1);
      dy.z = f.drop.apply(dy.z, bi + 2);
      dy.w = f.drop.apply(dy.w, bi + 3);
    }
    float4 dx = dy;
    if (cx.do_ln) {
      const float4 x = xv[u];
      const float mu = muv[u], rs = rsv[u];
      const float4 w = cx.w;
      const float4 xh = make_float4((x.x - mu) * rs, (x.y - mu) * rs, (x.z - mu) * rs, (x.w - mu) * rs);
      acc_w.x += dy.x * xh.x; acc_w.y += dy.y * xh.y; acc_w.z += dy.z * xh.z; acc_w.w += dy.w * xh.w;
      acc_b.x += dy.x; acc_b.y += dy.y; acc_b.z += dy.z; acc_b.w += dy.w;
      const float4 dh = make_float4(dy.x * w.x, dy.y * w.y, dy.z * w.z, dy.w * w.w);
      float c1 = (dh.x + dh.y) + (dh.z + dh.w);
      float c2 = dh.x * xh.x + dh.y * xh.y + dh.z * xh.z + dh.w * xh.w;
      c1 = lane_sum<LPR>(c1) / (float)D;
      c2 = lane_sum<LPR>(c2) / (float)D;
      dx.x = (dh.x - c1 - xh.x * c2) * rs;
      dx.y = (dh.y - c1 - xh.y * c2) * rs;
      dx.z = (dh.z - c1 - xh.z * c2) * rs;
      dx.w = (dh.w - c1 - xh.w * c2) * rs;
    }
    if (a.dbase && !(ABL & 4)) reinterpret_cast<float4*>(a.dbase + r * D)[c] = dx;
    if (ABL & 1) continue;
    if (!SC) {  // position / small-table sums come from seq_embed_keysum_k over dbase
      if (a.dgate) {
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          if (!(NL > 0 && (NL != kMaxTab || k < lv.n))) continue;
          const float4 e = ev[u][k];
          acc_l[k] += dx.x * e.x + dx.y * e.y + dx.z * e.z + dx.w * e.w;
        }
      }
      // a live table too large for the LDS image still takes the global scatter below
      bool big = false;
#pragma unroll
      for (int k = 0; k < NS; ++k)
        if (NL > 0 && (NL != kMaxTab || k < lv.n) && lv.dtab[k] && lv.soff[k] < 0) big = true;
      if (!big) continue;
    }
    // Scatter-adds take the row in lane-strided order (lane c holds elements c + LPR*k): each
    // atomic instruction then covers LPR consecutive floats (one 128-B line per row at D=128)
    // instead of LPR 16-B pieces over four lines — 4x fewer lines per L2 atomic and
    // conflict-free LDS adds. The exchange goes through a per-wave LDS row (same wave: LDS
    // operations complete in order, no barrier).
    float xs[4];
    reinterpret_cast<float4*>(cx.xr)[c] = dx;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) xs[k] = cx.xr[c + LPR * k];
    __builtin_amdgcn_wave_barrier();
    if (SC && a.dpos) {
      float* dst = cx.s_pos + lp[u] * D + c;
#pragma unroll
      for (int k = 0; k < 4; ++k) atomicAdd(dst + LPR * k, xs[k]);
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      if (!(NL > 0 && (NL != kMaxTab || k < lv.n))) continue;
      if (SC && a.dgate) {
        const float4 e = ev[u][k];
        acc_l[k] += dx.x * e.x + dx.y * e.y + dx.z * e.z + dx.w * e.w;
      }
      const int64_t i = id[u][k];
      if (lv.dtab[k] && i != lv.pad[k]) {
        const float gk = lv.g[k];
        if (lv.soff[k] >= 0) {
          if (!SC) continue;
          float* dst = cx.s_small + lv.soff[k] + i * D + c;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            __hip_atomic_fetch_add(dst + LPR * q, xs[q] * gk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          float* dst = lv.dtab[k] + i * D + c;
#pragma unroll
          for (int q = 0; q < 4; ++q) atomicAdd(dst + LPR * q, xs[q] * gk);
        }
      }
    }
  }
}

constexpr int kSmallMax = 8192;  // floats (32 KiB)

// One workgroup per contiguous chunk of tokens (~2 per CU). Position and small-table
// gradients accumulate in LDS (ds_add_f32) and are flushed once per workgroup; LN and gate
// gradients fold in registers; big-table rows are scatter-added with global float atomics.
// The LDS and global scatter paths are kept apart so no flat (address-space-generic)
// atomics are emitted.
// ABL: timing ablations only (results wrong): 1 no LDS / global scatter, 2 no table-row loads,
// 4 no dbase store (RSX_SEQ_EMBED_BWD_ABL, tools/seq_embed_step_micro.py)
// SC = false: no scatter at all (every table gradient and the positions come from the sorted
// segment sums / seq_embed_keysum_k over dbase); only LN weight / bias and gate sums, and only
// those columns of the partial row are written.
template <int D, int ABL, bool SC = true, int UB = 2>
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
  const int lds_total = SC ? f.L * D + a.small_total : 0;
  for (int i = tid; i < lds_total; i += blockDim.x) s_dyn[i] = 0.0f;
  if (SC) __syncthreads();

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
  // live tables (gate != 0) compacted into slots by wave-uniform selects over the kernarg fields,
  // so every register array below is indexed by compile-time slot numbers only
  BwdLive lv;
  lv.n = 0;
#pragma unroll
  for (int k = 0; k < kMaxTab; ++k) {
    lv.ids[k] = nullptr; lv.tab[k] = nullptr; lv.dtab[k] = nullptr;
    lv.g[k] = 0.0f; lv.pad[k] = 0; lv.soff[k] = -1; lv.j[k] = -1;
  }
#pragma unroll
  for (int j = 0; j < kMaxTab; ++j) {
    if (g[j] != 0.0f) {
#pragma unroll
      for (int k = 0; k < kMaxTab; ++k) {
        if (k == lv.n) {
          lv.ids[k] = f.ids[j]; lv.tab[k] = f.tab[j]; lv.dtab[k] = a.dtab[j];
          lv.g[k] = g[j]; lv.pad[k] = a.pad_idx[j]; lv.soff[k] = a.small_off[j]; lv.j[k] = j;
        }
      }
      ++lv.n;
    }
  }
  float acc_l[kMaxTab];
#pragma unroll
  for (int k = 0; k < kMaxTab; ++k) acc_l[k] = 0.0f;
  BwdCtx cx{&s_xr[wave][sub][0], s_pos, s_small, r_begin, r_end, wave, sub, c, w, do_ln};
  if (lv.n <= 2) {
    for (int64_t r00 = r_begin; r00 < r_end; r00 += UB * NW * RPW) {
      if (lv.n == 2) bwd_groups<D, UB, 2, ABL, SC>(a, lv, cx, r00, acc_w, acc_b, acc_l);
      else if (lv.n == 1) bwd_groups<D, UB, 1, ABL, SC>(a, lv, cx, r00, acc_w, acc_b, acc_l);
      else bwd_groups<D, UB, 0, ABL, SC>(a, lv, cx, r00, acc_w, acc_b, acc_l);
    }
  } else {
    for (int64_t r00 = r_begin; r00 < r_end; r00 += NW * RPW)
      bwd_groups<D, 1, kMaxTab, ABL, SC>(a, lv, cx, r00, acc_w, acc_b, acc_l);
  }
#pragma unroll
  for (int j = 0; j < kMaxTab; ++j) {
#pragma unroll
    for (int k = 0; k < kMaxTab; ++k)
      if (lv.j[k] == j) acc_g[j] = acc_l[k];
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
  if (a.partials) {
    // deterministic two-pass reduction: this block's sums in its own workspace row (plain
    // stores, zeros included), folded over blocks in a fixed order by seq_embed_bwd_reduce_k
    float* prow = a.partials + (int64_t)blockIdx.x * a.part_w;
    const int nlds = f.L * D + a.small_total;
    if (SC)
      for (int i = tid; i < nlds; i += blockDim.x) prow[i] = s_dyn[i];
    for (int i = tid; i < 2 * D; i += blockDim.x) {
      const int which = i / D, col = i % D;
      float v = 0.0f;
#pragma unroll
      for (int wv = 0; wv < NW; ++wv) v += s_red[wv][which][col];
      prow[nlds + i] = v;
    }
    if (tid < kMaxTab) {
      float v = 0.0f;
#pragma unroll
      for (int wv = 0; wv < NW; ++wv) v += s_gate[wv][tid];
      prow[nlds + 2 * D + tid] = v;
    }
    return;
  }
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

// Position and small-table gradients as one-hot products on the MFMA (D = 128), replacing the
// LDS float atomics (≈ 130 cycles per ds_add_f32 wave-instruction measured: 0.28 ms of the
// 0.65-ms backward at the bench shape, tools/seq_embed_step_micro.py):
//   S[key][dim] = sum_t onehot[t][key] * dx[t][dim],  key = position (0..L-1) or
//                 L + small_off_j / D + id_j(t) for each small table j (id != padding_idx)
// over dbase (= dx, written by seq_embed_bwd_k<.., SC = false>). Each wave streams 16-token steps:
// lane (c, h) loads dims 4c..4c+3 of tokens h + 2i (i = 0..7) — exactly the B fragment of
// v_mfma_f32_32x32x16_bf16 for n = c (dim 4c + j, one MFMA column tile per component j) with
// k-slot 8h + i <-> token h + 2i; the A fragment (one-hot, keys 32 kt + c) is built in registers
// from the same tokens' keys. dx = b1 + b2 + b3 split exactly into three bf16 parts (24 mantissa
// bits), so every product is exact and only the fp32 accumulation rounds. The four waves of a
// workgroup meet in LDS in wave order; one partial row [nkeys][D] per workgroup, folded by
// seq_embed_bwd_reduce_k (deterministic).
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct KeyArgs {
  const float* dx;            // [T][128]
  const int64_t* tok_pos;     // [T] or nullptr => r % L
  const int64_t* ids[2];      // small tables' ids (nullptr: slot unused)
  int key_off[2];             // first key of each small table
  int64_t pad[2];
  int64_t T;
  int L;
  int do_pos;                 // position keys wanted
  int nkeys;                  // <= 64
  int64_t rows_per_block;     // multiple of 64
  float* partials;            // [blocks][nkeys * 128]
};

__device__ __forceinline__ void split3(float x, __bf16& a, __bf16& b, __bf16& c) {
  a = (__bf16)x;
  const float r = x - (float)a;
  b = (__bf16)r;
  c = (__bf16)(r - (float)b);
}

// TP: tok_pos given (else r % L); NS: small tables (0..2). Compile-time so the loop has no
// branches: a branch join makes the waitcnt pass drain the prefetched step with vmcnt(0).
template <bool TP, int NS>
__global__ __launch_bounds__(256, 2) void seq_embed_keysum_k(KeyArgs a) {
  __shared__ __attribute__((aligned(16))) float s_acc[64 * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_block;
  int64_t r_end = r_begin + a.rows_per_block;
  if (r_end > a.T) r_end = a.T;
  f32x16 acc[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[kt][j][r] = 0.0f;

  // rows past the block are clamped to its last row (valid memory) and given no key, so their
  // one-hot column is zero: no per-row branches. load_step only issues loads (keys first); the
  // keys are formed in compute_step, so no wait lands between the loads of a step.
  struct Step {
    float4 x[8];
    int64_t p, i0, i1;
  };
  auto load_step = [&](int64_t s0, Step& st) {
    const int64_t r0 = s0 + (lane & 15);
    const int64_t rk = r0 < r_end ? r0 : r_end - 1;
    st.p = TP ? a.tok_pos[rk] : rk % a.L;
    st.i0 = NS > 0 ? a.ids[0][rk] : a.pad[0];
    st.i1 = NS > 1 ? a.ids[1][rk] : a.pad[1];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int64_t r = s0 + h + 2 * i;
      r = r < r_end ? r : r_end - 1;
      st.x[i] = reinterpret_cast<const float4*>(a.dx + r * 128)[c];
    }
  };
  auto compute_step = [&](int64_t s0, const Step& st) {
    const bool ok = s0 + (lane & 15) < r_end;
    const int kp = (ok && a.do_pos) ? (int)st.p : -1;
    const int k0 = (ok && st.i0 != a.pad[0]) ? a.key_off[0] + (int)st.i0 : -1;
    const int k1 = (ok && st.i1 != a.pad[1]) ? a.key_off[1] + (int)st.i1 : -1;
    bf16x8 am[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = h + 2 * i;
      const int p = __shfl(kp, t, 64), q0 = __shfl(k0, t, 64), q1 = __shfl(k1, t, 64);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const int key = 32 * kt + c;
        am[kt][i] = (p == key || q0 == key || q1 == key) ? (__bf16)1.0f : (__bf16)0.0f;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x8 b1, b2, b3;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float v = j == 0 ? st.x[i].x : (j == 1 ? st.x[i].y : (j == 2 ? st.x[i].z : st.x[i].w));
        __bf16 p1, p2, p3;
        split3(v, p1, p2, p3);
        b1[i] = p1; b2[i] = p2; b3[i] = p3;
      }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        acc[kt][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[kt], b3, acc[kt][j], 0, 0, 0);
        acc[kt][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[kt], b2, acc[kt][j], 0, 0, 0);
        acc[kt][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[kt], b1, acc[kt][j], 0, 0, 0);
      }
    }
  };

  // 16-token steps, the block's steps dealt to its waves round robin (stride 64 tokens). No
  // cross-step prefetch (its loop-carried registers made hipcc drain the loads at the loop
  // header); latency is hidden by two workgroups per CU instead (<= 256 registers per wave).
  const int64_t first = r_begin + 16 * wave;
  for (int64_t s0 = first; s0 < r_end; s0 += 64) {
    Step st;
    load_step(s0, st);
    compute_step(s0, st);
  }

  // waves meet in LDS in wave order: lane (c, h), register r of tile (kt, j) = S[32 kt + row(r, h)][4c + j]
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = 32 * kt + 8 * (r >> 2) + 4 * h + (r & 3);
          float4* p = reinterpret_cast<float4*>(&s_acc[key * 128 + 4 * c]);
          float4 v = make_float4(acc[kt][0][r], acc[kt][1][r], acc[kt][2][r], acc[kt][3][r]);
          if (w > 0) {
            const float4 o = *p;
            v.x = o.x + v.x; v.y = o.y + v.y; v.z = o.z + v.z; v.w = o.w + v.w;
          }
          *p = v;
        }
    }
    __syncthreads();
  }
  float* prow = a.partials + (int64_t)blockIdx.x * a.nkeys * 128;
  for (int i = tid; i < a.nkeys * 32; i += blockDim.x)
    reinterpret_cast<float4*>(prow)[i] = reinterpret_cast<const float4*>(s_acc)[i];
}

// Fold of the per-block partial rows: column j of [blocks][part_w] summed over blocks in block
// order, then added to its destination (positions, LDS-resident small tables, LN weight / bias,
// gates). One workgroup per 64 columns; its 4 waves take every 4th block row, 64 lanes read 256
// contiguous bytes of a row; the 4 wave sums are combined in LDS in wave order.
struct ReduceArgs {
  const float* partials;
  int64_t blocks;
  int part_w;
  int L, D, ntab;
  int small_total;
  int small_off[kMaxTab];
  int small_rows[kMaxTab];
  float* dtab[kMaxTab];
  float* dpos;
  float* dln_w;
  float* dln_b;
  float* dgate;
  // seq_embed_keysum_k partial rows [kblocks][kw] (kw = L*D + small_total): when present they,
  // not the LDS image columns of partials, hold positions and small tables (small-table sums
  // unscaled: multiplied by their gate here)
  const float* kpart;
  int64_t kblocks;
  const float* gate;
};

__global__ __launch_bounds__(256) void seq_embed_bwd_reduce_k(ReduceArgs a) {
  __shared__ float s_part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const int nlds = a.L * a.D + a.small_total;
  const bool from_k = a.kpart != nullptr && j < nlds;
  const float* src = from_k ? a.kpart : a.partials;
  const int64_t w = from_k ? nlds : a.part_w;
  const int64_t nb = from_k ? a.kblocks : a.blocks;
  float v = 0.0f;
  if (j < a.part_w) {
    const float* p = src + j;
    int64_t b = wave;
    for (; b + 28 < nb; b += 32) {
      float x[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = p[(b + 4 * i) * w];
#pragma unroll
      for (int i = 0; i < 8; ++i) v += x[i];
    }
    for (; b < nb; b += 4) v += p[b * w];
  }
  s_part[wave][lane] = v;
  __syncthreads();
  if (wave != 0 || j >= a.part_w) return;
  v = ((s_part[0][lane] + s_part[1][lane]) + s_part[2][lane]) + s_part[3][lane];
  const int npos = a.L * a.D;
  float* dst = nullptr;
  if (j < npos) {
    dst = a.dpos ? a.dpos + j : nullptr;
  } else if (j < nlds) {
    const int o = j - npos;
    for (int t = 0; t < a.ntab; ++t) {
      if (a.small_off[t] >= 0 && o >= a.small_off[t] && o < a.small_off[t] + a.small_rows[t] * a.D) {
        dst = a.dtab[t] ? a.dtab[t] + (o - a.small_off[t]) : nullptr;
        if (from_k) v *= a.gate ? a.gate[t] : 1.0f;
      }
    }
  } else if (j < nlds + a.D) {
    dst = a.dln_w ? a.dln_w + (j - nlds) : nullptr;
  } else if (j < nlds + 2 * a.D) {
    dst = a.dln_b ? a.dln_b + (j - nlds - a.D) : nullptr;
  } else if (j - nlds - 2 * a.D < a.ntab) {
    dst = a.dgate ? a.dgate + (j - nlds - 2 * a.D) : nullptr;
  }
  if (dst) *dst += v;
}

// row groups per wave iteration (seq_embed_fwd_k U); RSX_SEQ_EMBED_FWD_U in {1,2,4,8} overrides
// (tuning experiments)
int fwd_groups_setting() {
  static int u = [] {
    const char* s = getenv("RSX_SEQ_EMBED_FWD_U");
    const int v = s ? atoi(s) : 2;
    return (v == 1 || v == 2 || v == 4 || v == 8) ? v : 2;
  }();
  return u;
}

template <int D, int U>
void launch_fwd_u(const FwdArgs& a, hipStream_t st) {
  const int64_t rows_per_block = 4 * (64 / (D / 4)) * U;
  int64_t blocks = (a.T + rows_per_block - 1) / rows_per_block;
  if (blocks > 16384) blocks = 16384;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((seq_embed_fwd_k<D, U>), dim3((unsigned)blocks), dim3(256), 0, st, a);
}

template <int D>
int launch_fwd(const FwdArgs& a, hipStream_t st) {
  switch (fwd_groups_setting()) {
    case 1: launch_fwd_u<D, 1>(a, st); break;
    case 2: launch_fwd_u<D, 2>(a, st); break;
    case 8: launch_fwd_u<D, 8>(a, st); break;
    case 4: launch_fwd_u<D, 4>(a, st); break;
    default: launch_fwd_u<D, 2>(a, st); break;
  }
  return 0;
}

template <int D>
int launch_bwd(const BwdArgs& a, hipStream_t st, bool keysum) {
  const int64_t blocks = (a.f.T + a.rows_per_block - 1) / a.rows_per_block;
  if (keysum) {  // no scatter: positions / small tables from seq_embed_keysum_k
    static const int ub = [] {
      const char* e = getenv("RSX_SEQ_EMBED_BWD_U");
      return e ? atoi(e) : 2;
    }();
    if (ub == 4) hipLaunchKernelGGL((seq_embed_bwd_k<D, 0, false, 4>), dim3((unsigned)blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((seq_embed_bwd_k<D, 0, false, 2>), dim3((unsigned)blocks), dim3(256), 0, st, a);
    return 0;
  }
  const size_t lds = (size_t)(a.f.L * D + a.small_total) * sizeof(float);
  static const int abl = [] {
    const char* e = getenv("RSX_SEQ_EMBED_BWD_ABL");
    return e ? atoi(e) : 0;
  }();
  switch (abl) {
    case 1: hipLaunchKernelGGL((seq_embed_bwd_k<D, 1>), dim3((unsigned)blocks), dim3(256), lds, st, a); break;
    case 2: hipLaunchKernelGGL((seq_embed_bwd_k<D, 2>), dim3((unsigned)blocks), dim3(256), lds, st, a); break;
    case 3: hipLaunchKernelGGL((seq_embed_bwd_k<D, 3>), dim3((unsigned)blocks), dim3(256), lds, st, a); break;
    case 7: hipLaunchKernelGGL((seq_embed_bwd_k<D, 7>), dim3((unsigned)blocks), dim3(256), lds, st, a); break;
    default: hipLaunchKernelGGL((seq_embed_bwd_k<D, 0>), dim3((unsigned)blocks), dim3(256), lds, st, a); break;
  }
  return 0;
}

int64_t bwd_rows_per_block(int64_t T, int64_t D, int64_t target_blocks) {
  // target_blocks workgroups, each owning a contiguous token chunk
  int64_t rpb = (T + target_blocks - 1) / target_blocks;
  const int64_t quantum = 2 * 4 * (64 / (D / 4));  // two row groups per wave iteration
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

// Measurement hook (include/recsys_amd.h rsx_gather_events): HIP events around each forward gather launch,
// whichever caller issues it (the per-op path or the native tower program), for the bench's gather roofline.
struct GatherEvents {
  std::mutex mu;
  bool on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  std::vector<int64_t> tokens;
  void clear() {
    for (auto& e : ev) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
    ev.clear();
    tokens.clear();
  }
};
GatherEvents& gather_events() {
  static GatherEvents g;
  return g;
}
}  // namespace

RSX_API int rsx_gather_events(int on) {
  GatherEvents& g = gather_events();
  std::lock_guard<std::mutex> lk(g.mu);
  g.clear();
  g.on = on != 0;
  return 0;
}

RSX_API int rsx_gather_events_read(float* ms, int64_t* tokens, int max_n) {
  RSX_ARG((ms != nullptr && tokens != nullptr) || max_n == 0, "null output");
  GatherEvents& g = gather_events();
  std::lock_guard<std::mutex> lk(g.mu);
  int n = 0;
  for (size_t k = 0; k < g.ev.size() && n < max_n; ++k) {
    float t = 0.0f;
    hipError_t err = hipEventSynchronize(g.ev[k].second);
    if (err == hipSuccess) err = hipEventElapsedTime(&t, g.ev[k].first, g.ev[k].second);
    if (err != hipSuccess) {
      rsx::set_error("%s: %s", __func__, hipGetErrorString(err));
      return -1;
    }
    ms[n] = t;
    tokens[n] = g.tokens[k];
    ++n;
  }
  return n;
}

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
  GatherEvents& ge = gather_events();
  std::pair<hipEvent_t, hipEvent_t> evp{nullptr, nullptr};
  const bool timed = ge.on;  // read without the lock: toggled only between steps by the caller
  if (timed && hipEventCreate(&evp.first) == hipSuccess && hipEventCreate(&evp.second) == hipSuccess)
    (void)hipEventRecord(evp.first, st);
  if (D == 64) launch_fwd<64>(a, st);
  else if (D == 128) launch_fwd<128>(a, st);
  else launch_fwd<256>(a, st);
  RSX_LAUNCHED();
  if (timed && evp.second) {
    (void)hipEventRecord(evp.second, st);
    std::lock_guard<std::mutex> lk(ge.mu);
    ge.ev.push_back(evp);
    ge.tokens.push_back(T);
  }
  return 0;
}

// With a workspace the backward runs kBwdBlocksWs workgroups (3 per CU: the gathers of the
// LayerNorm recompute need the occupancy) that store per-block partial sums, folded by
// seq_embed_bwd_reduce_k (deterministic, no global atomics); without one, ~2 workgroups per CU
// flush their LDS sums with global float atomics.
constexpr int64_t kBwdBlocksWs = 768;  // 3 per CU: the two-group loop runs at 3 waves per SIMD
constexpr int64_t kBwdBlocksAtomic = 512;
constexpr int64_t kKeyBlocksMax = 512;  // seq_embed_keysum_k workgroups (2 per CU)

RSX_API int64_t rsx_seq_embed_bwd_workspace_floats(int64_t T, int64_t L, int64_t D) {
  if (T <= 0 || D <= 0) return 0;
  const int64_t rpb = bwd_rows_per_block(T, D, kBwdBlocksWs);
  const int64_t blocks = (T + rpb - 1) / rpb;
  return blocks * (L * D + kSmallMax + 2 * D + kMaxTab) + kKeyBlocksMax * 64 * D;
}

RSX_API int rsx_seq_embed_bwd(const float* base, const int64_t* const* ids, const float* const* tables,
                              const int64_t* table_rows, const int64_t* padding_idx, int ntab, const float* gate,
                              const float* pos, const int64_t* tok_pos, const float* ln_w, const float* mean,
                              const float* rstd, float eps, int64_t T, int64_t L, int64_t D, float p_drop,
                              uint64_t seed, const float* dout, float* dbase, float* const* dtables, float* dgate,
                              float* dpos, float* dln_w, float* dln_b, float* workspace, int64_t ws_floats,
                              void* stream) {
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
  const bool use_ws = workspace != nullptr;
  if (use_ws)
    RSX_ARG(ws_floats >= rsx_seq_embed_bwd_workspace_floats(T, L, D), "workspace too small");
  a.rows_per_block = bwd_rows_per_block(T, D, use_ws ? kBwdBlocksWs : kBwdBlocksAtomic);
  const int64_t blocks = (T + a.rows_per_block - 1) / a.rows_per_block;
  a.partials = use_ws ? workspace : nullptr;
  a.part_w = (int)(L * D + a.small_total + 2 * D + kMaxTab);
  // one-hot MFMA key sums instead of LDS atomics: D = 128 with a workspace and dbase, every live
  // table with a gradient LDS-sized (<= 2 of them), positions + small rows <= 64 keys
  KeyArgs k{};
  bool keysum = use_ws && D == 128 && dbase != nullptr && (L * D + a.small_total) <= 64 * D &&
                getenv("RSX_SEQ_EMBED_KEYSUM") == nullptr;  // =anything: the LDS-atomic kernel (A/B)
  int nsm = 0;
  for (int j = 0; j < ntab && keysum; ++j) {
    // tables too large for the LDS image keep the kernel's global scatter (when live: the gate is
    // on the device); small ones become keys (a gate of 0 scales their sums to 0 in the reduce)
    if (!a.dtab[j] || a.small_off[j] < 0) continue;
    if (nsm == 2) { keysum = false; break; }
    k.ids[nsm] = ids[j];
    k.key_off[nsm] = (int)(L + a.small_off[j] / D);
    k.pad[nsm] = a.pad_idx[j];
    ++nsm;
  }
  hipStream_t st = (hipStream_t)stream;
  if (D == 64) launch_bwd<64>(a, st, false);
  else if (D == 128) launch_bwd<128>(a, st, keysum);
  else launch_bwd<256>(a, st, false);
  const int64_t ws_a = blocks * a.part_w;
  int64_t kblocks = 0;
  if (keysum) {
    const int64_t nb = 2 * rsx::cu_count() < kKeyBlocksMax ? 2 * rsx::cu_count() : kKeyBlocksMax;  // 2 per CU
    int64_t rpb = (T + nb - 1) / nb;
    rpb = (rpb + 63) / 64 * 64;
    kblocks = (T + rpb - 1) / rpb;
    k.dx = dbase;
    k.tok_pos = tok_pos;
    k.T = T;
    k.L = (int)L;
    k.do_pos = dpos != nullptr;
    k.nkeys = (int)(L + a.small_total / D);
    k.rows_per_block = rpb;
    k.partials = workspace + ws_a;
    const dim3 g((unsigned)kblocks), b(256);
    if (tok_pos) {
      if (nsm == 0) hipLaunchKernelGGL((seq_embed_keysum_k<true, 0>), g, b, 0, st, k);
      else if (nsm == 1) hipLaunchKernelGGL((seq_embed_keysum_k<true, 1>), g, b, 0, st, k);
      else hipLaunchKernelGGL((seq_embed_keysum_k<true, 2>), g, b, 0, st, k);
    } else {
      if (nsm == 0) hipLaunchKernelGGL((seq_embed_keysum_k<false, 0>), g, b, 0, st, k);
      else if (nsm == 1) hipLaunchKernelGGL((seq_embed_keysum_k<false, 1>), g, b, 0, st, k);
      else hipLaunchKernelGGL((seq_embed_keysum_k<false, 2>), g, b, 0, st, k);
    }
  }
  if (use_ws) {
    ReduceArgs r;
    r.partials = workspace;
    r.blocks = blocks;
    r.part_w = a.part_w;
    r.L = (int)L;
    r.D = (int)D;
    r.ntab = ntab;
    r.small_total = a.small_total;
    for (int j = 0; j < kMaxTab; ++j) {
      r.small_off[j] = a.small_off[j];
      r.small_rows[j] = a.small_rows[j];
      r.dtab[j] = a.dtab[j];
    }
    r.dpos = dpos;
    r.dln_w = dln_w;
    r.dln_b = dln_b;
    r.dgate = dgate;
    r.kpart = keysum ? workspace + ws_a : nullptr;
    r.kblocks = kblocks;
    r.gate = gate;
    hipLaunchKernelGGL(seq_embed_bwd_reduce_k, dim3((unsigned)((a.part_w + 63) / 64)), dim3(256), 0, st, r);
  }
  RSX_LAUNCHED();
  return 0;
}

