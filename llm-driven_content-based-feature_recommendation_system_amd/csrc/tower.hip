// The user tower's packed-token training program as one native call per direction
// (include/recsys_amd.h rsx_tower_fwd / rsx_tower_bwd).
//
// Reference: SASRecUserTower.forward (tower_code/v1_refine_usertower.py:434-510) in training mode
// over the contrastive step's packed tokens, i.e. what forward_packed in the drop-in module runs
// op by op: item_proj, the gated embedding stage, the norm_first encoder stack (per layer: in_proj,
// causal + key-pad attention, out_proj + residual + norm2, feed-forward with GELU and dropout,
// residual + the next norm1), output_proj[0] over cat(token, profile[user]), LayerNorm + GELU,
// output_proj[3], F.normalize. The backward is autograd's order for that graph.
//
// Every launch below is one of this library's per-op entry points with exactly the arguments the
// per-op path passes (same kernels, same reduction orders, same dropout seeds), so the two paths
// give bit-identical results (tail mode aside: there the last layer's per-row ops past the
// attention key their dropout masks by the R kept rows' own index, so at p > 0 view 2's kept rows
// draw different -- equally independent -- masks than the all-rows program; view 1's rows and
// every p = 0 result are unchanged, see rsx_tower_fwd); what changes is the host side: ~45 forward and ~60 backward
// launches issued from here instead of one interpreted call (plus an autograd node and tensor
// allocations) each. Buffers: the caller's arena holds the activations the backward reads, the
// caller's workspace the backward's temporaries; nothing is allocated here.
#include "rsx_common.h"
#include "recsys_amd.h"

#include <utility>

namespace {

constexpr int64_t kD = 128, kQKV = 384, kF = 256, kHeads = 4, kDh = 32, kMaxLayers = 8;
constexpr int kEpiBias = 0, kEpiGeluDrop = 1, kEpiDgeluDrop = 2, kActGelu = 2;

int64_t al(int64_t floats) { return (floats + 63) / 64 * 64; }  // 256-B granules

struct LayerAct {
  int64_t qkv, a, lse, xs, hs, m2, r2, gg, act, f, xn, hn, mn, rn;
};
struct Layout {  // float offsets into the arena
  int64_t base, x0, m0, r0, h0, mh0, rh0;
  LayerAct l[kMaxLayers];
  int64_t prof, hp, g, mo, ro, o, nrm, aR, xR, tidx, tinv, tuser, tseg, lseq, total;
};

Layout layout(int64_t T, int64_t U, int nl) {
  Layout s{};
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += al(n); return r; };
  s.base = take(T * kD); s.x0 = take(T * kD); s.m0 = take(T); s.r0 = take(T);
  s.h0 = take(T * kD); s.mh0 = take(T); s.rh0 = take(T);
  for (int i = 0; i < nl; ++i) {
    LayerAct& a = s.l[i];
    a.qkv = take(T * kQKV); a.a = take(T * kD); a.lse = take(T * kHeads);
    a.xs = take(T * kD); a.hs = take(T * kD); a.m2 = take(T); a.r2 = take(T);
    a.gg = take(T * kF); a.act = take(T * kF); a.f = take(T * kD);
    a.xn = take(T * kD); a.hn = take(T * kD); a.mn = take(T); a.rn = take(T);
  }
  s.prof = take(U * kD); s.hp = take(T * kD); s.g = take(T * kD); s.mo = take(T); s.ro = take(T);
  s.o = take(T * kD); s.nrm = take(T);
  // the tail (rows the losses read, see rsx_tower_fwd): gathered attention output and layer input,
  // and the row maps (int64, two floats each)
  s.aR = take(T * kD); s.xR = take(T * kD); s.tidx = take(2 * T); s.tinv = take(2 * T); s.tuser = take(2 * T);
  s.tseg = take(2 * (U + 1)); s.lseq = take(kHeads * U);
  s.total = o;
  return s;
}

struct BwdLayout {  // float offsets into the workspace
  int64_t dO, dG, dHp, dX, dXs, dH, dHs, dF, dPre, dRes, dA, dQKV, dProf, dBase, part, dAR, dXR, wsw, wsl, wse, total;
  int64_t n_wsw, n_wsl, n_wse;
};

BwdLayout bwd_layout(int64_t T, int64_t U, int64_t L, int64_t C) {
  BwdLayout s{};
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += al(n); return r; };
  s.dO = take(T * kD); s.dG = take(T * kD); s.dHp = take(T * kD); s.dX = take(T * kD); s.dXs = take(T * kD);
  s.dH = take(T * kD); s.dHs = take(T * kD); s.dF = take(T * kD); s.dPre = take(T * kF); s.dRes = take(T * kD);
  s.dA = take(T * kD); s.dQKV = take(T * kQKV); s.dProf = take(U * kD); s.dBase = take(T * kD);
  s.part = take((C > 0 ? C : 1) * kD);
  s.dAR = take((T + 1) * kD); s.dXR = take((T + 1) * kD);  // tail rows + one zero row (the expand's source)
  int64_t w = 0;
  const int64_t nk[5][3] = {{T, kD, kD}, {T, kQKV, kD}, {T, kD, kF}, {T, kF, kD}, {U, kD, kD}};
  for (auto& q : nk) {
    const int64_t v = rsx_linear_wgrad_workspace_floats(q[0], q[1], q[2]);
    if (v > w) w = v;
  }
  s.n_wsw = w;
  s.n_wsl = rsx_ln_bwd_workspace_floats(T, kD);
  s.n_wse = rsx_seq_embed_bwd_workspace_floats(T, L, kD);
  s.wsw = take(s.n_wsw); s.wsl = take(s.n_wsl); s.wse = take(s.n_wse);
  s.total = o;
  return s;
}

int64_t n_ptrs(int nl) { return RSX_TW_LAYER0 + 12 * (int64_t)nl + 6 + 1; }  // + the tail's last rows

// The tail's row maps. Packed rows [0, T1) are view 1's tokens, [T1, 2 T1) view 2's in the same
// order; the kept rows are all of view 1 and view 2's "last" row of each user (T1 + last[j]):
// tidx[r] = the packed row of kept row r; tinv[t] = the kept row of packed row t, or R (a zero
// row) for the dropped ones; tuser[r] = its user (view 2's user j is B + j); tseg = the kept
// rows' user offsets (view 1's as they are, then one row per view-2 user).
__global__ __launch_bounds__(256) void tw_tail_k(const int64_t* __restrict__ last, int64_t T1, int64_t B,
                                                 const int64_t* __restrict__ tok_user, const int64_t* __restrict__ seg64,
                                                 int64_t* __restrict__ tidx, int64_t* __restrict__ tinv,
                                                 int64_t* __restrict__ tuser, int64_t* __restrict__ tseg) {
  const int64_t T = 2 * T1, R = T1 + B, n = T > 2 * B + 1 ? T : 2 * B + 1;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (i <= 2 * B) tseg[i] = i <= B ? seg64[i] : T1 + (i - B);
    if (i >= T) continue;
    if (i < R) {
      tidx[i] = i < T1 ? i : T1 + last[i - T1];
      tuser[i] = i < T1 ? tok_user[i] : B + (i - T1);
    }
    if (i < T1) {
      tinv[i] = i;
    } else {
      const int64_t j = tok_user[i] - B;
      tinv[i] = (i - T1 == last[j]) ? T1 + j : R;
    }
  }
}

#define TW_CALL(x)            \
  do {                        \
    const int rc_ = (x);      \
    if (rc_ != 0) return rc_; \
  } while (0)

struct View {  // typed views of the pointer table
  const void* const* p;
  const float* f(int i) const { return static_cast<const float*>(p[i]); }
  const int64_t* i64(int i) const { return static_cast<const int64_t*>(p[i]); }
};

// View 2's attention in the tail layer: only each user's "last" query row is read downstream, so
// instead of the whole causal attention of view 2's sequences, one wave per (user, head) forms
// that single row: lane k holds key k of the user's segment (L <= 64), fp32 scores over the
// head's 32 dims (scaled by 1/sqrt(32)), causal (key index <= query index) + key-padding mask,
// softmax, dropout on the probabilities (keep-mask hash(seed, ((q * 4 + h) * 64 + k)) with q the
// query's packed row: the key mha_fwd_x3 gives that row, so view 2's mask is the full program's and
// independent of view 1's), scaled by 1 / (1 - p)), out = P V. A query with no valid key gets zero output (the training path's
// fully-masked-row semantics). lse (natural log, -inf when masked) is kept for the backward.
struct LastQ {
  const float* qkv;        // [T, 384]
  const uint8_t* kpad;     // [T]
  const int64_t* seg64;    // [U + 1] packed user offsets (view 2's users are B + j)
  const int64_t* last;     // [B] view-1 token index of user j's last row (view 2: + T1)
  float* out;              // [B, 128] rows of the tail's attention output (view 2 part)
  float* lse;              // [B, 4]
  const float* dout;       // [B, 128] (backward)
  float* dqkv;             // [T, 384] (backward: view 2's rows written whole)
  int64_t T1, B;
  rsx::Dropout drop;
};

__global__ __launch_bounds__(256) void tw_lastq_fwd_k(LastQ a) {
  const int lane = threadIdx.x & 63, hd = threadIdx.x >> 6;
  const int64_t j = blockIdx.x;
  const int64_t s0 = a.seg64[a.B + j], len = a.seg64[a.B + j + 1] - s0;
  const int64_t q = a.T1 + a.last[j], qi = q - s0;
  const float* qr = a.qkv + q * kQKV + kDh * hd;
  const bool in = lane < len;
  const int64_t kr = s0 + lane;
  bool valid = in && lane <= qi && a.kpad[kr] == 0;
  float sc = -INFINITY;
  if (valid) {
    const float* kk = a.qkv + kr * kQKV + kD + kDh * hd;
    float d = 0.0f;
#pragma unroll
    for (int e = 0; e < kDh; e += 4) {
      const float4 x = *reinterpret_cast<const float4*>(qr + e), y = *reinterpret_cast<const float4*>(kk + e);
      d += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    sc = d * 0.17677669529663687f;
  }
  float m = sc;
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const float pe = valid ? expf(sc - m) : 0.0f;
  float l = pe;
  for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
  float* orow = a.out + j * kD + kDh * hd;
  if (m == -INFINITY) {  // fully masked query: zero row
    if (lane < kDh) orow[lane] = 0.0f;
    if (lane == 0) a.lse[j * kHeads + hd] = -INFINITY;
    return;
  }
  float pr = pe / l;
  pr = a.drop.apply(pr, ((uint64_t)q * kHeads + hd) * 64 + lane);
  // out[d] = sum_k pr_k V_k[d]: each lane writes its pr_k V_k row to LDS, lane d sums column d (one
  // pass over the keys instead of a 6-step wave reduction per output dim)
  __shared__ float sP[kHeads][64][kDh + 1];
  {
    const float* vr = a.qkv + kr * kQKV + 2 * kD + kDh * hd;
#pragma unroll
    for (int e = 0; e < kDh; e += 4) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (in && pr != 0.0f) v = *reinterpret_cast<const float4*>(vr + e);
      sP[hd][lane][e] = pr * v.x;
      sP[hd][lane][e + 1] = pr * v.y;
      sP[hd][lane][e + 2] = pr * v.z;
      sP[hd][lane][e + 3] = pr * v.w;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores done
  if (lane < kDh) {
    float acc = 0.0f;  // keys in order 0..len-1 (rows past len hold zeros)
    for (int k = 0; k < len; ++k) acc += sP[hd][k][lane];
    orow[lane] = acc;
  }
  if (lane == 0) a.lse[j * kHeads + hd] = m + logf(l);
}

// Its backward, writing every dqkv row of view 2's user j for head hd (32-column slices of q, k
// and v): dQ on the query row, dK / dV on the valid keys, zero elsewhere.
__global__ __launch_bounds__(256) void tw_lastq_bwd_k(LastQ a) {
  const int lane = threadIdx.x & 63, hd = threadIdx.x >> 6;
  const int64_t j = blockIdx.x;
  const int64_t s0 = a.seg64[a.B + j], len = a.seg64[a.B + j + 1] - s0;
  const int64_t q = a.T1 + a.last[j], qi = q - s0;
  const float* qr = a.qkv + q * kQKV + kDh * hd;
  const bool in = lane < len;
  const int64_t kr = s0 + lane;
  const float lse = a.lse[j * kHeads + hd];
  const bool valid = in && lane <= qi && a.kpad[kr] == 0 && lse != -INFINITY;
  const float* kk = a.qkv + kr * kQKV + kD + kDh * hd;
  const float* vr = a.qkv + kr * kQKV + 2 * kD + kDh * hd;
  const float* dor = a.dout + j * kD + kDh * hd;
  float p = 0.0f, dp = 0.0f;
  if (valid) {
    float d = 0.0f, dv = 0.0f;
#pragma unroll
    for (int e = 0; e < kDh; e += 4) {
      const float4 x = *reinterpret_cast<const float4*>(qr + e), y = *reinterpret_cast<const float4*>(kk + e);
      const float4 g = *reinterpret_cast<const float4*>(dor + e), w = *reinterpret_cast<const float4*>(vr + e);
      d += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
      dv += g.x * w.x + g.y * w.y + g.z * w.z + g.w * w.w;
    }
    p = expf(d * 0.17677669529663687f - lse);
    const uint64_t idx = ((uint64_t)q * kHeads + hd) * 64 + lane;
    dp = a.drop.apply(dv, idx);       // d/dP of out = sum_k D_k P_k v_k
  }
  float sdp = p * dp;
  for (int o = 32; o > 0; o >>= 1) sdp += __shfl_xor(sdp, o, 64);
  const float ds = valid ? p * (dp - sdp) * 0.17677669529663687f : 0.0f;  // dL/dscore, scale folded in
  // dQ = sum_k ds_k K_k: each lane's ds_k K_k row to LDS, lane d sums column d
  __shared__ float sP[kHeads][64][kDh + 1];
#pragma unroll
  for (int e = 0; e < kDh; e += 4) {
    float4 kv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid) kv = *reinterpret_cast<const float4*>(kk + e);
    sP[hd][lane][e] = ds * kv.x;
    sP[hd][lane][e + 1] = ds * kv.y;
    sP[hd][lane][e + 2] = ds * kv.z;
    sP[hd][lane][e + 3] = ds * kv.w;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores done
  float dq_d = 0.0f;  // lanes 0..31 hold dQ
  if (lane < kDh)
    for (int k = 0; k < len; ++k) dq_d += sP[hd][k][lane];
  if (in) {
    float* drow = a.dqkv + kr * kQKV;
    const float pd = valid ? a.drop.apply(p, ((uint64_t)q * kHeads + hd) * 64 + lane) : 0.0f;  // D_k P_k
#pragma unroll
    for (int e = 0; e < kDh; e += 4) {
      const float4 x = *reinterpret_cast<const float4*>(qr + e), g = *reinterpret_cast<const float4*>(dor + e);
      *reinterpret_cast<float4*>(drow + kD + kDh * hd + e) =
          make_float4(ds * x.x, ds * x.y, ds * x.z, ds * x.w);                     // dK
      *reinterpret_cast<float4*>(drow + 2 * kD + kDh * hd + e) =
          make_float4(pd * g.x, pd * g.y, pd * g.z, pd * g.w);                     // dV
    }
    if (lane != qi) {
#pragma unroll
      for (int e = 0; e < kDh; e += 4)
        *reinterpret_cast<float4*>(drow + kDh * hd + e) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // the query row's dQ slice: lane d writes dim d
  if (lane < kDh) a.dqkv[q * kQKV + kDh * hd + lane] = dq_d;
}

}  // namespace

RSX_API int64_t rsx_tower_n_ptrs(int layers) { return n_ptrs(layers); }

RSX_API int64_t rsx_tower_arena_bytes(int64_t T, int64_t U, int layers) {
  if (layers < 1 || layers > kMaxLayers || T < 0 || U < 0) return -1;
  return layout(T, U, layers).total * 4;
}

RSX_API int64_t rsx_tower_bwd_workspace_bytes(int64_t T, int64_t U, int64_t L, int layers, int64_t C) {
  if (layers < 1 || layers > kMaxLayers || T < 0 || U < 0) return -1;
  return bwd_layout(T, U, L, C).total * 4;
}

RSX_API int rsx_tower_fwd(const void* const* p, const int64_t* dims, const float* fargs, const uint64_t* seeds,
                          void* arena, int64_t arena_bytes, float* out, void* stream) {
  RSX_ARG(p && dims && fargs && seeds && arena && out, "null argument");
  const int64_t T = dims[0], U = dims[1], L = dims[2];
  const int nl = (int)dims[3];
  RSX_ARG(nl >= 1 && nl <= kMaxLayers, "1 <= layers <= 8");
  RSX_ARG(T > 0 && U > 0 && L > 0 && L <= 64, "need T, U > 0 and 0 < L <= 64");
  const Layout s = layout(T, U, nl);
  RSX_ARG(arena_bytes >= s.total * 4, "arena too small (rsx_tower_arena_bytes)");
  for (int64_t i = 0; i < n_ptrs(nl) - 1; ++i)
    if (i < RSX_TW_ITEMSEG || i >= RSX_TW_ITEM_PROJ) RSX_ARG(p[i] != nullptr, "null input / parameter pointer");
  // tail: dims[12] = B users per view (U = 2B), dims[13] = T1 view-1 tokens (T = 2 T1), p[last] =
  // view 1's "last" token of each user; 0 = every row
  const int64_t tB = dims[12], T1 = dims[13];
  const bool tail = tB > 0;
  RSX_ARG(!tail || (U == 2 * tB && T == 2 * T1 && p[n_ptrs(nl) - 1]), "tail needs U = 2B, T = 2 T1 and the last rows");
  const int64_t R = tail ? T1 + tB : T;
  const View v{p};
  float* A = static_cast<float*>(arena);
  const float pd = fargs[0];
  const int pl = RSX_TW_LAYER0 + 12 * nl;  // output head
  // item_proj (ops.linear_tok -> rsx_gemm_x3)
  TW_CALL(rsx_gemm_x3(v.f(RSX_TW_PV), kD, v.f(RSX_TW_ITEM_PROJ), kD, v.f(RSX_TW_ITEM_PROJ + 1), T, kD, kD, kEpiBias,
                      nullptr, 0, 0.0f, 0, A + s.base, kD, stream));
  // embedding stage (ops.seq_embed, packed form)
  const int64_t* ids[6];
  const float* tabs[6];
  for (int j = 0; j < 6; ++j) {
    ids[j] = v.i64(RSX_TW_IDS + j);
    tabs[j] = v.f(RSX_TW_TABLES + j);
  }
  TW_CALL(rsx_seq_embed_fwd(A + s.base, ids, tabs, 6, v.f(RSX_TW_GATE), v.f(RSX_TW_POS), v.i64(RSX_TW_TOK_POS),
                            v.f(RSX_TW_EMB_LN), v.f(RSX_TW_EMB_LN + 1), fargs[1], T, L, kD, pd, seeds[0], A + s.x0,
                            A + s.m0, A + s.r0, stream));
  // first norm1 (ops.layer_norm_pass)
  TW_CALL(rsx_ln_fwd(A + s.x0, nullptr, 0.0f, 0, v.f(RSX_TW_LAYER0), v.f(RSX_TW_LAYER0 + 1), fargs[2], 0, T, kD,
                     nullptr, A + s.h0, A + s.mh0, A + s.rh0, stream));
  const float* x = A + s.x0;
  const float* h = A + s.h0;
  const uint8_t* kp = static_cast<const uint8_t*>(p[RSX_TW_TOK_PAD]);
  const int* seg = static_cast<const int*>(p[RSX_TW_SEG32]);
  int64_t* tidx = reinterpret_cast<int64_t*>(A + s.tidx);
  int64_t* tuser = reinterpret_cast<int64_t*>(A + s.tuser);
  int64_t* tseg = reinterpret_cast<int64_t*>(A + s.tseg);
  if (tail) {
    const int64_t n = T > 2 * tB + 1 ? T : 2 * tB + 1;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(tw_tail_k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const int64_t*>(p[n_ptrs(nl) - 1]), T1, tB, v.i64(RSX_TW_TOK_USER),
                       v.i64(RSX_TW_SEG64), tidx, reinterpret_cast<int64_t*>(A + s.tinv), tuser, tseg);
    RSX_LAUNCHED();
  }
  for (int i = 0; i < nl; ++i) {
    const int q = RSX_TW_LAYER0 + 12 * i;
    const LayerAct& a = s.l[i];
    const uint64_t* sd = seeds + 1 + 4 * i;
    // in_proj + attention (ops.qkv_mha -> linear_tok + mha)
    TW_CALL(rsx_gemm_x3(h, kD, v.f(q + 2), kD, v.f(q + 3), T, (int)kQKV, (int)kD, kEpiBias, nullptr, 0, 0.0f, 0,
                        A + a.qkv, kQKV, stream));
    // the last layer from its attention on runs on the tail rows only (the losses read no other
    // row of view 2; every op past the attention is per row)
    const float* ain = A + a.a;
    const float* xin = x;
    int64_t rows = T;
    if (tail && i == nl - 1) {
      // view 1: the whole causal attention of its B sequences, written straight into tail rows
      // [0, T1); view 2: only each user's last query row (tw_lastq_fwd_k) into rows [T1, R)
      TW_CALL(rsx_mha_fwd_x3(A + a.qkv, kp, seg, tB, 64, kHeads, kDh, 1, pd, sd[0], A + s.aR, A + a.lse, stream));
      LastQ lq{};
      lq.qkv = A + a.qkv; lq.kpad = kp; lq.seg64 = v.i64(RSX_TW_SEG64); lq.last = v.i64(n_ptrs(nl) - 1);
      lq.out = A + s.aR + T1 * kD; lq.lse = A + s.lseq; lq.T1 = T1; lq.B = tB; lq.drop = rsx::make_dropout(pd, sd[0]);
      hipLaunchKernelGGL(tw_lastq_fwd_k, dim3((unsigned)tB), dim3(256), 0, (hipStream_t)stream, lq);
      RSX_LAUNCHED();
      TW_CALL(rsx_gather_rows(x, kD, tidx, R, kD, 0, 0.0f, A + s.xR, nullptr, stream));
      ain = A + s.aR;
      xin = A + s.xR;
      rows = R;
    } else {
      TW_CALL(rsx_mha_fwd_x3(A + a.qkv, kp, seg, U, 64, kHeads, kDh, 1, pd, sd[0], A + a.a, A + a.lse, stream));
    }
    // out_proj + residual + norm2 (ops.linear_add_layer_norm)
    TW_CALL(rsx_gemm_x3_addln(ain, kD, v.f(q + 4), kD, v.f(q + 5), rows, kD, kD, xin, kD, pd, sd[1], v.f(q + 6),
                              v.f(q + 7), fargs[3 + 2 * i], A + a.xs, kD, A + a.hs, kD, A + a.m2, A + a.r2, stream));
    // feed-forward (ops.ffn)
    TW_CALL(rsx_gemm_x3(A + a.hs, kD, v.f(q + 8), kD, v.f(q + 9), rows, (int)kF, (int)kD, kEpiGeluDrop, A + a.gg, kF,
                        pd, sd[2], A + a.act, kF, stream));
    TW_CALL(rsx_gemm_x3(A + a.act, kF, v.f(q + 10), kF, v.f(q + 11), rows, (int)kD, (int)kF, kEpiBias, nullptr, 0,
                        0.0f, 0, A + a.f, kD, stream));
    if (i + 1 < nl) {  // residual + the next layer's norm1 (ops.add_layer_norm)
      TW_CALL(rsx_ln_fwd(A + a.xs, A + a.f, pd, sd[3], v.f(q + 12), v.f(q + 13), fargs[2 + 2 * (i + 1)], 0, T, kD,
                         A + a.xn, A + a.hn, A + a.mn, A + a.rn, stream));
      h = A + a.hn;
    } else {  // the closing residual add (ops.add_dropout)
      TW_CALL(rsx_ln_fwd(A + a.xs, A + a.f, pd, sd[3], nullptr, nullptr, 0.0f, 0, rows, kD, A + a.xn, nullptr,
                         nullptr, nullptr, stream));
    }
    x = A + a.xn;
  }
  // output_proj[0] over cat(token, profile[user]) (ops.profile_linear): the profile half per user,
  // then the token half with those rows added in the epilogue
  const float* w0 = v.f(pl);
  TW_CALL(rsx_gemm_x3(v.f(RSX_TW_PROFILE), kD, w0 + kD, 2 * kD, v.f(pl + 1), U, kD, kD, kEpiBias, nullptr, 0, 0.0f, 0,
                      A + s.prof, kD, stream));
  TW_CALL(rsx_gemm_x3_rowadd(x, kD, w0, 2 * kD, nullptr, R, kD, kD, A + s.prof, kD,
                             tail ? tuser : v.i64(RSX_TW_TOK_USER), A + s.hp, kD, stream));
  // output_proj[1] + GELU (ops.layer_norm act), output_proj[3], F.normalize (ops.l2_normalize)
  TW_CALL(rsx_ln_fwd(A + s.hp, nullptr, 0.0f, 0, v.f(pl + 2), v.f(pl + 3), fargs[2 + 2 * nl], kActGelu, R, kD, nullptr,
                     A + s.g, A + s.mo, A + s.ro, stream));
  TW_CALL(rsx_gemm_x3(A + s.g, kD, v.f(pl + 4), kD, v.f(pl + 5), R, kD, kD, kEpiBias, nullptr, 0, 0.0f, 0, A + s.o, kD,
                      stream));
  TW_CALL(rsx_gather_rows(A + s.o, kD, nullptr, R, kD, 1, 1e-12f, out, A + s.nrm, stream));
  return 0;
}

RSX_API int rsx_tower_bwd(const void* const* p, const int64_t* dims, const float* fargs, const uint64_t* seeds,
                          const void* arena, const float* out, const float* dout, void* const* grads, void* ws,
                          int64_t ws_bytes, void* stream) {
  RSX_ARG(p && dims && fargs && seeds && arena && out && dout && grads && ws, "null argument");
  const int64_t T = dims[0], U = dims[1], L = dims[2], C = dims[4], Uq = dims[5];
  const int nl = (int)dims[3];
  RSX_ARG(nl >= 1 && nl <= kMaxLayers, "1 <= layers <= 8");
  RSX_ARG(T > 0 && U > 0 && L > 0 && L <= 64 && C >= 0 && Uq >= 0, "bad sizes");
  const Layout s = layout(T, U, nl);
  const BwdLayout b = bwd_layout(T, U, L, C);
  RSX_ARG(ws_bytes >= b.total * 4, "workspace too small (rsx_tower_bwd_workspace_bytes)");
  const int pl = RSX_TW_LAYER0 + 12 * nl;
  for (int64_t i = RSX_TW_ITEM_PROJ; i < n_ptrs(nl) - 1; ++i) RSX_ARG(grads[i] != nullptr, "null parameter gradient");
  const int64_t tB = dims[12], T1 = dims[13];
  const bool tail = tB > 0;
  RSX_ARG(!tail || (U == 2 * tB && T == 2 * T1), "tail needs U = 2B and T = 2 T1");
  const int64_t R = tail ? T1 + tB : T;
  RSX_ARG(grads[RSX_TW_GATE] && grads[RSX_TW_PROFILE], "null gate / profile gradient");
  RSX_ARG(C == 0 || (p[RSX_TW_ITEMSEG] && p[RSX_TW_ITEMSEG + 1] && p[RSX_TW_ITEMSEG + 2] && p[RSX_TW_ITEMSEG + 3] &&
                     p[RSX_TW_ITEMSEG + 4]), "item-id gradient plan required");
  const View v{p};
  const float* A = static_cast<const float*>(arena);
  float* W = static_cast<float*>(ws);
  auto G = [&](int i) { return static_cast<float*>(grads[i]); };
  const float pd = fargs[0];
  float* wsw = W + b.wsw;
  float* wsl = W + b.wsl;
  const uint8_t* kp = static_cast<const uint8_t*>(p[RSX_TW_TOK_PAD]);
  const int* seg = static_cast<const int*>(p[RSX_TW_SEG32]);
  // dW (+ db) of y = x W^T + b over the rows (ops.linear_wgrad -> rsx_linear_wgrad_x3)
  auto wgrad = [&](const float* dy, int64_t ldy, const float* xx, int64_t ldx, int64_t t, int64_t n, int64_t k,
                   float* dw, int64_t ldw, float* db) {
    return rsx_linear_wgrad_x3(dy, ldy, xx, ldx, t, n, k, dw, ldw, db, 0, wsw, b.n_wsw, stream);
  };
  // dX = dY W with W [K = out, N = in] as stored (ops._dx -> rsx_gemm_x3_tn)
  auto tn = [&](const float* dy, int64_t ldy, const float* w, int64_t ldw, int64_t m, int n, int k, float* c,
                int64_t ldc) {
    return rsx_gemm_x3_tn(dy, ldy, w, ldw, nullptr, m, n, k, kEpiBias, nullptr, 0, 0.0f, 0, c, ldc, stream);
  };
  // F.normalize (ops.l2_normalize: gather_rows backward, store); the head runs on the R output rows
  TW_CALL(rsx_scatter_rows(dout, out, A + s.nrm, nullptr, R, kD, 1, 1e-12f, 0, -1, W + b.dO, kD, stream));
  // output_proj[3] (_TokLinear: dX, then dW / db)
  TW_CALL(tn(W + b.dO, kD, v.f(pl + 4), kD, R, kD, kD, W + b.dG, kD));
  TW_CALL(wgrad(W + b.dO, kD, A + s.g, kD, R, kD, kD, G(pl + 4), kD, G(pl + 5)));
  // output_proj[1] + GELU (_LayerNorm)
  TW_CALL(rsx_ln_bwd(A + s.hp, A + s.mo, A + s.ro, v.f(pl + 2), v.f(pl + 3), kActGelu, W + b.dG, nullptr, 0.0f, 0, R,
                     kD, W + b.dHp, nullptr, G(pl + 2), G(pl + 3), wsl, b.n_wsl, stream));
  // output_proj[0] (_ProfileLinear): per-user sums, dX, d(profile), both weight halves and the bias
  const float* w0 = v.f(pl);
  const float* xl = A + s.l[nl - 1].xn;
  const int64_t* useg = tail ? reinterpret_cast<const int64_t*>(A + s.tseg) : v.i64(RSX_TW_SEG64);
  TW_CALL(rsx_segment_sum_rows(W + b.dHp, kD, nullptr, useg, nullptr, U, kD, nullptr, -1, W + b.dProf, kD, 0, stream));
  TW_CALL(tn(W + b.dHp, kD, w0, 2 * kD, R, kD, kD, W + b.dX, kD));
  TW_CALL(tn(W + b.dProf, kD, w0 + kD, 2 * kD, U, kD, kD, G(RSX_TW_PROFILE), kD));
  TW_CALL(wgrad(W + b.dHp, kD, xl, kD, R, kD, kD, G(pl), 2 * kD, nullptr));
  TW_CALL(wgrad(W + b.dProf, kD, v.f(RSX_TW_PROFILE), kD, U, kD, kD, G(pl) + kD, 2 * kD, G(pl + 1)));
  // encoder stack, last layer first. dX: gradient of the layer's output x; dH: of its output h
  // (the next layer's norm1 output, none for the last layer)
  float* dX = W + b.dX;
  float* dXs = W + b.dXs;
  float* dH = W + b.dH;
  for (int i = nl - 1; i >= 0; --i) {
    const int q = RSX_TW_LAYER0 + 12 * i;
    const LayerAct& a = s.l[i];
    const uint64_t* sd = seeds + 1 + 4 * i;
    const bool tl = tail && i == nl - 1;  // this layer's post-attention ops ran on the R tail rows
    const int64_t rows = tl ? R : T;
    float* dF = W + b.dF;
    if (i == nl - 1) {  // _AddDropout: d(xs) = dX itself, d(f) = the dropout mask applied to it
      TW_CALL(rsx_dropout_bwd(dX, rows, kD, pd, sd[3], dF, stream));
      std::swap(dX, dXs);  // dXs now names the gradient of xs
    } else {  // _AddLayerNorm of the next layer's norm1: (ds = dX, dy = dH) -> d(xs), d(f)
      const int qn = RSX_TW_LAYER0 + 12 * (i + 1);
      TW_CALL(rsx_ln_bwd(A + a.xn, A + a.mn, A + a.rn, v.f(qn), v.f(qn + 1), 0, dH, dX, pd, sd[3], T, kD, dXs, dF,
                         G(qn), G(qn + 1), wsl, b.n_wsl, stream));
    }
    // _FFN: dPre (dGELU + dropout epilogue), dW2 / db2, dW1 / db1, d(hs)
    float* dPre = W + b.dPre;
    float* dHs = W + b.dHs;
    TW_CALL(rsx_gemm_x3_tn(dF, kD, v.f(q + 10), kF, nullptr, rows, (int)kF, (int)kD, kEpiDgeluDrop,
                           const_cast<float*>(A + a.gg), kF, pd, sd[2], dPre, kF, stream));
    TW_CALL(wgrad(dF, kD, A + a.act, kF, rows, kD, kF, G(q + 10), kF, G(q + 11)));
    TW_CALL(wgrad(dPre, kF, A + a.hs, kD, rows, kF, kD, G(q + 8), kD, G(q + 9)));
    TW_CALL(tn(dPre, kF, v.f(q + 8), kD, rows, (int)kD, (int)kF, dHs, kD));
    // _LinearAddLayerNorm: (ds = d(xs), dy = d(hs)) -> d(x_in), d(out_proj output); then d(a), dWo, dbo
    float* dRes = W + b.dRes;
    float* dA = W + b.dA;
    float* dQKV = W + b.dQKV;
    if (tl) {
      // tail rows: d(x_in) lands in an R-row buffer with a zero row R and expands to every packed
      // row through the inverse map (dropped rows read the zero row); d(a) of view 1 feeds its
      // attention backward, view 2's last rows the last-query backward, which writes view 2's
      // whole dqkv rows
      float* dXR = W + b.dXR;
      float* dAR = W + b.dAR;
      (void)hipMemsetAsync(dXR + R * kD, 0, kD * sizeof(float), (hipStream_t)stream);
      TW_CALL(rsx_ln_bwd(A + a.xs, A + a.m2, A + a.r2, v.f(q + 6), v.f(q + 7), 0, dHs, dXs, pd, sd[1], R, kD, dXR, dRes,
                         G(q + 6), G(q + 7), wsl, b.n_wsl, stream));
      TW_CALL(tn(dRes, kD, v.f(q + 4), kD, R, kD, kD, dAR, kD));
      TW_CALL(wgrad(dRes, kD, A + s.aR, kD, R, kD, kD, G(q + 4), kD, G(q + 5)));
      const int64_t* tinv = reinterpret_cast<const int64_t*>(A + s.tinv);
      TW_CALL(rsx_gather_rows(dXR, kD, tinv, T, kD, 0, 0.0f, dX, nullptr, stream));
      TW_CALL(rsx_mha_bwd_x3(A + a.qkv, kp, seg, A + s.aR, A + a.lse, dAR, tB, 64, kHeads, kDh, 1, pd, sd[0], dQKV,
                             stream));
      LastQ lq{};
      lq.qkv = A + a.qkv; lq.kpad = kp; lq.seg64 = v.i64(RSX_TW_SEG64); lq.last = v.i64(n_ptrs(nl) - 1);
      lq.lse = const_cast<float*>(A + s.lseq); lq.dout = dAR + T1 * kD; lq.dqkv = dQKV; lq.T1 = T1; lq.B = tB;
      lq.drop = rsx::make_dropout(pd, sd[0]);
      hipLaunchKernelGGL(tw_lastq_bwd_k, dim3((unsigned)tB), dim3(256), 0, (hipStream_t)stream, lq);
      RSX_LAUNCHED();
    } else {
      TW_CALL(rsx_ln_bwd(A + a.xs, A + a.m2, A + a.r2, v.f(q + 6), v.f(q + 7), 0, dHs, dXs, pd, sd[1], T, kD, dX, dRes,
                         G(q + 6), G(q + 7), wsl, b.n_wsl, stream));
      TW_CALL(tn(dRes, kD, v.f(q + 4), kD, T, kD, kD, dA, kD));
      TW_CALL(wgrad(dRes, kD, A + a.a, kD, T, kD, kD, G(q + 4), kD, G(q + 5)));
      // _MHA
      TW_CALL(rsx_mha_bwd_x3(A + a.qkv, kp, seg, A + a.a, A + a.lse, dA, U, 64, kHeads, kDh, 1, pd, sd[0], dQKV,
                             stream));
    }
    // in_proj (_TokLinear)
    const float* h_in = (i == 0) ? A + s.h0 : A + s.l[i - 1].hn;
    TW_CALL(tn(dQKV, kQKV, v.f(q + 2), kD, T, (int)kD, (int)kQKV, dH, kD));
    TW_CALL(wgrad(dQKV, kQKV, h_in, kD, T, kQKV, kD, G(q + 2), kD, G(q + 3)));
  }
  // the first norm1 (_LayerNormPass: the residual gradient dX folded into its backward)
  float* dX0 = dXs;
  TW_CALL(rsx_ln_bwd(A + s.x0, A + s.mh0, A + s.rh0, v.f(RSX_TW_LAYER0), v.f(RSX_TW_LAYER0 + 1), 0, dH, dX, 0.0f, 0, T,
                     kD, dX0, nullptr, G(RSX_TW_LAYER0), G(RSX_TW_LAYER0 + 1), wsl, b.n_wsl, stream));
  // embedding stage (_SeqEmbed with the item-id sort plan): dbase; the small tables, positions,
  // LN and gates accumulated by the kernel; table 0 by the two sorted segment-sum passes
  const int64_t* ids[6];
  const float* tabs[6];
  float* dtabs[6];
  for (int j = 0; j < 6; ++j) {
    ids[j] = v.i64(RSX_TW_IDS + j);
    tabs[j] = v.f(RSX_TW_TABLES + j);
    dtabs[j] = j == 0 ? nullptr : G(RSX_TW_TABLES + j);
  }
  const int64_t rows[6] = {dims[6], dims[7], dims[8], dims[9], dims[10], dims[11]};
  const int64_t pad[6] = {0, 0, 0, 0, 0, 0};
  float* dBase = W + b.dBase;
  TW_CALL(rsx_seq_embed_bwd(A + s.base, ids, tabs, rows, pad, 6, v.f(RSX_TW_GATE), v.f(RSX_TW_POS),
                            v.i64(RSX_TW_TOK_POS), v.f(RSX_TW_EMB_LN), A + s.m0, A + s.r0, fargs[1], T, L, kD, pd,
                            seeds[0], dX0, dBase, dtabs, G(RSX_TW_GATE), G(RSX_TW_POS), G(RSX_TW_EMB_LN),
                            G(RSX_TW_EMB_LN + 1), W + b.wse, b.n_wse, stream));
  if (C > 0) {
    const int64_t* plan = v.i64(RSX_TW_ITEMSEG);  // perm
    TW_CALL(rsx_segment_sum_rows(dBase, kD, plan, v.i64(RSX_TW_ITEMSEG + 1), v.i64(RSX_TW_ITEMSEG + 2), C, kD, nullptr,
                                 -1, W + b.part, kD, 0, stream));
    TW_CALL(rsx_segment_sum_rows(W + b.part, kD, v.i64(RSX_TW_ITEMSEG + 2), v.i64(RSX_TW_ITEMSEG + 3),
                                 v.i64(RSX_TW_ITEMSEG + 4), Uq, kD, v.f(RSX_TW_GATE), 0, G(RSX_TW_TABLES), kD, 1,
                                 stream));
  }
  // item_proj (_TokLinear): d(pretrained rows) when asked, dW / db
  if (grads[RSX_TW_PV]) TW_CALL(tn(dBase, kD, v.f(RSX_TW_ITEM_PROJ), kD, T, kD, kD, G(RSX_TW_PV), kD));
  TW_CALL(wgrad(dBase, kD, v.f(RSX_TW_PV), kD, T, kD, kD, G(RSX_TW_ITEM_PROJ), kD, G(RSX_TW_ITEM_PROJ + 1)));
  return 0;
}
