// The user tower's static profile as one native call per direction (include/recsys_amd.h
// rsx_static_profile_fwd / rsx_static_profile_bwd).
//
// Reference: SASRecUserTower phase 2 (tower_code/v1_refine_usertower.py:472-494):
//   u_g  = sigmoid(static_gate)                                   [10]
//   x    = cat(E_j(id_j) * u_g[j] for the nine tables,            [U, 84]
//              relu(cont_proj(cont_feats)) * u_g[9])              [U, 16]
//   prof = Dropout(GELU(LayerNorm(static_mlp[0](x))))             [U, 128]
// PyTorch runs this as ~25 forward and ~35 backward launches (nine gathers, a library GEMM for
// the 4 -> 16 projection, ReLU / gate products, cat, the MLP GEMM, LayerNorm, GELU, dropout, and
// every op's backward node). Here: forward = one kernel that builds the whole [U, 128] input row
// (the nine gated gathers, the 4 -> 16 projection + ReLU + gate, zero padding to 128 columns) and
// the zero-padded [128, 128] MLP weight, then the library's bf16x3 GEMM, fused LayerNorm + GELU
// and dropout kernels. Backward = dropout, LayerNorm + GELU backward (dW / db of the norm), the
// MLP's weight gradient and input gradient, the nine tables' gradients (rsx_static_embed_bwd in
// write mode), the projection's gradients as per-workgroup partials and one tail kernel for their
// sum, the gates' sigmoid backward and the [128, 100] weight slice. All reductions have a fixed
// order (bit-reproducible).
#include "rsx_common.h"
#include "recsys_amd.h"

namespace {

constexpr int kD = 128, kKp = 128, kMaxTab = 16;

int64_t al(int64_t floats) { return (floats + 63) / 64 * 64; }  // 256-B granules

struct Cfg {
  int64_t U, src;  // output rows; input rows (row r reads input row r % src: both dropout views)
  int ntab, C, P, K, ncols;  // ncols = table columns (the projection's start column)
  int64_t rows[kMaxTab], dims[kMaxTab], pad[kMaxTab];
  int col_off[kMaxTab + 1];
};

struct ArenaLayout {
  int64_t flag, sid, X, Wp, H, mean, rstd, ug, total;
};
// flag (int32 at byte 0): set when an id was outside its table; sid: the ids as the forward read
// them (out-of-range ids replaced by 0), [ntab][src] int64, what the backward scatters by
ArenaLayout arena_layout(int64_t U) {
  ArenaLayout s{};
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += al(n); return r; };
  s.flag = take(1); s.sid = take(2 * kMaxTab * U);
  s.X = take(U * kKp); s.Wp = take(kD * kKp); s.H = take(U * kD); s.mean = take(U); s.rstd = take(U);
  s.ug = take(kMaxTab + 1);
  s.total = o;
  return s;
}

constexpr int kCP = 16, kCC = 4;            // cont_proj: 4 -> 16 (the reference's fixed shape)
constexpr int kNout = kCP * kCC + kCP + 1;  // dWc, dbc, the cont gate's gradient
constexpr int kRowsPerBlk = 256;

struct WsLayout {
  int64_t dY, dH, dX, dWp, dgu, wsw, wsl, wse, cpart, total, n_wsw, n_wsl, n_wse;
};
WsLayout ws_layout(int64_t U) {
  WsLayout s{};
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += al(n); return r; };
  s.dY = take(U * kD); s.dH = take(U * kD); s.dX = take(U * kKp); s.dWp = take(kD * kKp); s.dgu = take(kMaxTab + 1);
  s.n_wsw = rsx_linear_wgrad_workspace_floats(U, kD, kKp);
  s.n_wsl = rsx_ln_bwd_workspace_floats(U, kD);
  s.n_wse = ((U + 63) / 64) * (4096 + kMaxTab) + 1;  // >= rsx_static_embed_bwd_workspace_floats for any tables
  s.wsw = take(s.n_wsw); s.wsl = take(s.n_wsl); s.wse = take(s.n_wse);
  s.cpart = take(((U + kRowsPerBlk - 1) / kRowsPerBlk) * kNout);
  s.total = o;
  return s;
}

int parse(Cfg& c, const int64_t* dims) {
  c.U = dims[0];
  c.ntab = (int)dims[1];
  c.C = (int)dims[2];
  c.P = (int)dims[3];
  c.K = (int)dims[4];
  c.src = dims[5];
  RSX_ARG(c.U >= 0 && c.ntab >= 1 && c.ntab <= kMaxTab, "1..16 tables");
  RSX_ARG(c.src >= 1 && c.U % c.src == 0, "U must be a multiple of the input rows");
  RSX_ARG(c.C == 4 && c.P == 16, "cont_proj must be Linear(4, 16) (the reference's shape)");
  int off = 0;
  for (int j = 0; j < c.ntab; ++j) {
    c.rows[j] = dims[6 + j];
    c.dims[j] = dims[6 + c.ntab + j];
    c.pad[j] = dims[6 + 2 * c.ntab + j];
    RSX_ARG(c.rows[j] >= 1 && c.dims[j] >= 1, "empty table");
    c.col_off[j] = off;
    off += (int)c.dims[j];
  }
  c.col_off[c.ntab] = off;
  c.ncols = off;
  RSX_ARG(c.ncols + c.P == c.K && c.K <= kKp, "table columns + projection width must equal K <= 128");
  return 0;
}

struct InArgs {
  const int64_t* ids[kMaxTab];
  const float* tab[kMaxTab];
  int64_t rows[kMaxTab];
  int dim[kMaxTab];
  int col_off[kMaxTab + 1];
  int ntab, C, P, K, ncols;
  const float* gate;  // static_gate [ntab + 1] (raw parameter)
  const float* cont;  // [U, C]
  const float* wc;    // [P, C]
  const float* bc;    // [P]
  const float* wm;    // [128, K]
  float* X;           // [U, 128]
  float* Wp;          // [128, 128]
  float* ug;          // [ntab + 1] sigmoid(static_gate), for the backward
  int64_t* sid;       // [ntab][src] checked ids (0 where out of range)
  int* flag;          // set to 1 when any id was out of range
  int64_t U, src, x_blocks;
};

__device__ __forceinline__ float sigm(float g) { return 1.0f / (1.0f + __expf(-g)); }

__global__ __launch_bounds__(256) void prof_in_k(InArgs a) {
  if (blockIdx.x >= a.x_blocks) {  // the zero-padded MLP weight [128, 128]
    const int64_t e = (blockIdx.x - a.x_blocks) * 256 + threadIdx.x;
    if (e < kD * kKp) {
      const int n = (int)(e / kKp), k = (int)(e % kKp);
      a.Wp[e] = k < a.K ? a.wm[(int64_t)n * a.K + k] : 0.0f;
    }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x <= a.ntab) a.ug[threadIdx.x] = sigm(a.gate[threadIdx.x]);
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= a.U * kKp) return;
  const int64_t r = e / kKp % a.src;
  const int c = (int)(e % kKp);
  float v = 0.0f;
  if (c < a.ncols) {
    int j = 0;
    while (j + 1 < a.ntab && c >= a.col_off[j + 1]) ++j;
    int64_t id = a.ids[j][r];
    if (id < 0 || id >= a.rows[j]) {  // nn.Embedding raises here; this read stays in bounds
      id = 0;
      *a.flag = 1;
    }
    if (c == a.col_off[j] && e / kKp < a.src) a.sid[j * a.src + r] = id;
    v = a.tab[j][id * a.dim[j] + (c - a.col_off[j])] * sigm(a.gate[j]);
  } else if (c < a.K) {
    const int q = c - a.ncols;
    float pre = a.bc[q];
    for (int k = 0; k < a.C; ++k) pre += a.cont[r * a.C + k] * a.wc[q * a.C + k];
    v = fmaxf(pre, 0.0f) * sigm(a.gate[a.ntab]);
  }
  a.X[e] = v;
}

struct TailArgs {
  const float* dX;    // [U, 128]
  const float* cont;  // [src, C]
  const float* wc;
  const float* bc;
  const float* ug;    // [ntab + 1]
  const float* dgu;   // [ntab] table-gate gradients (rsx_static_embed_bwd)
  const float* dWp;   // [128, 128]
  float* cpart;       // [nblk][kNout] per-workgroup partials
  float* dwc;         // [P, C]
  float* dbc;         // [P]
  float* dgate;       // [ntab + 1] gradient of the raw static_gate
  float* dwm;         // [128, K]
  int64_t U, src;
  int ntab, K, ncols, nblk;
};

// The projection's backward, per-workgroup partials: thread = one output row r (input row
// r % src); its contributions to dWc [16, 4], dbc [16] and the cont gate's gradient
// sum_q dX[r, q] * relu(pre_q) are summed over the wave by a fixed shuffle tree and over the
// workgroup's four waves in order.
__global__ __launch_bounds__(kRowsPerBlk) void prof_cont_part_k(TailArgs a) {
  __shared__ float red[kRowsPerBlk / 64][kNout];
  const int64_t r = (int64_t)blockIdx.x * kRowsPerBlk + threadIdx.x;
  float acc[kNout];
#pragma unroll
  for (int o = 0; o < kNout; ++o) acc[o] = 0.0f;
  if (r < a.U) {
    const float* xr = a.cont + (r % a.src) * kCC;
    float x[kCC];
#pragma unroll
    for (int k = 0; k < kCC; ++k) x[k] = xr[k];
    const float g9 = a.ug[a.ntab];
    const float* dx = a.dX + r * kKp + a.ncols;
#pragma unroll
    for (int q = 0; q < kCP; ++q) {
      float pre = a.bc[q];
#pragma unroll
      for (int k = 0; k < kCC; ++k) pre += x[k] * a.wc[q * kCC + k];
      const float dc = dx[q];
      acc[kNout - 1] += dc * fmaxf(pre, 0.0f);
      const float dpre = pre > 0.0f ? dc * g9 : 0.0f;
#pragma unroll
      for (int k = 0; k < kCC; ++k) acc[q * kCC + k] = dpre * x[k];
      acc[kCP * kCC + q] = dpre;
    }
  }
#pragma unroll
  for (int o = 0; o < kNout; ++o) {
    float v = acc[o];
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][o] = v;
  }
  __syncthreads();
  if (threadIdx.x < kNout) {
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < kRowsPerBlk / 64; ++w) v += red[w][threadIdx.x];
    a.cpart[(int64_t)blockIdx.x * kNout + threadIdx.x] = v;
  }
}

// block 0: the partials summed in workgroup order -> dWc, dbc, the gates' sigmoid backward;
// blocks >= 1: the [128, K] slice of the padded weight gradient.
__global__ __launch_bounds__(256) void prof_tail_k(TailArgs a) {
  if (blockIdx.x > 0) {
    for (int64_t e = (int64_t)(blockIdx.x - 1) * 256 + threadIdx.x; e < (int64_t)kD * a.K;
         e += (int64_t)(gridDim.x - 1) * 256) {
      const int64_t n = e / a.K, k = e % a.K;
      a.dwm[e] = a.dWp[n * kKp + k];
    }
    return;
  }
  __shared__ float outs[kNout];
  const int t = threadIdx.x;
  if (t < kNout) {
    float v = 0.0f;
    for (int b = 0; b < a.nblk; ++b) v += a.cpart[(int64_t)b * kNout + t];
    outs[t] = v;
    if (t < kCP * kCC) a.dwc[t] = v;
    else if (t < kCP * kCC + kCP) a.dbc[t - kCP * kCC] = v;
  }
  __syncthreads();
  if (t <= a.ntab) {
    const float dg = t < a.ntab ? a.dgu[t] : outs[kNout - 1];
    const float sg = a.ug[t];
    a.dgate[t] = dg * (1.0f - sg) * sg;  // torch's sigmoid backward
  }
}

#define SP_CALL(x)            \
  do {                        \
    const int rc_ = (x);      \
    if (rc_ != 0) return rc_; \
  } while (0)

}  // namespace

RSX_API int64_t rsx_static_profile_arena_bytes(int64_t U) { return U < 0 ? -1 : arena_layout(U).total * 4; }
RSX_API int64_t rsx_static_profile_bwd_workspace_bytes(int64_t U) { return U < 0 ? -1 : ws_layout(U).total * 4; }

RSX_API int rsx_static_profile_fwd(const void* const* p, const int64_t* dims, float eps, float p_drop, uint64_t seed,
                                   void* arena, int64_t arena_bytes, float* out, void* stream) {
  RSX_ARG(p && dims && arena && out, "null argument");
  Cfg c;
  SP_CALL(parse(c, dims));
  const ArenaLayout s = arena_layout(c.U);
  RSX_ARG(arena_bytes >= s.total * 4, "arena too small (rsx_static_profile_arena_bytes)");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0, 1)");
  for (int i = 0; i < RSX_SP_N; ++i)
    if ((i < RSX_SP_IDS + c.ntab || i >= RSX_SP_IDS + kMaxTab) && (i < RSX_SP_TABLES + c.ntab || i >= RSX_SP_TABLES + kMaxTab))
      RSX_ARG(p[i] != nullptr, "null input / parameter pointer");
  hipStream_t st = (hipStream_t)stream;
  float* A = static_cast<float*>(arena);
  if (c.U == 0) {
    (void)hipMemsetAsync(A + s.flag, 0, sizeof(int), st);
    return 0;
  }
  InArgs a{};
  for (int j = 0; j < c.ntab; ++j) {
    a.ids[j] = static_cast<const int64_t*>(p[RSX_SP_IDS + j]);
    a.tab[j] = static_cast<const float*>(p[RSX_SP_TABLES + j]);
    a.dim[j] = (int)c.dims[j];
    a.rows[j] = c.rows[j];
  }
  for (int j = 0; j <= c.ntab; ++j) a.col_off[j] = c.col_off[j];
  a.ntab = c.ntab; a.C = c.C; a.P = c.P; a.K = c.K; a.ncols = c.ncols;
  a.gate = static_cast<const float*>(p[RSX_SP_GATE]);
  a.cont = static_cast<const float*>(p[RSX_SP_CONT]);
  a.wc = static_cast<const float*>(p[RSX_SP_WC]);
  a.bc = static_cast<const float*>(p[RSX_SP_BC]);
  a.wm = static_cast<const float*>(p[RSX_SP_WM]);
  a.X = A + s.X; a.Wp = A + s.Wp; a.ug = A + s.ug;
  a.sid = reinterpret_cast<int64_t*>(A + s.sid);
  a.flag = reinterpret_cast<int*>(A + s.flag);
  (void)hipMemsetAsync(a.flag, 0, sizeof(int), st);
  a.U = c.U;
  a.src = c.src;
  a.x_blocks = (c.U * kKp + 255) / 256;
  const int64_t blocks = a.x_blocks + (kD * kKp + 255) / 256;
  hipLaunchKernelGGL(prof_in_k, dim3((unsigned)blocks), dim3(256), 0, st, a);
  RSX_LAUNCHED();
  SP_CALL(rsx_gemm_x3(A + s.X, kKp, A + s.Wp, kKp, static_cast<const float*>(p[RSX_SP_BM]), c.U, kD, kKp, 0, nullptr,
                      0, 0.0f, 0, A + s.H, kD, stream));
  SP_CALL(rsx_ln_fwd(A + s.H, nullptr, 0.0f, 0, static_cast<const float*>(p[RSX_SP_LNW]),
                     static_cast<const float*>(p[RSX_SP_LNB]), eps, 2, c.U, kD, nullptr, out, A + s.mean, A + s.rstd,
                     stream));
  // Dropout(p) after the GELU: the keep-mask hash(seed, row * 128 + col) applied in place (the
  // dropout "backward" kernel is the same elementwise mask-and-scale)
  if (p_drop > 0.0f) SP_CALL(rsx_dropout_bwd(out, c.U, kD, p_drop, seed, out, stream));
  return 0;
}

RSX_API int rsx_static_profile_bwd(const void* const* p, const int64_t* dims, float p_drop, uint64_t seed,
                                   const void* arena, const float* dout, float* const* grads, void* ws,
                                   int64_t ws_bytes, void* stream) {
  RSX_ARG(p && dims && arena && dout && grads && ws, "null argument");
  Cfg c;
  SP_CALL(parse(c, dims));
  const WsLayout w = ws_layout(c.U);
  const ArenaLayout s = arena_layout(c.U);
  RSX_ARG(c.U > 0, "U must be > 0");
  RSX_ARG(ws_bytes >= w.total * 4, "workspace too small (rsx_static_profile_bwd_workspace_bytes)");
  for (int i = RSX_SP_GATE; i < RSX_SP_N; ++i)
    if (i != RSX_SP_CONT) RSX_ARG(grads[i] != nullptr, "null parameter gradient");
  for (int j = 0; j < c.ntab; ++j) RSX_ARG(grads[RSX_SP_TABLES + j] != nullptr, "null table gradient");
  hipStream_t st = (hipStream_t)stream;
  const float* A = static_cast<const float*>(arena);
  float* W = static_cast<float*>(ws);
  const float* dY = dout;
  if (c.U > 0 && p_drop > 0.0f) {
    SP_CALL(rsx_dropout_bwd(dout, c.U, kD, p_drop, seed, W + w.dY, stream));
    dY = W + w.dY;
  }
  SP_CALL(rsx_ln_bwd(A + s.H, A + s.mean, A + s.rstd, static_cast<const float*>(p[RSX_SP_LNW]),
                     static_cast<const float*>(p[RSX_SP_LNB]), 2, dY, nullptr, 0.0f, 0, c.U, kD, W + w.dH, nullptr,
                     grads[RSX_SP_LNW], grads[RSX_SP_LNB], W + w.wsl, w.n_wsl, stream));
  SP_CALL(rsx_linear_wgrad_x3(W + w.dH, kD, A + s.X, kKp, c.U, kD, kKp, W + w.dWp, kKp, grads[RSX_SP_BM], 0,
                              W + w.wsw, w.n_wsw, stream));
  if (c.U > 0)
    SP_CALL(rsx_gemm_x3_tn(W + w.dH, kD, A + s.Wp, kKp, nullptr, c.U, kKp, kD, 0, nullptr, 0, 0.0f, 0, W + w.dX, kKp,
                           stream));
  const int64_t* ids[kMaxTab];
  const float* tabs[kMaxTab];
  float* dtabs[kMaxTab];
  for (int j = 0; j < c.ntab; ++j) {  // the ids the forward checked (no out-of-range scatter)
    ids[j] = reinterpret_cast<const int64_t*>(A + s.sid) + j * c.src;
    tabs[j] = static_cast<const float*>(p[RSX_SP_TABLES + j]);
    dtabs[j] = grads[RSX_SP_TABLES + j];
  }
  // the tables' and their gates' gradients (written; row r reads user r % src)
  SP_CALL(rsx_static_embed_bwd(ids, tabs, c.rows, c.dims, c.pad, c.ntab, A + s.ug, W + w.dX, kKp, c.U, c.src, dtabs,
                               W + w.dgu, 0, W + w.wse, w.n_wse, stream));
  TailArgs t{};
  t.dX = W + w.dX;
  t.cont = static_cast<const float*>(p[RSX_SP_CONT]);
  t.wc = static_cast<const float*>(p[RSX_SP_WC]);
  t.bc = static_cast<const float*>(p[RSX_SP_BC]);
  t.ug = A + s.ug;
  t.dgu = W + w.dgu;
  t.dWp = W + w.dWp;
  t.dwc = grads[RSX_SP_WC];
  t.dbc = grads[RSX_SP_BC];
  t.dgate = grads[RSX_SP_GATE];
  t.dwm = grads[RSX_SP_WM];
  t.cpart = W + w.cpart;
  t.U = c.U;
  t.src = c.src;
  t.ntab = c.ntab; t.K = c.K; t.ncols = c.ncols;
  t.nblk = (int)((c.U + kRowsPerBlk - 1) / kRowsPerBlk);
  hipLaunchKernelGGL(prof_cont_part_k, dim3((unsigned)t.nblk), dim3(kRowsPerBlk), 0, st, t);
  RSX_LAUNCHED();
  hipLaunchKernelGGL(prof_tail_k, dim3(1 + 16), dim3(256), 0, st, t);
  RSX_LAUNCHED();
  return 0;
}
