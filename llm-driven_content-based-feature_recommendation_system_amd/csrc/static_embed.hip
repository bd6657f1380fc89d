// Gated lookups of the user tower's static-profile embeddings, concatenated:
//
//   out[b, off_j + c] = E_j[id_j[b]][c] * g_j        (j = 0..ntab-1, c < dim_j)
//
// Reference: SASRecUserTower static stage (tower_code/v1_refine_usertower.py:472-494:
// age/price/cnt/recency [11,16], channel/club [4,4], news/fn/active [3,4], each times
// u_g[j] = sigmoid(static_gate)[j], concatenated before cont_proj's part). PyTorch runs one
// gather per table forward and one sort-based embedding backward (~8 kernels) per table.
// Here: one forward kernel and one backward kernel for all tables. The tables are tiny (a
// few hundred floats): the backward sums each table's gradient and its gate gradient
// sum_b <dout_j, E_j[id_j[b]]> as per-workgroup partials reduced in a fixed order
// (deterministic, no atomics). padding_idx rows (nn.Embedding semantics) receive no gradient.
// The backward adds into dE / dgate (autograd accumulation) or, with accumulate = 0, writes them.
#include "rsx_common.h"

namespace {

constexpr int kMaxTab = 16;
constexpr int kMaxCols = 256;
constexpr int kMaxFloats = 4096;  // LDS budget for all table gradients

struct SArgs {
  const int64_t* ids[kMaxTab];
  const float* tab[kMaxTab];
  float* dtab[kMaxTab];
  int64_t pad_idx[kMaxTab];
  int dim[kMaxTab];
  int col_off[kMaxTab];   // column offset of table j in the output row
  int lds_off[kMaxTab + 1];  // offset of table j's gradient in the partial / LDS layout ([ntab] = total)
  int rows[kMaxTab];
  int ntab, ncols;
  int accumulate;         // backward: 1 adds into dE / dgate, 0 writes them (padding rows get 0)
  const float* gate;      // [ntab] (nullable: 1)
  float* dgate;           // [ntab] (nullable)
  const float* dout;      // [B, ld_out]
  float* out;             // [B, ld_out]
  int64_t B, ld_out, ids_rows;  // backward: dout row b reads user b % ids_rows
};

__device__ __forceinline__ int table_of(const SArgs& a, int c) {
  int j = 0;
#pragma unroll 1
  while (j + 1 < a.ntab && c >= a.col_off[j + 1]) ++j;
  return j;
}

__global__ __launch_bounds__(256) void static_embed_fwd_k(SArgs a) {
  const int64_t n = a.B * a.ncols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / a.ncols;
    const int c = (int)(e % a.ncols);
    const int j = table_of(a, c);
    const float g = a.gate ? a.gate[j] : 1.0f;
    const int64_t id = a.ids[j][b];
    a.out[b * a.ld_out + c] = a.tab[j][id * a.dim[j] + (c - a.col_off[j])] * g;
  }
}

// Backward, deterministic, two kernels.
// static_embed_bwd_part_k: workgroup w owns dout rows [w * kUsers, (w + 1) * kUsers). Thread
//   (slice, c) walks its rows in order keeping the column-c gradient of 16 table rows in registers
//   (a select per row: the tables have <= 11 rows; larger ones take further 16-row passes) and the
//   column's gate partial sum_b dout[b, c] * E_j[id_b][c]; the slices meet in LDS in slice order and
//   the workgroup writes one partial of every table entry and every gate to the workspace.
// static_embed_bwd_fin_k: one wave per output sums its partials over the workgroups (lane-strided
//   in order, then a fixed shuffle tree), scales table entries by the gate, zeroes / skips padding
//   rows and writes or adds the result. Same result on every run (no float atomics).
// Row b of dout reads the ids of user b % ids_rows (the contrastive step's two dropout views).
constexpr int kBwdThreads = 256, kRowChunk = 16, kUsers = 64;

__global__ __launch_bounds__(kBwdThreads) void static_embed_bwd_part_k(SArgs a, float* __restrict__ part_out) {
  __shared__ float part[kBwdThreads * kRowChunk];  // [slice][row][col]: nslice * ncols <= 256
  __shared__ float gcol[kBwdThreads];
  const int t = threadIdx.x;
  const int nslice = kBwdThreads / a.ncols;
  const int c = t % a.ncols, sl = t / a.ncols;
  const bool active = sl < nslice;
  const int j = table_of(a, c);
  const int dim = a.dim[j], R = a.rows[j], cc = c - a.col_off[j];
  const int64_t b0 = (int64_t)blockIdx.x * kUsers;
  const int64_t b1 = min(b0 + kUsers, a.B);
  const int64_t* ids = a.ids[j];
  const float* tab = a.tab[j];
  const int64_t S = a.lds_off[a.ntab] + a.ntab;  // partial floats per workgroup
  float* po = part_out + (int64_t)blockIdx.x * S;
  float gsum = 0.0f;
  int maxR = 0;
  for (int q = 0; q < a.ntab; ++q) maxR = max(maxR, a.rows[q]);
  for (int r0 = 0; r0 < maxR; r0 += kRowChunk) {
    float acc[kRowChunk];
#pragma unroll
    for (int r = 0; r < kRowChunk; ++r) acc[r] = 0.0f;
    if (active && r0 < R) {
      for (int64_t b = b0 + sl; b < b1; b += nslice) {
        const int64_t id = ids[b % a.ids_rows];
        const float d = a.dout[b * a.ld_out + c];
        if (r0 == 0) gsum += d * tab[id * dim + cc];
        const int64_t rel = id - r0;
#pragma unroll
        for (int r = 0; r < kRowChunk; ++r) acc[r] += rel == r ? d : 0.0f;
      }
    }
    if (active) {
#pragma unroll
      for (int r = 0; r < kRowChunk; ++r) part[(sl * kRowChunk + r) * a.ncols + c] = acc[r];
    }
    __syncthreads();
    for (int o = t; o < kRowChunk * a.ncols; o += kBwdThreads) {
      const int r = o / a.ncols, c2 = o % a.ncols;
      const int j2 = table_of(a, c2);
      if (r0 + r < a.rows[j2]) {
        float sum = 0.0f;
        for (int q = 0; q < nslice; ++q) sum += part[(q * kRowChunk + r) * a.ncols + c2];
        po[a.lds_off[j2] + (r0 + r) * a.dim[j2] + (c2 - a.col_off[j2])] = sum;
      }
    }
    __syncthreads();
  }
  part[t] = active ? gsum : 0.0f;
  __syncthreads();
  if (t < a.ncols) {
    float v = 0.0f;
    for (int q = 0; q < nslice; ++q) v += part[q * a.ncols + t];
    gcol[t] = v;
  }
  __syncthreads();
  if (t < a.ntab) {
    float v = 0.0f;
    for (int c2 = a.col_off[t]; c2 < a.col_off[t] + a.dim[t]; ++c2) v += gcol[c2];
    po[a.lds_off[a.ntab] + t] = v;
  }
}

__global__ __launch_bounds__(256) void static_embed_bwd_fin_k(SArgs a, const float* __restrict__ parts, int nblk) {
  const int64_t S = a.lds_off[a.ntab] + a.ntab;
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;  // one wave per output
  const int lane = threadIdx.x & 63;
  if (e >= S) return;
  float v = 0.0f;
  for (int w = lane; w < nblk; w += 64) v += parts[(int64_t)w * S + e];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane != 0) return;
  if (e >= a.lds_off[a.ntab]) {  // a gate
    const int j = (int)(e - a.lds_off[a.ntab]);
    if (a.dgate) {
      if (a.accumulate) a.dgate[j] += v; else a.dgate[j] = v;
    }
    return;
  }
  int j = 0;
  while (j + 1 < a.ntab && e >= a.lds_off[j + 1]) ++j;
  if (!a.dtab[j]) return;
  const int64_t o = e - a.lds_off[j];
  const int64_t row = o / a.dim[j];
  const float g = a.gate ? a.gate[j] : 1.0f;
  const float val = row == a.pad_idx[j] ? 0.0f : v * g;
  if (a.accumulate) {
    if (row != a.pad_idx[j]) a.dtab[j][o] += val;
  } else {
    a.dtab[j][o] = val;
  }
}

bool fill(SArgs& a, const int64_t* const* ids, const float* const* tables, const int64_t* rows, const int64_t* dims,
          int ntab) {
  if (ntab < 1 || ntab > kMaxTab) return false;
  int c = 0, l = 0;
  for (int j = 0; j <= kMaxTab; ++j) {
    if (j == kMaxTab) {
      a.lds_off[j] = l;
      break;
    }
    if (j < ntab) {
      if (!ids[j] || !tables[j] || dims[j] < 1 || rows[j] < 1) return false;
      a.ids[j] = ids[j];
      a.tab[j] = tables[j];
      a.dim[j] = (int)dims[j];
      a.rows[j] = (int)rows[j];
      a.col_off[j] = c;
      a.lds_off[j] = l;
      c += (int)dims[j];
      l += (int)(rows[j] * dims[j]);
    } else {
      a.ids[j] = nullptr; a.tab[j] = nullptr; a.dim[j] = 0; a.rows[j] = 0; a.col_off[j] = c; a.lds_off[j] = l;
    }
    a.dtab[j] = nullptr;
    a.pad_idx[j] = -1;
  }
  a.lds_off[ntab] = l;
  a.ntab = ntab;
  a.ncols = c;
  a.accumulate = 1;
  return c <= kMaxCols && l <= kMaxFloats;
}

}  // namespace

RSX_API int rsx_static_embed_fwd(const int64_t* const* ids, const float* const* tables, const int64_t* table_rows,
                                 const int64_t* dims, int ntab, const float* gate, int64_t B, float* out,
                                 int64_t ld_out, void* stream) {
  RSX_ARG(ids && tables && table_rows && dims && out, "null argument");
  SArgs a;
  RSX_ARG(fill(a, ids, tables, table_rows, dims, ntab), "tables: 1..16, <= 256 columns, <= 4096 floats in total");
  RSX_ARG(ld_out >= a.ncols, "ld_out must cover the concatenated columns");
  if (B == 0) return 0;
  a.gate = gate; a.dgate = nullptr; a.dout = nullptr; a.out = out; a.B = B; a.ld_out = ld_out; a.ids_rows = B > 0 ? B : 1;
  int64_t blocks = (B * a.ncols + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(static_embed_fwd_k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int64_t rsx_static_embed_bwd_workspace_floats(int64_t B, int ntab, const int64_t* table_rows,
                                                     const int64_t* dims) {
  if (B < 0 || ntab < 1 || ntab > kMaxTab || !table_rows || !dims) return -1;
  int64_t l = 0;
  for (int j = 0; j < ntab; ++j) l += table_rows[j] * dims[j];
  return ((B + kUsers - 1) / kUsers) * (l + ntab) + 1;
}

RSX_API int rsx_static_embed_bwd(const int64_t* const* ids, const float* const* tables, const int64_t* table_rows,
                                 const int64_t* dims, const int64_t* padding_idx, int ntab, const float* gate,
                                 const float* dout, int64_t ld_dout, int64_t B, int64_t ids_rows,
                                 float* const* dtables, float* dgate, int accumulate, float* ws, int64_t ws_floats,
                                 void* stream) {
  RSX_ARG(ids && tables && table_rows && dims && (dout || B == 0), "null argument");
  SArgs a;
  RSX_ARG(fill(a, ids, tables, table_rows, dims, ntab), "tables: 1..16, <= 256 columns, <= 4096 floats in total");
  RSX_ARG(ld_dout >= a.ncols, "ld_dout must cover the concatenated columns");
  RSX_ARG(B >= 0 && (B == 0 || (ids_rows >= 1 && B % ids_rows == 0)), "B must be a multiple of ids_rows");
  RSX_ARG(ws && ws_floats >= rsx_static_embed_bwd_workspace_floats(B, ntab, table_rows, dims),
          "workspace too small (rsx_static_embed_bwd_workspace_floats)");
  for (int j = 0; j < ntab; ++j) {
    a.dtab[j] = dtables ? dtables[j] : nullptr;
    a.pad_idx[j] = padding_idx ? padding_idx[j] : -1;
  }
  a.gate = gate; a.dgate = dgate; a.dout = dout; a.out = nullptr; a.B = B; a.ld_out = ld_dout;
  a.ids_rows = ids_rows > 0 ? ids_rows : 1;
  a.accumulate = accumulate ? 1 : 0;
  if (B == 0 && accumulate) return 0;
  const int nblk = (int)((B + kUsers - 1) / kUsers);
  const int64_t S = a.lds_off[ntab] + ntab;
  if (nblk > 0) {
    hipLaunchKernelGGL(static_embed_bwd_part_k, dim3((unsigned)nblk), dim3(kBwdThreads), 0, (hipStream_t)stream, a,
                       ws);
    RSX_LAUNCHED();
  }
  // B == 0 in write mode: nblk = 0 partials, the finishing kernel writes zeros
  hipLaunchKernelGGL(static_embed_bwd_fin_k, dim3((unsigned)((S * 64 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, a, ws, nblk);
  RSX_LAUNCHED();
  return 0;
}
