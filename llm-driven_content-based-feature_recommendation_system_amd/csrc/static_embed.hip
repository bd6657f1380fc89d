// Gated lookups of the user tower's static-profile embeddings, concatenated:
//
//   out[b, off_j + c] = E_j[id_j[b]][c] * g_j        (j = 0..ntab-1, c < dim_j)
//
// Reference: SASRecUserTower static stage (tower_code/v1_refine_usertower.py:472-494:
// age/price/cnt/recency [11,16], channel/club [4,4], news/fn/active [3,4], each times
// u_g[j] = sigmoid(static_gate)[j], concatenated before cont_proj's part). PyTorch runs one
// gather per table forward and one sort-based embedding backward (~8 kernels) per table.
// Here: one forward kernel and one backward kernel for all tables. The tables are tiny (a
// few hundred floats): the backward gives each table one workgroup that sums its gradient and
// its gate gradient sum_b <dout_j, E_j[id_j[b]]> over the users in a fixed order
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
  int lds_off[kMaxTab];   // offset of table j's gradient in LDS
  int rows[kMaxTab];
  int ntab, ncols;
  int accumulate;         // backward: 1 adds into dE / dgate, 0 writes them (padding rows get 0)
  const float* gate;      // [ntab] (nullable: 1)
  float* dgate;           // [ntab] (nullable)
  const float* dout;      // [B, ld_out]
  float* out;             // [B, ld_out]
  int64_t B, ld_out, rows_per_block;
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

// Backward, deterministic: one 1024-thread workgroup per table owns every entry of dE_j and
// dgate[j]. Thread (slice, c) walks the users b = slice, slice + nslice, ... in order, keeping
// the column-c gradient of 16 table rows in registers (a select per row: the tables have <= 11
// rows, larger ones take further 16-row passes); the slices' partials meet in LDS and are
// summed in slice order, the gate partials by a fixed shuffle tree. Same result on every run
// (no float atomics), added into dE_j / dgate like the atomics it replaces.
constexpr int kBwdThreads = 1024, kRowChunk = 16;

__global__ __launch_bounds__(1024) void static_embed_bwd_k(SArgs a) {
  __shared__ float part[kBwdThreads * kRowChunk];  // [slice][row][col]: nslice * dim <= 1024
  __shared__ float wsum[kBwdThreads / 64];
  const int j = blockIdx.x, t = threadIdx.x;
  const int dim = a.dim[j], R = a.rows[j], off = a.col_off[j];
  const int nslice = kBwdThreads / dim;
  const int cc = t % dim, sl = t / dim;
  const bool active = sl < nslice;
  const int64_t* ids = a.ids[j];
  const float* tab = a.tab[j];
  float* dtab = a.dtab[j];
  const float g = a.gate ? a.gate[j] : 1.0f;
  float gsum = 0.0f;
  for (int r0 = 0; r0 < R; r0 += kRowChunk) {
    float acc[kRowChunk];
#pragma unroll
    for (int r = 0; r < kRowChunk; ++r) acc[r] = 0.0f;
    if (active) {
      for (int64_t b = sl; b < a.B; b += nslice) {
        const int64_t id = ids[b];
        const float d = a.dout[b * a.ld_out + off + cc];
        if (r0 == 0 && a.dgate) gsum += d * tab[id * dim + cc];
        const int64_t rel = id - r0;
#pragma unroll
        for (int r = 0; r < kRowChunk; ++r) acc[r] += rel == r ? d : 0.0f;
      }
#pragma unroll
      for (int r = 0; r < kRowChunk; ++r) part[(sl * kRowChunk + r) * dim + cc] = acc[r];
    }
    __syncthreads();
    if (dtab) {
      for (int o = t; o < kRowChunk * dim; o += kBwdThreads) {
        const int r = o / dim, c2 = o % dim;
        if (r0 + r < R && r0 + r != a.pad_idx[j]) {
          float sum = 0.0f;
          for (int q = 0; q < nslice; ++q) sum += part[(q * kRowChunk + r) * dim + c2];
          if (a.accumulate)
            dtab[(int64_t)(r0 + r) * dim + c2] += sum * g;
          else
            dtab[(int64_t)(r0 + r) * dim + c2] = sum * g;
        } else if (r0 + r < R && !a.accumulate) {
          dtab[(int64_t)(r0 + r) * dim + c2] = 0.0f;
        }
      }
    }
    __syncthreads();
  }
  if (a.dgate) {
    const float w = rsx::wave_sum_width(gsum, 64);
    if ((t & 63) == 0) wsum[t >> 6] = w;
    __syncthreads();
    if (t == 0) {
      float total = 0.0f;
      for (int i = 0; i < kBwdThreads / 64; ++i) total += wsum[i];
      if (a.accumulate)
        a.dgate[j] += total;
      else
        a.dgate[j] = total;
    }
  }
}

bool fill(SArgs& a, const int64_t* const* ids, const float* const* tables, const int64_t* rows, const int64_t* dims,
          int ntab) {
  if (ntab < 1 || ntab > kMaxTab) return false;
  int c = 0, l = 0;
  for (int j = 0; j < kMaxTab; ++j) {
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
  a.gate = gate; a.dgate = nullptr; a.dout = nullptr; a.out = out; a.B = B; a.ld_out = ld_out; a.rows_per_block = 0;
  int64_t blocks = (B * a.ncols + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(static_embed_fwd_k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_static_embed_bwd(const int64_t* const* ids, const float* const* tables, const int64_t* table_rows,
                                 const int64_t* dims, const int64_t* padding_idx, int ntab, const float* gate,
                                 const float* dout, int64_t ld_dout, int64_t B, float* const* dtables, float* dgate,
                                 int accumulate, void* stream) {
  RSX_ARG(ids && tables && table_rows && dims && dout, "null argument");
  SArgs a;
  RSX_ARG(fill(a, ids, tables, table_rows, dims, ntab), "tables: 1..16, <= 256 columns, <= 4096 floats in total");
  RSX_ARG(ld_dout >= a.ncols, "ld_dout must cover the concatenated columns");
  for (int j = 0; j < ntab; ++j) {
    a.dtab[j] = dtables ? dtables[j] : nullptr;
    a.pad_idx[j] = padding_idx ? padding_idx[j] : -1;
  }
  if (B == 0 && accumulate) return 0;  // write mode still writes (zero) gradients
  a.gate = gate; a.dgate = dgate; a.dout = dout; a.out = nullptr; a.B = B; a.ld_out = ld_dout;
  a.rows_per_block = 0;
  a.accumulate = accumulate ? 1 : 0;
  hipLaunchKernelGGL(static_embed_bwd_k, dim3((unsigned)ntab), dim3(kBwdThreads), 0, (hipStream_t)stream, a);
  RSX_LAUNCHED();
  return 0;
}
