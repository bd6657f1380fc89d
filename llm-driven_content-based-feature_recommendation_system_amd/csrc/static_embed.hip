// Gated lookups of the user tower's static-profile embeddings, concatenated:
//
//   out[b, off_j + c] = E_j[id_j[b]][c] * g_j        (j = 0..ntab-1, c < dim_j)
//
// Reference: SASRecUserTower static stage (tower_code/v1_refine_usertower.py:472-494:
// age/price/cnt/recency [11,16], channel/club [4,4], news/fn/active [3,4], each times
// u_g[j] = sigmoid(static_gate)[j], concatenated before cont_proj's part). PyTorch runs one
// gather per table forward and one sort-based embedding backward (~8 kernels) per table.
// Here: one forward kernel and one backward kernel for all tables. The tables are tiny (a
// few hundred floats), so each backward workgroup accumulates the table gradients of its
// row chunk in LDS and flushes the non-zero entries with one global atomic each; the gate
// gradients sum_b <dout_j, E_j[id_j[b]]> take the same route. padding_idx rows (nn.Embedding
// semantics) receive no gradient.
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

__global__ __launch_bounds__(256) void static_embed_bwd_k(SArgs a) {
  __shared__ float s_grad[kMaxFloats];
  __shared__ float s_gate[kMaxTab];
  int total = 0;
  for (int j = 0; j < a.ntab; ++j) total = a.lds_off[j] + a.rows[j] * a.dim[j];
  for (int i = threadIdx.x; i < total; i += blockDim.x) s_grad[i] = 0.0f;
  if (threadIdx.x < kMaxTab) s_gate[threadIdx.x] = 0.0f;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * a.rows_per_block;
  int64_t b1 = b0 + a.rows_per_block;
  if (b1 > a.B) b1 = a.B;
  const int64_t n = (b1 - b0) * a.ncols;
  float gsum = 0.0f;
  int gj = -1;
  for (int64_t e = threadIdx.x; e < n; e += blockDim.x) {
    const int64_t b = b0 + e / a.ncols;
    const int c = (int)(e % a.ncols);
    const int j = table_of(a, c);
    const int cc = c - a.col_off[j];
    const int64_t id = a.ids[j][b];
    const float d = a.dout[b * a.ld_out + c];
    const float g = a.gate ? a.gate[j] : 1.0f;
    if (a.dtab[j] && id != a.pad_idx[j])
      __hip_atomic_fetch_add(&s_grad[a.lds_off[j] + id * a.dim[j] + cc], d * g, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    if (a.dgate) {
      if (j != gj) {  // flush the running gate partial when the table changes
        if (gj >= 0) __hip_atomic_fetch_add(&s_gate[gj], gsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        gsum = 0.0f;
        gj = j;
      }
      gsum += d * a.tab[j][id * a.dim[j] + cc];
    }
  }
  if (a.dgate && gj >= 0) __hip_atomic_fetch_add(&s_gate[gj], gsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  for (int j = 0; j < a.ntab; ++j) {
    if (!a.dtab[j]) continue;
    const int m = a.rows[j] * a.dim[j];
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
      const float v = s_grad[a.lds_off[j] + i];
      if (v != 0.0f) atomicAdd(a.dtab[j] + i, v);
    }
  }
  if (a.dgate && threadIdx.x < a.ntab) atomicAdd(a.dgate + threadIdx.x, s_gate[threadIdx.x]);
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
                                 void* stream) {
  RSX_ARG(ids && tables && table_rows && dims && dout, "null argument");
  SArgs a;
  RSX_ARG(fill(a, ids, tables, table_rows, dims, ntab), "tables: 1..16, <= 256 columns, <= 4096 floats in total");
  RSX_ARG(ld_dout >= a.ncols, "ld_dout must cover the concatenated columns");
  for (int j = 0; j < ntab; ++j) {
    a.dtab[j] = dtables ? dtables[j] : nullptr;
    a.pad_idx[j] = padding_idx ? padding_idx[j] : -1;
  }
  if (B == 0) return 0;
  a.gate = gate; a.dgate = dgate; a.dout = dout; a.out = nullptr; a.B = B; a.ld_out = ld_dout;
  a.rows_per_block = 128;
  const int64_t blocks = (B + a.rows_per_block - 1) / a.rows_per_block;
  hipLaunchKernelGGL(static_embed_bwd_k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  RSX_LAUNCHED();
  return 0;
}
