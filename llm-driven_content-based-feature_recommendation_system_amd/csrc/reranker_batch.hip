// GDCN reranker batch builder (reference utils/data_preprocessing/feature_processor.py:144-195:
// RerankerDataset.__getitem__ + reranker_collate_fn) on device-resident feature tables:
//
//   dense[b]  = [ user_scaled[u] (3) | item_scaled[i] (6) |
//                 avg_item_price_log[i] - user_avg_price_log[u],          (price gap, :104)
//                 velocity_1w[i] * total_cnt_log[u],                       (trend 1w,  :108)
//                 velocity_1m[i] * total_cnt_log[u] ]                      (trend 1m,  :109)
//   cat[b]    = preferred_channel[u] - 1                                   (:76)
//   seq[b, t] = the last min(len_u, max_len) ids of user u's sequence, right-padded with 0 to the
//               batch's longest (pad_sequence(batch_first, padding_value=0), :188)
//   mask[b,t] = seq[b, t] != 0                                             (:189)
//   target[b] = numeric item id (int(i_id) if it is all digits, else 0)    (:179)
//
// The cross features are computed in float64 from the float64 raw tables and rounded to fp32
// once, as the reference does (numpy float64 columns -> torch.tensor(..., float32)); scaled
// tables arrive as fp32 (StandardScaler output cast once on the host). Integer / byte work:
// one thread per output element, coalesced along the row.
#include "rsx_common.h"

namespace {

struct RBArgs {
  const int64_t* uidx;     // [B] user rows
  const int64_t* iidx;     // [B] item rows
  const float* u_scaled;   // [U, 3]
  const double* u_raw;     // [U, 2]: user_avg_price_log, total_cnt_log
  const int64_t* u_cat;    // [U] preferred_channel - 1
  const float* i_scaled;   // [I, 6]
  const double* i_raw;     // [I, 3]: avg_item_price_log, velocity_1w, velocity_1m
  const int64_t* i_num;    // [I] numeric item id
  const int64_t* seq_off;  // [U + 1] CSR offsets
  const int64_t* seq_ids;  // [nnz]
  int64_t B;
  int max_len;
  int64_t L;               // output sequence width (batch max of min(len, max_len))
  float* dense;            // [B, 12]
  int64_t* cat;            // [B]
  int64_t* target;         // [B]
  int64_t* seq;            // [B, L]
  int64_t* mask;           // [B, L]
};

__global__ __launch_bounds__(256) void reranker_rows_k(RBArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (row, feature) pairs
  if (i >= a.B * 14) return;
  const int64_t b = i / 14;
  const int k = (int)(i - b * 14);
  const int64_t u = a.uidx[b], it = a.iidx[b];
  if (k < 3) {
    a.dense[b * 12 + k] = a.u_scaled[u * 3 + k];
  } else if (k < 9) {
    a.dense[b * 12 + k] = a.i_scaled[it * 6 + (k - 3)];
  } else if (k == 9) {
    a.dense[b * 12 + 9] = (float)(a.i_raw[it * 3 + 0] - a.u_raw[u * 2 + 0]);
  } else if (k < 12) {
    a.dense[b * 12 + k] = (float)(a.i_raw[it * 3 + (k - 9)] * a.u_raw[u * 2 + 1]);
  } else if (k == 12) {
    a.cat[b] = a.u_cat[u];
  } else {
    a.target[b] = a.i_num[it];
  }
}

__global__ __launch_bounds__(256) void reranker_seq_k(RBArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (row, position) pairs
  if (i >= a.B * a.L) return;
  const int64_t b = i / a.L, t = i - b * a.L;
  const int64_t u = a.uidx[b];
  const int64_t s = a.seq_off[u], e = a.seq_off[u + 1];
  int64_t n = e - s;
  if (n > a.max_len) n = a.max_len;
  const int64_t v = t < n ? a.seq_ids[e - n + t] : 0;
  a.seq[i] = v;
  a.mask[i] = v != 0 ? 1 : 0;
}

__global__ __launch_bounds__(256) void reranker_len_k(const int64_t* uidx, const int64_t* seq_off, int64_t B,
                                                      int max_len, int64_t* lens) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t u = uidx[b];
  int64_t n = seq_off[u + 1] - seq_off[u];
  lens[b] = n < max_len ? n : max_len;
}

}  // namespace

RSX_API int rsx_reranker_seq_lens(const int64_t* uidx, const int64_t* seq_off, int64_t B, int max_len, int64_t* lens,
                                  void* stream) {
  RSX_ARG(uidx && seq_off && lens, "null tensor");
  RSX_ARG(B >= 0 && max_len >= 0, "need B >= 0 and max_len >= 0");
  if (B == 0) return 0;
  hipLaunchKernelGGL(reranker_len_k, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)stream, uidx,
                     seq_off, B, max_len, lens);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_reranker_batch(const int64_t* uidx, const int64_t* iidx, int64_t B, const float* u_scaled,
                               const double* u_raw, const int64_t* u_cat, const float* i_scaled, const double* i_raw,
                               const int64_t* i_num, const int64_t* seq_off, const int64_t* seq_ids, int max_len,
                               int64_t L, float* dense, int64_t* cat, int64_t* target, int64_t* seq, int64_t* mask,
                               void* stream) {
  RSX_ARG(uidx && iidx && u_scaled && u_raw && u_cat && i_scaled && i_raw && i_num && seq_off, "null tensor");
  RSX_ARG(dense && cat && target, "null output");
  RSX_ARG(B >= 0 && L >= 0 && max_len >= 0, "need B, L, max_len >= 0");
  RSX_ARG(L == 0 || (seq && mask && seq_ids), "seq/mask/seq_ids required when L > 0");
  if (B == 0) return 0;
  RBArgs a;
  a.uidx = uidx; a.iidx = iidx; a.u_scaled = u_scaled; a.u_raw = u_raw; a.u_cat = u_cat;
  a.i_scaled = i_scaled; a.i_raw = i_raw; a.i_num = i_num; a.seq_off = seq_off; a.seq_ids = seq_ids;
  a.B = B; a.max_len = max_len; a.L = L;
  a.dense = dense; a.cat = cat; a.target = target; a.seq = seq; a.mask = mask;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(reranker_rows_k, dim3((unsigned)((B * 14 + 255) / 256)), dim3(256), 0, st, a);
  RSX_LAUNCHED();
  if (L > 0) {
    hipLaunchKernelGGL(reranker_seq_k, dim3((unsigned)((B * L + 255) / 256)), dim3(256), 0, st, a);
    RSX_LAUNCHED();
  }
  return 0;
}
