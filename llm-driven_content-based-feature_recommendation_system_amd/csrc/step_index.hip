// Step index on the device: every data-dependent structure of one contrastive step, built from
// the batch's [B, L] tensors by a few kernels and two radix sorts, with ONE host read (the
// totals) instead of the ~12 size queries of the torch form (nonzero / unique /
// unique_consecutive / repeat_interleave / the count all-gather).
// Reference: the per-batch host work of train_user_tower_all_time (tower_code/
// v1_usertower_train.py:794-835: valid-step flattening, target / user ids, the DuoRec "last"
// index count-1) and the structures the grouped loss kernels read (csrc/infonce.hip GArgs).
// Same arrays, same orders, as the torch builders it replaces (PackedTokens, pack_inputs,
// ops.sort_segments, ops.TargetGroups): tests/test_gpu_step_index.py compares them element
// for element.
//
// Phase A (rsx_step_index_count, then rsx_step_index_totals after an optional all-gather):
//   si_user_k      one wave per user: token / valid-step / distinct-target counts, the user's
//                  valid targets sorted (wave bitonic sort), item-id and (user, target) pair
//                  histograms
//   si_scan_k      exclusive sums over users (token, row and pair offsets)
//   si_tloc_k      this rank's loss-row targets in flat order into a [B*L + 1] buffer (-1 pad,
//                  the row count in the last slot): the fixed-size block the ranks all-gather
//   si_colhist_k   target histogram over the gathered blocks (the global columns)
//   si_scan_k      over the item-id domain: column index, item segment offsets and chunk counts
//   si_totals_k    T, N, D, E, U, C (+ every rank's row count) -> the one host read
// Phase B (rsx_step_index_fill, sizes known): si_tokens_k (packed tokens of both views, per-token
//   ids, loss rows and their column / user ranges, per-user sorted columns, pair keys), a stable
//   radix sort of the view-1 tokens by item id and of the (user, target) pairs by column,
//   si_itemseg_k (the two-view segmented-sum plan), si_cols_k, si_pairs_k, si_pv_k (pretrained
//   rows of both views).
#include "rsx_common.h"
#include <hipcub/hipcub.hpp>
#include <limits.h>

namespace {

constexpr int kSegChunk = 64;  // ops._SEG_CHUNK

__device__ __forceinline__ uint64_t wballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ int below(uint64_t m, int lane) {
  return __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
}

// ascending bitonic sort of one value per lane across the 64-lane wave
__device__ __forceinline__ int wave_sort_asc(int v, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int o = __shfl_xor(v, j, 64);
      const bool asc = (lane & k) == 0, lower = (lane & j) == 0;
      v = (asc == lower) ? min(v, o) : max(v, o);
    }
  }
  return v;
}

struct User {
  int cnt, last;
  bool valid, sel;
  uint64_t vm, sm;
};

// the user's token selection (PackedTokens): every valid position plus the DuoRec "last"
// position count-1 (clamped at 0) when it is padding (v1_usertower_train.py:830-835)
__device__ __forceinline__ User user_sel(const uint8_t* pm, int64_t b, int L, int lane) {
  User u;
  const bool in = lane < L;
  const bool pad = in ? pm[b * L + lane] != 0 : true;
  u.valid = in && !pad;
  u.vm = wballot(u.valid);
  u.cnt = __popcll(u.vm);
  u.last = u.cnt > 0 ? u.cnt - 1 : 0;
  const bool extra = pm[b * L + u.last] != 0;
  u.sel = u.valid || (lane == u.last && extra);
  u.sm = wballot(u.sel);
  return u;
}

__device__ __forceinline__ int checked(int64_t v, int64_t n, int* err) {
  if (v < 0 || v >= n) {
    atomicOr(err, 1);
    return 0;
  }
  return (int)v;
}

// Block-level histogram aggregation in LDS (open addressing, linear probing) before the global
// atomics: the ids are heavy-tailed (Zipf-like item popularity: the most popular item carries ~9 % of
// a synthetic batch's tokens), and per-token global atomics on one hot address serialise at its L2
// channel. Counts are integers, so the histograms are exact and independent of the order.
template <int NSLOT>
struct LdsHist {
  int key[NSLOT];
  int cnt[NSLOT];
  __device__ __forceinline__ void init(int tid, int nthr) {
    for (int s = tid; s < NSLOT; s += nthr) {
      key[s] = -1;
      cnt[s] = 0;
    }
  }
  __device__ __forceinline__ void add(int v, int* global_hist) {
    int s = (int)(((unsigned)v * 2654435761u) >> 8) & (NSLOT - 1);
#pragma unroll 1
    for (int probe = 0; probe < 16; ++probe) {
      const int old = atomicCAS(&key[s], -1, v);
      if (old == -1 || old == v) {
        atomicAdd(&cnt[s], 1);
        return;
      }
      s = (s + 1) & (NSLOT - 1);
    }
    atomicAdd(&global_hist[v], 1);  // crowded table: straight to the global histogram
  }
  __device__ __forceinline__ void flush(int tid, int nthr, int* global_hist) {
    for (int s = tid; s < NSLOT; s += nthr)
      if (key[s] >= 0) atomicAdd(&global_hist[key[s]], cnt[s]);
  }
};

__global__ __launch_bounds__(256) void si_user_k(const uint8_t* pm, const int64_t* tgt, const int64_t* item, int64_t B,
                                                 int L, int64_t n_items, int* Tb, int* Nb, int* Eb, int* srt,
                                                 int* hist_i, int* hist_u, int* err) {
  __shared__ LdsHist<512> hi_, hu_;
  const int lane = threadIdx.x & 63;
  hi_.init(threadIdx.x, 256);
  hu_.init(threadIdx.x, 256);
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b < B) {  // wave-uniform (every wave reaches the barriers)
    const User u = user_sel(pm, b, L, lane);
    const int64_t o = b * L + lane;
    if (u.sel) hi_.add(checked(item[o], n_items, err), hist_i);
    int v = u.valid ? checked(tgt[o], n_items, err) : INT_MAX;
    v = wave_sort_asc(v, lane);
    const int pv = __shfl_up(v, 1, 64);
    const bool ds = lane < u.cnt && (lane == 0 || v != pv);
    const uint64_t dm = wballot(ds);
    if (lane < u.cnt) srt[b * L + lane] = v;
    if (ds) hu_.add(v, hist_u);
    if (lane == 0) {
      Tb[b] = __popcll(u.sm);
      Nb[b] = u.cnt;
      Eb[b] = __popcll(dm);
    }
  }
  __syncthreads();
  hi_.flush(threadIdx.x, 256, hist_i);
  hu_.flush(threadIdx.x, 256, hist_u);
}

__global__ __launch_bounds__(256) void si_tloc_k(const uint8_t* pm, const int64_t* tgt, int64_t B, int L,
                                                 int64_t n_items, const int* offN, int* tloc, int* err) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const User u = user_sel(pm, b, L, lane);
  if (u.valid) tloc[offN[b] + below(u.vm, lane)] = checked(tgt[b * L + lane], n_items, err);
}

// The block's row-count slot, with this rank's id-range error in bit 30 (written after every
// range check of the count phase): at world > 1 the slots are all-gathered with the targets, so
// every rank's totals see every rank's error and all of them raise together (no rank carries on
// into the step's collectives alone).
constexpr int kSlotErr = 1 << 30;
__global__ void si_slot_k(const int* offN, const int* err, int64_t B, int64_t L, int* tloc) {
  if (threadIdx.x == 0) tloc[B * L] = offN[B] | (*err ? kSlotErr : 0);
}

__global__ __launch_bounds__(256) void si_colhist_k(const int* tglob, int64_t n, int64_t blk, int64_t n_items,
                                                    int* hist_t) {
  __shared__ LdsHist<2048> h;
  h.init(threadIdx.x, 256);
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (i % blk == blk - 1) continue;  // a block's row-count slot
    const int v = tglob[i];
    if (v >= 0 && v < n_items) h.add(v, hist_t);
  }
  __syncthreads();
  h.flush(threadIdx.x, 256, hist_t);
}

__device__ __forceinline__ int scan_xform(int x, int mode) {
  return mode == 0 ? x : mode == 1 ? (x > 0 ? 1 : 0) : (2 * x + kSegChunk - 1) / kSegChunk;
}

// Exclusive sums of up to five int arrays, one workgroup per array (the arrays are short: B + 1
// users or n_items + 1 ids), each thread holding 4 consecutive elements of a 4096-element tile,
// with an optional transform of the input (mode 0 identity, 1 "> 0", 2 DuoRec-segment chunk
// count of an item id with x view-1 tokens). One launch instead of one multi-kernel library scan
// per array: the step index runs beside the step on a side stream, where every extra launch
// waits for CU slots.
struct ScanJob {
  const int* in;
  int* out;
  int n, mode;
};
struct ScanJobs {
  ScanJob j[5];
};

__global__ __launch_bounds__(1024) void si_scan_k(ScanJobs js) {
  const ScanJob J = js.j[blockIdx.x];
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int carry = 0;
  for (int base = 0; base < J.n; base += 4096) {
    const int i0 = base + tid * 4;
    int v[4], s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = i0 + k < J.n ? scan_xform(J.in[i0 + k], J.mode) : 0;
      s += v[k];
    }
    int x = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (w == 0) {
      int t = lane < 16 ? wsum[lane] : 0;
#pragma unroll
      for (int d = 1; d < 16; d <<= 1) {
        const int y = __shfl_up(t, d, 64);
        if (lane >= d) t += y;
      }
      if (lane < 16) wsum[lane] = t;
    }
    __syncthreads();
    int e = carry + (w > 0 ? wsum[w - 1] : 0) + x - s;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i0 + k < J.n) J.out[i0 + k] = e;
      e += v[k];
    }
    carry += wsum[15];
    __syncthreads();  // wsum is rewritten by the next tile
  }
}

__global__ void si_totals_k(const int* offT, const int* offN, const int* offE, const int* colidx, const int* itemidx,
                            const int* chunkoff, const int* err, const int* tglob, int world, int64_t B, int64_t L,
                            int64_t n_items, int64_t* tot) {
  if (threadIdx.x != 0) return;
  tot[0] = offT[B];
  tot[1] = offN[B];
  tot[2] = colidx[n_items];
  tot[3] = offE[B];
  tot[4] = itemidx[n_items];
  tot[5] = chunkoff[n_items];
  int e = *err ? 1 : 0;
  tot[7] = 0;
  for (int r = 0; r < world; ++r) {
    const int v = tglob[(int64_t)r * (B * L + 1) + B * L];
    e |= (v & kSlotErr) ? 1 : 0;
    tot[8 + r] = v & ~kSlotErr;
  }
  tot[6] = e;
}

struct FillOut {
  int64_t *flat1, *user1, *pos1;
  uint8_t* pad1;
  int* seg1;
  int64_t* seg1_64;
  int64_t *valid_tok, *last_tok;
  int64_t *flat2, *user2, *pos2;
  uint8_t* pad2;
  int* seg2;
  int64_t* seg2_64;
  int64_t* tok_ids;  // [6][2T]
  int *row_col, *row_beg, *row_end, *exc_cols;
  int* last_t;  // int32: the SupCon kernel's key type (ids < n_items < 2^31)
};

__global__ __launch_bounds__(256) void si_tokens_k(const uint8_t* pm, const int64_t* tgt, const int64_t* ids0,
                                                   const int64_t* ids1, const int64_t* ids2, const int64_t* ids3,
                                                   const int64_t* ids4, const int64_t* ids5, int64_t B, int L,
                                                   int64_t T, const int* offT, const int* offN, const int* offE,
                                                   const int* srt, const int* colidx, FillOut f, unsigned* ikeys,
                                                   int* ivals, unsigned* pkeys, int* pvals, int* pair_b, int* pair_n) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const User u = user_sel(pm, b, L, lane);
  const int64_t o = b * L + lane;
  const int64_t t0 = offT[b];
  if (u.sel) {
    const int64_t tok = t0 + below(u.sm, lane);
    const uint8_t pd = u.valid ? 0 : 1;
    f.flat1[tok] = o;
    f.user1[tok] = b;
    f.pos1[tok] = lane;
    f.pad1[tok] = pd;
    f.flat2[tok] = o;
    f.flat2[T + tok] = B * L + o;
    f.user2[tok] = b;
    f.user2[T + tok] = B + b;
    f.pos2[tok] = lane;
    f.pos2[T + tok] = lane;
    f.pad2[tok] = pd;
    f.pad2[T + tok] = pd;
    const int64_t* src[6] = {ids0, ids1, ids2, ids3, ids4, ids5};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int64_t v = src[k][o];
      f.tok_ids[(2 * k) * T + tok] = v;
      f.tok_ids[(2 * k + 1) * T + tok] = v;
    }
    ikeys[tok] = (unsigned)ids0[o];  // range-checked in phase A
    ivals[tok] = (int)tok;
    if (u.valid) {
      const int64_t r = offN[b] + below(u.vm, lane);
      f.valid_tok[r] = tok;
      f.row_col[r] = colidx[tgt[o]];
      f.row_beg[r] = offN[b];
      f.row_end[r] = offN[b + 1];
    }
  }
  if (lane < u.cnt) {  // the user's targets sorted (with repeats) -> its exception columns
    const int v = srt[b * L + lane];
    const int c = colidx[v];
    f.exc_cols[offN[b] + lane] = c;
    const int pv = __shfl_up(v, 1, 64);
    (void)pv;
  }
  {  // distinct (user, target) pairs with multiplicities, in user order, keyed by column
    const int v = lane < u.cnt ? srt[b * L + lane] : INT_MAX;
    const int pv = __shfl_up(v, 1, 64);
    const bool ds = lane < u.cnt && (lane == 0 || v != pv);
    const uint64_t dm = wballot(ds);
    if (ds) {
      const uint64_t higher = (lane == 63) ? 0ull : (dm & (~0ull << (lane + 1)));
      const int nxt = higher ? (__ffsll((long long)higher) - 1) : u.cnt;
      const int64_t e = offE[b] + below(dm, lane);
      pkeys[e] = (unsigned)colidx[v];
      pvals[e] = (int)e;
      pair_b[e] = (int)b;
      pair_n[e] = nxt - lane;
    }
  }
  if (lane == 0) {
    f.last_tok[b] = t0 + __popcll(u.sm & ((u.last == 0) ? 0ull : (~0ull >> (64 - u.last))));
    f.last_t[b] = (int)tgt[b * L + u.last];
    f.seg1[b] = (int)t0;
    f.seg1_64[b] = t0;
    f.seg2[b] = (int)t0;
    f.seg2_64[b] = t0;
    f.seg2[B + b] = (int)(T + t0);
    f.seg2_64[B + b] = T + t0;
    if (b == B - 1) {
      f.seg1[B] = (int)T;
      f.seg1_64[B] = T;
      f.seg2[2 * B] = (int)(2 * T);
      f.seg2_64[2 * B] = 2 * T;
    }
  }
}

// the two-view segmented-sum plan of ops.sort_segments over tok_ids[0] (2T tokens): the stable
// order lists, per item id u (ascending), its view-1 tokens then their view-2 copies (T + t);
// chunks of <= 64 sorted tokens never straddle two ids
__global__ __launch_bounds__(256) void si_itemseg_k(const unsigned* skeys, const int* svals, int64_t T,
                                                    const int* hist_i, const int* itemoff, const int* itemidx,
                                                    const int* chunkoff, int64_t U, int64_t C, int64_t* perm,
                                                    int64_t* cb, int64_t* chunk_ids, int64_t* ch_off,
                                                    int64_t* uniq_items) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < T; p += (int64_t)gridDim.x * 256) {
    const unsigned id = skeys[p];
    const int64_t a = itemoff[id], n = hist_i[id], w = p - a;
    const int64_t tok = svals[p];
    perm[2 * a + w] = tok;
    perm[2 * a + n + w] = T + tok;
    if (w == 0) {
      const int64_t ui = itemidx[id], c0 = chunkoff[id];
      uniq_items[ui] = id;
      ch_off[ui] = c0;
      const int64_t nch = (2 * n + kSegChunk - 1) / kSegChunk;
      for (int64_t k = 0; k < nch; ++k) {
        cb[c0 + k] = 2 * a + kSegChunk * k;
        chunk_ids[c0 + k] = c0 + k;
      }
    }
    if (p == 0) {
      ch_off[U] = C;
      cb[C] = 2 * T;
    }
  }
}

__global__ __launch_bounds__(256) void si_cols_k(const int* hist_t, const int* hist_u, const int* colidx,
                                                 const int* pairoff, int64_t n_items, int64_t* uniq, float* colcnt,
                                                 int* col_beg, int* col_end) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n_items; v += (int64_t)gridDim.x * 256) {
    const int h = hist_t[v];
    if (h == 0) continue;
    const int d = colidx[v];
    uniq[d] = v;
    colcnt[d] = (float)h;
    col_beg[d] = pairoff[v];
    col_end[d] = pairoff[v] + hist_u[v];
  }
}

__global__ __launch_bounds__(256) void si_pairs_k(const int* spvals, int64_t E, const int* pair_b, const int* pair_n,
                                                  const int* offN, int* exc_s, int* exc_e, int* exc_n) {
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < E; q += (int64_t)gridDim.x * 256) {
    const int e = spvals[q];
    const int b = pair_b[e];
    exc_s[q] = offN[b];
    exc_e[q] = offN[b + 1];
    exc_n[q] = pair_n[e];
  }
}

// pretrained rows of the view-1 tokens' item ids into both halves of [2T, 128]
__global__ __launch_bounds__(256) void si_pv_k(const float* lookup, int64_t ld, const int64_t* ids_tok, int64_t T,
                                               float* pv) {
  const int lane = threadIdx.x & 31;
  for (int64_t t = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 5; t < T; t += ((int64_t)gridDim.x * 256) >> 5) {
    const float4 v = reinterpret_cast<const float4*>(lookup + ids_tok[t] * ld)[lane];
    reinterpret_cast<float4*>(pv + t * 128)[lane] = v;
    reinterpret_cast<float4*>(pv + (T + t) * 128)[lane] = v;
  }
}

int64_t a256(int64_t x) { return (x + 255) / 256 * 256; }

struct SiLayout {
  int64_t err, Tb, Nb, Eb, offT, offN, offE, srt, hist_t, hist_u, hist_i, colidx, itemidx, itemoff, chunkoff,
      pairoff, ikeys, ivals, ikeys_o, ivals_o, pkeys, pvals, pkeys_o, pvals_o, pair_b, pair_n, temp, temp_bytes,
      total;
};

int bits_for(int64_t n) {  // bits of the largest key value n - 1
  int b = 1;
  while (b < 32 && ((int64_t)1 << b) < n) ++b;
  return b;
}

size_t temp_bytes(int64_t B, int64_t L, int64_t n_items) {
  size_t s = 0;
  int* ip = nullptr;
  unsigned* up = nullptr;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, s, up, up, ip, ip, (int)(B * L), 0, 32);
  return s;
}

SiLayout si_layout(int64_t B, int64_t L, int64_t n_items) {
  SiLayout l;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    const int64_t r = o;
    o += a256(bytes);
    return r;
  };
  const int64_t BL = B * L, ni = n_items + 1;
  l.err = take(4);
  l.Tb = take((B + 1) * 4);
  l.Nb = take((B + 1) * 4);
  l.Eb = take((B + 1) * 4);
  l.offT = take((B + 1) * 4);
  l.offN = take((B + 1) * 4);
  l.offE = take((B + 1) * 4);
  l.srt = take(BL * 4);
  l.hist_t = take(ni * 4);
  l.hist_u = take(ni * 4);
  l.hist_i = take(ni * 4);
  l.colidx = take(ni * 4);
  l.itemidx = take(ni * 4);
  l.itemoff = take(ni * 4);
  l.chunkoff = take(ni * 4);
  l.pairoff = take(ni * 4);
  l.ikeys = take(BL * 4);
  l.ivals = take(BL * 4);
  l.ikeys_o = take(BL * 4);
  l.ivals_o = take(BL * 4);
  l.pkeys = take(BL * 4);
  l.pvals = take(BL * 4);
  l.pkeys_o = take(BL * 4);
  l.pvals_o = take(BL * 4);
  l.pair_b = take(BL * 4);
  l.pair_n = take(BL * 4);
  l.temp_bytes = (int64_t)temp_bytes(B, L, n_items);
  l.temp = take(l.temp_bytes);
  l.total = o;
  return l;
}

template <typename P>
P* at(void* ws, int64_t off) {
  return reinterpret_cast<P*>(reinterpret_cast<char*>(ws) + off);
}

unsigned grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace

RSX_API int64_t rsx_step_index_workspace_bytes(int64_t B, int64_t L, int64_t n_items) {
  return si_layout(B, L, n_items).total;
}

RSX_API int rsx_step_index_count(const uint8_t* pm, const int64_t* tgt, const int64_t* item, int64_t B, int64_t L,
                                 int64_t n_items, void* ws, int64_t ws_bytes, int* tloc, void* stream) {
  RSX_ARG(pm && tgt && item && ws && tloc, "null tensor");
  RSX_ARG(B >= 1 && L >= 1 && L <= 64, "need B >= 1 and 1 <= L <= 64 (one wave per user)");
  RSX_ARG(n_items >= 1 && n_items < INT_MAX && B * L < (1 << 30), "sizes must fit int32 (B * L < 2^30)");
  const SiLayout l = si_layout(B, L, n_items);
  RSX_ARG(ws_bytes >= l.total, "workspace too small (rsx_step_index_workspace_bytes)");
  hipStream_t st = (hipStream_t)stream;
  // zero err .. Eb and the three histograms (the ranges are contiguous)
  (void)hipMemsetAsync(at<char>(ws, l.err), 0, l.offT - l.err, st);
  (void)hipMemsetAsync(at<char>(ws, l.hist_t), 0, l.colidx - l.hist_t, st);
  (void)hipMemsetAsync(tloc, 0xff, (B * L + 1) * 4, st);
  const unsigned gu = (unsigned)((B + 3) / 4);
  hipLaunchKernelGGL(si_user_k, dim3(gu), dim3(256), 0, st, pm, tgt, item, B, (int)L, n_items, at<int>(ws, l.Tb),
                     at<int>(ws, l.Nb), at<int>(ws, l.Eb), at<int>(ws, l.srt), at<int>(ws, l.hist_i),
                     at<int>(ws, l.hist_u), at<int>(ws, l.err));
  RSX_LAUNCHED();
  {
    ScanJobs js{};
    const int nb = (int)(B + 1);
    js.j[0] = {at<int>(ws, l.Tb), at<int>(ws, l.offT), nb, 0};
    js.j[1] = {at<int>(ws, l.Nb), at<int>(ws, l.offN), nb, 0};
    js.j[2] = {at<int>(ws, l.Eb), at<int>(ws, l.offE), nb, 0};
    hipLaunchKernelGGL(si_scan_k, dim3(3), dim3(1024), 0, st, js);
    RSX_LAUNCHED();
  }
  hipLaunchKernelGGL(si_tloc_k, dim3(gu), dim3(256), 0, st, pm, tgt, B, (int)L, n_items, at<int>(ws, l.offN), tloc,
                     at<int>(ws, l.err));
  RSX_LAUNCHED();
  hipLaunchKernelGGL(si_slot_k, dim3(1), dim3(64), 0, st, at<int>(ws, l.offN), at<int>(ws, l.err), B, L, tloc);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_step_index_totals(const int* tglob, int world, int64_t B, int64_t L, int64_t n_items, void* ws,
                                  int64_t ws_bytes, int64_t* totals, void* stream) {
  RSX_ARG(tglob && ws && totals, "null tensor");
  RSX_ARG(world >= 1, "world >= 1");
  const SiLayout l = si_layout(B, L, n_items);
  RSX_ARG(ws_bytes >= l.total, "workspace too small (rsx_step_index_workspace_bytes)");
  hipStream_t st = (hipStream_t)stream;
  const int64_t blk = B * L + 1, n = blk * world;
  // ~1,600 tokens per block: enough repeats of the popular ids for the LDS aggregation to pay
  hipLaunchKernelGGL(si_colhist_k, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(256, (n + 1023) / 1024))),
                     dim3(256), 0, st, tglob, n, blk, n_items,
                     at<int>(ws, l.hist_t));
  RSX_LAUNCHED();
  {
    const int ni = (int)(n_items + 1);  // the extra (zero) element makes entry n_items the total
    ScanJobs js{};
    js.j[0] = {at<int>(ws, l.hist_t), at<int>(ws, l.colidx), ni, 1};
    js.j[1] = {at<int>(ws, l.hist_i), at<int>(ws, l.itemidx), ni, 1};
    js.j[2] = {at<int>(ws, l.hist_i), at<int>(ws, l.itemoff), ni, 0};
    js.j[3] = {at<int>(ws, l.hist_i), at<int>(ws, l.chunkoff), ni, 2};
    js.j[4] = {at<int>(ws, l.hist_u), at<int>(ws, l.pairoff), ni, 0};
    hipLaunchKernelGGL(si_scan_k, dim3(5), dim3(1024), 0, st, js);
    RSX_LAUNCHED();
  }
  hipLaunchKernelGGL(si_totals_k, dim3(1), dim3(64), 0, st, at<int>(ws, l.offT), at<int>(ws, l.offN),
                     at<int>(ws, l.offE), at<int>(ws, l.colidx), at<int>(ws, l.itemidx), at<int>(ws, l.chunkoff),
                     at<int>(ws, l.err), tglob, world, B, L, n_items, totals);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_step_index_fill(const uint8_t* pm, const int64_t* tgt, const int64_t* const* seq_ids,
                                const float* lookup, int64_t ld_lookup, int64_t B, int64_t L, int64_t n_items,
                                const int64_t* sizes, void* ws, int64_t ws_bytes, void* const* out, void* stream) {
  RSX_ARG(pm && tgt && seq_ids && sizes && ws && out, "null tensor");
  const SiLayout l = si_layout(B, L, n_items);
  RSX_ARG(ws_bytes >= l.total, "workspace too small (rsx_step_index_workspace_bytes)");
  const int64_t T = sizes[0], N = sizes[1], D = sizes[2], E = sizes[3], U = sizes[4], C = sizes[5];
  RSX_ARG(T >= B && T <= B * L && N >= 0 && N <= T && D >= 0 && E >= 0 && E <= N && U >= 1 && C >= U,
          "inconsistent sizes (rsx_step_index_totals)");
  hipStream_t st = (hipStream_t)stream;
  FillOut f;
  f.flat1 = (int64_t*)out[0]; f.user1 = (int64_t*)out[1]; f.pos1 = (int64_t*)out[2]; f.pad1 = (uint8_t*)out[3];
  f.seg1 = (int*)out[4]; f.seg1_64 = (int64_t*)out[5]; f.valid_tok = (int64_t*)out[6]; f.last_tok = (int64_t*)out[7];
  f.flat2 = (int64_t*)out[8]; f.user2 = (int64_t*)out[9]; f.pos2 = (int64_t*)out[10]; f.pad2 = (uint8_t*)out[11];
  f.seg2 = (int*)out[12]; f.seg2_64 = (int64_t*)out[13]; f.tok_ids = (int64_t*)out[14];
  f.row_col = (int*)out[23]; f.row_beg = (int*)out[24]; f.row_end = (int*)out[25]; f.exc_cols = (int*)out[26];
  f.last_t = (int*)out[32];
  const unsigned gu = (unsigned)((B + 3) / 4);
  hipLaunchKernelGGL(si_tokens_k, dim3(gu), dim3(256), 0, st, pm, tgt, seq_ids[0], seq_ids[1], seq_ids[2],
                     seq_ids[3], seq_ids[4], seq_ids[5], B, (int)L, T, at<int>(ws, l.offT), at<int>(ws, l.offN),
                     at<int>(ws, l.offE), at<int>(ws, l.srt), at<int>(ws, l.colidx), f, at<unsigned>(ws, l.ikeys),
                     at<int>(ws, l.ivals), at<unsigned>(ws, l.pkeys), at<int>(ws, l.pvals), at<int>(ws, l.pair_b),
                     at<int>(ws, l.pair_n));
  RSX_LAUNCHED();
  size_t tb = (size_t)l.temp_bytes;
  void* tmp = at<void>(ws, l.temp);
  // stable LSD radix sorts: tokens by item id (token order kept within an id), pairs by column
  // (user order kept within a column)
  (void)hipcub::DeviceRadixSort::SortPairs(tmp, tb, at<unsigned>(ws, l.ikeys), at<unsigned>(ws, l.ikeys_o),
                                           at<int>(ws, l.ivals), at<int>(ws, l.ivals_o), (int)T, 0,
                                           bits_for(n_items), st);
  RSX_LAUNCHED();
  hipLaunchKernelGGL(si_itemseg_k, dim3(grid_for(T)), dim3(256), 0, st, at<unsigned>(ws, l.ikeys_o),
                     at<int>(ws, l.ivals_o), T, at<int>(ws, l.hist_i), at<int>(ws, l.itemoff), at<int>(ws, l.itemidx),
                     at<int>(ws, l.chunkoff), U, C, (int64_t*)out[16], (int64_t*)out[17], (int64_t*)out[18],
                     (int64_t*)out[19], (int64_t*)out[20]);
  RSX_LAUNCHED();
  if (D > 0) {
    hipLaunchKernelGGL(si_cols_k, dim3(grid_for(n_items)), dim3(256), 0, st, at<int>(ws, l.hist_t),
                       at<int>(ws, l.hist_u), at<int>(ws, l.colidx), at<int>(ws, l.pairoff), n_items,
                       (int64_t*)out[21], (float*)out[22], (int*)out[30], (int*)out[31]);
    RSX_LAUNCHED();
  }
  if (E > 0) {
    (void)hipcub::DeviceRadixSort::SortPairs(tmp, tb, at<unsigned>(ws, l.pkeys), at<unsigned>(ws, l.pkeys_o),
                                             at<int>(ws, l.pvals), at<int>(ws, l.pvals_o), (int)E, 0,
                                             bits_for(D > 1 ? D : 2), st);
    RSX_LAUNCHED();
    hipLaunchKernelGGL(si_pairs_k, dim3(grid_for(E)), dim3(256), 0, st, at<int>(ws, l.pvals_o), E,
                       at<int>(ws, l.pair_b), at<int>(ws, l.pair_n), at<int>(ws, l.offN), (int*)out[27],
                       (int*)out[28], (int*)out[29]);
    RSX_LAUNCHED();
  }
  if (lookup && out[15]) {
    RSX_ARG(ld_lookup >= 128 && ld_lookup % 4 == 0, "pretrained lookup rows must be 128 floats (stride % 4 == 0)");
    hipLaunchKernelGGL(si_pv_k, dim3(grid_for(T * 32)), dim3(256), 0, st, lookup, ld_lookup, f.tok_ids, T,
                       (float*)out[15]);
    RSX_LAUNCHED();
  }
  return 0;
}
