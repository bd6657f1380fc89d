// DeepFM rerank forward in ONE kernel (BASELINE configs[2]; semantics of
// deepctr-torch 0.2.9's DeepFM as in deepfm.hip): per 64-row block
//
//   gather   the 39 x 16 field embeddings (and first-order weights) of each row: FM term and
//            linear term in registers, the DNN input row split to bf16 hi/lo straight into LDS
//            (the [R, 624] activation never goes to HBM: it was written and re-read, 2/3 of
//            the unfused path's HBM traffic);
//   layer 1  H1^T = W1 . X^T on v_mfma_f32_32x32x16_bf16 in bf16x3 (hi*hi + hi*lo + lo*hi, fp32
//            accumulate, ~2^-17 relative per product); each 16-wide k-step is exactly one
//            field; W1 comes from a pre-split fragment-ordered bf16 image (L2-resident);
//   layer 2  H2^T = W2 . relu(H1 + b1)^T: the layer-1 accumulators ARE the layer-2 B
//            fragments (lane (c, h) register 4g + e holds n = 32j + 8g + 4h + e of row c, i.e.
//            the k-set {16s + 4h + e, 16s + 8 + 4h + e} of k-step s = 2j + g/2) — no data
//            movement; W2 from a pre-split image in the same permuted k order; each wave
//            reduces its 64 k, the four partials meet in LDS (fixed order: deterministic);
//   output   logit = bias + first + FM + w_o . relu(H2 + b2), prob = sigmoid(logit).
// Measured (tools/deepfm_micro.py, config 3): 0.19 ms per 65,536 rows against 0.50 ms for the
// three-kernel path; with the gathers disabled it still takes 0.11 ms, i.e. the per-block
// latency chain (id staging, W1 ring prologue, b1 / W2 fragment loads, four barriers) at one
// 123-KB workgroup per CU bounds it, not HBM (next: two row blocks in flight per workgroup).
// Fields are processed in chunks of 13 (three chunks at F = 39; missing fields are zero),
// double-buffered: loader waves stage the next chunk while the compute waves run this one.
// Barriers (both roles, in order): one per staged chunk (nchunk + 1 in all), then two per n2
// half of layer 2.
#include "rsx_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int kMaxF = 64;
constexpr int kFC = 13;          // fields per chunk
constexpr int kBM = 64;          // rows per workgroup
constexpr int kN1 = 256, kN2 = 128;

// element offset of lane half h's 8-element chunk of W2 row n2 in k-step ks ([16][128][2][8] image):
// the two 16-B halves of a row are swapped on bit 3 of n2, so the 16 lanes (c = 0..15 or 16..31, one
// h) of a ds_read_b128 group cover all 64 banks when the image is read from LDS (deepfm_rows2m_k);
// without it lanes c and c + 8 hit the same banks (1.05e6 conflicts per call, r05 PMC)
__device__ __host__ __forceinline__ int w2_off(int ks, int n2, int h) {
  return ((ks * kN2 + n2) * 2 + (h ^ ((n2 >> 3) & 1))) * 8;
}

constexpr int kChunkElems = kFC * kBM * 16;  // bf16 per image per chunk

struct FArgs {
  const int64_t* x;          // [R, F]
  const float* V[kMaxF];     // [vocab_f, 16]
  const float* W[kMaxF];     // [vocab_f] or nullptr
  int64_t R;
  int F, nchunk;
  float bias;
  const __bf16* w1hi;        // [nchunk*13][256][16]  (field, n, k-in-field)
  const __bf16* w1lo;
  const float* b1;           // [256]
  const __bf16* w2hi;        // [16 ksteps][128][2 h][8]  permuted k (see rsx_deepfm_prep)
  const __bf16* w2lo;
  const float* b2;           // [128]
  const float* wo;           // [128]
  float* logit;              // [R]
  float* prob;               // [R] (nullable)
};

__device__ __forceinline__ void split4(const float4& v, bf16x4& h, bf16x4& l) {
  const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const __bf16 hk = (__bf16)f[k];
    h[k] = hk;
    l[k] = (__bf16)(f[k] - (float)hk);
  }
}

struct Lds {
  union {
    struct {
      __bf16 hi[2][kChunkElems];   // [buf][field-in-chunk][row][16]
      __bf16 lo[2][kChunkElems];
    } x;
    float part[4][64][kBM];         // layer-2 partials of one 64-wide n2 half: [wave][n2][row]
  } u;
  int ids[kBM][kMaxF + 1];  // +1: rows on different banks
};

// 512 threads: waves 0-3 compute (layer-1 MFMAs on the staged chunk, then layer 2), waves
// 4-7 load (all ids of their rows up front, then one chunk's embedding rows ahead of the
// compute waves, FM and linear terms, the final reduction). The compute waves' vmcnt queue
// then holds only their own W1 fragment loads, so a 4-field register ring of W1 fragments
// hides the L2 latency (in-order vmcnt: a gather load queued in between would stall it).
constexpr int kRing = 4;

__global__ __launch_bounds__(512, 1) void deepfm_fused_k(FArgs a) {
  __shared__ __attribute__((aligned(16))) Lds s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int64_t m0 = (int64_t)blockIdx.x * kBM;
  const bool loader = wave >= 4;
  const int nf = a.nchunk * kFC;

  // the block's ids -> LDS (int32), all 512 threads, coalesced: the loaders then address
  // their embedding rows from LDS (lgkmcnt), so each chunk's row loads can be issued a chunk
  // ahead without an in-order vmcnt wait on an id load queued behind them
  for (int i = tid; i < kBM * a.F; i += 512) {
    const int r = i / a.F, f = i - r * a.F;
    const int64_t row = m0 + r < a.R ? m0 + r : a.R - 1;  // tail rows re-read the last row; never stored
    s.ids[r][f] = (int)a.x[row * a.F + f];
  }
  __syncthreads();

  if (loader) {
    // gather role: row gr, quarter q (floats 4q..4q+3 of every field); two register buffers:
    // chunk ch+1's rows are in flight while chunk ch is split and staged
    const int lt = tid - 256, gr = lt >> 2, q = lt & 3;
    float4 fs = make_float4(0.f, 0.f, 0.f, 0.f), fss = fs;
    float first = 0.0f;
    auto issue = [&](int ch, float4 (&vb)[kFC], float (&wv)[kFC]) {
#pragma unroll
      for (int j = 0; j < kFC; ++j) {
        const int f = ch * kFC + j;
        vb[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        wv[j] = 0.0f;
        if (f < a.F) {
          const int id = s.ids[gr][f];
          vb[j] = reinterpret_cast<const float4*>(a.V[f] + (int64_t)id * 16)[q];
          if (q == (f & 3) && a.W[f]) wv[j] = a.W[f][id];
        }
      }
    };
    auto consume = [&](int ch, const float4 (&vb)[kFC], const float (&wv)[kFC]) {
      const int buf = ch & 1;
#pragma unroll
      for (int j = 0; j < kFC; ++j) {
        const float4 v = vb[j];
        fs.x += v.x; fs.y += v.y; fs.z += v.z; fs.w += v.w;
        fss.x += v.x * v.x; fss.y += v.y * v.y; fss.z += v.z * v.z; fss.w += v.w * v.w;
        first += wv[j];
        bf16x4 hi, lo;
        split4(v, hi, lo);
        const int o = (j * kBM + gr) * 16 + 4 * q;
        *reinterpret_cast<u32x2*>(&s.u.x.hi[buf][o]) = __builtin_bit_cast(u32x2, hi);
        *reinterpret_cast<u32x2*>(&s.u.x.lo[buf][o]) = __builtin_bit_cast(u32x2, lo);
      }
      __syncthreads();  // chunk ch staged (the compute waves consume it before the next barrier)
    };
    float4 va[kFC], vbb[kFC];
    float wa[kFC], wb[kFC];
    issue(0, va, wa);
    for (int ch = 0; ch < a.nchunk; ch += 2) {
      if (ch + 1 < a.nchunk) issue(ch + 1, vbb, wb);
      consume(ch, va, wa);
      if (ch + 1 >= a.nchunk) break;
      if (ch + 2 < a.nchunk) issue(ch + 2, va, wa);
      consume(ch + 1, vbb, wb);
    }
    __syncthreads();    // compute waves finished the last chunk
    float fm = (fs.x * fs.x - fss.x) + (fs.y * fs.y - fss.y) + (fs.z * fs.z - fss.z) + (fs.w * fs.w - fss.w);
    fm += __shfl_xor(fm, 1, 64);
    fm += __shfl_xor(fm, 2, 64);
    first += __shfl_xor(first, 1, 64);
    first += __shfl_xor(first, 2, 64);
    float dnn_acc = 0.0f;
    for (int half = 0; half < 2; ++half) {
      __syncthreads();  // A: partials of this half may be written
      __syncthreads();  // B: partials written
      // n2 in [16q, 16q + 16) of this half, the four waves' partials summed in order
#pragma unroll 4
      for (int k = 0; k < 16; ++k) {
        const int nl = 16 * q + k, n2 = 64 * half + nl;
        float v = ((s.u.part[0][nl][gr] + s.u.part[1][nl][gr]) + s.u.part[2][nl][gr]) + s.u.part[3][nl][gr];
        v += a.b2[n2];
        v = v > 0.0f ? v : 0.0f;
        dnn_acc += v * a.wo[n2];
      }
    }
    dnn_acc += __shfl_xor(dnn_acc, 1, 64);
    dnn_acc += __shfl_xor(dnn_acc, 2, 64);
    if (q == 0 && m0 + gr < a.R) {
      const float v = a.bias + first + 0.5f * fm + dnn_acc;
      a.logit[m0 + gr] = v;
      if (a.prob) a.prob[m0 + gr] = 1.0f / (1.0f + expf(-v));
    }
    return;
  }

  // ---- compute waves: layer 1 over the staged chunks
  const int nw0 = 64 * wave;
  f32x16 acc[2][2];  // [m-tile i][n-tile j]: D[n = nw0 + 32j + tile_row][m = 32i + c]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  // W1 fragment of field f: lane (c, h) reads n = nw0 + 32j + c, k-in-field 8h..8h+7
  const __bf16* w1h = a.w1hi + ((int64_t)nw0 + c) * 16 + 8 * h;
  const __bf16* w1l = a.w1lo + ((int64_t)nw0 + c) * 16 + 8 * h;
  auto wload = [&](int f, bf16x8 (&wh)[2], bf16x8 (&wl)[2]) {
    const int ff = f < nf ? f : nf - 1;  // past the end: a harmless re-read, never used
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      wh[j] = *reinterpret_cast<const bf16x8*>(w1h + ((int64_t)ff * kN1 + 32 * j) * 16);
      wl[j] = *reinterpret_cast<const bf16x8*>(w1l + ((int64_t)ff * kN1 + 32 * j) * 16);
    }
  };
  bf16x8 rh[kRing][2], rl[kRing][2];
#pragma unroll
  for (int d = 0; d < kRing; ++d) wload(d, rh[d], rl[d]);
  __syncthreads();  // chunk 0 staged
  for (int ch = 0; ch < a.nchunk; ++ch) {
    const int buf = ch & 1;
#pragma unroll
    for (int f = 0; f < kFC; ++f) {
      bf16x8 xh[2], xl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = (f * kBM + 32 * i + c) * 16 + 8 * h;
        xh[i] = *reinterpret_cast<const bf16x8*>(&s.u.x.hi[buf][o]);
        xl[i] = *reinterpret_cast<const bf16x8*>(&s.u.x.lo[buf][o]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rl[0][j], xh[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rh[0][j], xl[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rh[0][j], xh[i], acc[i][j], 0, 0, 0);
        }
      // shift the ring, fetch field + kRing
#pragma unroll
      for (int d = 0; d + 1 < kRing; ++d)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          rh[d][j] = rh[d + 1][j];
          rl[d][j] = rl[d + 1][j];
        }
      wload(ch * kFC + f + kRing, rh[kRing - 1], rl[kRing - 1]);
    }
    __syncthreads();  // done with buf; the loaders' next chunk is staged (the last one pairs
                      // the loaders' post-loop barrier)
  }

  // layer-1 epilogue: relu(acc + b1) split to hi/lo = the layer-2 B fragments.
  // k-step t = 2j + p of this wave (k = nw0 + 16t + ..) takes registers 8p..8p+7 of acc[i][j].
  bf16x8 gh[2][4], gl[2][4];  // [m-tile][k-step]
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bb = *reinterpret_cast<const float4*>(a.b1 + nw0 + 32 * j + 8 * g + 4 * h);
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[i][j][4 * g + e] + bv[e];
          v = v > 0.0f ? v : 0.0f;
          const __bf16 hv = (__bf16)v;
          const int t = 2 * j + (g >> 1), el = 4 * (g & 1) + e;
          gh[i][t][el] = hv;
          gl[i][t][el] = (__bf16)(v - (float)hv);
        }
    }

  // layer 2 in two halves of n2 (64 each); partial over this wave's 64 k -> LDS
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    f32x16 acc2[2][2];  // [m-tile i][n2-tile j2 within half]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[i][j2][r] = 0.0f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ks = wave * 4 + t;  // global k-step over the 256 layer-1 outputs
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2) {
        const int n2 = 64 * half + 32 * j2 + c;
        const int64_t o = w2_off(ks, n2, h);
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(a.w2hi + o);
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(a.w2lo + o);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          acc2[i][j2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, gh[i][t], acc2[i][j2], 0, 0, 0);
          acc2[i][j2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, gl[i][t], acc2[i][j2], 0, 0, 0);
          acc2[i][j2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, gh[i][t], acc2[i][j2], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // A: the X images are dead (half 0) / the previous partials were consumed
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          s.u.part[wave][32 * j2 + (r & 3) + 8 * (r >> 2) + 4 * h][32 * i + c] = acc2[i][j2][r];
    __syncthreads();  // B
  }
}

// Weight images (one launch): W1 [256][F*16] -> [nchunk*13][256][16] hi/lo (zero past F);
// W2 [128][256] -> [16 ksteps][128][2][8] hi/lo with element (ks, n2, h, 4p + e) =
// W2[n2][16 ks + 8p + 4h + e]: the k order of the layer-1 accumulators (see the header).
__global__ __launch_bounds__(256) void deepfm_prep_k(const float* w1, int F, int nchunk, const float* w2,
                                                     __bf16* w1hi, __bf16* w1lo, __bf16* w2hi, __bf16* w2lo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n1 = (int64_t)nchunk * kFC * kN1 * 16;
  if (i < n1) {
    const int k = (int)(i % 16), n = (int)((i / 16) % kN1), f = (int)(i / (16 * kN1));
    const float v = f < F ? w1[(int64_t)n * F * 16 + f * 16 + k] : 0.0f;
    const __bf16 hv = (__bf16)v;
    w1hi[i] = hv;
    w1lo[i] = (__bf16)(v - (float)hv);
    return;
  }
  const int64_t j = i - n1;
  if (j < 16 * kN2 * 16) {
    const int el = (int)(j % 8), hs = (int)((j / 8) % 2), n2 = (int)((j / 16) % kN2), ks = (int)(j / (16 * kN2));
    const int hh = hs ^ ((n2 >> 3) & 1);  // the stored half (w2_off's swizzle)
    const int k = 16 * ks + 8 * (el >> 2) + 4 * hh + (el & 3);
    const float v = w2[(int64_t)n2 * kN1 + k];
    const __bf16 hv = (__bf16)v;
    w2hi[j] = hv;
    w2lo[j] = (__bf16)(v - (float)hv);
  }
}

// ---- persistent form (F in [25, 48]) ------------------------------------------------------
// One 512-thread workgroup per CU loops over 64-row blocks; fields in chunks of 8. The per-block
// latency chain of deepfm_fused_k (id staging, W1 ring prologue, the layer-2 barriers at one
// workgroup per CU: 0.11 ms of its 0.19 ms with the gathers disabled) overlaps with useful work:
//  * loader waves stage the next block's ids during chunk 0, its first two chunks during the
//    compute waves' layer-1 tail and epilogue, so every chunk is in LDS before it is needed;
//  * the compute waves' W1 fragment ring runs on across block boundaries (no prologue);
//  * layer 2 is split by n2 (each compute wave 32 outputs over all k) from relu(H1 + b1)
//    exchanged through LDS in bf16 hi/lo, so it needs no cross-wave partial sums; the four
//    waves' per-row dot products with w_o meet in LDS, the loaders add bias + first + FM.
// Barrier sequence per block (both roles, same order): A_0 .. A_{C-1} (chunk j staged),
// E1 (layer 1 done: its buffers free), E2 (h1 written), E3 (per-row partials written).
constexpr int kFC2 = 8;                   // fields per chunk
constexpr int kChunk2 = kFC2 * kBM * 16;  // bf16 per image per chunk
constexpr int kH1Stride = kN1 + 8;        // bf16 per h1 row (528 B: conflict-free row reads)
constexpr int kPersistMaxF = 48;
constexpr int kIdLoads = (kBM * kPersistMaxF + 255) / 256;  // id loads per loader thread per block
constexpr int kRing2 = 6;  // W1 fragment ring depth of the persistent kernel (fields ahead)

struct PArgs {
  const int64_t* x;
  const float* V[kMaxF];
  const float* W[kMaxF];
  const float* P[kMaxF];     // packed [vocab_f][32] (V row, W, pad: one 128-B line per id) or nullptr
  int64_t R;
  int F, nchunk, id_stride;
  int64_t nrb;               // row blocks
  float bias;
  const __bf16* w1hi;        // [nchunk*8][256][16]
  const __bf16* w1lo;
  const float* b1;
  const __bf16* w2hi;        // [128][256] natural k order
  const __bf16* w2lo;
  const float* b2;
  const float* wo;
  float* logit;
  float* prob;
};

__global__ __launch_bounds__(512, 1) void deepfm_persist_k(PArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __bf16* xhi = reinterpret_cast<__bf16*>(smem);                  // [2][8][64][16]
  __bf16* xlo = xhi + 2 * kChunk2;
  __bf16* h1hi = xlo + 2 * kChunk2;                               // [64][264]
  __bf16* h1lo = h1hi + kBM * kH1Stride;
  float* red = reinterpret_cast<float*>(h1lo + kBM * kH1Stride);  // [4][64]
  int* ids = reinterpret_cast<int*>(red + 4 * kBM);               // [2][64][id_stride]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int C = a.nchunk, nf = C * kFC2;
  const int64_t nit = (a.nrb - blockIdx.x + gridDim.x - 1) / gridDim.x;
  auto rb_of = [&](int64_t it) -> int64_t { return blockIdx.x + it * (int64_t)gridDim.x; };

  if (wave >= 4) {
    // ---------------- loaders: row gr, quarter q (floats 4q..4q+3 of every field)
    const int lt = tid - 256, gr = lt >> 2, q = lt & 3;
    float4 vA[kFC2], vB[kFC2], vC[kFC2];  // three register sets: global chunk g uses set g % 3
    float wA[kFC2], wB[kFC2], wC[kFC2];
    float4 fs = make_float4(0.f, 0.f, 0.f, 0.f), fss = fs;
    float first = 0.0f;
    // ids of block it -> ids[it & 1] (int32), coalesced: the block's [64][F] slice of x is
    // contiguous, so every load is issued before the first is used (one memory latency per
    // block instead of one per 256 ids); (row, field) from a float reciprocal (exact: the
    // quotient of i + 0.5 stays >= 0.5 / F away from an integer)
    const float invF = 1.0f / (float)a.F;
    auto load_ids = [&](int64_t it) {
      const int64_t m0 = rb_of(it) * kBM;
      int* dst = ids + (it & 1) * kBM * a.id_stride;
      const int n = kBM * a.F;
      const bool full = m0 + kBM <= a.R;
      int64_t v[kIdLoads];
#pragma unroll
      for (int k = 0; k < kIdLoads; ++k) {
        const int i = lt + 256 * k;
        v[k] = 0;
        if (i < n) {
          int64_t e = m0 * a.F + i;
          if (!full) {  // tail rows re-read the last row; never stored
            const int r = (int)(((float)i + 0.5f) * invF);
            if (m0 + r >= a.R) e = (a.R - 1) * a.F + (i - r * a.F);
          }
          v[k] = a.x[e];
        }
      }
#pragma unroll
      for (int k = 0; k < kIdLoads; ++k) {
        const int i = lt + 256 * k;
        if (i < n) {
          const int r = (int)(((float)i + 0.5f) * invF), f = i - r * a.F;
          dst[r * a.id_stride + f] = (int)v[k];
        }
      }
    };
    auto issue_set = [&](int64_t it, int j, float4 (&vb)[kFC2], float (&wv)[kFC2]) {
      const int* idr = ids + (it & 1) * kBM * a.id_stride + gr * a.id_stride;
#pragma unroll
      for (int k = 0; k < kFC2; ++k) {
        const int f = j * kFC2 + k;
        vb[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        wv[k] = 0.0f;
        if (f < a.F) {
          const int id = idr[f];
          if (a.P[0]) {  // packed: the V row and W of one id share a 128-B line
            const float* pr = a.P[f] + (int64_t)id * 32;
            vb[k] = reinterpret_cast<const float4*>(pr)[q];
            if (q == (f & 3)) wv[k] = pr[16];
          } else {
            vb[k] = reinterpret_cast<const float4*>(a.V[f] + (int64_t)id * 16)[q];
            if (q == (f & 3) && a.W[f]) wv[k] = a.W[f][id];
          }
        }
      }
    };
    auto consume_set = [&](int buf, const float4 (&vb)[kFC2], const float (&wv)[kFC2]) {
#pragma unroll
      for (int k = 0; k < kFC2; ++k) {
        const float4 v = vb[k];
        fs.x += v.x; fs.y += v.y; fs.z += v.z; fs.w += v.w;
        fss.x += v.x * v.x; fss.y += v.y * v.y; fss.z += v.z * v.z; fss.w += v.w * v.w;
        first += wv[k];
        bf16x4 hi, lo;
        split4(v, hi, lo);
        const int o = buf * kChunk2 + (k * kBM + gr) * 16 + 4 * q;
        *reinterpret_cast<u32x2*>(&xhi[o]) = __builtin_bit_cast(u32x2, hi);
        *reinterpret_cast<u32x2*>(&xlo[o]) = __builtin_bit_cast(u32x2, lo);
      }
    };
    float fm_out = 0.0f, first_out = 0.0f;
    auto finalize_fm = [&]() {  // the block's FM / first terms per row (4 quarters summed)
      float fm = (fs.x * fs.x - fss.x) + (fs.y * fs.y - fss.y) + (fs.z * fs.z - fss.z) + (fs.w * fs.w - fss.w);
      fm += __shfl_xor(fm, 1, 64);
      fm += __shfl_xor(fm, 2, 64);
      float fi = first + __shfl_xor(first, 1, 64);
      fi += __shfl_xor(fi, 2, 64);
      fm_out = fm;
      first_out = fi;
      fs = make_float4(0.f, 0.f, 0.f, 0.f);
      fss = fs;
      first = 0.0f;
    };
    auto write_logits = [&](int64_t it) {  // after E3(it): the compute waves' per-row partials
      const int64_t row = rb_of(it) * kBM + gr;
      if (q == 0 && row < a.R) {
        const float dnn = ((red[gr] + red[kBM + gr]) + red[2 * kBM + gr]) + red[3 * kBM + gr];
        const float v = a.bias + first_out + 0.5f * fm_out + dnn;
        a.logit[row] = v;
        if (a.prob) a.prob[row] = 1.0f / (1.0f + expf(-v));
      }
    };
    // One step per global chunk g = (it, j) = (g / C, g % C): rows of chunk g+2 issued into the
    // third register set (two chunks of gathers in flight), chunk g consumed into LDS buffer
    // g & 1, then the barriers that separate staging chunk g from staging chunk g+1 (see the
    // sequence above): chunks (it, 0) and (it, 1) are staged during block it-1's layer-1 tail /
    // epilogue, chunk (it, j >= 2) between A_{j-1} and A_j; the next block's ids are loaded
    // between A_0 and A_1 (C >= 4: they are visible before chunk (it+1, 0) is issued at step
    // (it, C-2), which follows A_{C-3}).
    const int64_t G = nit * C;
    auto step = [&](int64_t g, float4 (&vc)[kFC2], float (&wc)[kFC2], float4 (&vn)[kFC2], float (&wn)[kFC2]) {
      const int64_t it = g / C;
      const int j = (int)(g - it * C);
      if (j == 0 && it > 0) finalize_fm();
      if (g + 2 < G) issue_set((g + 2) / C, (int)((g + 2) % C), vn, wn);
      consume_set((int)(g & 1), vc, wc);
      if (j == 0) {
        if (it > 0) __syncthreads();  // E1(it-1)
      } else if (j == 1) {
        if (it > 0) {
          __syncthreads();  // E2(it-1)
          __syncthreads();  // E3(it-1)
          write_logits(it - 1);
        }
        __syncthreads();  // A_0(it)
        if (it + 1 < nit) load_ids(it + 1);
        __syncthreads();  // A_1(it)
      } else {
        __syncthreads();  // A_j(it)
      }
    };
    if (nit > 0) load_ids(0);
    __syncthreads();  // P
    if (G > 0) issue_set(0, 0, vA, wA);
    if (G > 1) issue_set(1 / C, 1 % C, vB, wB);
    for (int64_t g = 0; g < G; g += 3) {
      step(g, vA, wA, vC, wC);
      if (g + 1 < G) step(g + 1, vB, wB, vA, wA);
      if (g + 2 < G) step(g + 2, vC, wC, vB, wB);
    }
    if (nit > 0) {
      finalize_fm();
      __syncthreads();  // E1(last)
      __syncthreads();  // E2(last)
      __syncthreads();  // E3(last)
      write_logits(nit - 1);
    }
    return;
  }

  // ---------------- compute waves
  const int nw0 = 64 * wave;
  const __bf16* w1h = a.w1hi + ((int64_t)nw0 + c) * 16 + 8 * h;
  const __bf16* w1l = a.w1lo + ((int64_t)nw0 + c) * 16 + 8 * h;
  auto wload = [&](int f, bf16x8 (&wh)[2], bf16x8 (&wl)[2]) {
    const int ff = f % nf;  // the ring runs on into the next block's fields
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      wh[j] = *reinterpret_cast<const bf16x8*>(w1h + ((int64_t)ff * kN1 + 32 * j) * 16);
      wl[j] = *reinterpret_cast<const bf16x8*>(w1l + ((int64_t)ff * kN1 + 32 * j) * 16);
    }
  };
  bf16x8 rh[kRing2][2], rl[kRing2][2];
#pragma unroll
  for (int d = 0; d < kRing2; ++d) wload(d, rh[d], rl[d]);
  __syncthreads();  // P
  for (int64_t it = 0; it < nit; ++it) {
    f32x16 acc[2][2];  // [m-tile i][n-tile j]: D[n = nw0 + 32j + tile_row][m = 32i + c]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    for (int ch = 0; ch < C; ++ch) {
      __syncthreads();  // A_ch
      const int buf = (int)((it * C + ch) & 1);
#pragma unroll
      for (int f = 0; f < kFC2; ++f) {
        bf16x8 xh[2], xl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int o = buf * kChunk2 + (f * kBM + 32 * i + c) * 16 + 8 * h;
          xh[i] = *reinterpret_cast<const bf16x8*>(&xhi[o]);
          xl[i] = *reinterpret_cast<const bf16x8*>(&xlo[o]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rl[0][j], xh[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rh[0][j], xl[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rh[0][j], xh[i], acc[i][j], 0, 0, 0);
          }
#pragma unroll
        for (int d = 0; d + 1 < kRing2; ++d)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            rh[d][j] = rh[d + 1][j];
            rl[d][j] = rl[d + 1][j];
          }
        wload(ch * kFC2 + f + kRing2, rh[kRing2 - 1], rl[kRing2 - 1]);
      }
    }
    __syncthreads();  // E1
    // h1 = relu(H1 + b1) -> LDS hi/lo: lane (c, h) holds rows 32i + c, n = nw0 + 32j + 8g + 4h + e
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bb = *reinterpret_cast<const float4*>(a.b1 + nw0 + 32 * j + 8 * g + 4 * h);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const float4 v = make_float4(fmaxf(acc[i][j][4 * g + 0] + bb.x, 0.0f), fmaxf(acc[i][j][4 * g + 1] + bb.y, 0.0f),
                                       fmaxf(acc[i][j][4 * g + 2] + bb.z, 0.0f), fmaxf(acc[i][j][4 * g + 3] + bb.w, 0.0f));
          bf16x4 hi, lo;
          split4(v, hi, lo);
          const int o = (32 * i + c) * kH1Stride + nw0 + 32 * j + 8 * g + 4 * h;
          *reinterpret_cast<u32x2*>(&h1hi[o]) = __builtin_bit_cast(u32x2, hi);
          *reinterpret_cast<u32x2*>(&h1lo[o]) = __builtin_bit_cast(u32x2, lo);
        }
      }
    __syncthreads();  // E2
    // layer 2, n2 in [32 wave, 32 wave + 32): D[n2][m] = sum_k W2[n2][k] h1[m][k]
    f32x16 acc2[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc2[i][r] = 0.0f;
    const int n2 = 32 * wave + c;
    const __bf16* w2h = a.w2hi + (int64_t)n2 * kN1 + 8 * h;
    const __bf16* w2l = a.w2lo + (int64_t)n2 * kN1 + 8 * h;
#pragma unroll 4
    for (int s = 0; s < kN1 / 16; ++s) {
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(w2h + 16 * s);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(w2l + 16 * s);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = (32 * i + c) * kH1Stride + 16 * s + 8 * h;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&h1hi[o]);
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&h1lo[o]);
        acc2[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc2[i], 0, 0, 0);
        acc2[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc2[i], 0, 0, 0);
        acc2[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc2[i], 0, 0, 0);
      }
    }
    // relu(H2 + b2) . w_o over this wave's 32 n2 (register r: n2 = 32 wave + tile_row(r, h))
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float sdot = 0.0f;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nb = 32 * wave + 8 * g + 4 * h;
        const float4 bb = *reinterpret_cast<const float4*>(a.b2 + nb);
        const float4 ww = *reinterpret_cast<const float4*>(a.wo + nb);
        sdot += fmaxf(acc2[i][4 * g + 0] + bb.x, 0.0f) * ww.x;
        sdot += fmaxf(acc2[i][4 * g + 1] + bb.y, 0.0f) * ww.y;
        sdot += fmaxf(acc2[i][4 * g + 2] + bb.z, 0.0f) * ww.z;
        sdot += fmaxf(acc2[i][4 * g + 3] + bb.w, 0.0f) * ww.w;
      }
      sdot += __shfl_xor(sdot, 32, 64);
      if (h == 0) red[wave * kBM + 32 * i + c] = sdot;
    }
    __syncthreads();  // E3
  }
}

// Weight images of the persistent form: W1 [256][F*16] -> [nchunk*8][256][16] hi/lo (zero past
// F); W2 [128][256] -> [128][256] hi/lo (natural k order).
__global__ __launch_bounds__(256) void deepfm_prep2_k(const float* w1, int F, int nchunk, const float* w2,
                                                      __bf16* w1hi, __bf16* w1lo, __bf16* w2hi, __bf16* w2lo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n1 = (int64_t)nchunk * kFC2 * kN1 * 16;
  float v;
  __bf16 *dh, *dl;
  if (i < n1) {
    const int k = (int)(i % 16), n = (int)((i / 16) % kN1), f = (int)(i / (16 * kN1));
    v = f < F ? w1[(int64_t)n * F * 16 + f * 16 + k] : 0.0f;
    dh = w1hi + i;
    dl = w1lo + i;
  } else if (i - n1 < (int64_t)kN2 * kN1) {
    v = w2[i - n1];
    dh = w2hi + (i - n1);
    dl = w2lo + (i - n1);
  } else {
    return;
  }
  const __bf16 hv = (__bf16)v;
  *dh = hv;
  *dl = (__bf16)(v - (float)hv);
}

// packed table of one field: out[id][0..15] = V[id], out[id][16] = W[id] (0 if W is null),
// out[id][17..31] = 0; one thread per 16-B chunk
__global__ __launch_bounds__(256) void deepfm_pack_k(const float* V, const float* W, int64_t vocab, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (id, chunk 0..7)
  if (i >= vocab * 8) return;
  const int64_t id = i >> 3;
  const int ch = (int)(i & 7);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ch < 4) v = reinterpret_cast<const float4*>(V + id * 16)[ch];
  else if (ch == 4 && W) v.x = W[id];
  reinterpret_cast<float4*>(out + id * 32)[ch] = v;
}

// ---- row-owning form (F = 39: the config-3 field count; other F take deepfm_persist_k) -------
// Every wave owns 64 rows and gathers them itself, straight into MFMA fragment registers: no
// loader / compute hand-off (the persistent kernel's bound: its compute waves waited a third of
// their time for the loaders). Per field f and m-tile i (32 rows), lane (c, h) issues three
// 16-B loads of row 32i + c's packed 128-B line: bytes 16h (V[4h..4h+3]), 32 + 16h
// (V[8+4h..]) and 64 + 16h (W at byte 64, read by h = 0). A random-line probe reads 53 G lines/s
// with the first two (one line request per pair, as one 4-lane instruction: 52 G) and 48 G with
// the third (tools/probe/gather_pieces.hip). The lane's eight values are the B fragment of
// v_mfma_f32_32x32x16_bf16 for k-slots 8h..8h+7 <-> V[kperm(slot)], kperm = {0-3, 8-11, 4-7,
// 12-15} (the W1 image uses the same order). W1 (the A operand, [256][16] per field, hi / lo)
// streams through a two-slot LDS ring: each wave register-loads a quarter of field f + R's
// image along with its own gathers for f + R, writes it at field f, one barrier per field (no
// glds: beside it hipcc drains ordinary loads with vmcnt(0)). The field loop is fully unrolled
// (F is a template parameter) so the R-deep register ring is straight-line code: loop-carried
// load registers make hipcc drain the loads at the loop header. Layer 2 takes its B fragments
// from the layer-1 accumulators (the deepfm_fused_k order; W2 image of deepfm_prep_k).
constexpr int kRowsF = 39;
constexpr int kRowsR = 8;           // fields of loads in flight ahead of the one computed
constexpr int kW1Field = 8192;      // bf16 per field image: hi [256][16] then lo [256][16]

struct RArgs {
  const int64_t* x;          // [R, F]
  const float* P[kMaxF];     // packed [vocab][32]: V[16], W, pad
  const float* V[kMaxF];     // unpacked form (deepfm_rows5_k<F, false>): V [vocab][16], W [vocab] or null
  const float* W[kMaxF];
  int64_t R;
  int64_t nit;               // task rounds (4 tasks of 64 rows per workgroup per round)
  float bias;
  const __bf16* w1;          // [F][8192] (swizzled, kperm order; deepfm_prep3_k)
  const float* b1;
  const __bf16* w2hi;        // [16 ksteps][128][2][8] (deepfm_prep_k order)
  const __bf16* w2lo;
  const float* b2;
  const float* wo;
  float* logit;
  float* prob;
};

// element index of (n, slot) in a field image's hi half; the 16-B halves of a row are swapped
// on bit 3 of n, so the 16 lanes of each ds_read_b128 lane group hit all 64 banks
__device__ __host__ __forceinline__ int w1_idx(int n, int slot) {
  return n * 16 + 8 * ((slot >> 3) ^ ((n >> 3) & 1)) + (slot & 7);
}

// ABL (timing ablations, results wrong; RSX_DEEPFM_ABL): 1 no per-field barrier, 2 no W1 LDS
// writes, 4 no layer-1 MFMAs, 8 no layer 2
template <int F, int ABL = 0>
__global__ __launch_bounds__(256, 1) void deepfm_rows_k(RArgs a) {
  constexpr int R = kRowsR, NB = R + 1;
  __shared__ __attribute__((aligned(16))) __bf16 w1s[2][kW1Field];
  __shared__ int ids_s[4][32 * F];
  // b1 / b2 / w_o via LDS: a global load in layer 2 would wait out its W2 prefetch
  __shared__ __attribute__((aligned(16))) float b1s[kN1], b2s[kN2], wos[kN2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 31, h = lane >> 5;
  b1s[tid] = a.b1[tid];  // visible after barrier 0
  if (tid < kN2) b2s[tid] = a.b2[tid];
  else wos[tid - kN2] = a.wo[tid - kN2];
  int* my_ids = ids_s[wave];
  const int64_t m0 = ((int64_t)blockIdx.x * 4 + wave) * 32;  // this wave's 32 rows
  const uint4* w1g = reinterpret_cast<const uint4*>(a.w1);
  uint4* w1l0 = reinterpret_cast<uint4*>(w1s[0]);
  uint4* w1l1 = reinterpret_cast<uint4*>(w1s[1]);

  // ---- ids of the 32 rows -> LDS (int32); rows past R re-read the last row, never stored
  {
    const int64_t last = a.R - 1;
    constexpr int NT = (32 * F + 63) / 64;
    int64_t v[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int e = lane + 64 * t;
      const int row = e / F, f = e - row * F;
      const int64_t gr = m0 + row <= last ? m0 + row : last;
      v[t] = e < 32 * F ? a.x[gr * F + f] : 0;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (lane + 64 * t < 32 * F) my_ids[lane + 64 * t] = (int)v[t];
  }
  // ---- layer 1 over the fields: the gathers of fields f+1..f+R and this wave's quarter of
  // their W1 images in flight (one register ring: both are waited for at the same depth, so the
  // in-order vmcnt never waits on a younger field)
  float4 xa[NB], xb[NB], xw[NB];
  uint4 wq[NB][4];
  f32x16 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
  float fs[8], fq = 0.0f, fw = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) fs[k] = 0.0f;
  auto issue = [&](int f, int sl) {
#pragma unroll
    for (int k = 0; k < 4; ++k) wq[sl][k] = w1g[f * (kW1Field / 8) + 256 * wave + lane + 64 * k];
    const int id = my_ids[c * F + f];
    const float4* line = reinterpret_cast<const float4*>(a.P[f] + (int64_t)id * 32);
    xa[sl] = line[h];
    xb[sl] = line[2 + h];
    xw[sl] = line[4 + h];
  };
#pragma unroll
  for (int f = 0; f < R; ++f) issue(f, f);
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const int sl = f % NB;
    if (f + R < F) issue(f + R, (f + R) % NB);
    __builtin_amdgcn_sched_barrier(0);
    // field f's registers "redefined" here: left alone, hipcc consumes each field's loads right
    // after issuing them (fewer live registers) and so waits on them at once
    asm volatile("" : "+v"(wq[sl][0].x), "+v"(wq[sl][0].y), "+v"(wq[sl][0].z), "+v"(wq[sl][0].w),
                 "+v"(wq[sl][1].x), "+v"(wq[sl][1].y), "+v"(wq[sl][1].z), "+v"(wq[sl][1].w));
    asm volatile("" : "+v"(wq[sl][2].x), "+v"(wq[sl][2].y), "+v"(wq[sl][2].z), "+v"(wq[sl][2].w),
                 "+v"(wq[sl][3].x), "+v"(wq[sl][3].y), "+v"(wq[sl][3].z), "+v"(wq[sl][3].w));
    uint4* slot = (f & 1) ? w1l1 : w1l0;
    if (!(ABL & 2)) {
#pragma unroll
      for (int k = 0; k < 4; ++k) slot[256 * wave + lane + 64 * k] = wq[sl][k];
    } else {
      asm volatile("" :: "v"(wq[sl][0].x), "v"(wq[sl][1].x), "v"(wq[sl][2].x), "v"(wq[sl][3].x));
    }
    if (!(ABL & 1)) __syncthreads();  // barrier f: slot f & 1 holds field f (plain global loads survive it)
    asm volatile("" : "+v"(xa[sl].x), "+v"(xa[sl].y), "+v"(xa[sl].z), "+v"(xa[sl].w), "+v"(xb[sl].x),
                 "+v"(xb[sl].y), "+v"(xb[sl].z), "+v"(xb[sl].w), "+v"(xw[sl].x), "+v"(xw[sl].y), "+v"(xw[sl].z),
                 "+v"(xw[sl].w));
    const __bf16* ws = (f & 1) ? w1s[1] : w1s[0];
    // W1 fragments of n-tile pair jp + 1 read while pair jp's MFMAs run; pair 0's reads are
    // issued before the split, whose VALU then covers their latency
    bf16x8 ah[2][2], al[2][2];
    auto wread = [&](int jp, int b) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int n = 32 * (2 * jp + q) + c;
        ah[b][q] = *reinterpret_cast<const bf16x8*>(ws + w1_idx(n, 8 * h));
        al[b][q] = *reinterpret_cast<const bf16x8*>(ws + 4096 + w1_idx(n, 8 * h));
      }
    };
    wread(0, 0);
    bf16x8 bh, bl;
    {
      const float4 p = xa[sl], q = xb[sl], w = xw[sl];
      const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        fs[k] += v[k];
        fq += v[k] * v[k];
        const __bf16 hv = (__bf16)v[k];
        bh[k] = hv;
        bl[k] = (__bf16)(v[k] - (float)hv);
      }
      // bytes 64..95 of the line: W then zeros (deepfm_pack_k), so the whole 16-B piece sums
      // to W on h = 0 and to 0 on h = 1 (all four components used: a dword load of the same
      // line runs at 38 G lines/s in the probe, a 16-B piece at 48 G)
      fw += (w.x + w.y) + (w.z + w.w);
    }
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      if (jp + 1 < 4) wread(jp + 1, (jp + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
      const int b = jp & 1;
      if (ABL & 4) {
        asm volatile("" :: "v"(al[b][0]), "v"(ah[b][0]), "v"(al[b][1]), "v"(ah[b][1]), "v"(bh), "v"(bl));
        __builtin_amdgcn_sched_barrier(0);
        continue;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j = 2 * jp + q;
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[b][q], bh, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[b][q], bl, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[b][q], bh, acc[j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // ---- layer 2 in two halves of n2 (64 outputs each: the half's accumulators, the layer-1
  // accumulators and a 6-deep W2 prefetch ring fit the registers the layer-1 rings leave free).
  // The 32 (half, k-step) steps are one flat unrolled sequence, so the ring runs across the
  // halves; B fragments of k-step t = 2j + g2 from acc[j] (deepfm_fused_k order), rebuilt per
  // half. b1 / b2 / w_o come from LDS: a global load here would wait out the W2 prefetch.
  float dot = 0.0f;
  if (ABL & 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" :: "v"(acc[j]));
  }
  constexpr int P = 6, NS = 32;
  bf16x8 w2h[P + 1][2], w2l[P + 1][2];
  auto w2load = [&](int st) {
    const int half = st >> 4, t = st & 15, b = st % (P + 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = w2_off(t, 32 * (2 * half + q) + c, h);
      w2h[b][q] = *reinterpret_cast<const bf16x8*>(a.w2hi + o);
      w2l[b][q] = *reinterpret_cast<const bf16x8*>(a.w2lo + o);
    }
  };
  if (!(ABL & 8)) {
#pragma unroll
    for (int st = 0; st < P; ++st) w2load(st);
  }
  f32x16 acc2[2];
#pragma unroll
  for (int st = 0; st < (ABL & 8 ? 0 : NS); ++st) {
    const int half = st >> 4, t = st & 15, j = t >> 1, g2 = t & 1, b = st % (P + 1);
    if (t == 0) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[q][r] = 0.0f;
    }
    if (st + P < NS) w2load(st + P);
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 gh, gl;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float4 bb = *reinterpret_cast<const float4*>(b1s + 16 * t + 8 * p + 4 * h);
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[j][4 * (2 * g2 + p) + e] + bv[e];
        v = v > 0.0f ? v : 0.0f;
        const __bf16 hv = (__bf16)v;
        gh[4 * p + e] = hv;
        gl[4 * p + e] = (__bf16)(v - (float)hv);
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const bf16x8 ah = w2h[b][q], al = w2l[b][q];
      acc2[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, gh, acc2[q], 0, 0, 0);
      acc2[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, gl, acc2[q], 0, 0, 0);
      acc2[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, gh, acc2[q], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t == 15) {  // relu(H2 + b2) . wo over this half's 64 outputs
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int nb = 32 * (2 * half + q) + 8 * g + 4 * h;
          const float4 bb = *reinterpret_cast<const float4*>(b2s + nb);
          const float4 ww = *reinterpret_cast<const float4*>(wos + nb);
          dot += fmaxf(acc2[q][4 * g + 0] + bb.x, 0.0f) * ww.x;
          dot += fmaxf(acc2[q][4 * g + 1] + bb.y, 0.0f) * ww.y;
          dot += fmaxf(acc2[q][4 * g + 2] + bb.z, 0.0f) * ww.z;
          dot += fmaxf(acc2[q][4 * g + 3] + bb.w, 0.0f) * ww.w;
        }
    }
  }
  float fm = -fq;
#pragma unroll
  for (int k = 0; k < 8; ++k) fm += fs[k] * fs[k];
  dot += __shfl_xor(dot, 32, 64);
  fm += __shfl_xor(fm, 32, 64);
  const float first = fw + __shfl_xor(fw, 32, 64);
  const int64_t row = m0 + c;
  if (h == 0 && row < a.R) {
    const float v = a.bias + first + 0.5f * fm + dot;
    a.logit[row] = v;
    if (a.prob) a.prob[row] = 1.0f / (1.0f + expf(-v));
  }
}

// deepfm_rows_k with W1 staged by a fifth wave through LDS-DMA instead of the compute waves'
// register ring + ds_write (timing ablations: the per-field W1 writes and barrier were half of the
// kernel with L2-resident gathers): the compute waves' only global loads are their gathers.
// 320 threads (the stager shares a SIMD): 256 registers per wave, so R = 5 and a 3-deep W2 ring.
// PK = false: the tables as given (V row: two 16-B pieces of its 64 B; W: one dword), for callers
// without the packed images (rsx_deepfm_fused, or no table cache).
template <int F, bool PK = true>
__global__ __launch_bounds__(320, 1) void deepfm_rows5_k(RArgs a) {
  constexpr int R = 4, NB = R + 1, ABL = 0;
  __shared__ __attribute__((aligned(16))) __bf16 w1s[3][kW1Field];
  __shared__ int ids_s[4][32 * F];
  // b1 / b2 / w_o via LDS: a global load in layer 2 would wait out its W2 prefetch
  __shared__ __attribute__((aligned(16))) float b1s[kN1], b2s[kN2], wos[kN2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 31, h = lane >> 5;
  if (tid < kN1) b1s[tid] = a.b1[tid];  // visible after barrier 0
  if (tid < kN2) b2s[tid] = a.b2[tid];
  else if (tid < kN1) wos[tid - kN2] = a.wo[tid - kN2];
  if (wave == 4) {
    // ---- W1 stager: field f + 2 into slot (f + 2) % 3 after barrier f (its previous field,
    // f - 1, was finished by every compute wave before barrier f); a counted vmcnt retires field
    // f + 1's 16 pieces before barrier f + 1; raw s_barrier (__syncthreads() would drain the DMA)
    const char* w1b = reinterpret_cast<const char*>(a.w1);
    auto dma = [&](int f) {
      char* dst = reinterpret_cast<char*>(w1s[f % 3]);
#pragma unroll
      for (int k = 0; k < 16; ++k)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(w1b + (int64_t)f * (kW1Field * 2) + 1024 * k + 16 * lane),
            (__attribute__((address_space(3))) void*)(dst + 1024 * k), 16, 0, 0);
    };
    dma(0);
    dma(1);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // field 0 landed
    __builtin_amdgcn_s_barrier();                      // barrier 0
#pragma unroll
    for (int f = 0; f + 1 < F; ++f) {
      if (f + 2 < F) {
        dma(f + 2);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // field f + 1 landed
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();  // barrier f + 1
    }
    return;
  }
  int* my_ids = ids_s[wave];
  const int64_t m0 = ((int64_t)blockIdx.x * 4 + wave) * 32;  // this wave's 32 rows

  // ---- ids of the 32 rows -> LDS (int32); rows past R re-read the last row, never stored
  {
    const int64_t last = a.R - 1;
    constexpr int NT = (32 * F + 63) / 64;
    int64_t v[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int e = lane + 64 * t;
      const int row = e / F, f = e - row * F;
      const int64_t gr = m0 + row <= last ? m0 + row : last;
      v[t] = e < 32 * F ? a.x[gr * F + f] : 0;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (lane + 64 * t < 32 * F) my_ids[lane + 64 * t] = (int)v[t];
  }
  // ---- layer 1 over the fields: the gathers of fields f+1..f+R and this wave's quarter of
  // their W1 images in flight (one register ring: both are waited for at the same depth, so the
  // in-order vmcnt never waits on a younger field)
  float4 xa[NB], xb[NB], xw[NB];
  f32x16 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
  float fs[8], fq = 0.0f, fw = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) fs[k] = 0.0f;
  auto issue = [&](int f, int sl) {
    const int id = my_ids[c * F + f];
    if constexpr (PK) {
      const float4* line = reinterpret_cast<const float4*>(a.P[f] + (int64_t)id * 32);
      xa[sl] = line[h];
      xb[sl] = line[2 + h];
      xw[sl] = line[4 + h];
    } else {
      const float4* vr = reinterpret_cast<const float4*>(a.V[f] + (int64_t)id * 16);
      xa[sl] = vr[h];
      xb[sl] = vr[2 + h];
      const float wv = (a.W[f] != nullptr && h == 0) ? a.W[f][id] : 0.0f;
      xw[sl] = make_float4(wv, 0.0f, 0.0f, 0.0f);
    }
  };
#pragma unroll
  for (int f = 0; f < R; ++f) issue(f, f);
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const int sl = f % NB;
    if (f + R < F) issue(f + R, (f + R) % NB);
    __builtin_amdgcn_sched_barrier(0);
    // field f's registers "redefined" here: left alone, hipcc consumes each field's loads right
    // after issuing them (fewer live registers) and so waits on them at once
    __syncthreads();  // barrier f: slot f % 3 holds field f (plain global loads survive it)
    asm volatile("" : "+v"(xa[sl].x), "+v"(xa[sl].y), "+v"(xa[sl].z), "+v"(xa[sl].w), "+v"(xb[sl].x),
                 "+v"(xb[sl].y), "+v"(xb[sl].z), "+v"(xb[sl].w), "+v"(xw[sl].x), "+v"(xw[sl].y), "+v"(xw[sl].z),
                 "+v"(xw[sl].w));
    const __bf16* ws = w1s[f % 3];
    // W1 fragments of n-tile pair jp + 1 read while pair jp's MFMAs run; pair 0's reads are
    // issued before the split, whose VALU then covers their latency
    bf16x8 ah[2][2], al[2][2];
    auto wread = [&](int jp, int b) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int n = 32 * (2 * jp + q) + c;
        ah[b][q] = *reinterpret_cast<const bf16x8*>(ws + w1_idx(n, 8 * h));
        al[b][q] = *reinterpret_cast<const bf16x8*>(ws + 4096 + w1_idx(n, 8 * h));
      }
    };
    wread(0, 0);
    bf16x8 bh, bl;
    {
      const float4 p = xa[sl], q = xb[sl], w = xw[sl];
      const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        fs[k] += v[k];
        fq += v[k] * v[k];
        const __bf16 hv = (__bf16)v[k];
        bh[k] = hv;
        bl[k] = (__bf16)(v[k] - (float)hv);
      }
      // bytes 64..95 of the line: W then zeros (deepfm_pack_k), so the whole 16-B piece sums
      // to W on h = 0 and to 0 on h = 1 (all four components used: a dword load of the same
      // line runs at 38 G lines/s in the probe, a 16-B piece at 48 G)
      fw += (w.x + w.y) + (w.z + w.w);
    }
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      if (jp + 1 < 4) wread(jp + 1, (jp + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
      const int b = jp & 1;
      if (ABL & 4) {
        asm volatile("" :: "v"(al[b][0]), "v"(ah[b][0]), "v"(al[b][1]), "v"(ah[b][1]), "v"(bh), "v"(bl));
        __builtin_amdgcn_sched_barrier(0);
        continue;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j = 2 * jp + q;
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[b][q], bh, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[b][q], bl, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[b][q], bh, acc[j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // ---- layer 2 in two halves of n2 (64 outputs each: the half's accumulators, the layer-1
  // accumulators and a 6-deep W2 prefetch ring fit the registers the layer-1 rings leave free).
  // The 32 (half, k-step) steps are one flat unrolled sequence, so the ring runs across the
  // halves; B fragments of k-step t = 2j + g2 from acc[j] (deepfm_fused_k order), rebuilt per
  // half. b1 / b2 / w_o come from LDS: a global load here would wait out the W2 prefetch.
  float dot = 0.0f;
  if (ABL & 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" :: "v"(acc[j]));
  }
  constexpr int P = 3, NS = 32;
  bf16x8 w2h[P + 1][2], w2l[P + 1][2];
  auto w2load = [&](int st) {
    const int half = st >> 4, t = st & 15, b = st % (P + 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = w2_off(t, 32 * (2 * half + q) + c, h);
      w2h[b][q] = *reinterpret_cast<const bf16x8*>(a.w2hi + o);
      w2l[b][q] = *reinterpret_cast<const bf16x8*>(a.w2lo + o);
    }
  };
  if (!(ABL & 8)) {
#pragma unroll
    for (int st = 0; st < P; ++st) w2load(st);
  }
  f32x16 acc2[2];
#pragma unroll
  for (int st = 0; st < (ABL & 8 ? 0 : NS); ++st) {
    const int half = st >> 4, t = st & 15, j = t >> 1, g2 = t & 1, b = st % (P + 1);
    if (t == 0) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[q][r] = 0.0f;
    }
    if (st + P < NS) w2load(st + P);
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 gh, gl;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float4 bb = *reinterpret_cast<const float4*>(b1s + 16 * t + 8 * p + 4 * h);
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[j][4 * (2 * g2 + p) + e] + bv[e];
        v = v > 0.0f ? v : 0.0f;
        const __bf16 hv = (__bf16)v;
        gh[4 * p + e] = hv;
        gl[4 * p + e] = (__bf16)(v - (float)hv);
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const bf16x8 ah = w2h[b][q], al = w2l[b][q];
      acc2[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, gh, acc2[q], 0, 0, 0);
      acc2[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, gl, acc2[q], 0, 0, 0);
      acc2[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, gh, acc2[q], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t == 15) {  // relu(H2 + b2) . wo over this half's 64 outputs
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int nb = 32 * (2 * half + q) + 8 * g + 4 * h;
          const float4 bb = *reinterpret_cast<const float4*>(b2s + nb);
          const float4 ww = *reinterpret_cast<const float4*>(wos + nb);
          dot += fmaxf(acc2[q][4 * g + 0] + bb.x, 0.0f) * ww.x;
          dot += fmaxf(acc2[q][4 * g + 1] + bb.y, 0.0f) * ww.y;
          dot += fmaxf(acc2[q][4 * g + 2] + bb.z, 0.0f) * ww.z;
          dot += fmaxf(acc2[q][4 * g + 3] + bb.w, 0.0f) * ww.w;
        }
    }
  }
  float fm = -fq;
#pragma unroll
  for (int k = 0; k < 8; ++k) fm += fs[k] * fs[k];
  dot += __shfl_xor(dot, 32, 64);
  fm += __shfl_xor(fm, 32, 64);
  const float first = fw + __shfl_xor(fw, 32, 64);
  const int64_t row = m0 + c;
  if (h == 0 && row < a.R) {
    const float v = a.bias + first + 0.5f * fm + dot;
    a.logit[row] = v;
    if (a.prob) a.prob[row] = 1.0f / (1.0f + expf(-v));
  }
}

template <int I, int N, typename Fn>
__device__ __forceinline__ void static_for_(Fn&& fn) {
  if constexpr (I < N) {
    fn(std::integral_constant<int, I>{});
    static_for_<I + 1, N>(fn);
  }
}

// s_waitcnt vmcnt(n) for a count known after unrolling (the switch folds to one instruction)
#define RSX_VMW(N) \
  case N:          \
    asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); \
    break;
__device__ __forceinline__ void vm_wait_n(int n) {
  switch (n) {
    RSX_VMW(0) RSX_VMW(1) RSX_VMW(2) RSX_VMW(3) RSX_VMW(4) RSX_VMW(5) RSX_VMW(6) RSX_VMW(7)
    RSX_VMW(8) RSX_VMW(9) RSX_VMW(10) RSX_VMW(11) RSX_VMW(12) RSX_VMW(13) RSX_VMW(14) RSX_VMW(15)
    RSX_VMW(16) RSX_VMW(17) RSX_VMW(18) RSX_VMW(19) RSX_VMW(20) RSX_VMW(21) RSX_VMW(22) RSX_VMW(23)
    RSX_VMW(24) RSX_VMW(25) RSX_VMW(26) RSX_VMW(27) RSX_VMW(28) RSX_VMW(29) RSX_VMW(30) RSX_VMW(31)
    RSX_VMW(32) RSX_VMW(33) RSX_VMW(34) RSX_VMW(35) RSX_VMW(36) RSX_VMW(37) RSX_VMW(38) RSX_VMW(39)
    RSX_VMW(40) RSX_VMW(41) RSX_VMW(42) RSX_VMW(43) RSX_VMW(44) RSX_VMW(45) RSX_VMW(46) RSX_VMW(47)
    RSX_VMW(48) RSX_VMW(49) RSX_VMW(50) RSX_VMW(51) RSX_VMW(52) RSX_VMW(53) RSX_VMW(54) RSX_VMW(55)
    RSX_VMW(56) RSX_VMW(57) RSX_VMW(58) RSX_VMW(59) RSX_VMW(60) RSX_VMW(61) RSX_VMW(62) RSX_VMW(63)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;  // > 63: the counter's limit
  }
}
#undef RSX_VMW

// deepfm_rows5_k reorganised around 256-row workgroups (65,536 rows: one round of the grid
// instead of two) with the layer-1 accumulators in the AGPR file, in two shapes:
//   MT = 2: four waves of 64 rows (two 32-row m-tiles sharing every W1 fragment read, half the LDS
//           read traffic per MFMA; 256 accumulator floats, one wave per SIMD);
//   MT = 1: eight waves of 32 rows (128 accumulator floats, two waves per SIMD).
// There is no stager wave (no room beside AGPR-holding compute waves): each wave stages its share
// of a field's W1 image by LDS-DMA (inline asm: hipcc would drain vmcnt in front of every LDS read
// if it saw a pending DMA) and waits for it with a counted vmcnt. Field f's work is software-
// pipelined around barrier B_{f+1}, which sits after its first two n-tile pairs: behind B_{f+1}
// (slot (f+1) % 4 complete everywhere) the wave issues the DMA of field f + 3 into slot (f + 3) % 4
// (field f - 1's, finished before B_{f+1}), splits field f + 1's gathered rows and reads its first
// W1 fragments under field f's last two pairs of MFMAs. Layer 2 reads W2 from LDS: the 128-KiB
// image (1-KiB pieces, piece p at byte 1024 p of the union) is staged as space frees up -- pieces
// 104..127 (unused by layer 1) in the prologue, each wave's id region after its last gather, the
// slots of fields F-4 / F-3 after B_{F-1}, the last two slots after layer 1 -- and each step's B
// fragments are built under the previous step's MFMAs.
template <int F>
__host__ __device__ constexpr int rows2m_after_dma(int g, int R, int iss, int idp, int dp) {
  // loads a wave issues between its DMA of field g and its wait for it (before B_g): gathers,
  // the next field's DMA and the W2 pieces staged into the wave's id region at field F - 1 - R
  // (idp of them). An exact count: a smaller one would also wait for younger loads.
  const int fi = F - 1 - R;
  return g == 0 ? dp + iss * R
       : g == 1 ? iss * R + dp + (R < F ? iss : 0) + (fi == 0 ? idp : 0)
                : (g - 2 + R < F ? iss : 0) + (g + 1 < F ? dp : 0) + (g - 1 + R < F ? iss : 0) +
                      ((fi == g - 2 || fi == g - 1) ? idp : 0);
}

constexpr int kRows2mLds = 2 * 16 * kN2 * 16 * 2;  // bytes: the W2 hi + lo images (128 KiB)

#ifndef RSX_DFM_R
#define RSX_DFM_R 3
#endif
#ifndef RSX_DFM_L2PIPE
#define RSX_DFM_L2PIPE 1  // layer 2: the next step's B fragments built under this step's MFMAs
#endif
#ifndef RSX_DFM_ABL
#define RSX_DFM_ABL 0  // timing probes (wrong results): 1 no field barriers, 2 no W1 DMA in the loop
#endif

template <int F, int MT, bool L2 = true>
__global__ __launch_bounds__(512 / MT, 1) void deepfm_rows2m_k(RArgs a) {
  constexpr int NW = 8 / MT;        // waves per workgroup (256 rows)
  constexpr int R = RSX_DFM_R, NB = R + 1;  // gather ring: fields in flight ahead of the one computed
  constexpr int kIss = 3 * MT;      // global loads per issue() (m-tiles x three 16-B pieces)
  constexpr int kDp = 16 / NW;      // 1-KiB W1 pieces a wave stages per field
  constexpr int kSlots = 4;         // W1 ring
  constexpr int kIdBlk = 5 * MT;    // 1-KiB blocks per wave's id region (32 MT F ints)
  constexpr int kIdp = kIdBlk;      // W2 pieces a wave stages into its id region
  static_assert(32 * MT * F * 4 <= kIdBlk * 1024 && 64 + NW * kIdBlk <= 104, "id regions must fit blocks 64..103");
  static_assert(F - 1 - R >= 2, "the staging schedule assumes F >= R + 3");
  // union (1-KiB blocks): layer 1 = W1 ring blocks 0..63 + ids blocks 64..103 (104..127 free);
  // layer 2 = W2 hi | lo, piece p in block p
  __shared__ __attribute__((aligned(16))) unsigned char lds[kRows2mLds];
  __shared__ __attribute__((aligned(16))) float b1s[kN1], b2s[kN2], wos[kN2];
  __bf16* w1s = reinterpret_cast<__bf16*>(lds);
  int* ids_all = reinterpret_cast<int*>(lds + kSlots * kW1Field * 2);
  // MT = 2: an AGPR operand anywhere in the kernel keeps hipcc from inferring "no AGPRs", which
  // selects the VGPR form of every MFMA (the 256 accumulators would then spill). MT = 1: the VGPR
  // form, 256 architectural registers per wave at two waves per SIMD (with AGPR-form MFMAs the
  // layer-2 accumulators would not fit beside the layer-1 ones in a 128 / 128 split)
  if (MT == 2) asm volatile("" ::"a"(0.0f));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 31, h = lane >> 5;
  if (tid < kN1) b1s[tid] = a.b1[tid];
  if (tid < kN2) b2s[tid] = a.b2[tid];
  else if (tid < kN1) wos[tid - kN2] = a.wo[tid - kN2];
  int* my_ids = ids_all + wave * (kIdBlk * 256);
  const int64_t m0 = ((int64_t)blockIdx.x * NW + wave) * (32 * MT);  // this wave's 32 MT rows
  const char* w1g = reinterpret_cast<const char*>(a.w1);
  // LDS-DMA from inline asm (M0 = the LDS base; M0 has no other user in this kernel; one wait state
  // between the M0 write and the DMA that reads it)
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)lds;
  auto dma1k = [&](const char* src_block, unsigned dst_block) {
    const char* src = src_block + 16 * lane;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(dst_block) : "memory");
  };
  auto dma = [&](int f) {  // pieces kDp wave .. kDp wave + kDp - 1 (1 KiB each) of field f's image
#pragma unroll
    for (int k = 0; k < kDp; ++k) {
      const int piece = kDp * wave_u + k;
      dma1k(w1g + (int64_t)f * (kW1Field * 2) + 1024 * piece, lds_base + (f % kSlots) * (kW1Field * 2) + 1024 * piece);
    }
  };

  const char* w2g = reinterpret_cast<const char*>(a.w2hi);  // w2lo follows w2hi (deepfm_prep_images)
  auto w2dma = [&](int piece) { dma1k(w2g + 1024 * piece, lds_base + 1024 * piece); };
  if (L2) {
#pragma unroll
    for (int k = 0; k < 24 / NW; ++k) w2dma(104 + (24 / NW) * wave_u + k);  // blocks no layer-1 data uses
  }
  // ---- ids of the 32 MT rows -> LDS (int32); rows past R re-read the last row, never stored
  {
    const int64_t last = a.R - 1;
    constexpr int NE = 32 * MT * F, NT = (NE + 63) / 64;
#pragma unroll
    for (int t0 = 0; t0 < NT; t0 += 13) {
      int64_t v[13];
#pragma unroll
      for (int t = 0; t < 13; ++t) {
        const int e = lane + 64 * (t0 + t);
        const int row = e / F, f = e - row * F;
        const int64_t gr = m0 + row <= last ? m0 + row : last;
        v[t] = (t0 + t < NT && e < NE) ? a.x[gr * F + f] : 0;
      }
#pragma unroll
      for (int t = 0; t < 13; ++t)
        if (t0 + t < NT && lane + 64 * (t0 + t) < NE) my_ids[lane + 64 * (t0 + t)] = (int)v[t];
    }
  }
  float4 xa[MT][NB], xb[MT][NB], xw[MT][NB];
  f32x16 acc[MT][8];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][j][r] = 0.0f;
  float fs[MT][8], fq[MT], fw[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    fq[m] = 0.0f;
    fw[m] = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) fs[m][k] = 0.0f;
  }
  auto issue = [&](int f, int sl) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int id = my_ids[(32 * m + c) * F + f];
      const float4* line = reinterpret_cast<const float4*>(a.P[f] + (int64_t)id * 32);
      xa[m][sl] = line[h];
      xb[m][sl] = line[2 + h];
      xw[m][sl] = line[4 + h];
    }
  };
  // field f's gathered rows (ring slot sl) -> split fragments (set st) + the FM sums
  bf16x8 bh[2][MT], bl[2][MT];  // [set][m-tile]
  auto split = [&](int sl, int st) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
      asm volatile("" : "+v"(xa[m][sl].x), "+v"(xa[m][sl].y), "+v"(xa[m][sl].z), "+v"(xa[m][sl].w), "+v"(xb[m][sl].x),
                   "+v"(xb[m][sl].y), "+v"(xb[m][sl].z), "+v"(xb[m][sl].w), "+v"(xw[m][sl].x), "+v"(xw[m][sl].y),
                   "+v"(xw[m][sl].z), "+v"(xw[m][sl].w));
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float4 p = xa[m][sl], q = xb[m][sl], w = xw[m][sl];
      const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        fs[m][k] += v[k];
        fq[m] += v[k] * v[k];
        const __bf16 hv = (__bf16)v[k];
        bh[st][m][k] = hv;
        bl[st][m][k] = (__bf16)(v[k] - (float)hv);
      }
      fw[m] += (w.x + w.y) + (w.z + w.w);  // W then zeros (deepfm_pack_k): see deepfm_rows5_k
      // the FM sums are formed here, field by field: left alone, hipcc sinks the 39-term chains to
      // their use after the field loop and keeps every gathered piece alive until then (spills)
      asm volatile("" : "+v"(fs[m][0]), "+v"(fs[m][1]), "+v"(fs[m][2]), "+v"(fs[m][3]), "+v"(fs[m][4]),
                   "+v"(fs[m][5]), "+v"(fs[m][6]), "+v"(fs[m][7]), "+v"(fq[m]), "+v"(fw[m]));
    }
  };
  bf16x8 ah[2][2], al[2][2];  // W1 fragments [buffer][n-tile of the pair]
  auto wread = [&](int f, int jp, int b) {
    const __bf16* ws = w1s + (f % kSlots) * kW1Field;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int n = 32 * (2 * jp + q) + c;
      ah[b][q] = *reinterpret_cast<const bf16x8*>(ws + w1_idx(n, 8 * h));
      al[b][q] = *reinterpret_cast<const bf16x8*>(ws + 4096 + w1_idx(n, 8 * h));
    }
  };
  auto pair_mfma = [&](int jp, int b, int st) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int j = 2 * jp + q;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[b][q], bh[st][m], acc[m][j], 0, 0, 0);
        acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[b][q], bl[st][m], acc[m][j], 0, 0, 0);
        acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[b][q], bh[st][m], acc[m][j], 0, 0, 0);
      }
    }
  };
  dma(0);
  dma(1);
#pragma unroll
  for (int f = 0; f < R; ++f) issue(f, f);
  __builtin_amdgcn_sched_barrier(0);
  vm_wait_n(rows2m_after_dma<F>(0, R, kIss, L2 ? kIdp : 0, kDp));  // this wave's quarter of field 0 landed
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ids, b1 / b2 / w_o stores
  __builtin_amdgcn_s_barrier();  // B_0
  __builtin_amdgcn_sched_barrier(0);
  dma(2);
  split(0, 0);
  wread(0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  static_for_<0, F>([&](auto fc) __attribute__((always_inline)) {
    constexpr int f = decltype(fc)::value;
    constexpr int cs = f & 1;
    if (f + R < F) issue(f + R, (f + R) % NB);
    if (L2 && f == F - 1 - R) {  // last gather issued: this wave's id region takes W2 pieces
#pragma unroll
      for (int k = 0; k < kIdp; ++k) w2dma(64 + kIdBlk * wave_u + k);
    }
    __builtin_amdgcn_sched_barrier(0);
    // pairs 0 and 1 of field f (the next pair's fragments read under each pair's MFMAs)
    wread(f, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    pair_mfma(0, 0, cs);
    __builtin_amdgcn_sched_barrier(0);
    wread(f, 2, 0);
    __builtin_amdgcn_sched_barrier(0);
    pair_mfma(1, 1, cs);
    __builtin_amdgcn_sched_barrier(0);
    if (f + 1 < F) {
      if (!(RSX_DFM_ABL & 1)) {
        vm_wait_n(rows2m_after_dma<F>(f + 1, R, kIss, L2 ? kIdp : 0, kDp));  // this wave's quarter of field f + 1
        __builtin_amdgcn_s_barrier();                                    // B_{f+1}
      }
      __builtin_amdgcn_sched_barrier(0);
      if (f + 3 < F && !(RSX_DFM_ABL & 2)) dma(f + 3);
      if (L2 && f + 1 == F - 1) {  // slots of fields F-4 and F-3 are free: W2 pieces into them
        constexpr int s0 = (F - 4) % kSlots, s1 = (F - 3) % kSlots;
#pragma unroll
        for (int k = 0; k < kDp; ++k) {
          w2dma(16 * s0 + kDp * wave_u + k);
          w2dma(16 * s1 + kDp * wave_u + k);
        }
      }
    }
    // pair 2 with field f + 1's split in its MFMA issue gaps, then pair 3 with field f + 1's
    // first fragments read under it
    wread(f, 3, 1);
    if (f + 1 < F) split((f + 1) % NB, cs ^ 1);
    pair_mfma(2, 0, cs);
    if (f + 1 < F) {
#pragma unroll
      for (int i = 0; i < 6 * MT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);  // six VALU
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (f + 1 < F) wread(f + 1, 0, 0);
    pair_mfma(3, 1, cs);
    __builtin_amdgcn_sched_barrier(0);
  });
  // ---- W2 (hi | lo, 128 KiB) into the layer-1 space: every wave is past its last W1 / id read
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (L2) {  // the last two slots (fields F-2, F-1)
    constexpr int s0 = (F - 2) % kSlots, s1 = (F - 1) % kSlots;
#pragma unroll
    for (int k = 0; k < kDp; ++k) {
      w2dma(16 * s0 + kDp * wave_u + k);
      w2dma(16 * s1 + kDp * wave_u + k);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  // ---- layer 2 (deepfm_rows5_k's flat 32-step sequence, each W2 fragment used by both m-tiles)
  float dot[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) dot[m] = 0.0f;
  constexpr int NS = 32;
  bf16x8 w2h[2][2], w2l[2][2];
  auto w2read = [&](int st) {
    const int half = st >> 4, t = st & 15, b = st & 1;
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // piece 4 t + 2 half + q of each image; 16 B at lane (c, h)
      const int p = 4 * t + 2 * half + q, o = 2 * (w2_off(0, c, h));  // bytes within the piece
      w2h[b][q] = *reinterpret_cast<const bf16x8*>(lds + 1024 * p + o);
      w2l[b][q] = *reinterpret_cast<const bf16x8*>(lds + 1024 * (64 + p) + o);
    }
  };
  f32x16 acc2[MT][2];
  if (!L2) {  // timing ablation (wrong results): layer 1 only (one element per tile kept live)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 8; ++j) dot[m] += acc[m][j][0] * 1e-30f;
  }
  // B fragments of step st (relu(H1 + b1) of k-step t = st & 15, split), both m-tiles
  bf16x8 gh[2][MT], gl[2][MT];  // [set][m-tile]
  auto build = [&](int st, int set) {
    const int t = st & 15, j = t >> 1, g2 = t & 1;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float4 bb = *reinterpret_cast<const float4*>(b1s + 16 * t + 8 * p + 4 * h);
        const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[m][j][4 * (2 * g2 + p) + e] + bv[e];
          v = v > 0.0f ? v : 0.0f;
          const __bf16 hv = (__bf16)v;
          gh[set][m][4 * p + e] = hv;
          gl[set][m][4 * p + e] = (__bf16)(v - (float)hv);
        }
      }
    }
  };
  if (L2) {
    w2read(0);
    if (RSX_DFM_L2PIPE) build(0, 0);
  }
  auto step = [&](int st) __attribute__((always_inline)) {
    const int half = st >> 4, t = st & 15, b = st & 1;
    if (t == 0) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc2[m][q][r] = 0.0f;
    }
    if (st + 1 < NS) w2read(st + 1);
    if (!RSX_DFM_L2PIPE) build(st, b);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const bf16x8 wh = w2h[b][q], wl = w2l[b][q];
        acc2[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, gh[b][m], acc2[m][q], 0, 0, 0);
        acc2[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, gl[b][m], acc2[m][q], 0, 0, 0);
        acc2[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, gh[b][m], acc2[m][q], 0, 0, 0);
      }
    }
    if (RSX_DFM_L2PIPE && st + 1 < NS) {  // the next step's fragments in this step's MFMA issue gaps
      build(st + 1, b ^ 1);
#pragma unroll
      for (int i = 0; i < 6 * MT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t == 15) {  // relu(H2 + b2) . wo over this half's 64 outputs
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int nb = 32 * (2 * half + q) + 8 * g + 4 * h;
            const float4 bb = *reinterpret_cast<const float4*>(b2s + nb);
            const float4 ww = *reinterpret_cast<const float4*>(wos + nb);
            dot[m] += fmaxf(acc2[m][q][4 * g + 0] + bb.x, 0.0f) * ww.x;
            dot[m] += fmaxf(acc2[m][q][4 * g + 1] + bb.y, 0.0f) * ww.y;
            dot[m] += fmaxf(acc2[m][q][4 * g + 2] + bb.z, 0.0f) * ww.z;
            dot[m] += fmaxf(acc2[m][q][4 * g + 3] + bb.w, 0.0f) * ww.w;
          }
    }
  };
#pragma unroll
  for (int st = 0; st < (L2 ? NS : 0); ++st) step(st);
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    float fm = -fq[m];
#pragma unroll
    for (int k = 0; k < 8; ++k) fm += fs[m][k] * fs[m][k];
    const float d = dot[m] + __shfl_xor(dot[m], 32, 64);
    fm += __shfl_xor(fm, 32, 64);
    const float first = fw[m] + __shfl_xor(fw[m], 32, 64);
    const int64_t row = m0 + 32 * m + c;
    if (h == 0 && row < a.R) {
      const float v = a.bias + first + 0.5f * fm + d;
      a.logit[row] = v;
      if (a.prob) a.prob[row] = 1.0f / (1.0f + expf(-v));
    }
  }
}

// W1 [256][F*16] -> [F][8192]: hi at w1_idx(n, s), lo at 4096 + w1_idx(n, s), s = k-slot with
// V index kperm(s) = (s & 3) + 8 * ((s >> 2) & 1) + 4 * (s >> 3)
__global__ __launch_bounds__(256) void deepfm_prep3_k(const float* w1, int F, __bf16* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)F * 256 * 16) return;
  const int s = (int)(i & 15), n = (int)((i >> 4) & 255), f = (int)(i >> 12);
  const int k = (s & 3) + 8 * ((s >> 2) & 1) + 4 * (s >> 3);
  const float v = w1[(int64_t)n * F * 16 + f * 16 + k];
  const __bf16 hv = (__bf16)v;
  __bf16* img = out + (int64_t)f * kW1Field;
  img[w1_idx(n, s)] = hv;
  img[4096 + w1_idx(n, s)] = (__bf16)(v - (float)hv);
}

size_t persist_lds_bytes(int id_stride) {
  return (size_t)4 * kChunk2 * sizeof(__bf16) + 2 * (size_t)kBM * kH1Stride * sizeof(__bf16) +
         4 * kBM * sizeof(float) + 2 * (size_t)kBM * id_stride * sizeof(int);
}

using rsx::cu_count;

bool persist_ok(int F) { return F >= 3 * kFC2 + 1 && F <= kPersistMaxF && getenv("RSX_DEEPFM_PERSIST") == nullptr; }

// row-owning kernel for F = 39 (RSX_DEEPFM_ROWS=0: the persistent kernel, A/B)
bool rows_ok(int F) {
  static const bool off = [] {
    const char* e = getenv("RSX_DEEPFM_ROWS");
    return e && e[0] == '0';
  }();
  return F == kRowsF && !off;
}

}  // namespace

RSX_API int64_t rsx_deepfm_fused_workspace_bytes(int F) {
  if (F < 1 || F > kMaxF) return -1;
  const int64_t nchunk = (F + kFC - 1) / kFC, nchunk2 = (F + kFC2 - 1) / kFC2;
  const int64_t w1 = nchunk * kFC * kN1 * 16 > nchunk2 * kFC2 * kN1 * 16 ? nchunk * kFC * kN1 * 16
                                                                          : nchunk2 * kFC2 * kN1 * 16;
  return 2 * (w1 + 16 * kN2 * 16) * (int64_t)sizeof(__bf16);
}

namespace {
// Builds the weight images of the kernel form rsx_deepfm_fused_run takes for F fields.
int deepfm_prep_images(int F, const float* w1, const float* w2, __bf16* wsb, hipStream_t st) {
  if (rows_ok(F)) {  // W1 [F][8192] (deepfm_prep3_k), then W2 in deepfm_prep_k's permuted order
    const int64_t n1 = (int64_t)F * 256 * 16, m1 = (int64_t)F * kW1Field, n2 = 16 * kN2 * 16;
    hipLaunchKernelGGL(deepfm_prep3_k, dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, st, w1, F, wsb);
    hipLaunchKernelGGL(deepfm_prep_k, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, st, w1, F, 0, w2, wsb, wsb,
                       wsb + m1, wsb + m1 + n2);
    return 0;
  }
  if (persist_ok(F)) {
    const int nchunk = (F + kFC2 - 1) / kFC2;
    const int64_t m1 = (int64_t)nchunk * kFC2 * kN1 * 16, m2 = (int64_t)kN2 * kN1;
    hipLaunchKernelGGL(deepfm_prep2_k, dim3((unsigned)((m1 + m2 + 255) / 256)), dim3(256), 0, st, w1, F, nchunk,
                       w2, wsb, wsb + m1, wsb + 2 * m1, wsb + 2 * m1 + m2);
  } else {
    const int nchunk = (F + kFC - 1) / kFC;
    const int64_t n1 = (int64_t)nchunk * kFC * kN1 * 16, n2 = 16 * kN2 * 16;
    hipLaunchKernelGGL(deepfm_prep_k, dim3((unsigned)((n1 + n2 + 255) / 256)), dim3(256), 0, st, w1, F, nchunk, w2,
                       wsb, wsb + n1, wsb + 2 * n1, wsb + 2 * n1 + n2);
  }
  return 0;
}
}  // namespace

RSX_API int rsx_deepfm_fused_prep(int F, const float* w1, const float* w2, void* ws, void* stream) {
  RSX_ARG(w1 && w2 && ws, "null tensor");
  RSX_ARG(F >= 1 && F <= kMaxF, "F must be in [1,64]");
  deepfm_prep_images(F, w1, w2, reinterpret_cast<__bf16*>(ws), (hipStream_t)stream);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_deepfm_pack(const float* V, const float* W, int64_t vocab, float* packed, void* stream) {
  RSX_ARG(V && packed, "null tensor");
  RSX_ARG(vocab >= 0, "vocab must be >= 0");
  if (vocab == 0) return 0;
  hipLaunchKernelGGL(deepfm_pack_k, dim3((unsigned)((vocab * 8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, V, W,
                     vocab, packed);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_deepfm_fused_uses_packed(int F) { return (persist_ok(F) || rows_ok(F)) ? 1 : 0; }

RSX_API int rsx_deepfm_fused_run(const int64_t* x, int64_t R, int F, const float* const* V, const float* const* W,
                                 const float* const* packed, float bias, const float* b1, const float* b2,
                                 const float* wo, const void* ws, float* logit, float* prob, void* stream) {
  RSX_ARG(x && V && b1 && b2 && wo && ws && logit, "null tensor");
  RSX_ARG(F >= 1 && F <= kMaxF, "F must be in [1,64]");
  if (R == 0) return 0;
  for (int f = 0; f < F; ++f) RSX_ARG(V[f] != nullptr, "null field table");
  const __bf16* wsb = reinterpret_cast<const __bf16*>(ws);
  hipStream_t st = (hipStream_t)stream;
  if (rows_ok(F)) {  // the weight images are in this kernel's layout (deepfm_prep_images)
    if (packed)
      for (int f = 0; f < F; ++f) RSX_ARG(packed[f] != nullptr, "null packed table");
    RArgs r;
    r.x = x;
    for (int f = 0; f < kMaxF; ++f) {
      r.P[f] = (f < F && packed) ? packed[f] : nullptr;
      r.V[f] = f < F ? V[f] : nullptr;
      r.W[f] = (f < F && W) ? W[f] : nullptr;
    }
    r.R = R;
    const int64_t grid = (R + 127) / 128;  // 4 compute waves x 32 rows
    r.nit = 1;
    r.bias = bias;
    const int64_t m1 = (int64_t)F * kW1Field, n2 = 16 * kN2 * 16;
    r.w1 = wsb;
    r.w2hi = wsb + m1;
    r.w2lo = wsb + m1 + n2;
    r.b1 = b1; r.b2 = b2; r.wo = wo; r.logit = logit; r.prob = prob;
    // RSX_DEEPFM_ROWS (A/B): unset = deepfm_rows2m_k<F, 1> (eight 32-row waves), 2 = <F, 2> (four
    // 64-row waves), 5 = deepfm_rows5_k, 4 = deepfm_rows_k with RSX_DEEPFM_ABL ablations;
    // RSX_DEEPFM_ABL with rows2m: layer 1 only (timing, wrong results)
    static const char mode = [] {
      const char* e = getenv("RSX_DEEPFM_ROWS");
      return e && (e[0] == '2' || e[0] == '4' || e[0] == '5') ? e[0] : 'w';
    }();
    if (!packed) {
      hipLaunchKernelGGL((deepfm_rows5_k<kRowsF, false>), dim3((unsigned)grid), dim3(320), 0, st, r);
      RSX_LAUNCHED();
      return 0;
    }
    if (mode == 'w' || mode == '2') {
      const bool l1 = getenv("RSX_DEEPFM_ABL") != nullptr;
      const dim3 g((unsigned)((R + 255) / 256));  // 256 rows per workgroup
      if (mode == 'w' && l1) hipLaunchKernelGGL((deepfm_rows2m_k<kRowsF, 1, false>), g, dim3(512), 0, st, r);
      else if (mode == 'w') hipLaunchKernelGGL((deepfm_rows2m_k<kRowsF, 1>), g, dim3(512), 0, st, r);
      else if (l1) hipLaunchKernelGGL((deepfm_rows2m_k<kRowsF, 2, false>), g, dim3(256), 0, st, r);
      else hipLaunchKernelGGL((deepfm_rows2m_k<kRowsF, 2>), g, dim3(256), 0, st, r);
      RSX_LAUNCHED();
      return 0;
    }
    if (mode == '5') {
      hipLaunchKernelGGL((deepfm_rows5_k<kRowsF, true>), dim3((unsigned)grid), dim3(320), 0, st, r);
      RSX_LAUNCHED();
      return 0;
    }
    const char* abl_env = getenv("RSX_DEEPFM_ABL");  // timing ablations (diagnostic only)
    const int abl = abl_env ? atoi(abl_env) : 0;
    switch (abl) {
      case 1: hipLaunchKernelGGL((deepfm_rows_k<kRowsF, 1>), dim3((unsigned)grid), dim3(256), 0, st, r); break;
      case 3: hipLaunchKernelGGL((deepfm_rows_k<kRowsF, 3>), dim3((unsigned)grid), dim3(256), 0, st, r); break;
      case 4: hipLaunchKernelGGL((deepfm_rows_k<kRowsF, 4>), dim3((unsigned)grid), dim3(256), 0, st, r); break;
      case 8: hipLaunchKernelGGL((deepfm_rows_k<kRowsF, 8>), dim3((unsigned)grid), dim3(256), 0, st, r); break;
      case 12: hipLaunchKernelGGL((deepfm_rows_k<kRowsF, 12>), dim3((unsigned)grid), dim3(256), 0, st, r); break;
      case 15: hipLaunchKernelGGL((deepfm_rows_k<kRowsF, 15>), dim3((unsigned)grid), dim3(256), 0, st, r); break;
      default: hipLaunchKernelGGL((deepfm_rows_k<kRowsF, 0>), dim3((unsigned)grid), dim3(256), 0, st, r); break;
    }
    RSX_LAUNCHED();
    return 0;
  }
  if (persist_ok(F)) {
    PArgs p;
    p.x = x;
    for (int f = 0; f < kMaxF; ++f) {
      p.V[f] = f < F ? V[f] : nullptr;
      p.W[f] = (f < F && W) ? W[f] : nullptr;
      p.P[f] = (f < F && packed) ? packed[f] : nullptr;
    }
    if (packed)
      for (int f = 0; f < F; ++f) RSX_ARG(packed[f] != nullptr, "null packed table");
    p.R = R;
    p.F = F;
    p.nchunk = (F + kFC2 - 1) / kFC2;
    p.id_stride = F | 1;  // odd: the loaders' per-row id reads fall on distinct banks
    p.nrb = (R + kBM - 1) / kBM;
    p.bias = bias;
    const int64_t m1 = (int64_t)p.nchunk * kFC2 * kN1 * 16, m2 = (int64_t)kN2 * kN1;
    p.w1hi = wsb;
    p.w1lo = wsb + m1;
    p.w2hi = wsb + 2 * m1;
    p.w2lo = wsb + 2 * m1 + m2;
    p.b1 = b1; p.b2 = b2; p.wo = wo; p.logit = logit; p.prob = prob;
    const int64_t grid = p.nrb < cu_count() ? p.nrb : cu_count();
    static const bool attr = [] {  // > 64 KB of dynamic LDS per workgroup
      return hipFuncSetAttribute(reinterpret_cast<const void*>(&deepfm_persist_k),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    }();
    (void)attr;
    hipLaunchKernelGGL(deepfm_persist_k, dim3((unsigned)grid), dim3(512), persist_lds_bytes(p.id_stride), st, p);
    RSX_LAUNCHED();
    return 0;
  }
  FArgs a;
  a.x = x;
  for (int f = 0; f < kMaxF; ++f) {
    a.V[f] = f < F ? V[f] : nullptr;
    a.W[f] = (f < F && W) ? W[f] : nullptr;
  }
  a.R = R;
  a.F = F;
  a.nchunk = (F + kFC - 1) / kFC;
  a.bias = bias;
  const int64_t n1 = (int64_t)a.nchunk * kFC * kN1 * 16, n2 = 16 * kN2 * 16;
  a.w1hi = wsb;
  a.w1lo = wsb + n1;
  a.w2hi = wsb + 2 * n1;
  a.w2lo = wsb + 2 * n1 + n2;
  a.b1 = b1; a.b2 = b2; a.wo = wo; a.logit = logit; a.prob = prob;
  hipLaunchKernelGGL(deepfm_fused_k, dim3((unsigned)((R + kBM - 1) / kBM)), dim3(512), 0, st, a);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_deepfm_fused(const int64_t* x, int64_t R, int F, const float* const* V, const float* const* W,
                             float bias, const float* w1, const float* b1, const float* w2, const float* b2,
                             const float* wo, void* ws, float* logit, float* prob, void* stream) {
  RSX_ARG(x && V && w1 && b1 && w2 && b2 && wo && ws && logit, "null tensor");
  RSX_ARG(F >= 1 && F <= kMaxF, "F must be in [1,64]");
  if (R == 0) return 0;
  const int rc = rsx_deepfm_fused_prep(F, w1, w2, ws, stream);
  if (rc != 0) return rc;
  return rsx_deepfm_fused_run(x, R, F, V, W, nullptr, bias, b1, b2, wo, ws, logit, prob, stream);
}
