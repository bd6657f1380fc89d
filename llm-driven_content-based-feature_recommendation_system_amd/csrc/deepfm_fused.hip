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
        const int64_t o = (((int64_t)ks * kN2 + n2) * 2 + h) * 8;
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
    const int el = (int)(j % 8), hh = (int)((j / 8) % 2), n2 = (int)((j / 16) % kN2), ks = (int)(j / (16 * kN2));
    const int k = 16 * ks + 8 * (el >> 2) + 4 * hh + (el & 3);
    const float v = w2[(int64_t)n2 * kN1 + k];
    const __bf16 hv = (__bf16)v;
    w2hi[j] = hv;
    w2lo[j] = (__bf16)(v - (float)hv);
  }
}

}  // namespace

RSX_API int64_t rsx_deepfm_fused_workspace_bytes(int F) {
  if (F < 1 || F > kMaxF) return -1;
  const int64_t nchunk = (F + kFC - 1) / kFC;
  return 2 * (nchunk * kFC * kN1 * 16 + 16 * kN2 * 16) * (int64_t)sizeof(__bf16);
}

RSX_API int rsx_deepfm_fused(const int64_t* x, int64_t R, int F, const float* const* V, const float* const* W,
                             float bias, const float* w1, const float* b1, const float* w2, const float* b2,
                             const float* wo, void* ws, float* logit, float* prob, void* stream) {
  RSX_ARG(x && V && w1 && b1 && w2 && b2 && wo && ws && logit, "null tensor");
  RSX_ARG(F >= 1 && F <= kMaxF, "F must be in [1,64]");
  if (R == 0) return 0;
  FArgs a;
  a.x = x;
  for (int f = 0; f < kMaxF; ++f) {
    a.V[f] = f < F ? V[f] : nullptr;
    a.W[f] = (f < F && W) ? W[f] : nullptr;
  }
  for (int f = 0; f < F; ++f) RSX_ARG(a.V[f] != nullptr, "null field table");
  a.R = R;
  a.F = F;
  a.nchunk = (F + kFC - 1) / kFC;
  a.bias = bias;
  __bf16* wsb = reinterpret_cast<__bf16*>(ws);
  const int64_t n1 = (int64_t)a.nchunk * kFC * kN1 * 16, n2 = 16 * kN2 * 16;
  a.w1hi = wsb;
  a.w1lo = wsb + n1;
  a.w2hi = wsb + 2 * n1;
  a.w2lo = wsb + 2 * n1 + n2;
  a.b1 = b1; a.b2 = b2; a.wo = wo; a.logit = logit; a.prob = prob;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(deepfm_prep_k, dim3((unsigned)((n1 + n2 + 255) / 256)), dim3(256), 0, st, w1, F, a.nchunk, w2,
                     wsb, wsb + n1, wsb + 2 * n1, wsb + 2 * n1 + n2);
  RSX_LAUNCHED();
  hipLaunchKernelGGL(deepfm_fused_k, dim3((unsigned)((R + kBM - 1) / kBM)), dim3(512), 0, st, a);
  RSX_LAUNCHED();
  return 0;
}
