// Masked multi-head self-attention core for short sequences (L <= 64), the attention of
// nn.TransformerEncoderLayer as used by
//   * SASRecUserTower   tower_code/v1_refine_usertower.py:343-352, 461-466
//     (causal mask triu(ones,1) + src_key_padding_mask, left padding, L = 50, dh = 32)
//   * HybridItemTower   item_tower.py:169-182, 281 (no mask, 16 field tokens, dh = d/4)
// Input is the in_proj output qkv[T, 3*D] (q | k | v, heads contiguous inside each part,
// exactly torch's in_proj_weight layout) for T tokens: dense sequences (T = B*L) or packed
// variable-length segments (seg_off, used by the training step to skip left padding);
// output is the concatenated head output [T, D] that feeds out_proj.
//
// Semantics pinned to the training-mode (non fast-path) reference: a query row whose keys
// are all masked (left-padded positions under the causal mask) gets all-zero
// probabilities, so its attention output is exactly 0 (=> out_proj.bias after out_proj).
// Attention-probability dropout (p > 0) uses the counter-based hash in rsx_common.h.
//
// One 64-lane workgroup per (batch, head): lane i owns query row i. K/V rows of the head
// are staged in LDS and read by broadcast; scores live in registers (L <= 64).
#include "rsx_common.h"
#include <math.h>
#include <stdlib.h>

namespace {

constexpr int kLMax = 64;

struct FwdArgs {
  const float* qkv;      // [T, 3D] tokens (dense: T = B*L, token b*L+l; packed: segments by seg)
  const uint8_t* kpad;   // [T] 1 = pad (masked key) or nullptr
  const int* seg;        // [B+1] token offsets of each sequence (packed) or nullptr (dense, length L)
  float* out;            // [T, D]
  float* lse;            // [T, H] (natural log-sum-exp of the scaled scores; -inf if fully masked)
  int B, L, H, causal;
  float scale;
  rsx::Dropout drop;
};

template <int DH>
__global__ __launch_bounds__(64) void mha_fwd_k(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) float sK[kLMax][DH];
  __shared__ __attribute__((aligned(16))) float sV[kLMax][DH];
  __shared__ int sPad[kLMax];
  const int D = a.H * DH;
  const int b = blockIdx.x / a.H, hd = blockIdx.x % a.H;
  const int i = threadIdx.x;
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;  // packed segments are <= 51 by construction
  const float* base = a.qkv + tok0 * 3 * D;

  constexpr int V4 = DH / 4;
  for (int t = threadIdx.x; t < L * V4; t += 64) {
    const int r = t / V4, c4 = t % V4;
    const float4* rowp = reinterpret_cast<const float4*>(base + (int64_t)r * 3 * D);
    reinterpret_cast<float4*>(&sK[r][0])[c4] = rowp[(D + hd * DH) / 4 + c4];
    reinterpret_cast<float4*>(&sV[r][0])[c4] = rowp[(2 * D + hd * DH) / 4 + c4];
  }
  if (i < L) sPad[i] = a.kpad ? (int)a.kpad[tok0 + i] : 0;
  __syncthreads();
  if (i >= L) return;

  float q[DH];
  {
    const float4* qp = reinterpret_cast<const float4*>(base + (int64_t)i * 3 * D + hd * DH);
#pragma unroll
    for (int t = 0; t < V4; ++t) {
      const float4 v = qp[t];
      q[4 * t] = v.x; q[4 * t + 1] = v.y; q[4 * t + 2] = v.z; q[4 * t + 3] = v.w;
    }
  }
  float s[kLMax];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < kLMax; ++j) {
    s[j] = -INFINITY;
    if (j < L) {
      const bool allowed = !sPad[j] && (!a.causal || j <= i);
      float d = 0.0f;
#pragma unroll
      for (int t = 0; t < V4; ++t) {
        const float4 kv = reinterpret_cast<const float4*>(&sK[j][0])[t];
        d = fmaf(q[4 * t], kv.x, d);
        d = fmaf(q[4 * t + 1], kv.y, d);
        d = fmaf(q[4 * t + 2], kv.z, d);
        d = fmaf(q[4 * t + 3], kv.w, d);
      }
      if (allowed) {
        s[j] = d * a.scale;
        mx = fmaxf(mx, s[j]);
      }
    }
  }
  float o[DH];
#pragma unroll
  for (int e = 0; e < DH; ++e) o[e] = 0.0f;
  float lse = -INFINITY;
  if (mx != -INFINITY) {
    float sum = 0.0f;
#pragma unroll
    for (int j = 0; j < kLMax; ++j) {
      const float p = (s[j] == -INFINITY) ? 0.0f : __expf(s[j] - mx);
      s[j] = p;
      sum += p;
    }
    const float inv = 1.0f / sum;
    lse = mx + logf(sum);
    const uint64_t rowidx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax;
#pragma unroll
    for (int j = 0; j < kLMax; ++j) {
      if (j < L) {
        float p = s[j] * inv;
        p = a.drop.apply(p, rowidx + j);
        if (p != 0.0f) {
#pragma unroll
          for (int t = 0; t < V4; ++t) {
            const float4 vv = reinterpret_cast<const float4*>(&sV[j][0])[t];
            o[4 * t] = fmaf(p, vv.x, o[4 * t]);
            o[4 * t + 1] = fmaf(p, vv.y, o[4 * t + 1]);
            o[4 * t + 2] = fmaf(p, vv.z, o[4 * t + 2]);
            o[4 * t + 3] = fmaf(p, vv.w, o[4 * t + 3]);
          }
        }
      }
    }
  }
  float4* op = reinterpret_cast<float4*>(a.out + (tok0 + i) * D + hd * DH);
#pragma unroll
  for (int t = 0; t < V4; ++t) op[t] = make_float4(o[4 * t], o[4 * t + 1], o[4 * t + 2], o[4 * t + 3]);
  if (a.lse) a.lse[(tok0 + i) * a.H + hd] = lse;
}

struct BwdArgs {
  const float* qkv;
  const uint8_t* kpad;
  const int* seg;
  const float* out;   // forward output O [T, D]
  const float* lse;   // [T, H]
  const float* dout;  // [T, D]
  float* dqkv;        // [T, 3D] (written)
  int B, L, H, causal;
  float scale;
  rsx::Dropout drop;
};

template <int DH>
__global__ __launch_bounds__(64) void mha_bwd_k(BwdArgs a) {
  __shared__ __attribute__((aligned(16))) float sQ[kLMax][DH];
  __shared__ __attribute__((aligned(16))) float sK[kLMax][DH];
  __shared__ __attribute__((aligned(16))) float sdO[kLMax][DH];
  __shared__ float sLse[kLMax], sDelta[kLMax];
  __shared__ int sPad[kLMax];
  __shared__ float sdS[kLMax][kLMax + 1];
  const int D = a.H * DH;
  const int b = blockIdx.x / a.H, hd = blockIdx.x % a.H;
  const int lane = threadIdx.x;
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;  // packed segments are <= 51 by construction
  const float* base = a.qkv + tok0 * 3 * D;
  const float* dob = a.dout + tok0 * D;
  constexpr int V4 = DH / 4;

  for (int t = threadIdx.x; t < L * V4; t += 64) {
    const int r = t / V4, c4 = t % V4;
    const float4* rowp = reinterpret_cast<const float4*>(base + (int64_t)r * 3 * D);
    reinterpret_cast<float4*>(&sQ[r][0])[c4] = rowp[(hd * DH) / 4 + c4];
    reinterpret_cast<float4*>(&sK[r][0])[c4] = rowp[(D + hd * DH) / 4 + c4];
    reinterpret_cast<float4*>(&sdO[r][0])[c4] = reinterpret_cast<const float4*>(dob + (int64_t)r * D + hd * DH)[c4];
  }
  if (lane < L) {
    sPad[lane] = a.kpad ? (int)a.kpad[tok0 + lane] : 0;
    sLse[lane] = a.lse[(tok0 + lane) * a.H + hd];
    // delta_i = dO_i . O_i  (holds with dropout: sum_j P_ij dP_ij = dO_i . O_i)
    const float4* op = reinterpret_cast<const float4*>(a.out + (tok0 + lane) * D + hd * DH);
    const float4* dp = reinterpret_cast<const float4*>(dob + (int64_t)lane * D + hd * DH);
    float d = 0.0f;
#pragma unroll
    for (int t = 0; t < V4; ++t) {
      const float4 x = op[t], y = dp[t];
      d += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    sDelta[lane] = d;
  }
  __syncthreads();

  // ---- pass A: lane j owns key/value row j: dK_j, dV_j, and dS column j into LDS ----
  const int j = lane;
  float kj[DH], vj[DH], dk[DH], dv[DH];
  const bool jok = j < L;
  if (jok) {
    const float4* vp = reinterpret_cast<const float4*>(base + (int64_t)j * 3 * D + 2 * D + hd * DH);
#pragma unroll
    for (int t = 0; t < V4; ++t) {
      const float4 kk = reinterpret_cast<const float4*>(&sK[j][0])[t];
      const float4 vv = vp[t];
      kj[4 * t] = kk.x; kj[4 * t + 1] = kk.y; kj[4 * t + 2] = kk.z; kj[4 * t + 3] = kk.w;
      vj[4 * t] = vv.x; vj[4 * t + 1] = vv.y; vj[4 * t + 2] = vv.z; vj[4 * t + 3] = vv.w;
    }
  } else {
#pragma unroll
    for (int e = 0; e < DH; ++e) { kj[e] = 0.0f; vj[e] = 0.0f; }
  }
#pragma unroll
  for (int e = 0; e < DH; ++e) { dk[e] = 0.0f; dv[e] = 0.0f; }
  const bool jpad = jok ? (sPad[j] != 0) : true;

  for (int i = 0; i < L; ++i) {
    const float lse_i = sLse[i];
    float ds = 0.0f;
    const bool allowed = jok && !jpad && (!a.causal || j <= i) && lse_i != -INFINITY;
    if (allowed) {
      float sdot = 0.0f, pdot = 0.0f;
#pragma unroll
      for (int t = 0; t < V4; ++t) {
        const float4 qv = reinterpret_cast<const float4*>(&sQ[i][0])[t];
        const float4 gv = reinterpret_cast<const float4*>(&sdO[i][0])[t];
        sdot = fmaf(qv.x, kj[4 * t], sdot); sdot = fmaf(qv.y, kj[4 * t + 1], sdot);
        sdot = fmaf(qv.z, kj[4 * t + 2], sdot); sdot = fmaf(qv.w, kj[4 * t + 3], sdot);
        pdot = fmaf(gv.x, vj[4 * t], pdot); pdot = fmaf(gv.y, vj[4 * t + 1], pdot);
        pdot = fmaf(gv.z, vj[4 * t + 2], pdot); pdot = fmaf(gv.w, vj[4 * t + 3], pdot);
      }
      const float p = __expf(sdot * a.scale - lse_i);
      const uint64_t idx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax + j;
      float pd = p, dp = pdot;
      if (a.drop.active()) {
        const bool keep = rsx::hash_u32(a.drop.seed, idx) >= a.drop.thresh;
        pd = keep ? p * a.drop.scale : 0.0f;
        dp = keep ? pdot * a.drop.scale : 0.0f;
      }
      ds = p * (dp - sDelta[i]) * a.scale;
#pragma unroll
      for (int t = 0; t < V4; ++t) {
        const float4 qv = reinterpret_cast<const float4*>(&sQ[i][0])[t];
        const float4 gv = reinterpret_cast<const float4*>(&sdO[i][0])[t];
        dv[4 * t] = fmaf(pd, gv.x, dv[4 * t]); dv[4 * t + 1] = fmaf(pd, gv.y, dv[4 * t + 1]);
        dv[4 * t + 2] = fmaf(pd, gv.z, dv[4 * t + 2]); dv[4 * t + 3] = fmaf(pd, gv.w, dv[4 * t + 3]);
        dk[4 * t] = fmaf(ds, qv.x, dk[4 * t]); dk[4 * t + 1] = fmaf(ds, qv.y, dk[4 * t + 1]);
        dk[4 * t + 2] = fmaf(ds, qv.z, dk[4 * t + 2]); dk[4 * t + 3] = fmaf(ds, qv.w, dk[4 * t + 3]);
      }
    }
    if (j < kLMax) sdS[i][j] = ds;
  }
  __syncthreads();

  float* db = a.dqkv + tok0 * 3 * D;
  if (jok) {
    float4* kp = reinterpret_cast<float4*>(db + (int64_t)j * 3 * D + D + hd * DH);
    float4* vp = reinterpret_cast<float4*>(db + (int64_t)j * 3 * D + 2 * D + hd * DH);
#pragma unroll
    for (int t = 0; t < V4; ++t) {
      kp[t] = make_float4(dk[4 * t], dk[4 * t + 1], dk[4 * t + 2], dk[4 * t + 3]);
      vp[t] = make_float4(dv[4 * t], dv[4 * t + 1], dv[4 * t + 2], dv[4 * t + 3]);
    }
  }

  // ---- pass B: lane i owns query row i: dQ_i = sum_j dS_ij K_j ----
  const int i = lane;
  if (i < L) {
    float dq[DH];
#pragma unroll
    for (int e = 0; e < DH; ++e) dq[e] = 0.0f;
    for (int jj = 0; jj < L; ++jj) {
      const float ds = sdS[i][jj];
      if (ds != 0.0f) {
#pragma unroll
        for (int t = 0; t < V4; ++t) {
          const float4 kv = reinterpret_cast<const float4*>(&sK[jj][0])[t];
          dq[4 * t] = fmaf(ds, kv.x, dq[4 * t]); dq[4 * t + 1] = fmaf(ds, kv.y, dq[4 * t + 1]);
          dq[4 * t + 2] = fmaf(ds, kv.z, dq[4 * t + 2]); dq[4 * t + 3] = fmaf(ds, kv.w, dq[4 * t + 3]);
        }
      }
    }
    float4* qp = reinterpret_cast<float4*>(db + (int64_t)i * 3 * D + hd * DH);
#pragma unroll
    for (int t = 0; t < V4; ++t) qp[t] = make_float4(dq[4 * t], dq[4 * t + 1], dq[4 * t + 2], dq[4 * t + 3]);
  }
}

// ---- backward for head dim 64 (the item tower's bert-base text encoder under grad) -------------
// One wave per (sequence, head), fp32 on the VALU (the attention is ~1 % of a BERT layer's FLOPs; the
// GEMMs around it carry the step). Pass 0: lane j holds key / value row j in registers and walks the
// queries i (Q_i, dO_i broadcast from LDS), writing dS_ij and the dropped-out probability Pd_ij to LDS
// (mha_bwd_k's formulas: same mask, dropout hash and softmax). Then dK_j = sum_i dS_ij Q_i and
// dV_j = sum_i Pd_ij dO_i (lane j), and dQ_i = sum_j dS_ij K_j (lane i), 64 accumulators each.
// LM = the longest sequence the launch may hold (32: 33 KB of LDS, four waves per CU; 64: 81 KB).
template <int LM>
__global__ __launch_bounds__(64) void mha_bwd64_k(BwdArgs a) {
  constexpr int DH = 64, V4 = DH / 4;
  __shared__ __attribute__((aligned(16))) float sQ[LM][DH];
  __shared__ __attribute__((aligned(16))) float sK[LM][DH];
  __shared__ __attribute__((aligned(16))) float sdO[LM][DH];
  __shared__ float sDS[LM][LM + 1], sPD[LM][LM + 1];
  __shared__ float sLse[LM], sDelta[LM];
  __shared__ int sPad[LM];
  const int D = a.H * DH;
  const int b = blockIdx.x / a.H, hd = blockIdx.x % a.H;
  const int lane = threadIdx.x;
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > LM) L = LM;  // the host sizes LM by the longest sequence
  const float* base = a.qkv + tok0 * 3 * D;
  const float* dob = a.dout + tok0 * D;
  for (int t = lane; t < L * V4; t += 64) {
    const int r = t / V4, c4 = t % V4;
    const float4* rowp = reinterpret_cast<const float4*>(base + (int64_t)r * 3 * D);
    reinterpret_cast<float4*>(&sQ[r][0])[c4] = rowp[(hd * DH) / 4 + c4];
    reinterpret_cast<float4*>(&sK[r][0])[c4] = rowp[(D + hd * DH) / 4 + c4];
    reinterpret_cast<float4*>(&sdO[r][0])[c4] = reinterpret_cast<const float4*>(dob + (int64_t)r * D + hd * DH)[c4];
  }
  if (lane < L) {
    sPad[lane] = a.kpad ? (int)a.kpad[tok0 + lane] : 0;
    sLse[lane] = a.lse[(tok0 + lane) * a.H + hd];
    const float4* op = reinterpret_cast<const float4*>(a.out + (tok0 + lane) * D + hd * DH);
    const float4* dp = reinterpret_cast<const float4*>(dob + (int64_t)lane * D + hd * DH);
    float d = 0.0f;
#pragma unroll
    for (int t = 0; t < V4; ++t) {
      const float4 x = op[t], y = dp[t];
      d += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    sDelta[lane] = d;
  }
  __syncthreads();
  const int j = lane;
  const bool jok = j < L;
  {  // pass 0
    float kj[DH], vj[DH];
    if (jok) {
      const float4* vp = reinterpret_cast<const float4*>(base + (int64_t)j * 3 * D + 2 * D + hd * DH);
#pragma unroll
      for (int t = 0; t < V4; ++t) {
        const float4 kk = reinterpret_cast<const float4*>(&sK[j][0])[t];
        const float4 vv = vp[t];
        kj[4 * t] = kk.x; kj[4 * t + 1] = kk.y; kj[4 * t + 2] = kk.z; kj[4 * t + 3] = kk.w;
        vj[4 * t] = vv.x; vj[4 * t + 1] = vv.y; vj[4 * t + 2] = vv.z; vj[4 * t + 3] = vv.w;
      }
    }
    const bool jpad = jok ? (sPad[j] != 0) : true;
    for (int i = 0; i < L; ++i) {
      const float lse_i = sLse[i];
      float ds = 0.0f, pd = 0.0f;
      if (jok && !jpad && (!a.causal || j <= i) && lse_i != -INFINITY) {
        float sdot = 0.0f, pdot = 0.0f;
#pragma unroll
        for (int t = 0; t < V4; ++t) {
          const float4 qv = reinterpret_cast<const float4*>(&sQ[i][0])[t];
          const float4 gv = reinterpret_cast<const float4*>(&sdO[i][0])[t];
          sdot = fmaf(qv.x, kj[4 * t], sdot); sdot = fmaf(qv.y, kj[4 * t + 1], sdot);
          sdot = fmaf(qv.z, kj[4 * t + 2], sdot); sdot = fmaf(qv.w, kj[4 * t + 3], sdot);
          pdot = fmaf(gv.x, vj[4 * t], pdot); pdot = fmaf(gv.y, vj[4 * t + 1], pdot);
          pdot = fmaf(gv.z, vj[4 * t + 2], pdot); pdot = fmaf(gv.w, vj[4 * t + 3], pdot);
        }
        const float p = __expf(sdot * a.scale - lse_i);
        const uint64_t idx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax + j;
        pd = p;
        float dp = pdot;
        if (a.drop.active()) {
          const bool keep = rsx::hash_u32(a.drop.seed, idx) >= a.drop.thresh;
          pd = keep ? p * a.drop.scale : 0.0f;
          dp = keep ? pdot * a.drop.scale : 0.0f;
        }
        ds = p * (dp - sDelta[i]) * a.scale;
      }
      if (j < LM) {
        sDS[i][j] = ds;
        sPD[i][j] = pd;
      }
    }
  }
  __syncthreads();
  float* db = a.dqkv + tok0 * 3 * D;
  float acc[DH];
  if (jok) {  // dK_j
#pragma unroll
    for (int e = 0; e < DH; ++e) acc[e] = 0.0f;
    for (int i = 0; i < L; ++i) {
      const float w = sDS[i][j];
#pragma unroll
      for (int t = 0; t < V4; ++t) {
        const float4 qv = reinterpret_cast<const float4*>(&sQ[i][0])[t];
        acc[4 * t] = fmaf(w, qv.x, acc[4 * t]); acc[4 * t + 1] = fmaf(w, qv.y, acc[4 * t + 1]);
        acc[4 * t + 2] = fmaf(w, qv.z, acc[4 * t + 2]); acc[4 * t + 3] = fmaf(w, qv.w, acc[4 * t + 3]);
      }
    }
    float4* kp = reinterpret_cast<float4*>(db + (int64_t)j * 3 * D + D + hd * DH);
#pragma unroll
    for (int t = 0; t < V4; ++t) kp[t] = make_float4(acc[4 * t], acc[4 * t + 1], acc[4 * t + 2], acc[4 * t + 3]);
#pragma unroll
    for (int e = 0; e < DH; ++e) acc[e] = 0.0f;  // dV_j
    for (int i = 0; i < L; ++i) {
      const float w = sPD[i][j];
#pragma unroll
      for (int t = 0; t < V4; ++t) {
        const float4 gv = reinterpret_cast<const float4*>(&sdO[i][0])[t];
        acc[4 * t] = fmaf(w, gv.x, acc[4 * t]); acc[4 * t + 1] = fmaf(w, gv.y, acc[4 * t + 1]);
        acc[4 * t + 2] = fmaf(w, gv.z, acc[4 * t + 2]); acc[4 * t + 3] = fmaf(w, gv.w, acc[4 * t + 3]);
      }
    }
    float4* vq = reinterpret_cast<float4*>(db + (int64_t)j * 3 * D + 2 * D + hd * DH);
#pragma unroll
    for (int t = 0; t < V4; ++t) vq[t] = make_float4(acc[4 * t], acc[4 * t + 1], acc[4 * t + 2], acc[4 * t + 3]);
  }
  const int i = lane;
  if (i < L) {  // dQ_i
#pragma unroll
    for (int e = 0; e < DH; ++e) acc[e] = 0.0f;
    for (int jj = 0; jj < L; ++jj) {
      const float w = sDS[i][jj];
#pragma unroll
      for (int t = 0; t < V4; ++t) {
        const float4 kv = reinterpret_cast<const float4*>(&sK[jj][0])[t];
        acc[4 * t] = fmaf(w, kv.x, acc[4 * t]); acc[4 * t + 1] = fmaf(w, kv.y, acc[4 * t + 1]);
        acc[4 * t + 2] = fmaf(w, kv.z, acc[4 * t + 2]); acc[4 * t + 3] = fmaf(w, kv.w, acc[4 * t + 3]);
      }
    }
    float4* qp = reinterpret_cast<float4*>(db + (int64_t)i * 3 * D + hd * DH);
#pragma unroll
    for (int t = 0; t < V4; ++t) qp[t] = make_float4(acc[4 * t], acc[4 * t + 1], acc[4 * t + 2], acc[4 * t + 3]);
  }
}

// ---- backward on the fp32-input MFMA (head dim 32) ---------------------------------------
// One wave per (sequence, head), four independent waves per workgroup, no LDS: every MFMA
// operand is either a token row the lane loads itself (16 contiguous floats of dims
// 16h..16h+15 for k-step (s, h) -> dim 16h + s) or a column slice X[row_s][e] read by 32
// consecutive lanes (coalesced), and every accumulator tile is consumed in place:
//   key on the lane (dK, dV):  S = Q K^T, dP' = dO V^T   -> dS, Pd   -> dV^T += dO^T Pd,
//                                                                        dK^T += Q^T dS
//   query on the lane (dQ):    S^T = K Q^T, dP'^T = V dO^T -> dS^T   -> dQ^T += K^T dS^T
// S and dP' are computed in both orientations (the MFMA work is small; no transposes). The
// per-element mask, dropout hash, softmax and dS formulas are those of mha_bwd_k.
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// 16 dims (16h .. 16h+15) of token row `row` of matrix base (row stride ld), zeros if !ok
__device__ __forceinline__ void load_row16(float (&x)[16], const float* base, int64_t ld, int64_t row, bool ok,
                                           int h) {
  if (ok) {
    const float4* p = reinterpret_cast<const float4*>(base + row * ld + 16 * h);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 v = p[t];
      x[4 * t] = v.x; x[4 * t + 1] = v.y; x[4 * t + 2] = v.z; x[4 * t + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < 16; ++t) x[t] = 0.0f;
  }
}

// acc[r] = sum_e A_row(lane-a)[e] * B_row(lane-b)[e] over 32 dims: rows on A's lanes become
// the accumulator rows, B's lanes the columns
__device__ __forceinline__ f32x16 dot_tile(const float (&a)[16], const float (&b)[16]) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
  return acc;
}

// acc += X^T T: X = 32 rows (row0 + tile_row(s,h)) of a matrix, column e = lane&31 (coalesced),
// T = an accumulator tile whose register s holds row tile_row(s,h): k index (s, h)
__device__ __forceinline__ void acc_colT(f32x16& acc, const float* base, int64_t ld, int64_t row0, int nrows,
                                         const f32x16& t, int c, int h) {
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int rr = tile_row(s, h);
    const float x = (rr < nrows) ? base[(row0 + rr) * ld + c] : 0.0f;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x, t[s], acc, 0, 0, 0);
  }
}

__global__ __launch_bounds__(256) void mha_bwd_mfma_k(BwdArgs a) {
  constexpr int DH = 32;
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const int64_t unit = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (unit >= (int64_t)a.B * a.H) return;  // whole wave exits together
  const int b = (int)(unit / a.H), hd = (int)(unit % a.H);
  const int D = a.H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;
  if (L <= 0) return;
  const int nb = (L + 31) >> 5;
  const float* Qb = a.qkv + tok0 * ld + hd * DH;
  const float* Kb = Qb + D;
  const float* Vb = Qb + 2 * D;
  const float* dOb = a.dout + tok0 * D + hd * DH;
  const float* Ob = a.out + tok0 * D + hd * DH;
  float* dQb = a.dqkv + tok0 * ld + hd * DH;
  float* dKb = dQb + D;
  float* dVb = dQb + 2 * D;
  const float sc = a.scale;

  // per-token softmax statistics of this head: lse_i and delta_i = dO_i . O_i
  // (token t < L lives on lane t; fetched by shuffle where needed)
  float my_lse = -INFINITY, my_delta = 0.0f;
  int my_pad = 1;
  if (lane < L) {
    my_lse = a.lse[(tok0 + lane) * a.H + hd];
    const float4* op = reinterpret_cast<const float4*>(Ob + (int64_t)lane * D);
    const float4* gp = reinterpret_cast<const float4*>(dOb + (int64_t)lane * D);
    float d = 0.0f;
#pragma unroll
    for (int t = 0; t < DH / 4; ++t) {
      const float4 x = op[t], y = gp[t];
      d += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    my_delta = d;
    my_pad = a.kpad ? (int)a.kpad[tok0 + lane] : 0;
  }

  // element (query i, key j) -> (p, pd, dpd factor) ; returns dS and Pd
  auto grad_elem = [&](int i, int j, float s, float dp, float lse_i, float delta_i, bool allowed, float& pd_out) {
    pd_out = 0.0f;
    if (!allowed) return 0.0f;
    const float p = __expf(s * sc - lse_i);
    float pd = p, dpd = dp;
    if (a.drop.active()) {
      const uint64_t idx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax + j;
      const bool keep = rsx::hash_u32(a.drop.seed, idx) >= a.drop.thresh;
      pd = keep ? p * a.drop.scale : 0.0f;
      dpd = keep ? dp * a.drop.scale : 0.0f;
    }
    pd_out = pd;
    return p * (dpd - delta_i) * sc;
  };

  // ---- key block on the lanes: dK, dV ----
  for (int kb = 0; kb < nb; ++kb) {
    const int j = 32 * kb + c;
    const bool jok = j < L;
    const int jpad = __shfl(my_pad, j & 63, 64);
    float kr[16], vr[16];
    load_row16(kr, Kb, ld, j, jok, h);
    load_row16(vr, Vb, ld, j, jok, h);
    f32x16 dkT, dvT;
#pragma unroll
    for (int r = 0; r < 16; ++r) { dkT[r] = 0.0f; dvT[r] = 0.0f; }
    for (int qb = a.causal ? kb : 0; qb < nb; ++qb) {  // non-causal: every query block
      float qr[16], gr[16];
      const int iq = 32 * qb + c;
      load_row16(qr, Qb, ld, iq, iq < L, h);
      load_row16(gr, dOb, D, iq, iq < L, h);
      f32x16 S = dot_tile(qr, kr);   // [i][j]
      f32x16 dP = dot_tile(gr, vr);  // [i][j]
      f32x16 Pd;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = 32 * qb + tile_row(r, h);
        const float lse_i = __shfl(my_lse, i & 63, 64);
        const float del_i = __shfl(my_delta, i & 63, 64);
        const bool allowed = jok && i < L && !jpad && (!a.causal || j <= i) && lse_i != -INFINITY;
        float pd;
        S[r] = grad_elem(i, j, S[r], dP[r], lse_i, del_i, allowed, pd);
        Pd[r] = pd;
      }
      const int nrows = L - 32 * qb;
      acc_colT(dvT, dOb, D, 32 * qb, nrows, Pd, c, h);  // dV^T[e][j] += sum_i dO[i][e] Pd[i][j]
      acc_colT(dkT, Qb, ld, 32 * qb, nrows, S, c, h);   // dK^T[e][j] += sum_i Q[i][e] dS[i][j]
    }
    if (jok) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int e = tile_row(r, h);
        dKb[(int64_t)j * ld + e] = dkT[r];
        dVb[(int64_t)j * ld + e] = dvT[r];
      }
    }
  }

  // ---- query block on the lanes: dQ ----
  for (int qb = 0; qb < nb; ++qb) {
    const int i = 32 * qb + c;
    const bool iok = i < L;
    const float lse_i = __shfl(my_lse, i & 63, 64);
    const float del_i = __shfl(my_delta, i & 63, 64);
    float qr[16], gr[16];
    load_row16(qr, Qb, ld, i, iok, h);
    load_row16(gr, dOb, D, i, iok, h);
    f32x16 dqT;
#pragma unroll
    for (int r = 0; r < 16; ++r) dqT[r] = 0.0f;
    const int kb_end = a.causal ? qb + 1 : nb;
    for (int kb = 0; kb < kb_end; ++kb) {
      float kr[16], vr[16];
      const int jk = 32 * kb + c;
      load_row16(kr, Kb, ld, jk, jk < L, h);
      load_row16(vr, Vb, ld, jk, jk < L, h);
      f32x16 S = dot_tile(kr, qr);   // [j][i]
      f32x16 dP = dot_tile(vr, gr);  // [j][i]
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = 32 * kb + tile_row(r, h);
        const int jpad = __shfl(my_pad, j & 63, 64);
        const bool allowed = iok && j < L && !jpad && (!a.causal || j <= i) && lse_i != -INFINITY;
        float pd;
        S[r] = grad_elem(i, j, S[r], dP[r], lse_i, del_i, allowed, pd);
      }
      acc_colT(dqT, Kb, ld, 32 * kb, L - 32 * kb, S, c, h);  // dQ^T[e][i] += sum_j K[j][e] dS^T[j][i]
    }
    if (iok) {
#pragma unroll
      for (int r = 0; r < 16; ++r) dQb[(int64_t)i * ld + tile_row(r, h)] = dqT[r];
    }
  }
}

// ---- bf16x3 forward and backward (head dim 32) ------------------------------------------
// Same semantics, masks, dropout hash and lse as the kernels above, on 16x16 tiles of the bf16
// MFMA: every fp32 operand x is split x = hi + lo (hi = bf16(x), lo = bf16(x - hi)) and a
// product is hi*hi' + hi*lo' + lo*hi' with fp32 accumulation (~2^-17 relative error per term,
// the precision of the bf16x3 InfoNCE and token GEMMs).
//   score tiles  S = Q K^T, dP = dO V^T over the 32 head dims: one v_mfma_f32_16x16x32_bf16
//                per split product (lane (c,g) holds row c, dims 8g..8g+7 of each operand);
//   token sums   O = P V, dV = Pd^T dO, dK = dS^T Q, dQ = dS K over 16 tokens:
//                v_mfma_f32_16x16x16_bf16 with the A operand taken straight from the score
//                accumulator (lane (c,g) register r holds tile row 4g+r, column c = exactly the
//                A fragment of the transposed product) and the B operand gathered as columns
//                (4 rows x 1 float per lane, L1/L2 hits of rows this wave just read).
// One wave per (sequence, head), four per workgroup, no LDS; 16-token blocks waste less of
// the tile than 32 on the H&M lengths (mean ~19 tokens). MFMA cycles per 16x16 block pair:
// fwd 3x16 + 6x8, bwd (two passes) 12x16 + 18x8, against 8x(16x4 f32) = 256 per product on
// the fp32 MFMA.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Row8 {  // dims 8g .. 8g+7 of one token row, split
  bf16x8 hi, lo;
};
struct Col4 {  // 4 consecutive token rows of one column, split
  s16x4 hi, lo;
};

__device__ __forceinline__ Row8 load_row8(const float* base, int64_t ld, int row, bool ok, int g) {
  float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
  if (ok) {
    const float4* p = reinterpret_cast<const float4*>(base + (int64_t)row * ld + 8 * g);
    v0 = p[0];
    v1 = p[1];
  }
  const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  Row8 r;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const __bf16 h = (__bf16)f[k];
    r.hi[k] = h;
    r.lo[k] = (__bf16)(f[k] - (float)h);
  }
  return r;
}

__device__ __forceinline__ Col4 split4(const float (&f)[4]) {
  bf16x4 h, l;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const __bf16 hk = (__bf16)f[k];
    h[k] = hk;
    l[k] = (__bf16)(f[k] - (float)hk);
  }
  Col4 c;
  c.hi = __builtin_bit_cast(s16x4, h);
  c.lo = __builtin_bit_cast(s16x4, l);
  return c;
}

// column col of rows row0 .. row0+3 (zero past L)
__device__ __forceinline__ Col4 load_col4(const float* base, int64_t ld, int row0, int L, int col) {
  float f[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) f[t] = (row0 + t < L) ? base[(int64_t)(row0 + t) * ld + col] : 0.0f;
  return split4(f);
}

__device__ __forceinline__ f32x4 dot16_x3(const Row8& a, const Row8& b) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ f32x4 sum16_x3(const Col4& a, const Col4& b, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a.hi, b.lo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a.lo, b.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a.hi, b.hi, acc, 0, 0, 0);
  return acc;
}

__global__ __launch_bounds__(256) void mha_fwd_x3_k(FwdArgs a) {
  constexpr int DH = 32;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int64_t unit = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (unit >= (int64_t)a.B * a.H) return;  // whole wave exits together
  const int b = (int)(unit / a.H), hd = (int)(unit % a.H);
  const int D = a.H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;
  if (L <= 0) return;
  const int nb = (L + 15) >> 4;
  const float* Qb = a.qkv + tok0 * ld + hd * DH;
  const float* Kb = Qb + D;
  const float* Vb = Qb + 2 * D;
  float* Ob = a.out + tok0 * D + hd * DH;
  const int my_pad = (lane < L) ? (a.kpad ? (int)a.kpad[tok0 + lane] : 0) : 1;

  for (int qb = 0; qb < nb; ++qb) {
    const int i = 16 * qb + c;  // query of this lane's score column
    const bool iok = i < L;
    const Row8 qx = load_row8(Qb, ld, i, iok, g);
    const int kb_end = a.causal ? qb : nb - 1;
    f32x4 s[4];
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb <= kb_end) {
        const Row8 kx = load_row8(Kb, ld, 16 * kb + c, 16 * kb + c < L, g);
        s[kb] = dot16_x3(kx, qx);  // S^T: [key 16kb+4g+r][query i]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 16 * kb + 4 * g + r;
          const int jpad = __shfl(my_pad, j & 63, 64);
          const bool allowed = iok && j < L && !jpad && (!a.causal || j <= i);
          s[kb][r] = allowed ? s[kb][r] * a.scale : -INFINITY;
          m = fmaxf(m, s[kb][r]);
        }
      }
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.0f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb <= kb_end) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = (s[kb][r] == -INFINITY) ? 0.0f : __expf(s[kb][r] - m);
          s[kb][r] = p;
          l += p;
        }
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = (l > 0.0f) ? 1.0f / l : 0.0f;
    f32x4 o[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const uint64_t rowidx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb <= kb_end) {
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = a.drop.apply(s[kb][r] * inv, rowidx + 16 * kb + 4 * g + r);
        const Col4 pa = split4(p);
#pragma unroll
        for (int et = 0; et < 2; ++et) o[et] = sum16_x3(pa, load_col4(Vb, ld, 16 * kb + 4 * g, L, 16 * et + c), o[et]);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * qb + 4 * g + r;
      if (row < L) {
        Ob[(int64_t)row * D + c] = o[0][r];
        Ob[(int64_t)row * D + 16 + c] = o[1][r];
      }
    }
    if (a.lse && g == 0 && iok) a.lse[(tok0 + i) * a.H + hd] = (l > 0.0f) ? m + logf(l) : -INFINITY;
  }
}

// Forward with every operand load issued before the first use: the sequence's Q and K rows and
// V columns of this head for all NB 16-token blocks come in through one buffer resource over the
// sequence's rows (rows >= L read as zero by the range check: no branches, no per-load waits),
// so a wave pays one memory latency instead of one or two per query block (mha_fwd_x3_k
// re-loads K / V per query block behind data-dependent branches). Same arithmetic, masks,
// dropout hash and lse as mha_fwd_x3_k.
typedef unsigned int u32x4b __attribute__((ext_vector_type(4)));
__device__ __forceinline__ Row8 split_row8(const u32x4b& x0, const u32x4b& x1) {
  const float f[8] = {__uint_as_float(x0.x), __uint_as_float(x0.y), __uint_as_float(x0.z), __uint_as_float(x0.w),
                      __uint_as_float(x1.x), __uint_as_float(x1.y), __uint_as_float(x1.z), __uint_as_float(x1.w)};
  Row8 r;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const __bf16 h = (__bf16)f[k];
    r.hi[k] = h;
    r.lo[k] = (__bf16)(f[k] - (float)h);
  }
  return r;
}
template <int NB>
__device__ __forceinline__ void mha_fwd_x3b_seq(const FwdArgs& a, int hd, int64_t tok0, int L, int lane) {
  constexpr int DH = 32;
  const int c = lane & 15, g = lane >> 4;
  const int D = a.H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const uintptr_t bp = (uintptr_t)(a.qkv + tok0 * ld);
  const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)bp), bhi = __builtin_amdgcn_readfirstlane((unsigned)(bp >> 32));
  const unsigned nbytes = __builtin_amdgcn_readfirstlane((unsigned)(L * ld * 4));
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(((uintptr_t)bhi << 32) | blo), 0, (int)nbytes, 0x00020000);
  u32x4b qr[NB][2], kr[NB][2];
  unsigned vr[NB][2][4];
#pragma unroll
  for (int bb = 0; bb < NB; ++bb) {
    const unsigned oq = (unsigned)(((16 * bb + c) * ld + hd * DH + 8 * g) * 4);
    qr[bb][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, oq, 0, 0);
    qr[bb][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, oq + 16, 0, 0);
    kr[bb][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, oq + 4 * D, 0, 0);
    kr[bb][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, oq + 4 * D + 16, 0, 0);
#pragma unroll
    for (int et = 0; et < 2; ++et)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        vr[bb][et][t] = __builtin_amdgcn_raw_buffer_load_b32(
            rs, (unsigned)(((16 * bb + 4 * g + t) * ld + 2 * D + hd * DH + 16 * et + c) * 4), 0, 0);
  }
  const int my_pad = (lane < L) ? (a.kpad ? (int)a.kpad[tok0 + lane] : 0) : 1;
  float* Ob = a.out + tok0 * D + hd * DH;
  Row8 kx[NB];
#pragma unroll
  for (int bb = 0; bb < NB; ++bb) kx[bb] = split_row8(kr[bb][0], kr[bb][1]);
#pragma unroll
  for (int qb = 0; qb < NB; ++qb) {
    const int i = 16 * qb + c;  // query of this lane's score column
    const bool iok = i < L;
    const Row8 qx = split_row8(qr[qb][0], qr[qb][1]);
    const int kb_end = a.causal ? qb : NB - 1;
    f32x4 sv[NB];
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb <= kb_end) {
        sv[kb] = dot16_x3(kx[kb], qx);  // S^T: [key 16kb+4g+r][query i]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 16 * kb + 4 * g + r;
          const int jpad = __shfl(my_pad, j & 63, 64);
          const bool allowed = iok && j < L && !jpad && (!a.causal || j <= i);
          sv[kb][r] = allowed ? sv[kb][r] * a.scale : -INFINITY;
          m = fmaxf(m, sv[kb][r]);
        }
      }
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.0f;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb <= kb_end) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = (sv[kb][r] == -INFINITY) ? 0.0f : __expf(sv[kb][r] - m);
          sv[kb][r] = pv;
          l += pv;
        }
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = (l > 0.0f) ? 1.0f / l : 0.0f;
    f32x4 o[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const uint64_t rowidx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb <= kb_end) {
        float pr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) pr[r] = a.drop.apply(sv[kb][r] * inv, rowidx + 16 * kb + 4 * g + r);
        const Col4 pa = split4(pr);
#pragma unroll
        for (int et = 0; et < 2; ++et) {
          const float vf[4] = {__uint_as_float(vr[kb][et][0]), __uint_as_float(vr[kb][et][1]),
                               __uint_as_float(vr[kb][et][2]), __uint_as_float(vr[kb][et][3])};
          o[et] = sum16_x3(pa, split4(vf), o[et]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * qb + 4 * g + r;
      if (row < L) {
        Ob[(int64_t)row * D + c] = o[0][r];
        Ob[(int64_t)row * D + 16 + c] = o[1][r];
      }
    }
    if (a.lse && g == 0 && iok) a.lse[(tok0 + i) * a.H + hd] = (l > 0.0f) ? m + logf(l) : -INFINITY;
  }
}

// Head dim 64 (the item tower's BERT, inference): mha_fwd_x3b_seq with each token row in two
// 32-dim halves — S = Q_a K_a^T + Q_b K_b^T on the same 16x16 tile, four 16-column output groups.
template <int NB>
__device__ __forceinline__ void mha_fwd_x3b64_seq(const FwdArgs& a, int hd, int64_t tok0, int L, int lane) {
  constexpr int DH = 64;
  const int c = lane & 15, g = lane >> 4;
  const int D = a.H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const uintptr_t bp = (uintptr_t)(a.qkv + tok0 * ld);
  const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)bp), bhi = __builtin_amdgcn_readfirstlane((unsigned)(bp >> 32));
  const unsigned nbytes = __builtin_amdgcn_readfirstlane((unsigned)(L * ld * 4));
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(((uintptr_t)bhi << 32) | blo), 0, (int)nbytes, 0x00020000);
  u32x4b qr[NB][2][2], kr[NB][2][2];
  unsigned vr[NB][4][4];
#pragma unroll
  for (int bb = 0; bb < NB; ++bb) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const unsigned oq = (unsigned)(((16 * bb + c) * ld + hd * DH + 32 * hf + 8 * g) * 4);
      qr[bb][hf][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, oq, 0, 0);
      qr[bb][hf][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, oq + 16, 0, 0);
      kr[bb][hf][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, oq + 4 * D, 0, 0);
      kr[bb][hf][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, oq + 4 * D + 16, 0, 0);
    }
#pragma unroll
    for (int et = 0; et < 4; ++et)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        vr[bb][et][t] = __builtin_amdgcn_raw_buffer_load_b32(
            rs, (unsigned)(((16 * bb + 4 * g + t) * ld + 2 * D + hd * DH + 16 * et + c) * 4), 0, 0);
  }
  const int my_pad = (lane < L) ? (a.kpad ? (int)a.kpad[tok0 + lane] : 0) : 1;
  float* Ob = a.out + tok0 * D + hd * DH;
#pragma unroll
  for (int qb = 0; qb < NB; ++qb) {
    const int i = 16 * qb + c;  // query of this lane's score column
    const bool iok = i < L;
    const Row8 qa = split_row8(qr[qb][0][0], qr[qb][0][1]), qc = split_row8(qr[qb][1][0], qr[qb][1][1]);
    const int kb_end = a.causal ? qb : NB - 1;
    f32x4 sv[NB];
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb <= kb_end) {
        const f32x4 s0 = dot16_x3(split_row8(kr[kb][0][0], kr[kb][0][1]), qa);  // S^T: [key][query i]
        const f32x4 s1 = dot16_x3(split_row8(kr[kb][1][0], kr[kb][1][1]), qc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 16 * kb + 4 * g + r;
          const int jpad = __shfl(my_pad, j & 63, 64);
          const bool allowed = iok && j < L && !jpad && (!a.causal || j <= i);
          sv[kb][r] = allowed ? (s0[r] + s1[r]) * a.scale : -INFINITY;
          m = fmaxf(m, sv[kb][r]);
        }
      }
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.0f;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb <= kb_end) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = (sv[kb][r] == -INFINITY) ? 0.0f : __expf(sv[kb][r] - m);
          sv[kb][r] = pv;
          l += pv;
        }
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = (l > 0.0f) ? 1.0f / l : 0.0f;
    f32x4 o[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const uint64_t rowidx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb <= kb_end) {
        float pr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) pr[r] = a.drop.apply(sv[kb][r] * inv, rowidx + 16 * kb + 4 * g + r);
        const Col4 pa = split4(pr);
#pragma unroll
        for (int et = 0; et < 4; ++et) {
          const float vf[4] = {__uint_as_float(vr[kb][et][0]), __uint_as_float(vr[kb][et][1]),
                               __uint_as_float(vr[kb][et][2]), __uint_as_float(vr[kb][et][3])};
          o[et] = sum16_x3(pa, split4(vf), o[et]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * qb + 4 * g + r;
      if (row < L) {
#pragma unroll
        for (int et = 0; et < 4; ++et) Ob[(int64_t)row * D + 16 * et + c] = o[et][r];
      }
    }
    if (a.lse && g == 0 && iok) a.lse[(tok0 + i) * a.H + hd] = (l > 0.0f) ? m + logf(l) : -INFINITY;
  }
}

__global__ __launch_bounds__(256) void mha_fwd_x3b64_k(FwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= (int64_t)a.B * a.H) return;  // whole wave exits together
  const int b = (int)(unit / a.H), hd = (int)(unit % a.H);
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;
  if (L <= 0) return;
  const int nb = __builtin_amdgcn_readfirstlane((L + 15) >> 4);
  if (nb == 1) mha_fwd_x3b64_seq<1>(a, hd, tok0, L, lane);
  else if (nb == 2) mha_fwd_x3b64_seq<2>(a, hd, tok0, L, lane);
  else if (nb == 3) mha_fwd_x3b64_seq<3>(a, hd, tok0, L, lane);
  else mha_fwd_x3b64_seq<4>(a, hd, tok0, L, lane);
}

// three waves per SIMD (168 VGPRs, no spills; the default allocation took 176 and ran two): 166.6 ->
// 136.7 us on the headline tower's first layer (round 6, tools/tower_micro.py under rocprofv3)
__global__ __launch_bounds__(256, 3) void mha_fwd_x3b_k(FwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= (int64_t)a.B * a.H) return;  // whole wave exits together
  const int b = (int)(unit / a.H), hd = (int)(unit % a.H);
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;
  if (L <= 0) return;
  const int nb = __builtin_amdgcn_readfirstlane((L + 15) >> 4);
  if (nb == 1) mha_fwd_x3b_seq<1>(a, hd, tok0, L, lane);
  else if (nb == 2) mha_fwd_x3b_seq<2>(a, hd, tok0, L, lane);
  else if (nb == 3) mha_fwd_x3b_seq<3>(a, hd, tok0, L, lane);
  else mha_fwd_x3b_seq<4>(a, hd, tok0, L, lane);
}

__global__ __launch_bounds__(256) void mha_bwd_x3_k(BwdArgs a) {
  constexpr int DH = 32;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int64_t unit = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (unit >= (int64_t)a.B * a.H) return;  // whole wave exits together
  const int b = (int)(unit / a.H), hd = (int)(unit % a.H);
  const int D = a.H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;
  if (L <= 0) return;
  const int nb = (L + 15) >> 4;
  const float* Qb = a.qkv + tok0 * ld + hd * DH;
  const float* Kb = Qb + D;
  const float* Vb = Qb + 2 * D;
  const float* dOb = a.dout + tok0 * D + hd * DH;
  const float* Ob = a.out + tok0 * D + hd * DH;
  float* dQb = a.dqkv + tok0 * ld + hd * DH;
  float* dKb = dQb + D;
  float* dVb = dQb + 2 * D;
  const float sc = a.scale;

  // per-token softmax statistics (token t < L on lane t): lse_t, delta_t = dO_t . O_t, key pad
  float my_lse = -INFINITY, my_delta = 0.0f;
  int my_pad = 1;
  if (lane < L) {
    my_lse = a.lse[(tok0 + lane) * a.H + hd];
    const float4* op = reinterpret_cast<const float4*>(Ob + (int64_t)lane * D);
    const float4* gp = reinterpret_cast<const float4*>(dOb + (int64_t)lane * D);
    float d = 0.0f;
#pragma unroll
    for (int t = 0; t < DH / 4; ++t) {
      const float4 x = op[t], y = gp[t];
      d += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    my_delta = d;
    my_pad = a.kpad ? (int)a.kpad[tok0 + lane] : 0;
  }
  // dS_ij and the dropped-out probability Pd_ij of one score element (mha_bwd_k's formulas)
  auto grad_elem = [&](int i, int j, float s, float dp, float lse_i, float delta_i, bool allowed, float& pd_out) {
    pd_out = 0.0f;
    if (!allowed) return 0.0f;
    const float p = __expf(s * sc - lse_i);
    float pd = p, dpd = dp;
    if (a.drop.active()) {
      const uint64_t idx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax + j;
      const bool keep = rsx::hash_u32(a.drop.seed, idx) >= a.drop.thresh;
      pd = keep ? p * a.drop.scale : 0.0f;
      dpd = keep ? dp * a.drop.scale : 0.0f;
    }
    pd_out = pd;
    return p * (dpd - delta_i) * sc;
  };

  // ---- pass 1: key block on the score columns (j = 16kb + c): dK, dV ----
  for (int kb = 0; kb < nb; ++kb) {
    const int j = 16 * kb + c;
    const bool jok = j < L;
    const int jpad = __shfl(my_pad, j & 63, 64);
    const Row8 kx = load_row8(Kb, ld, j, jok, g);
    const Row8 vx = load_row8(Vb, ld, j, jok, g);
    f32x4 dk[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    f32x4 dv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    for (int qb = a.causal ? kb : 0; qb < nb; ++qb) {
      const int iq = 16 * qb + c;
      const Row8 qx = load_row8(Qb, ld, iq, iq < L, g);
      const Row8 gx = load_row8(dOb, D, iq, iq < L, g);
      f32x4 S = dot16_x3(qx, kx);   // [query 16qb+4g+r][key j]
      f32x4 dP = dot16_x3(gx, vx);  // [query][key]
      float ds[4], pd[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * qb + 4 * g + r;
        const float lse_i = __shfl(my_lse, i & 63, 64);
        const float del_i = __shfl(my_delta, i & 63, 64);
        const bool allowed = jok && i < L && !jpad && (!a.causal || j <= i) && lse_i != -INFINITY;
        ds[r] = grad_elem(i, j, S[r], dP[r], lse_i, del_i, allowed, pd[r]);
      }
      const Col4 pa = split4(pd), sa = split4(ds);
#pragma unroll
      for (int et = 0; et < 2; ++et) {
        dv[et] = sum16_x3(pa, load_col4(dOb, D, 16 * qb + 4 * g, L, 16 * et + c), dv[et]);  // dV[j][e]
        dk[et] = sum16_x3(sa, load_col4(Qb, ld, 16 * qb + 4 * g, L, 16 * et + c), dk[et]);  // dK[j][e]
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * kb + 4 * g + r;
      if (row < L) {
#pragma unroll
        for (int et = 0; et < 2; ++et) {
          dKb[(int64_t)row * ld + 16 * et + c] = dk[et][r];
          dVb[(int64_t)row * ld + 16 * et + c] = dv[et][r];
        }
      }
    }
  }

  // ---- pass 2: query block on the score columns (i = 16qb + c): dQ ----
  for (int qb = 0; qb < nb; ++qb) {
    const int i = 16 * qb + c;
    const bool iok = i < L;
    const float lse_i = __shfl(my_lse, i & 63, 64);
    const float del_i = __shfl(my_delta, i & 63, 64);
    const Row8 qx = load_row8(Qb, ld, i, iok, g);
    const Row8 gx = load_row8(dOb, D, i, iok, g);
    f32x4 dq[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int kb_end = a.causal ? qb : nb - 1;
    for (int kb = 0; kb <= kb_end; ++kb) {
      const int jr = 16 * kb + c;
      const Row8 kx = load_row8(Kb, ld, jr, jr < L, g);
      const Row8 vx = load_row8(Vb, ld, jr, jr < L, g);
      f32x4 St = dot16_x3(kx, qx);   // [key 16kb+4g+r][query i]
      f32x4 dPt = dot16_x3(vx, gx);  // [key][query]
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * kb + 4 * g + r;
        const int jpad = __shfl(my_pad, j & 63, 64);
        const bool allowed = iok && j < L && !jpad && (!a.causal || j <= i) && lse_i != -INFINITY;
        float pd;
        ds[r] = grad_elem(i, j, St[r], dPt[r], lse_i, del_i, allowed, pd);
      }
      const Col4 sa = split4(ds);
#pragma unroll
      for (int et = 0; et < 2; ++et)
        dq[et] = sum16_x3(sa, load_col4(Kb, ld, 16 * kb + 4 * g, L, 16 * et + c), dq[et]);  // dQ[i][e]
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * qb + 4 * g + r;
      if (row < L) {
        dQb[(int64_t)row * ld + c] = dq[0][r];
        dQb[(int64_t)row * ld + 16 + c] = dq[1][r];
      }
    }
  }
}

// ---- bf16x3 backward, software-pipelined ----------------------------------------------------
// mha_bwd_x3_k's wave per (sequence, head) and its two passes, with each pass's (key block,
// query block) pairs walked as one flat sequence: the operands of pair n+1 are loaded (buffer
// loads over the sequence's rows: rows past L, and the pair after the last, read as zero by the
// range check, so no load is predicated) while pair n computes, in two ping-pong register sets
// so that no in-flight load is copied. mha_bwd_x3_k waits one memory latency per pair.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t seq_rsrc(const void* base, unsigned bytes) {
  const uintptr_t bp = (uintptr_t)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)bp);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(bp >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uintptr_t)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
struct RawRow {  // dims 8g .. 8g+7 of one token row, as loaded
  u32x4b x0, x1;
};
__device__ __forceinline__ RawRow load_rawrow(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  RawRow r;
  r.x0 = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
  r.x1 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0);
  return r;
}
__device__ __forceinline__ void load_rawcols(__amdgpu_buffer_rsrc_t rs, int row0, int ld, int col,
                                             unsigned (&v)[2][4]) {
#pragma unroll
  for (int et = 0; et < 2; ++et)
#pragma unroll
    for (int t = 0; t < 4; ++t)
      v[et][t] = __builtin_amdgcn_raw_buffer_load_b32(rs, (unsigned)(((row0 + t) * ld + col + 16 * et) * 4), 0, 0);
}
__device__ __forceinline__ Col4 split_col4(const unsigned (&v)[4]) {
  const float f[4] = {__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3])};
  return split4(f);
}
struct Pair1 {  // pass 1 operands: key block rows (K, V), query block rows (Q, dO) and columns
  RawRow k, v, q, d;
  unsigned qc[2][4], dc[2][4];
};
struct Pair2 {  // pass 2 operands: query block rows (Q, dO), key block rows (K, V) and K columns
  RawRow q, d, k, v;
  unsigned kc[2][4];
};

__global__ __launch_bounds__(256) void mha_bwd_x3p_k(BwdArgs a) {
  constexpr int DH = 32;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int64_t unit = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= (int64_t)a.B * a.H) return;  // whole wave exits together
  const int b = (int)(unit / a.H), hd = (int)(unit % a.H);
  const int D = a.H * DH;
  const int ld = 3 * D;
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;
  if (L <= 0) return;
  const int nb = __builtin_amdgcn_readfirstlane((L + 15) >> 4);
  const auto rq = seq_rsrc(a.qkv + tok0 * ld, (unsigned)(L * ld * 4));
  const auto rd = seq_rsrc(a.dout + tok0 * D, (unsigned)(L * D * 4));
  const float sc = a.scale;
  const int cq = hd * DH, ck = D + hd * DH, cv = 2 * D + hd * DH;  // column offsets in a qkv row

  // per-token softmax statistics (token t < L on lane t): lse_t, delta_t = dO_t . O_t, key pad
  float my_lse = -INFINITY, my_delta = 0.0f;
  int my_pad = 1;
  if (lane < L) {
    my_lse = a.lse[(tok0 + lane) * a.H + hd];
    const float4* op = reinterpret_cast<const float4*>(a.out + (tok0 + lane) * D + hd * DH);
    const float4* gp = reinterpret_cast<const float4*>(a.dout + (tok0 + lane) * D + hd * DH);
    float d = 0.0f;
#pragma unroll
    for (int t = 0; t < DH / 4; ++t) {
      const float4 x = op[t], y = gp[t];
      d += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    my_delta = d;
    my_pad = a.kpad ? (int)a.kpad[tok0 + lane] : 0;
  }
  auto grad_elem = [&](int i, int j, float s, float dp, float lse_i, float delta_i, bool allowed, float& pd_out) {
    pd_out = 0.0f;
    if (!allowed) return 0.0f;
    const float p = __expf(s * sc - lse_i);
    float pd = p, dpd = dp;
    if (a.drop.active()) {
      const uint64_t idx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax + j;
      const bool keep = rsx::hash_u32(a.drop.seed, idx) >= a.drop.thresh;
      pd = keep ? p * a.drop.scale : 0.0f;
      dpd = keep ? dp * a.drop.scale : 0.0f;
    }
    pd_out = pd;
    return p * (dpd - delta_i) * sc;
  };

  // ---- pass 1: pairs (kb, qb >= kb) in kb-major order; key j = 16kb + c on the score columns ----
  {
    auto load1 = [&](Pair1& P, int kb, int qb) {
      const int j = 16 * kb + c, iq = 16 * qb + c;
      P.k = load_rawrow(rq, (unsigned)((j * ld + ck + 8 * g) * 4));
      P.v = load_rawrow(rq, (unsigned)((j * ld + cv + 8 * g) * 4));
      P.q = load_rawrow(rq, (unsigned)((iq * ld + cq + 8 * g) * 4));
      P.d = load_rawrow(rd, (unsigned)((iq * D + hd * DH + 8 * g) * 4));
      load_rawcols(rq, 16 * qb + 4 * g, ld, cq + c, P.qc);
      load_rawcols(rd, 16 * qb + 4 * g, D, hd * DH + c, P.dc);
    };
    f32x4 dk[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    f32x4 dv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    int kb = 0, qb = 0;
    // one pair: prefetch the next one into `fill`, compute this one from `use`; false when done
    auto step = [&](const Pair1& use, Pair1& fill) -> bool {
      int nkb = kb, nqb = qb + 1;
      if (nqb >= nb) { nkb = kb + 1; nqb = a.causal ? nkb : 0; }
      load1(fill, nkb, nqb);
      const int j = 16 * kb + c;
      const bool jok = j < L;
      const int jpad = __shfl(my_pad, j & 63, 64);
      const f32x4 S = dot16_x3(split_row8(use.q.x0, use.q.x1), split_row8(use.k.x0, use.k.x1));
      const f32x4 dP = dot16_x3(split_row8(use.d.x0, use.d.x1), split_row8(use.v.x0, use.v.x1));
      float ds[4], pd[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * qb + 4 * g + r;
        const float lse_i = __shfl(my_lse, i & 63, 64);
        const float del_i = __shfl(my_delta, i & 63, 64);
        const bool allowed = jok && i < L && !jpad && (!a.causal || j <= i) && lse_i != -INFINITY;
        ds[r] = grad_elem(i, j, S[r], dP[r], lse_i, del_i, allowed, pd[r]);
      }
      const Col4 pa = split4(pd), sa = split4(ds);
#pragma unroll
      for (int et = 0; et < 2; ++et) {
        dv[et] = sum16_x3(pa, split_col4(use.dc[et]), dv[et]);  // dV[j][e]
        dk[et] = sum16_x3(sa, split_col4(use.qc[et]), dk[et]);  // dK[j][e]
      }
      if (nkb != kb) {
        float* dKb = a.dqkv + tok0 * ld + ck;
        float* dVb = a.dqkv + tok0 * ld + cv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * kb + 4 * g + r;
          if (row < L) {
#pragma unroll
            for (int et = 0; et < 2; ++et) {
              dKb[(int64_t)row * ld + 16 * et + c] = dk[et][r];
              dVb[(int64_t)row * ld + 16 * et + c] = dv[et][r];
            }
          }
        }
#pragma unroll
        for (int et = 0; et < 2; ++et) dk[et] = dv[et] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      kb = nkb;
      qb = nqb;
      return kb < nb;
    };
    Pair1 p0, p1;
    load1(p0, 0, 0);
    for (;;) {
      if (!step(p0, p1)) break;
      if (!step(p1, p0)) break;
    }
  }

  // ---- pass 2: pairs (qb, kb <= qb) in qb-major order; query i = 16qb + c on the score columns ----
  {
    auto load2 = [&](Pair2& P, int qb, int kb) {
      const int i = 16 * qb + c, jr = 16 * kb + c;
      P.q = load_rawrow(rq, (unsigned)((i * ld + cq + 8 * g) * 4));
      P.d = load_rawrow(rd, (unsigned)((i * D + hd * DH + 8 * g) * 4));
      P.k = load_rawrow(rq, (unsigned)((jr * ld + ck + 8 * g) * 4));
      P.v = load_rawrow(rq, (unsigned)((jr * ld + cv + 8 * g) * 4));
      load_rawcols(rq, 16 * kb + 4 * g, ld, ck + c, P.kc);
    };
    f32x4 dq[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    int qb = 0, kb = 0;
    auto step = [&](const Pair2& use, Pair2& fill) -> bool {
      int nqb = qb, nkb = kb + 1;
      if (nkb > (a.causal ? qb : nb - 1)) { nqb = qb + 1; nkb = 0; }
      load2(fill, nqb, nkb);
      const int i = 16 * qb + c;
      const bool iok = i < L;
      const float lse_i = __shfl(my_lse, i & 63, 64);
      const float del_i = __shfl(my_delta, i & 63, 64);
      const f32x4 St = dot16_x3(split_row8(use.k.x0, use.k.x1), split_row8(use.q.x0, use.q.x1));
      const f32x4 dPt = dot16_x3(split_row8(use.v.x0, use.v.x1), split_row8(use.d.x0, use.d.x1));
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * kb + 4 * g + r;
        const int jpad = __shfl(my_pad, j & 63, 64);
        const bool allowed = iok && j < L && !jpad && (!a.causal || j <= i) && lse_i != -INFINITY;
        float pd;
        ds[r] = grad_elem(i, j, St[r], dPt[r], lse_i, del_i, allowed, pd);
      }
      const Col4 sa = split4(ds);
#pragma unroll
      for (int et = 0; et < 2; ++et) dq[et] = sum16_x3(sa, split_col4(use.kc[et]), dq[et]);  // dQ[i][e]
      if (nqb != qb) {
        float* dQb = a.dqkv + tok0 * ld + cq;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * qb + 4 * g + r;
          if (row < L) {
            dQb[(int64_t)row * ld + c] = dq[0][r];
            dQb[(int64_t)row * ld + 16 + c] = dq[1][r];
          }
        }
        dq[0] = dq[1] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      qb = nqb;
      kb = nkb;
      return qb < nb;
    };
    Pair2 p0, p1;
    load2(p0, 0, 0);
    for (;;) {
      if (!step(p0, p1)) break;
      if (!step(p1, p0)) break;
    }
  }
}


// ---- bf16x3 backward, causal, one dS evaluation per pair ---------------------------------------
// mha_bwd_x3p_k's pass 1 (key block on the lanes: S, dP, the softmax gradient dS and the dropped-out
// P, then dK and dV) also writes each pair's dS tile to LDS (1.25 KB per pair, <= 10 causal pairs
// per (sequence, head) at L <= 64: 51 KB per 4-wave workgroup, three workgroups per CU as the
// registers allow). Pass 2 then reads the tiles transposed and forms dQ = dS K with K's columns as
// its only loads, instead of recomputing S and dP (6 MFMAs), the exp / dropout hash of 16
// elements and four row splits per pair.
constexpr int kStashLd = 20;     // tile row stride (floats): conflict-free writes, aligned b128 reads
constexpr int kStashPairs = 10;  // causal pairs kb <= qb < 4
__device__ __forceinline__ int stash_slot(int kb, int qb) { return (qb * (qb + 1) >> 1) + kb; }

// Measured and not kept (round 6): a second instance for sequences of <= 32 tokens with a 3-pair stash
// (15 KB of LDS) at four waves per SIMD: 128 VGPRs with 49 spilled, 319 + 245 us against 367 us for this
// kernel alone on the headline tower's first layer.
__global__ __launch_bounds__(256) void mha_bwd_x3s_k(BwdArgs a) {
  // dS tiles of this wave's (kb, qb <= ... ) pairs, [16 query rows][16 key columns] at row stride 20
  __shared__ __attribute__((aligned(16))) float sDS[4][kStashPairs][16 * kStashLd];
  constexpr int DH = 32;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t unit = (int64_t)blockIdx.x * 4 + wave;
  if (unit >= (int64_t)a.B * a.H) return;  // whole wave exits together
  const int b = (int)(unit / a.H), hd = (int)(unit % a.H);
  const int D = a.H * DH;
  const int ld = 3 * D;
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;
  if (L <= 0) return;
  const int nb = __builtin_amdgcn_readfirstlane((L + 15) >> 4);
  const auto rq = seq_rsrc(a.qkv + tok0 * ld, (unsigned)(L * ld * 4));
  const auto rd = seq_rsrc(a.dout + tok0 * D, (unsigned)(L * D * 4));
  const float sc = a.scale;
  const int cq = hd * DH, ck = D + hd * DH, cv = 2 * D + hd * DH;  // column offsets in a qkv row

  // per-token softmax statistics (token t < L on lane t): lse_t, delta_t = dO_t . O_t, key pad
  float my_lse = -INFINITY, my_delta = 0.0f;
  int my_pad = 1;
  if (lane < L) {
    my_lse = a.lse[(tok0 + lane) * a.H + hd];
    const float4* op = reinterpret_cast<const float4*>(a.out + (tok0 + lane) * D + hd * DH);
    const float4* gp = reinterpret_cast<const float4*>(a.dout + (tok0 + lane) * D + hd * DH);
    float d = 0.0f;
#pragma unroll
    for (int t = 0; t < DH / 4; ++t) {
      const float4 x = op[t], y = gp[t];
      d += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    my_delta = d;
    my_pad = a.kpad ? (int)a.kpad[tok0 + lane] : 0;
  }
  auto grad_elem = [&](int i, int j, float s, float dp, float lse_i, float delta_i, bool allowed, float& pd_out) {
    pd_out = 0.0f;
    if (!allowed) return 0.0f;
    const float p = __expf(s * sc - lse_i);
    float pd = p, dpd = dp;
    if (a.drop.active()) {
      const uint64_t idx = ((uint64_t)(tok0 + i) * a.H + hd) * kLMax + j;
      const bool keep = rsx::hash_u32(a.drop.seed, idx) >= a.drop.thresh;
      pd = keep ? p * a.drop.scale : 0.0f;
      dpd = keep ? dp * a.drop.scale : 0.0f;
    }
    pd_out = pd;
    return p * (dpd - delta_i) * sc;
  };

  // ---- pass 1: pairs (kb, qb >= kb) in kb-major order; key j = 16kb + c on the score columns ----
  {
    auto load1 = [&](Pair1& P, int kb, int qb) {
      const int j = 16 * kb + c, iq = 16 * qb + c;
      P.k = load_rawrow(rq, (unsigned)((j * ld + ck + 8 * g) * 4));
      P.v = load_rawrow(rq, (unsigned)((j * ld + cv + 8 * g) * 4));
      P.q = load_rawrow(rq, (unsigned)((iq * ld + cq + 8 * g) * 4));
      P.d = load_rawrow(rd, (unsigned)((iq * D + hd * DH + 8 * g) * 4));
      load_rawcols(rq, 16 * qb + 4 * g, ld, cq + c, P.qc);
      load_rawcols(rd, 16 * qb + 4 * g, D, hd * DH + c, P.dc);
    };
    f32x4 dk[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    f32x4 dv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    int kb = 0, qb = 0;
    // one pair: prefetch the next one into `fill`, compute this one from `use`; false when done
    auto step = [&](const Pair1& use, Pair1& fill) -> bool {
      int nkb = kb, nqb = qb + 1;
      if (nqb >= nb) { nkb = kb + 1; nqb = a.causal ? nkb : 0; }
      load1(fill, nkb, nqb);
      const int j = 16 * kb + c;
      const bool jok = j < L;
      const int jpad = __shfl(my_pad, j & 63, 64);
      const f32x4 S = dot16_x3(split_row8(use.q.x0, use.q.x1), split_row8(use.k.x0, use.k.x1));
      const f32x4 dP = dot16_x3(split_row8(use.d.x0, use.d.x1), split_row8(use.v.x0, use.v.x1));
      float ds[4], pd[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * qb + 4 * g + r;
        const float lse_i = __shfl(my_lse, i & 63, 64);
        const float del_i = __shfl(my_delta, i & 63, 64);
        const bool allowed = jok && i < L && !jpad && (!a.causal || j <= i) && lse_i != -INFINITY;
        ds[r] = grad_elem(i, j, S[r], dP[r], lse_i, del_i, allowed, pd[r]);
      }
      {  // dS[16qb + 4g + r][16kb + c] -> tile row 4g + r, column c (read transposed in pass 2)
        float* t = sDS[wave][stash_slot(kb, qb)];
#pragma unroll
        for (int r = 0; r < 4; ++r) t[(4 * g + r) * kStashLd + c] = ds[r];
      }
      const Col4 pa = split4(pd), sa = split4(ds);
#pragma unroll
      for (int et = 0; et < 2; ++et) {
        dv[et] = sum16_x3(pa, split_col4(use.dc[et]), dv[et]);  // dV[j][e]
        dk[et] = sum16_x3(sa, split_col4(use.qc[et]), dk[et]);  // dK[j][e]
      }
      if (nkb != kb) {
        float* dKb = a.dqkv + tok0 * ld + ck;
        float* dVb = a.dqkv + tok0 * ld + cv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * kb + 4 * g + r;
          if (row < L) {
#pragma unroll
            for (int et = 0; et < 2; ++et) {
              dKb[(int64_t)row * ld + 16 * et + c] = dk[et][r];
              dVb[(int64_t)row * ld + 16 * et + c] = dv[et][r];
            }
          }
        }
#pragma unroll
        for (int et = 0; et < 2; ++et) dk[et] = dv[et] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      kb = nkb;
      qb = nqb;
      return kb < nb;
    };
    Pair1 p0, p1;
    load1(p0, 0, 0);
    for (;;) {
      if (!step(p0, p1)) break;
      if (!step(p1, p0)) break;
    }
  }

  // pass 2 reads dS entries other lanes of this wave wrote in pass 1: order the wave's LDS
  // writes before those reads explicitly (the per-wave stash is never touched by other waves)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // ---- pass 2: dQ[i] = sum_j dS[i][j] K[j] from the stashed tiles (qb-major, kb <= qb): the
  // tile is read transposed (lane (c, g): query 16qb + c, keys 16kb + 4g + 0..3 = the A operand),
  // K's columns are the only loads; S, dP and the softmax gradient are not recomputed ----
  {
    f32x4 dq[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    int qb = 0, kb = 0;
    auto step = [&](const unsigned (&use)[2][4], unsigned (&fill)[2][4]) -> bool {
      int nqb = qb, nkb = kb + 1;
      if (nkb > qb) { nqb = qb + 1; nkb = 0; }
      load_rawcols(rq, 16 * nkb + 4 * g, ld, ck + c, fill);
      const float4 t = *reinterpret_cast<const float4*>(&sDS[wave][stash_slot(kb, qb)][c * kStashLd + 4 * g]);
      const float ds[4] = {t.x, t.y, t.z, t.w};
      const Col4 sa = split4(ds);
#pragma unroll
      for (int et = 0; et < 2; ++et) dq[et] = sum16_x3(sa, split_col4(use[et]), dq[et]);  // dQ[i][e]
      if (nqb != qb) {
        float* dQb = a.dqkv + tok0 * ld + cq;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * qb + 4 * g + r;
          if (row < L) {
            dQb[(int64_t)row * ld + c] = dq[0][r];
            dQb[(int64_t)row * ld + 16 + c] = dq[1][r];
          }
        }
        dq[0] = dq[1] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      qb = nqb;
      kb = nkb;
      return qb < nb;
    };
    unsigned k0[2][4], k1[2][4];
    load_rawcols(rq, 4 * g, ld, ck + c, k0);
    for (;;) {
      if (!step(k0, k1)) break;
      if (!step(k1, k0)) break;
    }
  }
}



// ---- fused in-projection + attention forward (head dim 32, bf16x3) -------------------------
// The user tower's `qkv = in_proj(h); mha(qkv)` (v1_refine_usertower.py:343-352 through
// nn.TransformerEncoderLayer's self_attn) as ONE kernel: each wave (sequence, head) computes its
// head's Q, K and V for all of the sequence's 16-token blocks from the LayerNorm output h and
// in_proj_weight / in_proj_bias, then runs mha_fwd_x3b_seq's masked safe-softmax attention on them
// straight from registers (no qkv round trip through HBM before the attention). The projections
// are bf16x3 16x16x32 MFMAs (K = D in 32-wide k-steps) whose outputs land in exactly the attention's
// operand layouts:
//   Q^T, K^T tiles  A = W rows (dim), B = h rows (token): lane (c, g) register r holds dim
//                   16 dt + 4g + r of token c — the Row8 operand of the score MFMA with the head
//                   dims permuted ({4g..4g+3} U {16+4g..16+4g+3} on lane group g, the same
//                   permutation for Q and K, so S is unchanged);
//   V tiles         A = h rows, B = W rows: lane (c, g) register r holds token 4g + r, dim c —
//                   the Col4 operand of P V.
// qkv is still written (the attention backward, mha_bwd_x3p_k, and the in_proj weight gradient
// read it), with float4 stores for Q / K; the saving is the attention's qkv read and one launch.
struct QArgs {
  const float* x;        // [T, D] in_proj input
  const float* w;        // [3D, D] in_proj_weight
  const float* bias;     // [3D] or nullptr
  const uint8_t* kpad;
  const int* seg;
  float* qkv;            // [T, 3D] (for the backward) or nullptr
  float* out;            // [T, D]
  float* lse;            // [T, H] or nullptr
  int B, L, H, causal;
  float scale;
  rsx::Dropout drop;
};

__device__ __forceinline__ f32x4 dot16_x3_acc(const Row8& a, const Row8& b, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ Row8 split_f8(const float (&f)[8]) {
  Row8 r;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const __bf16 h = (__bf16)f[k];
    r.hi[k] = h;
    r.lo[k] = (__bf16)(f[k] - (float)h);
  }
  return r;
}

template <int NB, int KS>
__device__ __forceinline__ void mha_qkv_fwd_x3_seq(const QArgs& a, int hd, int64_t tok0, int L, int lane) {
  constexpr int DH = 32, D = 32 * KS;
  const int c = lane & 15, g = lane >> 4;
  const int H = a.H;
  // h rows of the sequence through one buffer resource (rows >= L read as zero)
  const uintptr_t bp = (uintptr_t)(a.x + tok0 * D);
  const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)bp), bhi = __builtin_amdgcn_readfirstlane((unsigned)(bp >> 32));
  const unsigned nbytes = __builtin_amdgcn_readfirstlane((unsigned)(L * D * 4));
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(((uintptr_t)bhi << 32) | blo), 0, (int)nbytes, 0x00020000);
  u32x4b xr[KS][NB][2];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
      const unsigned o = (unsigned)(((16 * bb + c) * D + 32 * s + 8 * g) * 4);
      xr[s][bb][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
      xr[s][bb][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16, 0, 0);
    }
  // projections: q/k/v accumulators of block bb, 16-dim tile dt
  f32x4 qa[NB][2], ka[NB][2], va[NB][2];
#pragma unroll
  for (int bb = 0; bb < NB; ++bb)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      qa[bb][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
      ka[bb][dt] = qa[bb][dt];
      va[bb][dt] = qa[bb][dt];
    }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    Row8 wf[3][2];  // [q|k|v][dt]: row 16 dt + c of the head's part, k-step s
#pragma unroll
    for (int pt = 0; pt < 3; ++pt)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const float4* p = reinterpret_cast<const float4*>(a.w + (int64_t)(pt * D + hd * DH + 16 * dt + c) * D + 32 * s + 8 * g);
        const float4 v0 = p[0], v1 = p[1];
        const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        wf[pt][dt] = split_f8(f);
      }
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
      const Row8 xx = split_row8(xr[s][bb][0], xr[s][bb][1]);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        qa[bb][dt] = dot16_x3_acc(wf[0][dt], xx, qa[bb][dt]);  // [dim 4g+r][token c]
        ka[bb][dt] = dot16_x3_acc(wf[1][dt], xx, ka[bb][dt]);
        va[bb][dt] = dot16_x3_acc(xx, wf[2][dt], va[bb][dt]);  // [token 4g+r][dim c]
      }
    }
  }
  // + bias; Q / K / V values of the attention operands; qkv for the backward
  float bq[2][4], bk[2][4], bv[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bq[dt][r] = a.bias ? a.bias[hd * DH + 16 * dt + 4 * g + r] : 0.0f;
      bk[dt][r] = a.bias ? a.bias[D + hd * DH + 16 * dt + 4 * g + r] : 0.0f;
    }
    bv[dt] = a.bias ? a.bias[2 * D + hd * DH + 16 * dt + c] : 0.0f;
  }
  Row8 kx[NB], qxs[NB];
  Col4 vc[NB][2];
#pragma unroll
  for (int bb = 0; bb < NB; ++bb) {
    float qf[8], kf[8];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        qf[4 * dt + r] = qa[bb][dt][r] + bq[dt][r];
        kf[4 * dt + r] = ka[bb][dt][r] + bk[dt][r];
      }
    qxs[bb] = split_f8(qf);
    kx[bb] = split_f8(kf);
    float vf[2][4];
#pragma unroll
    for (int et = 0; et < 2; ++et)
#pragma unroll
      for (int t = 0; t < 4; ++t) vf[et][t] = va[bb][et][t] + bv[et];
    vc[bb][0] = split4(vf[0]);
    vc[bb][1] = split4(vf[1]);
    if (a.qkv) {
      const int64_t D3 = 3 * (int64_t)D;
      const int tq = 16 * bb + c;
      if (tq < L) {
        float* qrow = a.qkv + (tok0 + tq) * D3 + hd * DH + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          *reinterpret_cast<float4*>(qrow + 16 * dt) = make_float4(qf[4 * dt], qf[4 * dt + 1], qf[4 * dt + 2], qf[4 * dt + 3]);
          *reinterpret_cast<float4*>(qrow + D + 16 * dt) =
              make_float4(kf[4 * dt], kf[4 * dt + 1], kf[4 * dt + 2], kf[4 * dt + 3]);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int tv = 16 * bb + 4 * g + t;
        if (tv < L) {
#pragma unroll
          for (int et = 0; et < 2; ++et) a.qkv[(tok0 + tv) * D3 + 2 * D + hd * DH + 16 * et + c] = vf[et][t];
        }
      }
    }
  }
  // ---- attention (mha_fwd_x3b_seq's masks, safe softmax, dropout hash, lse)
  const int my_pad = (lane < L) ? (a.kpad ? (int)a.kpad[tok0 + lane] : 0) : 1;
  float* Ob = a.out + tok0 * D + hd * DH;
#pragma unroll
  for (int qb = 0; qb < NB; ++qb) {
    const int i = 16 * qb + c;
    const bool iok = i < L;
    const int kb_end = a.causal ? qb : NB - 1;
    f32x4 sv[NB];
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb <= kb_end) {
        sv[kb] = dot16_x3(kx[kb], qxs[qb]);  // S^T: [key 16kb+4g+r][query i]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 16 * kb + 4 * g + r;
          const int jpad = __shfl(my_pad, j & 63, 64);
          const bool allowed = iok && j < L && !jpad && (!a.causal || j <= i);
          sv[kb][r] = allowed ? sv[kb][r] * a.scale : -INFINITY;
          m = fmaxf(m, sv[kb][r]);
        }
      }
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.0f;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb <= kb_end) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = (sv[kb][r] == -INFINITY) ? 0.0f : __expf(sv[kb][r] - m);
          sv[kb][r] = pv;
          l += pv;
        }
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = (l > 0.0f) ? 1.0f / l : 0.0f;
    f32x4 o[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const uint64_t rowidx = ((uint64_t)(tok0 + i) * H + hd) * kLMax;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb <= kb_end) {
        float pr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) pr[r] = a.drop.apply(sv[kb][r] * inv, rowidx + 16 * kb + 4 * g + r);
        const Col4 pa = split4(pr);
#pragma unroll
        for (int et = 0; et < 2; ++et) o[et] = sum16_x3(pa, vc[kb][et], o[et]);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * qb + 4 * g + r;
      if (row < L) {
        Ob[(int64_t)row * D + c] = o[0][r];
        Ob[(int64_t)row * D + 16 + c] = o[1][r];
      }
    }
    if (a.lse && g == 0 && iok) a.lse[(tok0 + i) * H + hd] = (l > 0.0f) ? m + logf(l) : -INFINITY;
  }
}

template <int KS>
__global__ __launch_bounds__(256) void mha_qkv_fwd_x3_k(QArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= (int64_t)a.B * a.H) return;  // whole wave exits together
  const int b = (int)(unit / a.H), hd = (int)(unit % a.H);
  const int64_t tok0 = a.seg ? (int64_t)a.seg[b] : (int64_t)b * a.L;
  int L = a.seg ? (a.seg[b + 1] - a.seg[b]) : a.L;
  if (L > kLMax) L = kLMax;
  if (L <= 0) return;
  const int nb = __builtin_amdgcn_readfirstlane((L + 15) >> 4);
  if (nb == 1) mha_qkv_fwd_x3_seq<1, KS>(a, hd, tok0, L, lane);
  else if (nb == 2) mha_qkv_fwd_x3_seq<2, KS>(a, hd, tok0, L, lane);
  else if (nb == 3) mha_qkv_fwd_x3_seq<3, KS>(a, hd, tok0, L, lane);
  else mha_qkv_fwd_x3_seq<4, KS>(a, hd, tok0, L, lane);
}

}  // namespace

RSX_API int rsx_mha_fwd(const float* qkv, const uint8_t* key_pad, const int* seg_off, int64_t B, int64_t L,
                        int64_t H, int64_t Dh, int causal, float p_drop, uint64_t seed, float* out, float* lse,
                        void* stream) {
  RSX_ARG(qkv && out, "null tensor");
  RSX_ARG(L >= 1 && L <= kLMax, "L must be in [1,64]");
  RSX_ARG(Dh == 16 || Dh == 32 || Dh == 64, "head dim must be 16, 32 or 64");
  RSX_ARG(H >= 1, "H must be >= 1");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0,1)");
  if (B == 0) return 0;
  FwdArgs a;
  a.qkv = qkv; a.kpad = key_pad; a.seg = seg_off; a.out = out; a.lse = lse;
  a.B = (int)B; a.L = (int)L; a.H = (int)H; a.causal = causal;
  a.scale = 1.0f / sqrtf((float)Dh);
  a.drop = rsx::make_dropout(p_drop, seed);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(B * H));
  if (Dh == 16) hipLaunchKernelGGL(mha_fwd_k<16>, grid, dim3(64), 0, st, a);
  else if (Dh == 32) hipLaunchKernelGGL(mha_fwd_k<32>, grid, dim3(64), 0, st, a);
  else hipLaunchKernelGGL(mha_fwd_k<64>, grid, dim3(64), 0, st, a);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_mha_bwd(const float* qkv, const uint8_t* key_pad, const int* seg_off, const float* out,
                        const float* lse, const float* dout, int64_t B, int64_t L, int64_t H, int64_t Dh, int causal,
                        float p_drop, uint64_t seed, float* dqkv, void* stream) {
  RSX_ARG(qkv && out && lse && dout && dqkv, "null tensor");
  RSX_ARG(L >= 1 && L <= kLMax, "L must be in [1,64]");
  RSX_ARG(Dh == 16 || Dh == 32 || Dh == 64, "backward head dim must be 16, 32 or 64");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0,1)");
  if (B == 0) return 0;
  BwdArgs a;
  a.qkv = qkv; a.kpad = key_pad; a.seg = seg_off; a.out = out; a.lse = lse; a.dout = dout; a.dqkv = dqkv;
  a.B = (int)B; a.L = (int)L; a.H = (int)H; a.causal = causal;
  a.scale = 1.0f / sqrtf((float)Dh);
  a.drop = rsx::make_dropout(p_drop, seed);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(B * H));
  if (Dh == 16) hipLaunchKernelGGL(mha_bwd_k<16>, grid, dim3(64), 0, st, a);
  else if (Dh == 64 && L <= 32) hipLaunchKernelGGL(mha_bwd64_k<32>, grid, dim3(64), 0, st, a);  // L: the longest sequence
  else if (Dh == 64) hipLaunchKernelGGL(mha_bwd64_k<64>, grid, dim3(64), 0, st, a);
  else hipLaunchKernelGGL(mha_bwd_mfma_k, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, st, a);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_mha_fwd_x3(const float* qkv, const uint8_t* key_pad, const int* seg_off, int64_t B, int64_t L,
                           int64_t H, int64_t Dh, int causal, float p_drop, uint64_t seed, float* out, float* lse,
                           void* stream) {
  RSX_ARG(qkv && out, "null tensor");
  RSX_ARG(L >= 1 && L <= kLMax, "L must be in [1,64]");
  RSX_ARG(Dh == 32 || Dh == 64, "bf16x3 attention forward head dim must be 32 or 64");
  RSX_ARG(H >= 1, "H must be >= 1");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0,1)");
  if (B == 0) return 0;
  FwdArgs a;
  a.qkv = qkv; a.kpad = key_pad; a.seg = seg_off; a.out = out; a.lse = lse;
  a.B = (int)B; a.L = (int)L; a.H = (int)H; a.causal = causal;
  a.scale = 1.0f / sqrtf((float)Dh);
  a.drop = rsx::make_dropout(p_drop, seed);
  static const bool legacy = getenv("RSX_MHA_FWD_LEGACY") != nullptr;  // A/B: the per-block-load kernel
  if (Dh == 64)
    hipLaunchKernelGGL(mha_fwd_x3b64_k, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a);
  else if (legacy)
    hipLaunchKernelGGL(mha_fwd_x3_k, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(mha_fwd_x3b_k, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a);
  RSX_LAUNCHED();
  return 0;
}

// Fused in_proj + attention forward (head dim 32, model width D = 32 H in {128}): see
// mha_qkv_fwd_x3_k. x [T, D], w [3D, D] (torch in_proj_weight), bias [3D] or null; qkv [T, 3D]
// written when non-null (what rsx_mha_bwd_x3 and the in_proj gradient read).
RSX_API int rsx_mha_qkv_fwd_x3(const float* x, const float* w, const float* bias, const uint8_t* key_pad,
                               const int* seg_off, int64_t B, int64_t L, int64_t H, int causal, float p_drop,
                               uint64_t seed, float* qkv, float* out, float* lse, void* stream) {
  RSX_ARG(x && w && out, "null tensor");
  RSX_ARG(L >= 1 && L <= kLMax, "L must be in [1,64]");
  RSX_ARG(H == 4, "fused in_proj + attention: D = 128 (4 heads of 32)");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0,1)");
  if (B == 0) return 0;
  QArgs a;
  a.x = x; a.w = w; a.bias = bias; a.kpad = key_pad; a.seg = seg_off; a.qkv = qkv; a.out = out; a.lse = lse;
  a.B = (int)B; a.L = (int)L; a.H = (int)H; a.causal = causal;
  a.scale = 1.0f / sqrtf(32.0f);
  a.drop = rsx::make_dropout(p_drop, seed);
  hipLaunchKernelGGL(mha_qkv_fwd_x3_k<4>, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a);
  RSX_LAUNCHED();
  return 0;
}

RSX_API int rsx_mha_bwd_x3(const float* qkv, const uint8_t* key_pad, const int* seg_off, const float* out,
                           const float* lse, const float* dout, int64_t B, int64_t L, int64_t H, int64_t Dh,
                           int causal, float p_drop, uint64_t seed, float* dqkv, void* stream) {
  RSX_ARG(qkv && out && lse && dout && dqkv, "null tensor");
  RSX_ARG(L >= 1 && L <= kLMax, "L must be in [1,64]");
  RSX_ARG(Dh == 32, "bf16x3 attention head dim must be 32");
  RSX_ARG(p_drop >= 0.0f && p_drop < 1.0f, "p_drop must be in [0,1)");
  if (B == 0) return 0;
  BwdArgs a;
  a.qkv = qkv; a.kpad = key_pad; a.seg = seg_off; a.out = out; a.lse = lse; a.dout = dout; a.dqkv = dqkv;
  a.B = (int)B; a.L = (int)L; a.H = (int)H; a.causal = causal;
  a.scale = 1.0f / sqrtf((float)Dh);
  a.drop = rsx::make_dropout(p_drop, seed);
  static const bool legacy = getenv("RSX_MHA_BWD_LEGACY") != nullptr;  // A/B: one latency per pair
  static const bool stash = getenv("RSX_MHA_BWD_STASH") == nullptr || getenv("RSX_MHA_BWD_STASH")[0] != '0';
  if (legacy)
    hipLaunchKernelGGL(mha_bwd_x3_k, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a);
  else if (causal && stash)
    hipLaunchKernelGGL(mha_bwd_x3s_k, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(mha_bwd_x3p_k, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a);
  RSX_LAUNCHED();
  return 0;
}
