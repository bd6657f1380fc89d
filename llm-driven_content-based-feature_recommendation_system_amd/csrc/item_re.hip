// BERT input embeddings over a packed token list (the RE fields of the item tower):
//
//   out[t] = LayerNorm( (word[ids[t]] + type_row) + pos[tok_pos[t]] ) * w + b      (eps 1e-12)
//
// Reference: HybridItemTower.forward's RE path, item_tower.py:247-262:
//   word = self.bert_model.embeddings(input_ids=re_ids)   (no_grad; BertEmbeddings: word +
//   token_type(0) + absolute position, LayerNorm, dropout inactive in eval)
// followed by re_proj and a masked mean over each field's 32 tokens. Only the valid (mask = 1)
// tokens contribute to that mean, so the tower runs this on the packed valid tokens: the
// [B*9, 32, 768] activation (3.6 GB at B = 4096) and its GEMM shrink to the valid share.
// One wave per token: D/256 float4 per lane, two-pass row statistics in fp32.
#include "rsx_common.h"

namespace {

struct EArgs {
  const float* word;     // [V, ld_word]
  int64_t ld_word;
  const float* pos;      // [P, D]
  const float* type_row; // [D] (token type 0)
  const float* w;        // LayerNorm weight [D]
  const float* b;        // LayerNorm bias [D]
  const int64_t* ids;    // [T]
  const int64_t* tok_pos;  // [T]
  int64_t T;
  float eps;
  float* out;            // [T, D]
};

template <int V4>  // D = 256 * V4
__global__ __launch_bounds__(256) void embed3_ln_k(EArgs a) {
  constexpr int D = 256 * V4;
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t t = wave_g; t < a.T; t += nw) {
    const float4* wr = reinterpret_cast<const float4*>(a.word + a.ids[t] * a.ld_word);
    const float4* pr = reinterpret_cast<const float4*>(a.pos + a.tok_pos[t] * D);
    const float4* tr = reinterpret_cast<const float4*>(a.type_row);
    float4 x[V4];
    float s = 0.0f;
#pragma unroll
    for (int v = 0; v < V4; ++v) {
      const int c = v * 64 + lane;
      const float4 e = wr[c], ty = tr[c], p = pr[c];
      x[v] = make_float4((e.x + ty.x) + p.x, (e.y + ty.y) + p.y, (e.z + ty.z) + p.z, (e.w + ty.w) + p.w);
      s += (x[v].x + x[v].y) + (x[v].z + x[v].w);
    }
    const float mu = rsx::wave_sum_width(s, 64) * (1.0f / D);
    float q = 0.0f;
#pragma unroll
    for (int v = 0; v < V4; ++v) {
      x[v] = make_float4(x[v].x - mu, x[v].y - mu, x[v].z - mu, x[v].w - mu);
      q += x[v].x * x[v].x + x[v].y * x[v].y + x[v].z * x[v].z + x[v].w * x[v].w;
    }
    const float rs = 1.0f / sqrtf(rsx::wave_sum_width(q, 64) * (1.0f / D) + a.eps);
    float4* o = reinterpret_cast<float4*>(a.out + t * D);
#pragma unroll
    for (int v = 0; v < V4; ++v) {
      const int c = v * 64 + lane;
      const float4 g = reinterpret_cast<const float4*>(a.w)[c], bb = reinterpret_cast<const float4*>(a.b)[c];
      o[c] = make_float4(x[v].x * rs * g.x + bb.x, x[v].y * rs * g.y + bb.y, x[v].z * rs * g.z + bb.z,
                         x[v].w * rs * g.w + bb.w);
    }
  }
}

}  // namespace

RSX_API int rsx_embed3_ln(const float* word, int64_t ld_word, const float* pos, const float* type_row,
                          const float* ln_w, const float* ln_b, float eps, const int64_t* ids, const int64_t* tok_pos,
                          int64_t T, int64_t D, float* out, void* stream) {
  RSX_ARG(word && pos && type_row && ln_w && ln_b && ids && tok_pos && out, "null tensor");
  RSX_ARG(D % 256 == 0 && D >= 256 && D <= 1024, "D must be 256, 512, 768 or 1024");
  RSX_ARG(ld_word >= D && ld_word % 4 == 0, "bad ld_word");
  if (T == 0) return 0;
  EArgs a;
  a.word = word; a.ld_word = ld_word; a.pos = pos; a.type_row = type_row; a.w = ln_w; a.b = ln_b;
  a.ids = ids; a.tok_pos = tok_pos; a.T = T; a.eps = eps; a.out = out;
  int64_t blocks = (T + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  hipStream_t st = (hipStream_t)stream;
  switch (D / 256) {
    case 1: hipLaunchKernelGGL(embed3_ln_k<1>, dim3((unsigned)blocks), dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL(embed3_ln_k<2>, dim3((unsigned)blocks), dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL(embed3_ln_k<3>, dim3((unsigned)blocks), dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(embed3_ln_k<4>, dim3((unsigned)blocks), dim3(256), 0, st, a); break;
  }
  RSX_LAUNCHED();
  return 0;
}
