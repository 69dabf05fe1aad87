// The two ends of the generic-width CLIP encoder (models/gemm_encoder.py: n_embd
// other than the fused kernels' 128, e.g. the reference CLI's default
// clip_{t,i}model_deb = 64, utils/config.py:58-59), whose layers run on the
// split-bf16 GEMM (ghm_gemm.hip), the row LayerNorms (ghm_vlm.hip) and the
// split-bf16 attention (ghm_vlm_x3.hip, D = 64 / 128 / 256):
//
//   embedding  H0[n, t, :] = tok_w[x[n, t]] + pos_w[t]        (models/model.py:764-765)
//   readout    emb[n, c]   = b_out + sum_t w_out[t] Z[n, t, c],
//              Z = H_L W_ro^T + b_ro (ghm_rows_linear)          (model.py:802-805)
//   and the readout's backward through the token-axis Linear(n_token -> 1):
//              dZ[n, t, c] = w_out[t] d_emb[n, c],
//              d_w_out[t]  = sum_{n, c} d_emb[n, c] Z[n, t, c],  d_b_out = sum d_emb
// Every sum runs in a fixed order (one thread or one workgroup tree per output):
// replays are bit-identical.
#include "ghm_launch.h"

namespace {

__global__ __launch_bounds__(256) void k_tok_embed_fwd(const uint8_t* __restrict__ tok, const float* __restrict__ tok_w,
                                                       const float* __restrict__ pos_w, float* __restrict__ H0,
                                                       int64_t n_tok, int T, int V, int D) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int D4 = D / 4;
  if (idx >= n_tok * D4) return;
  const int q = static_cast<int>(idx % D4);
  const int64_t m = idx / D4;
  const int t = static_cast<int>(m % T);
  int x = tok[m];
  x = x < V ? x : V - 1;  // (the module checks the range; the trainer's tokens come from the sampler)
  const float4 w = *reinterpret_cast<const float4*>(tok_w + static_cast<int64_t>(x) * D + 4 * q);
  const float4 p = *reinterpret_cast<const float4*>(pos_w + static_cast<int64_t>(t) * D + 4 * q);
  *reinterpret_cast<float4*>(H0 + m * D + 4 * q) = make_float4(w.x + p.x, w.y + p.y, w.z + p.z, w.w + p.w);
}

// one thread per (n, c): the token sum in t order
__global__ __launch_bounds__(256) void k_tok_readout_fwd(const float* __restrict__ Z, const float* __restrict__ w_out,
                                                         const float* __restrict__ b_out, float* __restrict__ emb,
                                                         int64_t n_seq, int T, int C) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (idx >= n_seq * C) return;
  const int64_t n = idx / C;
  const int c = static_cast<int>(idx % C);
  const float* z = Z + n * T * C + c;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s = __builtin_fmaf(w_out[t], z[static_cast<int64_t>(t) * C], s);
  emb[idx] = s + b_out[0];
}

// fixed-order workgroup sum of 256 per-thread partials
__device__ __forceinline__ float block_sum256(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  return red[0];
}

// workgroups 0 .. T-1: d_w_out[t]; workgroup T: d_b_out; the rest: dZ elementwise
__global__ __launch_bounds__(256) void k_tok_readout_bwd(const float* __restrict__ Z, const float* __restrict__ d_emb,
                                                         const float* __restrict__ w_out, float* __restrict__ dZ,
                                                         float* __restrict__ d_wout, float* __restrict__ d_bout,
                                                         int64_t n_seq, int T, int C) {
  __shared__ float red[256];
  const int64_t nc = n_seq * C;
  const int b = static_cast<int>(blockIdx.x);
  if (b <= T) {
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < nc; i += 256) {
      const int64_t n = i / C;
      const int c = static_cast<int>(i % C);
      s += b < T ? d_emb[i] * Z[(n * T + b) * C + c] : d_emb[i];
    }
    s = block_sum256(s, red);
    if (threadIdx.x == 0) {
      if (b < T) d_wout[b] = s;
      else d_bout[0] = s;
    }
    return;
  }
  const int64_t idx = static_cast<int64_t>(b - T - 1) * 256 + threadIdx.x;
  if (idx >= nc * T) return;
  const int64_t n = idx / (static_cast<int64_t>(T) * C);
  const int64_t r = idx % (static_cast<int64_t>(T) * C);
  const int t = static_cast<int>(r / C), c = static_cast<int>(r % C);
  dZ[idx] = w_out[t] * d_emb[n * C + c];
}

}  // namespace

extern "C" int ghm_tok_embed_fwd(const uint8_t* tokens, const float* tok_w, const float* pos_w, float* H0,
                                 int64_t n_seq, int T, int V, int D, void* stream) {
  GHM_CHECK(tokens && tok_w && pos_w && H0, "null pointer");
  GHM_CHECK(n_seq >= 1 && T >= 1 && V >= 1 && V <= 256 && D >= 4 && D % 4 == 0, "shape");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(tok_w) | reinterpret_cast<uintptr_t>(pos_w) |
              reinterpret_cast<uintptr_t>(H0)) & 15) == 0, "16-byte aligned tables and H0");
  const int64_t n = n_seq * T * (D / 4);
  hipLaunchKernelGGL(k_tok_embed_fwd, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, ghm_stream(stream),
                     tokens, tok_w, pos_w, H0, n_seq * T, T, V, D);
  return ghm_launch_status();
}

extern "C" int ghm_tok_readout_fwd(const float* Z, const float* w_out, const float* b_out, float* emb, int64_t n_seq,
                                   int T, int C, void* stream) {
  GHM_CHECK(Z && w_out && b_out && emb, "null pointer");
  GHM_CHECK(n_seq >= 1 && T >= 1 && C >= 1, "shape");
  const int64_t n = n_seq * C;
  hipLaunchKernelGGL(k_tok_readout_fwd, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     ghm_stream(stream), Z, w_out, b_out, emb, n_seq, T, C);
  return ghm_launch_status();
}

extern "C" int ghm_tok_readout_bwd(const float* Z, const float* d_emb, const float* w_out, float* dZ, float* d_wout,
                                   float* d_bout, int64_t n_seq, int T, int C, void* stream) {
  GHM_CHECK(Z && d_emb && w_out && dZ && d_wout && d_bout, "null pointer");
  GHM_CHECK(n_seq >= 1 && T >= 1 && C >= 1 && n_seq * T * C < (int64_t(1) << 40), "shape");
  const int64_t nz = (n_seq * T * C + 255) / 256;
  hipLaunchKernelGGL(k_tok_readout_bwd, dim3(static_cast<unsigned>(T + 1 + nz)), dim3(256), 0, ghm_stream(stream), Z,
                     d_emb, w_out, dZ, d_wout, d_bout, n_seq, T, C);
  return ghm_launch_status();
}
