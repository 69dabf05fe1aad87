// Shared device helpers for the GHM CLIP kernels (gfx950 / CDNA4 only).
//
// Compute model:
//   * fp32 everywhere (the reference trains in fp32).  Matrix products use the
//     exact-f32 MFMA v_mfma_f32_32x32x2_f32: a k-ordered fmaf chain, no TF32.
//   * "tokens on lanes": a wave owns 32 tokens; lane l = (j = l&31, h = l>>5).
//     Activations enter MFMAs as the B operand (column j = token), weights as
//     the A operand (row i = output feature), so every output tile is Yᵀ with
//     the token on the lane and features in the 16 accumulator registers:
//         feature(r, h) = (r & 3) + 8 * (r >> 2) + 4 * h      (r = 0..15)
//     That accumulator is directly the B operand of the next product that sums
//     over those features (MLP up -> GELU -> down stays in registers).
//   * row layout: a token row of 128 features is held as x[s] = row[64h + s].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define GHM_D 128     // embedding width (n_embd); the kernels are built for 128
#define GHM_F 512     // MLP hidden width = 4 * n_embd
#define GHM_MAXT 96   // longest sequence (tokens) the attention kernels take

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Transition matrix of a GHM tree edge for the device BP kernels: layer `layer`
// (parent at depth layer, child at depth layer + 1), child = the child's index
// among the C^(layer+1) nodes of its depth (breadth first: parent * C + slot).
// per_edge 0: translation-invariant templates [L][C][V][V] (slot = child % C);
// per_edge 1: every edge's own matrix, layer by layer ([sum_l C^(l+1)][V][V],
// GenTransition(translation_invariance=False), data_random_GHM.py:43-89).
__device__ __forceinline__ const double* bp_edge(const double* tr, int layer, int child, int C, int V, int per_edge) {
  int64_t idx;
  if (per_edge) {
    int64_t off = 0, w = C;
    for (int k = 0; k < layer; ++k) {
      off += w;
      w *= C;
    }
    idx = off + child;
  } else {
    idx = static_cast<int64_t>(layer) * C + child % C;
  }
  return tr + idx * V * V;
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// feature / row index held in accumulator register r by lane half h
__device__ __forceinline__ constexpr int acc_row(int r, int h) {
  return (r & 3) + 8 * (r >> 2) + 4 * h;
}

// Accumulator registers 4q..4q+3 of a lane hold 4 consecutive features
// 8q + 4h + t: epilogue loads/stores use one float4 per quad.
__device__ __forceinline__ constexpr int quad_off(int q, int h) { return 8 * q + 4 * h; }

__device__ __forceinline__ void st4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}

// lane-pair (l, l^32) exchange on the VALU (v_permlane32_swap: the lower half
// of one copy trades places with the upper half of the other), not through the
// LDS crossbar (ds_bpermute)
__device__ __forceinline__ float xhalf(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((__lane_id() & 32) ? r[0] : r[1]);
}

// sum over the 32 lanes of one half (lanes j = 0..31 for fixed h)
__device__ __forceinline__ float sum32(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 1, 64);
  return v;
}

// load 64 consecutive floats (16 x float4) into x[0..63]
__device__ __forceinline__ void load64(const float* __restrict__ p, float* x) {
  const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float4 v = q[i];
    x[4 * i + 0] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
  }
}

// exact GELU, torch approximate='none': x * 0.5 * (1 + erf(x / sqrt(2)))
__device__ __forceinline__ float gelu_f(float x) {
  return x * 0.5f * (1.f + erff(x * 0.70710678118654752440f));
}
// attention activation (model.py:121-130 get_activation): the ACT template
// parameter of the attention kernels and the `act` argument of their *_act entry points
constexpr int ACT_SOFTMAX = 0, ACT_RELU = 1, ACT_GELU = 2;

// GELU and its derivative from one erf evaluation (same formulas as torch's
// forward and GeluBackward, approximate='none')
__device__ __forceinline__ void gelu_and_grad(float x, float& g, float& d) {
  const float e = erff(x * 0.70710678118654752440f);
  g = x * 0.5f * (1.f + e);
  const float cdf = 0.5f * (1.f + e);
  const float pdf = 0.39894228040143267794f * expf(-0.5f * x * x);
  d = cdf + x * pdf;
}
// torch GeluBackward (approximate='none'): dy * (cdf + x * pdf)
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// Reduce-scatter of 16 values over the 32 lanes of a half (j = lane & 31):
// lanes j and j^1 both return the 32-lane sum of element j >> 1.  Four
// halving butterfly levels plus one pairwise sum: 16 exchanges instead of
// 16 x 5.  Fixed exchange/sum order -> deterministic.
__device__ __forceinline__ float reduce_scatter16(float* v, int j) {
#pragma unroll
  for (int lvl = 0; lvl < 4; ++lvl) {
    const int half = 8 >> lvl;  // live values 16 >> lvl
    const int d = 16 >> lvl;
    const bool upper = (j & d) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float lo = v[i], hi = v[i + half];
      const float send = upper ? lo : hi;
      const float keep = upper ? hi : lo;
      v[i] = keep + __shfl_xor(send, d, 64);
    }
  }
  return v[0] + __shfl_xor(v[0], 1, 64);
}

// Row LayerNorm statistics for a token held in row layout by lane pair (j,h):
// two-pass mean / biased variance over 128 features.
__device__ __forceinline__ void ln_stats64(const float* x, float eps, float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 64; ++k) s += x[k];
  s += xhalf(s);
  mean = s * (1.f / 128.f);
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    const float d = x[k] - mean;
    v += d * d;
  }
  v += xhalf(v);
  rstd = 1.f / sqrtf(v * (1.f / 128.f) + eps);
}

// Register-staged global -> LDS copy of an R x C fp32 tile (row stride ld in
// global, pitch P floats in LDS) by a 256-thread workgroup, split so the global
// loads can be issued early (stage_load) and written to LDS after a barrier
// (stage_store).  v must be a local array of stage_n<R, C>() float4.
template <int R, int C>
__device__ __forceinline__ constexpr int stage_n() { return R * (C / 4) / 256; }

template <int R, int C>
__device__ __forceinline__ void stage_load(float4* v, const float* __restrict__ g, int ld) {
  constexpr int C4 = C / 4, N = R * C4 / 256;
  static_assert(R * C4 % 256 == 0, "tile must be a multiple of 256 float4");
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const int idx = threadIdx.x + 256 * k;
    v[k] = *reinterpret_cast<const float4*>(g + static_cast<size_t>(idx / C4) * ld + 4 * (idx % C4));
  }
}

template <int R, int C, int P>
__device__ __forceinline__ void stage_store(const float4* v, float* lds) {
  constexpr int C4 = C / 4, N = R * C4 / 256;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const int idx = threadIdx.x + 256 * k;
    *reinterpret_cast<float4*>(lds + (idx / C4) * P + 4 * (idx % C4)) = v[k];
  }
}

__device__ __forceinline__ float4 lds4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Per-token LayerNorm statistics (mean, rstd) written by a forward kernel and
// read by a backward one.  ld_stats_sys: a system-scope buffer load (sc0 sc1),
// served past the XCD's L2; ld_stats: agent scope (sc1, served by L2).  The
// round-2 plain load of this buffer in k_qkv_bwd_x3 returned wrong 128-B lines
// beside a k_wgrad_x3 workgroup; on the same probe the agent-scope load was
// wrong in 32 of 39 repetitions and the system-scope load in none of 3 x 39
// (tools/race_probe.py; DESIGN.md §4 "Determinism").  The backward kernels
// read the statistics with ld_stats_sys (8 bytes per token: free), and
// k_qkv_bwd_x3 recomputes them.  Byte offsets must fit 31 bits (host-checked).
__device__ __forceinline__ float2 ld_stats_sys(const float2* base, int64_t idx) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(base), static_cast<short>(0), 0x7fffffff,
                                                    0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, static_cast<int>(idx * 8), 0, 1 | 16);  // sc0 sc1
  return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
}
__device__ __forceinline__ float2 ld_stats(const float2* p) {
  const uint64_t v = __hip_atomic_load(reinterpret_cast<uint64_t*>(const_cast<float2*>(p)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float(static_cast<uint32_t>(v)), __uint_as_float(static_cast<uint32_t>(v >> 32)));
}
