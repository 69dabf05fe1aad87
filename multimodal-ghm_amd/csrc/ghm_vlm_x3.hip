// Split-bf16 (x3) MFMA attention of the sequential VLM (gfx950).
//
// AutoRegressiveTransformer's attention (models/model.py:329-341): single head,
// S = (Q K^T + mask) / scale_div with generate_mask's prefix-causal mask
// (:24-33: a prefix query sees the prefix, a text query sees every earlier
// token), A = softmax(S), and the reference's double residual
// H_mid = H + A V + (A / D) V, evaluated as (H + o) + o / D.
//
// Same compute model as the CLIP attention (ghm_x3.hip): one workgroup per
// sequence, one wave per 32 queries with the query on the lane; scores S^T come
// out of v_mfma_f32_32x32x16_bf16 as keys-on-rows accumulators, so the row
// softmax is a per-lane loop plus one lane-pair exchange, and the probabilities
// (split in registers) are directly the B operand of O^T = V^T P^T.  K and V are
// staged through LDS as split (hi, lo) images; V / K / dO / Q column blocks are
// read with ds_read_b64_tr_b16 transposed reads.  D = 128 or 256 features are
// processed as 128-feature halves so the query fragments stay at 64 VGPRs.
// q, k, v live in one [M][3D] buffer (the fused QKV GEMM's output); the
// backward writes dq, dk, dv into the same layout for the fused data / weight
// gradient GEMMs.
#include "ghm_launch.h"
#include "ghm_split.h"

namespace {

// padded sequence length of the P / dS layouts: 96 for T <= 96 (NKT <= 3), 192 above
template <int NKT>
__device__ __forceinline__ constexpr int vx_pad() { return NKT <= 3 ? 96 : 192; }
constexpr int VX_PITCH = 64 + 8;  // [row][h][32] half image row (bf16)

typedef __attribute__((address_space(3))) bf16x4 vx_lds_bf16x4;
__device__ __forceinline__ bf16x4 vx_ldtr(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((vx_lds_bf16x4*)(p));
}
// 8-row transposed fragment of a [row][32] image: lane l of group g = l >> 4
// receives column 16(g & 1) + (l & 15) of rows r0..r0+3 and r1..r1+3
__device__ __forceinline__ bf16x8 vx_tr_frag(const __bf16* img, int r0, int r1, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = 16 * (g & 1) + 4 * p;
  const bf16x4 a = vx_ldtr(img + (r0 + q) * 32 + col);
  const bf16x4 b = vx_ldtr(img + (r1 + q) * 32 + col);
  bf16x8 v;
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  return v;
}

// 64 consecutive floats at p -> 8 split k-steps (zeros when inactive)
__device__ __forceinline__ void vx_load_split64(const float* __restrict__ p, bool active, bf16x8* xh, bf16x8* xl) {
  float x[64];
  if (active) {
    load64(p, x);
  } else {
#pragma unroll
    for (int k = 0; k < 64; ++k) x[k] = 0.f;
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) split8(x + 8 * t, xh[t], xl[t]);
}

// largest chunk <= 8 that divides n (float4 loads in flight per thread while staging)
__device__ __forceinline__ constexpr int vx_chunk(int n) {
  return n % 8 == 0 ? 8 : (n % 6 == 0 ? 6 : (n % 4 == 0 ? 4 : (n % 3 == 0 ? 3 : (n % 2 == 0 ? 2 : 1))));
}

// columns col + HS hh + 0..31 (hh = 0, 1) of rows 0..TP-1 (row stride ld) as a
// split [row][hh][32] image; rows >= T clamp to T - 1.  NW waves stage it in
// chunks of at most 8 float4 per thread.  HS = 64: a 32-column slab of each
// 64-feature half of a 128-feature block; HS = 32: the two halves of D = 64.
template <int NKT, int NW, int HS = 64>
__device__ __forceinline__ void vx_stage_half(const float* __restrict__ seq, int64_t ld, int T, int col, __bf16* ih,
                                              __bf16* il) {
  constexpr int NT = NW * 64, NIT = NKT * 32 * 16 / NT, CH = vx_chunk(NIT);
  static_assert(NKT * 32 * 16 % NT == 0 && NIT % CH == 0, "staging split");
#pragma unroll 1  // one chunk of loads in flight: unrolled, the compiler hoists every chunk's loads
  for (int c0 = 0; c0 < NIT; c0 += CH) {
    float4 v[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int idx = threadIdx.x + NT * (c0 + k);
      const int row = idx >> 4, hh = (idx >> 3) & 1, q4 = idx & 7;
      const int rc = row < T ? row : T - 1;
      v[k] = *reinterpret_cast<const float4*>(seq + static_cast<int64_t>(rc) * ld + col + HS * hh + 4 * q4);
    }
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int idx = threadIdx.x + NT * (c0 + k);
      const int row = idx >> 4, hh = (idx >> 3) & 1, q4 = idx & 7;
      bf16x4 a, b;
      split4(v[k], a, b);
      stb4(ih + row * VX_PITCH + 32 * hh + 4 * q4, a);
      stb4(il + row * VX_PITCH + 32 * hh + 4 * q4, b);
    }
  }
}

// columns col .. col+31 of rows 0..TP-1 (row stride ld) as a split [row][32]
// image for transposed reads; rows >= T clamp
template <int NKT, int NW>
__device__ __forceinline__ void vx_stage_cols(const float* __restrict__ base, int64_t ld, int T, int col, __bf16* ih,
                                              __bf16* il) {
  constexpr int NT = NW * 64, NIT = NKT * 32 * 8 / NT, CH = vx_chunk(NIT);
  static_assert(NKT * 32 * 8 % NT == 0 && NIT % CH == 0, "staging split");
#pragma unroll 1  // one chunk of loads in flight: unrolled, the compiler hoists every chunk's loads
  for (int c0 = 0; c0 < NIT; c0 += CH) {
    float4 v[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int idx = threadIdx.x + NT * (c0 + k);
      const int row = idx >> 3, q4 = idx & 7;
      const int rc = row < T ? row : T - 1;
      v[k] = *reinterpret_cast<const float4*>(base + static_cast<int64_t>(rc) * ld + col + 4 * q4);
    }
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int idx = threadIdx.x + NT * (c0 + k);
      bf16x4 a, b;
      split4(v[k], a, b);
      stb4(ih + idx * 4, a);
      stb4(il + idx * 4, b);
    }
  }
}

// S^T[key][query] += X_rows . Y over the 32-column slab c of a half image
template <int NKT>
__device__ __forceinline__ void vx_rows_dot(const __bf16* ih, const __bf16* il, const bf16x8* yh, const bf16x8* yl,
                                           int c, int j, int h, int nk, f32x16* acc) {
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    if (kt >= nk) break;  // key tiles past the mask bound stay 0 (masked to -inf / P = 0)
    const int off = (32 * kt + j) * VX_PITCH + 32 * h;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
      acc[kt] = mfma_x3(ldsb8(ih + off + 8 * tt), ldsb8(il + off + 8 * tt), yh[4 * c + tt], yl[4 * c + tt], acc[kt]);
  }
}

// S^T (keys on rows, this wave's queries on lanes) = X[keys] . Y[query]^T over
// DD features; X columns xcol.. of the sequence block (row stride ldx), the
// query-side row at yrow (DD floats)
template <int NKT, int DD, int NW>
__device__ __forceinline__ void vx_scores(const float* __restrict__ xseq, int64_t ldx, int xcol,
                                          const float* __restrict__ yrow, int T, int j, int h, int nk, __bf16* sh,
                                          __bf16* sl, f32x16* s) {
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) s[kt] = zero16();
  if constexpr (DD == 64) {
    // D = 64 (the generic-width CLIP encoder, n_embd = 64): lane half h holds
    // features 32 h .. 32 h + 31 of Y; one [row][hh][32] image of both halves
    bf16x8 yh[4], yl[4];
    float y[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(yrow + 32 * h + 4 * k);
      y[4 * k] = v.x; y[4 * k + 1] = v.y; y[4 * k + 2] = v.z; y[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) split8(y + 8 * t, yh[t], yl[t]);
    vx_stage_half<NKT, NW, 32>(xseq, ldx, T, xcol, sh, sl);
    __syncthreads();
    vx_rows_dot<NKT>(sh, sl, yh, yl, 0, j, h, nk, s);
    __syncthreads();
    return;
  }
#pragma unroll 1
  for (int e = 0; e < DD / 128; ++e) {
    bf16x8 yh[8], yl[8];
    vx_load_split64(yrow + 128 * e + 64 * h, true, yh, yl);  // Y[128e + 64h + 8t + i]
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      vx_stage_half<NKT, NW>(xseq, ldx, T, xcol + 128 * e + 32 * c, sh, sl);
      __syncthreads();
      vx_rows_dot<NKT>(sh, sl, yh, yl, c, j, h, nk, s);
      __syncthreads();
    }
  }
}

__device__ __forceinline__ bool vx_allowed(int q, int key, int npre) { return q < npre ? key < npre : key <= q; }

// key tiles a workgroup of query tiles [32 q0, 32 q1) needs under the prefix-causal
// mask: keys <= max(npre - 1, last query) (npre = T: all)
__device__ __forceinline__ int vx_key_tiles(int q1, int T, int npre) {
  const int qmax = (32 * q1 < T ? 32 * q1 : T) - 1;
  const int kmax = qmax > npre - 1 ? qmax : npre - 1;
  return (kmax < T ? kmax : T - 1) / 32 + 1;
}

// attention activation (model.py:121-130 get_activation): softmax, or relu / gelu
// of the scaled score elementwise (no row normalisation; masked entries 0); gelu
// also stores GELU'(score) in Pd for the backward
constexpr int VACT_SOFTMAX = 0, VACT_RELU = 1, VACT_GELU = 2;

// NS: the output's DD / 32 column blocks split over NS workgroups (blockIdx.z);
// each recomputes the scores and the softmax of its query tiles (P / GELU' stored
// by z = 0 only), so a batch of 128 one-tile-per-wave sequences puts NS x as many
// waves on the chip and each runs 1 / NS of the V staging round trips
template <int NKT, int DD, int NW, int ACT = VACT_SOFTMAX, int NS = 1>
__global__ __launch_bounds__(NW * 64, 2) void k_vlm_attn_fwd_x3(const float* __restrict__ qkv,
                                                                 const float* __restrict__ H,
                                                                 float* __restrict__ Hmid, float* __restrict__ P,
                                                                 int T, int npre, float scale_div, float dbl,
                                                                 float* __restrict__ Pd = nullptr) {
  // no fp contraction in the attention kernels: the compiler fused, e.g., the
  // normalised P's product into its split's subtraction in some instantiations and
  // not in others (GHM_VX_SPLIT); every product now rounds where the source does
#pragma clang fp contract(off)
  constexpr int VX_PAD = vx_pad<NKT>();
  constexpr int TP = NKT * 32;
  constexpr int64_t LD = 3 * DD;
  __shared__ __attribute__((aligned(16))) __bf16 sh[TP * VX_PITCH];
  __shared__ __attribute__((aligned(16))) __bf16 sl[TP * VX_PITCH];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const float* seq = qkv + base * LD;
  // workgroup y takes query tiles NW y .. NW y + NW - 1 (one per wave)
  const int q = 32 * (NW * static_cast<int>(blockIdx.y) + w) + j;
  const bool qv = q < T;
  const int qc = qv ? q : T - 1;
  const int nk = vx_key_tiles(NW * (static_cast<int>(blockIdx.y) + 1), T, npre);
  const bool first = NS == 1 || blockIdx.z == 0;  // the split that stores P (and GELU')
  f32x16 s[NKT];
  vx_scores<NKT, DD, NW>(seq, LD, DD, seq + qc * LD, T, j, h, nk, sh, sl, s);
  // one reciprocal and a base-2 exponent per score (as k_attn_fwd_x3)
  const float inv_scale = 1.f / scale_div, l2e = 1.4426950408889634f;
  float inv;
  if constexpr (ACT == VACT_SOFTMAX) {
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + acc_row(r, h);
        const float v = (key < T && vx_allowed(qc, key, npre)) ? s[kt][r] * inv_scale : -INFINITY;
        s[kt][r] = v;
        mx = fmaxf(mx, v);
      }
    }
    mx = fmaxf(mx, xhalf(mx));
    const float mx2 = mx * l2e;
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(fmaf(s[kt][r], l2e, -mx2));
        s[kt][r] = e;
        sum += e;
      }
    }
    sum += xhalf(sum);
    inv = qv ? 1.f / sum : 0.f;
  } else {
    inv = qv ? 1.f : 0.f;
    float* drow = ACT == VACT_GELU ? Pd + (static_cast<int64_t>(blockIdx.x) * VX_PAD + q) * VX_PAD : nullptr;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      float dv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + acc_row(r, h);
        const float x = s[kt][r] * inv_scale;
        float a, d;
        if constexpr (ACT == VACT_RELU) {
          a = fmaxf(x, 0.f);
          d = 0.f;
        } else {
          gelu_fast(x, a, d);
        }
        const bool ok = qv && key < T && vx_allowed(qc, key, npre);
        s[kt][r] = ok ? a : 0.f;
        dv[r] = ok ? d : 0.f;
      }
      if constexpr (ACT == VACT_GELU) {
        if (qv && first) {
#pragma unroll
          for (int qd = 0; qd < 4; ++qd)
            st4(drow + 32 * kt + quad_off(qd, h), dv[4 * qd], dv[4 * qd + 1], dv[4 * qd + 2], dv[4 * qd + 3]);
        }
      }
    }
  }
  float* prow = P + (static_cast<int64_t>(blockIdx.x) * VX_PAD + q) * VX_PAD;
  bf16x8 ph[2 * NKT], pl[2 * NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kt][r] *= inv;
    if (first) {
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        st4(prow + 32 * kt + quad_off(qd, h), s[kt][4 * qd], s[kt][4 * qd + 1], s[kt][4 * qd + 2], s[kt][4 * qd + 3]);
    }
    float pv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) pv[r] = s[kt][r];
    split_acc(pv, 0, ph[2 * kt], pl[2 * kt]);
    split_acc(pv, 1, ph[2 * kt + 1], pl[2 * kt + 1]);
  }
  // O^T[d][q] = sum_key V[key][d] P[q][key], V column blocks of 32 through LDS
  constexpr int NDT = DD / 32 / NS;
  const int dt0 = NS == 1 ? 0 : NDT * static_cast<int>(blockIdx.z);
#pragma unroll 1
  for (int dt = dt0; dt < dt0 + NDT; ++dt) {
    vx_stage_cols<NKT, NW>(seq, LD, T, 2 * DD + 32 * dt, sh, sl);
    __syncthreads();
    f32x16 acc = zero16();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (kt >= nk) break;  // P = 0 past the mask bound
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int r0 = 32 * kt + 16 * ss + 4 * h;
        acc = mfma_x3(vx_tr_frag(sh, r0, r0 + 8, lane), vx_tr_frag(sl, r0, r0 + 8, lane), ph[2 * kt + ss],
                      pl[2 * kt + ss], acc);
      }
    }
    __syncthreads();
    if (qv) {
      const int64_t row = (base + q) * DD + 32 * dt;
      float4 hv[4];
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) hv[qd] = *reinterpret_cast<const float4*>(H + row + quad_off(qd, h));
#pragma unroll
      // explicit fma: the same rounding in every instantiation (the compiler's own
      // contraction of o * dbl + (h + o) differed between NS = 1 and NS > 1)
      for (int qd = 0; qd < 4; ++qd) {
        const float o0 = acc[4 * qd], o1 = acc[4 * qd + 1], o2 = acc[4 * qd + 2], o3 = acc[4 * qd + 3];
        st4(Hmid + row + quad_off(qd, h), __builtin_fmaf(o0, dbl, hv[qd].x + o0), __builtin_fmaf(o1, dbl, hv[qd].y + o1),
            __builtin_fmaf(o2, dbl, hv[qd].z + o2), __builtin_fmaf(o3, dbl, hv[qd].w + o3));
      }
    }
  }
}

// dA^T = (V dO^T)(1 + 1/D), dS = P (dA - rowsum(P dA)) / scale_div (stored dense),
// dQ^T = K^T dS^T
// NS: dQ's column blocks over NS workgroups (blockIdx.z), each recomputing dS (stored by z = 0)
template <int NKT, int DD, int NW, int ACT = VACT_SOFTMAX, int NS = 1>
__global__ __launch_bounds__(NW * 64, 2) void k_vlm_attn_bwd_q_x3(const float* __restrict__ qkv,
                                                                   const float* __restrict__ P,
                                                                   const float* __restrict__ dHmid,
                                                                   float* __restrict__ dS_out,
                                                                   float* __restrict__ dqkv, int T, float scale_div,
                                                                   int npre, float dbl,
                                                                   const float* __restrict__ Pd = nullptr) {
  // no fp contraction in the attention kernels: the compiler fused, e.g., the
  // normalised P's product into its split's subtraction in some instantiations and
  // not in others (GHM_VX_SPLIT); every product now rounds where the source does
#pragma clang fp contract(off)
  constexpr int VX_PAD = vx_pad<NKT>();
  constexpr int TP = NKT * 32;
  constexpr int64_t LD = 3 * DD;
  __shared__ __attribute__((aligned(16))) __bf16 sh[TP * VX_PITCH];
  __shared__ __attribute__((aligned(16))) __bf16 sl[TP * VX_PITCH];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const float* seq = qkv + base * LD;
  const int q = 32 * (NW * static_cast<int>(blockIdx.y) + w) + j;
  const bool qv = q < T;
  const int qc = qv ? q : T - 1;
  const int nk = vx_key_tiles(NW * (static_cast<int>(blockIdx.y) + 1), T, npre);
  f32x16 dp[NKT];
  vx_scores<NKT, DD, NW>(seq, LD, 2 * DD, dHmid + (base + qc) * DD, T, j, h, nk, sh, sl, dp);
  // gelu: dS = GELU'(score) dA / scale_div, so the saved derivative replaces P here
  const float* prow = (ACT == VACT_GELU ? Pd : P) + (static_cast<int64_t>(blockIdx.x) * VX_PAD + q) * VX_PAD;
  const float inv_scale = 1.f / scale_div;
  float delta = 0.f;
  f32x16 p[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      const float4 pv = *reinterpret_cast<const float4*>(prow + 32 * kt + quad_off(qd, h));
      p[kt][4 * qd + 0] = qv ? pv.x : 0.f;
      p[kt][4 * qd + 1] = qv ? pv.y : 0.f;
      p[kt][4 * qd + 2] = qv ? pv.z : 0.f;
      p[kt][4 * qd + 3] = qv ? pv.w : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {  // explicit fmas: the same rounding in every instantiation
      dp[kt][r] = __builtin_fmaf(dp[kt][r], dbl, dp[kt][r]);
      if (ACT == VACT_SOFTMAX) delta = __builtin_fmaf(p[kt][r], dp[kt][r], delta);
    }
  }
  if (ACT == VACT_SOFTMAX) delta += xhalf(delta);
  float* srow = dS_out + (static_cast<int64_t>(blockIdx.x) * VX_PAD + q) * VX_PAD;
  bf16x8 dh[2 * NKT], dl[2 * NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    float dv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if constexpr (ACT == VACT_SOFTMAX)
        dv[r] = (p[kt][r] * (dp[kt][r] - delta)) * inv_scale;
      else if constexpr (ACT == VACT_RELU)
        dv[r] = (p[kt][r] > 0.f ? dp[kt][r] : 0.f) * inv_scale;
      else
        dv[r] = (p[kt][r] * dp[kt][r]) * inv_scale;
    }
    if (NS == 1 || blockIdx.z == 0) {
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        st4(srow + 32 * kt + quad_off(qd, h), dv[4 * qd], dv[4 * qd + 1], dv[4 * qd + 2], dv[4 * qd + 3]);
    }
    split_acc(dv, 0, dh[2 * kt], dl[2 * kt]);
    split_acc(dv, 1, dh[2 * kt + 1], dl[2 * kt + 1]);
  }
  constexpr int NDT = DD / 32 / NS;
  const int dt0 = NS == 1 ? 0 : NDT * static_cast<int>(blockIdx.z);
#pragma unroll 1
  for (int dt = dt0; dt < dt0 + NDT; ++dt) {
    vx_stage_cols<NKT, NW>(seq, LD, T, DD + 32 * dt, sh, sl);  // K
    __syncthreads();
    f32x16 acc = zero16();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (kt >= nk) break;  // dS = 0 past the mask bound
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int r0 = 32 * kt + 16 * ss + 4 * h;
        acc = mfma_x3(vx_tr_frag(sh, r0, r0 + 8, lane), vx_tr_frag(sl, r0, r0 + 8, lane), dh[2 * kt + ss],
                      dl[2 * kt + ss], acc);
      }
    }
    __syncthreads();
    if (qv) {
      float* o = dqkv + (base + q) * LD + 32 * dt;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        st4(o + quad_off(qd, h), acc[4 * qd], acc[4 * qd + 1], acc[4 * qd + 2], acc[4 * qd + 3]);
    }
  }
}

// dV^T = dO^T P (1 + 1/D) and dK^T = Q^T dS, summed over queries; the key on the lane
// NS: the DD / 32 column blocks of dK / dV over NS workgroups (blockIdx.z)
template <int NKT, int DD, int NW, int NS = 1>
__global__ __launch_bounds__(NW * 64, 2) void k_vlm_attn_bwd_kv_x3(const float* __restrict__ qkv,
                                                                    const float* __restrict__ P,
                                                                    const float* __restrict__ dS,
                                                                    const float* __restrict__ dHmid,
                                                                    float* __restrict__ dqkv, int T, int npre, float dbl) {
  // no fp contraction in the attention kernels: the compiler fused, e.g., the
  // normalised P's product into its split's subtraction in some instantiations and
  // not in others (GHM_VX_SPLIT); every product now rounds where the source does
#pragma clang fp contract(off)
  constexpr int VX_PAD = vx_pad<NKT>();
  constexpr int TP = NKT * 32, KS = TP / 16;
  constexpr int64_t LD = 3 * DD;
  __shared__ __attribute__((aligned(16))) __bf16 soh[TP * 32];
  __shared__ __attribute__((aligned(16))) __bf16 sol[TP * 32];
  __shared__ __attribute__((aligned(16))) __bf16 sqh[TP * 32];
  __shared__ __attribute__((aligned(16))) __bf16 sql[TP * 32];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const int key = 32 * (NW * static_cast<int>(blockIdx.y) + w) + j;
  const bool kv = key < T;
  // queries that see this workgroup's keys: all when a key is in the prefix,
  // else q >= the first key (P = dS = 0 above the diagonal)
  const int klo = 32 * NW * static_cast<int>(blockIdx.y);
  const int st0 = klo >= npre ? klo / 16 : 0;
  const float* pc = P + static_cast<int64_t>(blockIdx.x) * VX_PAD * VX_PAD + key;
  const float* sc = dS + static_cast<int64_t>(blockIdx.x) * VX_PAD * VX_PAD + key;
  if constexpr (NKT <= 3) {
    bf16x8 pbh[KS], pbl[KS], sbh[KS], sbl[KS];
  #pragma unroll
    for (int st = 0; st < KS; ++st) {
      if (st < st0) continue;
      float pv[8], sv[8];
  #pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int qq = 16 * st + 8 * h + i;
        pv[i] = pc[qq * VX_PAD];
        sv[i] = sc[qq * VX_PAD];
      }
      split8(pv, pbh[st], pbl[st]);
      split8(sv, sbh[st], sbl[st]);
    }
    constexpr int NDT = DD / 32 / NS;
    const int dt0 = NS == 1 ? 0 : NDT * static_cast<int>(blockIdx.z);
  #pragma unroll 1
    for (int dt = dt0; dt < dt0 + NDT; ++dt) {
      vx_stage_cols<NKT, NW>(dHmid + base * DD, DD, T, 32 * dt, soh, sol);
      vx_stage_cols<NKT, NW>(qkv + base * LD, LD, T, 32 * dt, sqh, sql);
      __syncthreads();
      f32x16 aV = zero16(), aK = zero16();
  #pragma unroll
      for (int st = 0; st < KS; ++st) {
        if (st < st0) continue;
        const int r0 = 16 * st + 8 * h;
        aV = mfma_x3(vx_tr_frag(soh, r0, r0 + 4, lane), vx_tr_frag(sol, r0, r0 + 4, lane), pbh[st], pbl[st], aV);
        aK = mfma_x3(vx_tr_frag(sqh, r0, r0 + 4, lane), vx_tr_frag(sql, r0, r0 + 4, lane), sbh[st], sbl[st], aK);
      }
      __syncthreads();
      if (kv) {
        float* o = dqkv + (base + key) * LD + 32 * dt;
  #pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          const float v0 = aV[4 * qd], v1 = aV[4 * qd + 1], v2 = aV[4 * qd + 2], v3 = aV[4 * qd + 3];
          st4(o + 2 * DD + quad_off(qd, h), __builtin_fmaf(v0, dbl, v0), __builtin_fmaf(v1, dbl, v1),
              __builtin_fmaf(v2, dbl, v2), __builtin_fmaf(v3, dbl, v3));
          st4(o + DD + quad_off(qd, h), aK[4 * qd], aK[4 * qd + 1], aK[4 * qd + 2], aK[4 * qd + 3]);
        }
      }
    }
  } else {
    // T > 96: both products' B fragments (4 x KS x 8 VGPRs) no longer fit beside
    // the accumulators, so dV^T = dO^T P and dK^T = Q^T dS run as two passes
#pragma unroll 1
    for (int which = 0; which < 2; ++which) {
      const float* src = which == 0 ? pc : sc;
      bf16x8 bh[KS], bl[KS];
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        if (st < st0) continue;
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = src[(16 * st + 8 * h + i) * VX_PAD];
        split8(v, bh[st], bl[st]);
      }
      constexpr int NDT = DD / 32 / NS;
      const int dt0 = NS == 1 ? 0 : NDT * static_cast<int>(blockIdx.z);
#pragma unroll 1
      for (int dt = dt0; dt < dt0 + NDT; ++dt) {
        if (which == 0) vx_stage_cols<NKT, NW>(dHmid + base * DD, DD, T, 32 * dt, soh, sol);
        else vx_stage_cols<NKT, NW>(qkv + base * LD, LD, T, 32 * dt, soh, sol);
        __syncthreads();
        f32x16 acc = zero16();
#pragma unroll
        for (int st = 0; st < KS; ++st) {
          if (st < st0) continue;
          const int r0 = 16 * st + 8 * h;
          acc = mfma_x3(vx_tr_frag(soh, r0, r0 + 4, lane), vx_tr_frag(sol, r0, r0 + 4, lane), bh[st], bl[st], acc);
        }
        __syncthreads();
        if (kv) {
          float* o = dqkv + (base + key) * LD + 32 * dt + (which == 0 ? 2 * DD : DD);
          const float f = which == 0 ? dbl : 0.f;
#pragma unroll
          for (int qd = 0; qd < 4; ++qd) {
            const float v0 = acc[4 * qd], v1 = acc[4 * qd + 1], v2 = acc[4 * qd + 2], v3 = acc[4 * qd + 3];
            st4(o + quad_off(qd, h), __builtin_fmaf(v0, f, v0), __builtin_fmaf(v1, f, v1), __builtin_fmaf(v2, f, v2),
                __builtin_fmaf(v3, f, v3));
          }
        }
      }
    }
  }
}

// waves (query or key tiles) per workgroup: several workgroups per sequence so a
// batch of 128 sequences fills the 256 CUs; NW must divide the staging split
template <int NKT>
constexpr int vx_nw() { return NKT == 6 ? 3 : (NKT == 4 ? 2 : (NKT == 5 ? 5 : 1)); }

// NS, the column blocks' split over workgroups (round 5, profiles/r5_vx_ab.txt):
// the forward and the dQ kernel recompute scores / dS per split, so 2 (two splits
// 30.6 -> 25.5 and 33.3 -> 27.6 us, four slower again); the dK / dV kernel only
// reloads P and dS, so 4 (32.2 -> 17.2 us).  GHM_VX_SPLIT / GHM_VX_SPLIT_KV = 1 / 2
// / 4 override them (A/B knobs, read per call).
inline int vx_split(const char* var = "GHM_VX_SPLIT", int dflt = 2) {
  const char* e = getenv(var);
  const int v = e ? atoi(e) : dflt;
  return v == 2 || v == 4 ? v : 1;
}

template <int NKT, int DD, int ACT = VACT_SOFTMAX>
void launch_fwd_n(unsigned g, hipStream_t s, const float* qkv, const float* H, float* Hm, float* P, int T, int npre,
                  float sd, float dbl, float* Pd = nullptr) {
  constexpr int NW = vx_nw<NKT>();
  const int ns = vx_split() <= DD / 32 ? vx_split() : DD / 32;  // at least one 32-column block per split
  if (ns == 2)
    hipLaunchKernelGGL((k_vlm_attn_fwd_x3<NKT, DD, NW, ACT, 2>), dim3(g, NKT / NW, 2), dim3(NW * 64), 0, s, qkv, H, Hm,
                       P, T, npre, sd, dbl, Pd);
  else if (ns == 4)
    hipLaunchKernelGGL((k_vlm_attn_fwd_x3<NKT, DD, NW, ACT, 4>), dim3(g, NKT / NW, 4), dim3(NW * 64), 0, s, qkv, H, Hm,
                       P, T, npre, sd, dbl, Pd);
  else
    hipLaunchKernelGGL((k_vlm_attn_fwd_x3<NKT, DD, NW, ACT>), dim3(g, NKT / NW), dim3(NW * 64), 0, s, qkv, H, Hm, P, T,
                       npre, sd, dbl, Pd);
}

template <int DD, int ACT = VACT_SOFTMAX>
void launch_fwd(int T, unsigned g, hipStream_t s, const float* qkv, const float* H, float* Hm, float* P, int npre,
                float sd, float dbl, float* Pd = nullptr) {
  if (T <= 32) launch_fwd_n<1, DD, ACT>(g, s, qkv, H, Hm, P, T, npre, sd, dbl, Pd);
  else if (T <= 64) launch_fwd_n<2, DD, ACT>(g, s, qkv, H, Hm, P, T, npre, sd, dbl, Pd);
  else if (T <= 96) launch_fwd_n<3, DD, ACT>(g, s, qkv, H, Hm, P, T, npre, sd, dbl, Pd);
  else if (T <= 128) launch_fwd_n<4, DD, ACT>(g, s, qkv, H, Hm, P, T, npre, sd, dbl, Pd);
  else if (T <= 160) launch_fwd_n<5, DD, ACT>(g, s, qkv, H, Hm, P, T, npre, sd, dbl, Pd);
  else launch_fwd_n<6, DD, ACT>(g, s, qkv, H, Hm, P, T, npre, sd, dbl, Pd);  // D = 256: spills 5-12 VGPRs (correct, slower)
}

template <int NKT, int DD, int ACT = VACT_SOFTMAX>
void launch_bwd_n(unsigned g, hipStream_t s, const float* qkv, const float* P, const float* dHm, float* dS,
                  float* dqkv, int T, int npre, float sd, float dbl, const float* Pd = nullptr) {
  constexpr int NW = vx_nw<NKT>();
  int ns = vx_split(), nkv = vx_split("GHM_VX_SPLIT_KV", 4);
  if (ns > DD / 32) ns = DD / 32;  // at least one 32-column block per split
  if (nkv > DD / 32) nkv = DD / 32;
  if (ns == 2)
    hipLaunchKernelGGL((k_vlm_attn_bwd_q_x3<NKT, DD, NW, ACT, 2>), dim3(g, NKT / NW, 2), dim3(NW * 64), 0, s, qkv, P,
                       dHm, dS, dqkv, T, sd, npre, dbl, Pd);
  else if (ns == 4)
    hipLaunchKernelGGL((k_vlm_attn_bwd_q_x3<NKT, DD, NW, ACT, 4>), dim3(g, NKT / NW, 4), dim3(NW * 64), 0, s, qkv, P,
                       dHm, dS, dqkv, T, sd, npre, dbl, Pd);
  else
    hipLaunchKernelGGL((k_vlm_attn_bwd_q_x3<NKT, DD, NW, ACT>), dim3(g, NKT / NW), dim3(NW * 64), 0, s, qkv, P, dHm,
                       dS, dqkv, T, sd, npre, dbl, Pd);
  if (nkv == 2)
    hipLaunchKernelGGL((k_vlm_attn_bwd_kv_x3<NKT, DD, NW, 2>), dim3(g, NKT / NW, 2), dim3(NW * 64), 0, s, qkv, P, dS,
                       dHm, dqkv, T, npre, dbl);
  else if (nkv == 4)
    hipLaunchKernelGGL((k_vlm_attn_bwd_kv_x3<NKT, DD, NW, 4>), dim3(g, NKT / NW, 4), dim3(NW * 64), 0, s, qkv, P, dS,
                       dHm, dqkv, T, npre, dbl);
  else
    hipLaunchKernelGGL((k_vlm_attn_bwd_kv_x3<NKT, DD, NW>), dim3(g, NKT / NW), dim3(NW * 64), 0, s, qkv, P, dS, dHm,
                       dqkv, T, npre, dbl);
}

template <int DD, int ACT = VACT_SOFTMAX>
void launch_bwd(int T, unsigned g, hipStream_t s, const float* qkv, const float* P, const float* dHm, float* dS,
                float* dqkv, int npre, float sd, float dbl, const float* Pd = nullptr) {
  if (T <= 32) launch_bwd_n<1, DD, ACT>(g, s, qkv, P, dHm, dS, dqkv, T, npre, sd, dbl, Pd);
  else if (T <= 64) launch_bwd_n<2, DD, ACT>(g, s, qkv, P, dHm, dS, dqkv, T, npre, sd, dbl, Pd);
  else if (T <= 96) launch_bwd_n<3, DD, ACT>(g, s, qkv, P, dHm, dS, dqkv, T, npre, sd, dbl, Pd);
  else if (T <= 128) launch_bwd_n<4, DD, ACT>(g, s, qkv, P, dHm, dS, dqkv, T, npre, sd, dbl, Pd);
  else if (T <= 160) launch_bwd_n<5, DD, ACT>(g, s, qkv, P, dHm, dS, dqkv, T, npre, sd, dbl, Pd);
  else launch_bwd_n<6, DD, ACT>(g, s, qkv, P, dHm, dS, dqkv, T, npre, sd, dbl, Pd);
}

}  // namespace

extern "C" int ghm_vlm_attn_fwd_x3(const float* qkv, const float* H, float* H_mid, float* P, int64_t n_seq, int T,
                                   int D, int n_prefix, float scale_div, void* stream) {
  GHM_CHECK(qkv && H && H_mid && P, "null pointer");
  GHM_CHECK((D == 128 || D == 256) && T >= 1 && T <= 96 && n_seq >= 1 && n_prefix >= 0 && n_prefix <= T,
            "shape (T <= 96, D in {128, 256})");
  return ghm_attn_ext_fwd_x3(qkv, H, H_mid, P, n_seq, T, D, n_prefix, scale_div, 1.f / static_cast<float>(D),
                             stream);
}

extern "C" int ghm_vlm_attn_bwd_x3(const float* qkv, const float* P, const float* dH_mid, float* dS, float* dqkv,
                                   int64_t n_seq, int T, int D, float scale_div, void* stream) {
  GHM_CHECK(qkv && P && dH_mid && dS && dqkv, "null pointer");
  GHM_CHECK((D == 128 || D == 256) && T >= 1 && T <= 96 && n_seq >= 1, "shape (T <= 96, D in {128, 256})");
  // no mask bound known here: n_prefix = T (no key / query tile skipping; P = 0 masks)
  return ghm_attn_ext_bwd_x3(qkv, P, dH_mid, dS, dqkv, n_seq, T, D, T, scale_div, 1.f / static_cast<float>(D), stream);
}

extern "C" int ghm_attn_ext_fwd_x3(const float* qkv, const float* H, float* H_mid, float* P, int64_t n_seq, int T,
                                   int D, int n_prefix, float scale_div, float dbl, void* stream) {
  GHM_CHECK(qkv && H && H_mid && P, "null pointer");
  GHM_CHECK((D == 64 || D == 128 || D == 256) && T >= 1 && T <= 192, "shape (D in {64, 128, 256}, T <= 192)");
  GHM_CHECK(n_seq >= 1 && n_prefix >= 0 && n_prefix <= T, "n_seq >= 1, 0 <= n_prefix <= T");
  const unsigned g = static_cast<unsigned>(n_seq);
  if (D == 64) launch_fwd<64>(T, g, ghm_stream(stream), qkv, H, H_mid, P, n_prefix, scale_div, dbl);
  else if (D == 128) launch_fwd<128>(T, g, ghm_stream(stream), qkv, H, H_mid, P, n_prefix, scale_div, dbl);
  else launch_fwd<256>(T, g, ghm_stream(stream), qkv, H, H_mid, P, n_prefix, scale_div, dbl);
  return ghm_launch_status();
}

extern "C" int ghm_attn_ext_bwd_x3(const float* qkv, const float* P, const float* dH_mid, float* dS, float* dqkv,
                                   int64_t n_seq, int T, int D, int n_prefix, float scale_div, float dbl,
                                   void* stream) {
  GHM_CHECK(qkv && P && dH_mid && dS && dqkv, "null pointer");
  GHM_CHECK((D == 64 || D == 128 || D == 256) && T >= 1 && T <= 192, "shape (D in {64, 128, 256}, T <= 192)");
  GHM_CHECK(n_seq >= 1 && n_prefix >= 0 && n_prefix <= T, "n_seq >= 1, 0 <= n_prefix <= T");
  const unsigned g = static_cast<unsigned>(n_seq);
  if (D == 64) launch_bwd<64>(T, g, ghm_stream(stream), qkv, P, dH_mid, dS, dqkv, n_prefix, scale_div, dbl);
  else if (D == 128) launch_bwd<128>(T, g, ghm_stream(stream), qkv, P, dH_mid, dS, dqkv, n_prefix, scale_div, dbl);
  else launch_bwd<256>(T, g, ghm_stream(stream), qkv, P, dH_mid, dS, dqkv, n_prefix, scale_div, dbl);
  return ghm_launch_status();
}

extern "C" int ghm_attn_ext_fwd_x3_act(const float* qkv, const float* H, float* H_mid, float* P, float* Pd,
                                       int64_t n_seq, int T, int D, int n_prefix, float scale_div, float dbl, int act,
                                       void* stream) {
  GHM_CHECK(qkv && H && H_mid && P, "null pointer");
  GHM_CHECK(act == VACT_RELU || (act == VACT_GELU && Pd), "act: 1 relu, 2 gelu (with Pd)");
  GHM_CHECK((D == 64 || D == 128 || D == 256) && T >= 1 && T <= 192, "shape (D in {64, 128, 256}, T <= 192)");
  GHM_CHECK(n_seq >= 1 && n_prefix >= 0 && n_prefix <= T, "n_seq >= 1, 0 <= n_prefix <= T");
  const unsigned g = static_cast<unsigned>(n_seq);
  hipStream_t s = ghm_stream(stream);
  if (D == 64) {
    if (act == VACT_RELU) launch_fwd<64, VACT_RELU>(T, g, s, qkv, H, H_mid, P, n_prefix, scale_div, dbl, Pd);
    else launch_fwd<64, VACT_GELU>(T, g, s, qkv, H, H_mid, P, n_prefix, scale_div, dbl, Pd);
  } else if (D == 128) {
    if (act == VACT_RELU) launch_fwd<128, VACT_RELU>(T, g, s, qkv, H, H_mid, P, n_prefix, scale_div, dbl, Pd);
    else launch_fwd<128, VACT_GELU>(T, g, s, qkv, H, H_mid, P, n_prefix, scale_div, dbl, Pd);
  } else {  // D = 256: the VLM (AutoRegressiveTransformer(activation=...), model.py:163, 287)
    if (act == VACT_RELU) launch_fwd<256, VACT_RELU>(T, g, s, qkv, H, H_mid, P, n_prefix, scale_div, dbl, Pd);
    else launch_fwd<256, VACT_GELU>(T, g, s, qkv, H, H_mid, P, n_prefix, scale_div, dbl, Pd);
  }
  return ghm_launch_status();
}

extern "C" int ghm_attn_ext_bwd_x3_act(const float* qkv, const float* P, const float* Pd, const float* dH_mid,
                                       float* dS, float* dqkv, int64_t n_seq, int T, int D, int n_prefix,
                                       float scale_div, float dbl, int act, void* stream) {
  GHM_CHECK(qkv && P && dH_mid && dS && dqkv, "null pointer");
  GHM_CHECK(act == VACT_RELU || (act == VACT_GELU && Pd), "act: 1 relu, 2 gelu (with Pd)");
  GHM_CHECK((D == 64 || D == 128 || D == 256) && T >= 1 && T <= 192, "shape (D in {64, 128, 256}, T <= 192)");
  GHM_CHECK(n_seq >= 1 && n_prefix >= 0 && n_prefix <= T, "n_seq >= 1, 0 <= n_prefix <= T");
  const unsigned g = static_cast<unsigned>(n_seq);
  hipStream_t s = ghm_stream(stream);
  if (D == 64) {
    if (act == VACT_RELU) launch_bwd<64, VACT_RELU>(T, g, s, qkv, P, dH_mid, dS, dqkv, n_prefix, scale_div, dbl, Pd);
    else launch_bwd<64, VACT_GELU>(T, g, s, qkv, P, dH_mid, dS, dqkv, n_prefix, scale_div, dbl, Pd);
  } else if (D == 128) {
    if (act == VACT_RELU) launch_bwd<128, VACT_RELU>(T, g, s, qkv, P, dH_mid, dS, dqkv, n_prefix, scale_div, dbl, Pd);
    else launch_bwd<128, VACT_GELU>(T, g, s, qkv, P, dH_mid, dS, dqkv, n_prefix, scale_div, dbl, Pd);
  } else {
    if (act == VACT_RELU) launch_bwd<256, VACT_RELU>(T, g, s, qkv, P, dH_mid, dS, dqkv, n_prefix, scale_div, dbl, Pd);
    else launch_bwd<256, VACT_GELU>(T, g, s, qkv, P, dH_mid, dS, dqkv, n_prefix, scale_div, dbl, Pd);
  }
  return ghm_launch_status();
}
