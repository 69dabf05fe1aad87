// Split-bf16 ("bf16x3") matrix products for gfx950.
//
// An f32 value x is carried as two bf16 parts, hi = bf16(x) and
// lo = bf16(x - hi), so x = hi + lo to ~2^-17 relative.  A product is
// a·b ≈ hi_a·hi_b + hi_a·lo_b + lo_a·hi_b; each term is an exact bf16×bf16
// product accumulated in f32 by v_mfma_f32_32x32x16_bf16, so a K=16 step costs
// 3 bf16 MFMAs (96 cycles) instead of 8 f32 MFMAs (512 cycles), at a relative
// error of ~2^-16 per product (the dropped lo·lo and truncation terms).
//
// Operand maps (32x32x16 bf16): lane (r = l&31, h = l>>5) holds A[r][8h + i]
// and B[8h + i][r], i = 0..7.  The accumulator layout equals the f32 MFMA's
// (ghm_common.h acc_row), so a "tokens on lanes" accumulator feeds the next
// product as the B operand: registers 8s..8s+7 form k-step s with element i of
// half h = row 16s + 8(i>>2) + 4h + (i&3).  Weight tiles that meet such an
// operand are stored in LDS with that k permutation (perm16 below) so each lane
// reads its 8 elements with one 16-byte load.
#pragma once
#include "ghm_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma_bf(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// acc += A·B with A = ah + al, B = bh + bl (lo·lo dropped)
__device__ __forceinline__ f32x16 mfma_x3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x16 c) {
  c = mfma_bf(al, bh, c);
  c = mfma_bf(ah, bl, c);
  return mfma_bf(ah, bh, c);
}

// six products of three-way split operands on the 32x32x16 MFMA (see mfma16_x6),
// chained: for accumulators that start from zero per output tile
__device__ __forceinline__ f32x16 mfma_x6(bf16x8 a0, bf16x8 a1, bf16x8 a2, bf16x8 b0, bf16x8 b1, bf16x8 b2,
                                         f32x16 c) {
  c = mfma_bf(a2, b0, c);
  c = mfma_bf(a1, b1, c);
  c = mfma_bf(a0, b2, c);
  c = mfma_bf(a1, b0, c);
  c = mfma_bf(a0, b1, c);
  return mfma_bf(a0, b0, c);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16x16x32 bf16: lane l holds A[row l&15][k = 8(l>>4) + i], B[k = 8(l>>4) + i][col l&15];
// C/D: col = l&15, row = 4(l>>4) + r
__device__ __forceinline__ f32x4 mfma16_bf(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16_x3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x4 c) {
  c = mfma16_bf(al, bh, c);
  c = mfma16_bf(ah, bl, c);
  return mfma16_bf(ah, bh, c);
}
// six products of three-way split operands, a.b ~ a2 b0 + a1 b1 + a0 b2 + a1 b0 +
// a0 b1 + a0 b0 (the dropped terms ~2^-27 |a||b|), smallest first, chained into one
// accumulator: for sums that start from zero and stay at the magnitude of their own
// terms (an MFMA adding products into a much larger accumulator drops their low bits)
__device__ __forceinline__ f32x4 mfma16_x6(bf16x8 a0, bf16x8 a1, bf16x8 a2, bf16x8 b0, bf16x8 b1, bf16x8 b2,
                                           f32x4 c) {
  c = mfma16_bf(a2, b0, c);
  c = mfma16_bf(a1, b1, c);
  c = mfma16_bf(a0, b2, c);
  c = mfma16_bf(a1, b0, c);
  c = mfma16_bf(a0, b1, c);
  return mfma16_bf(a0, b0, c);
}
__device__ __forceinline__ f32x4 zero4() {
  f32x4 z;
  z[0] = z[1] = z[2] = z[3] = 0.f;
  return z;
}

__device__ __forceinline__ void split1(float x, __bf16& hi, __bf16& lo) {
  hi = static_cast<__bf16>(x);
  lo = static_cast<__bf16>(x - static_cast<float>(hi));
}

// 8 consecutive floats -> (hi, lo) fragments
__device__ __forceinline__ void split8(const float* x, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    __bf16 a, b;
    split1(x[i], a, b);
    hi[i] = a;
    lo[i] = b;
  }
}

// three-way split: x = hi + lo + lo2 to ~2^-26 relative (hi, lo as split1; lo2 the
// bf16 of what is left, exact in f32 before its rounding)
__device__ __forceinline__ void split3_8(const float* x, bf16x8& hi, bf16x8& lo, bf16x8& lo2) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const __bf16 a = static_cast<__bf16>(x[i]);
    const float r = x[i] - static_cast<float>(a);
    const __bf16 b = static_cast<__bf16>(r);
    hi[i] = a;
    lo[i] = b;
    lo2[i] = static_cast<__bf16>(r - static_cast<float>(b));
  }
}

__device__ __forceinline__ void split4(float4 v, bf16x4& hi, bf16x4& lo) {
  __bf16 a, b;
  split1(v.x, a, b); hi[0] = a; lo[0] = b;
  split1(v.y, a, b); hi[1] = a; lo[1] = b;
  split1(v.z, a, b); hi[2] = a; lo[2] = b;
  split1(v.w, a, b); hi[3] = a; lo[3] = b;
}

// accumulator registers 8s..8s+7 as a (hi, lo) B/A fragment of k-step s
__device__ __forceinline__ void split_acc(const float* g, int s, bf16x8& hi, bf16x8& lo) {
  split8(g + 8 * s, hi, lo);
}

// Position inside a 16-column group at which original column c (0..15) is
// stored so that an accumulator-derived operand reads 8 contiguous elements:
// the 4-column groups 1 and 2 swap.
__device__ __forceinline__ constexpr int perm16_group(int g4) { return g4 == 1 ? 2 : (g4 == 2 ? 1 : g4); }

// Keep prefetch loads where they are written: without it the compiler sinks a
// next-tile global load down to its first use (the LDS store after the compute),
// which serialises its full latency into every loop iteration.
__device__ __forceinline__ void issue_fence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ bf16x8 ldsb8(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void stb4(__bf16* p, bf16x4 v) { *reinterpret_cast<bf16x4*>(p) = v; }

// Split-store a register-staged R x C f32 tile (stage_load order) into LDS hi/lo
// images of pitch P bf16.  PERM: apply perm16_group to the columns.
template <int R, int C, int P, bool PERM>
__device__ __forceinline__ void stage_store_split(const float4* v, __bf16* hi, __bf16* lo) {
  constexpr int C4 = C / 4, N = R * C4 / 256;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const int idx = threadIdx.x + 256 * k;
    const int row = idx / C4, c4 = idx % C4;
    const int col = PERM ? 16 * (c4 >> 2) + 4 * perm16_group(c4 & 3) : 4 * c4;
    bf16x4 a, b;
    split4(v[k], a, b);
    stb4(hi + row * P + col, a);
    stb4(lo + row * P + col, b);
  }
}

// GELU (approximate='none') and its derivative, branch-free, for the split
// path: Phi(-|x|) = erfc(z)/2 with z = |x|/sqrt(2) evaluated as
// t * exp(-z^2) * R(t), t = 1/(1 + z/2), R a degree-8 polynomial fitted to
// erfc(z) e^{z^2} / (2t) in relative error (fit 5e-8; f32 evaluation 2.5e-7
// relative on erfc).  exp(-z^2) = exp(-x^2/2) is shared with the derivative
// pdf term, so the pair costs one v_exp_f32 and one v_rcp_f32.  Against the
// float64 formula: |G err| <= 4e-7, |G' err| <= 2e-7 on [-12, 12]; torch's f32
// x/2 (1 + erf(x/sqrt 2)) is itself 1.2e-6 off (cancellation for x < -3).
__device__ __forceinline__ void gelu_fast(float x, float& g, float& d) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.f));
  float r = -0.02965068817138672f;
  r = fmaf(r, t, 0.14285887777805328f);
  r = fmaf(r, t, -0.24479423463344574f);
  r = fmaf(r, t, 0.1404150128364563f);
  r = fmaf(r, t, -0.014276500791311264f);
  r = fmaf(r, t, 0.10175687074661255f);
  r = fmaf(r, t, 0.12144583463668823f);
  r = fmaf(r, t, 0.14120244979858398f);
  r = fmaf(r, t, 0.14104235172271729f);
  const float e = __builtin_amdgcn_exp2f((x * x) * -0.72134752044448170368f);  // exp(-x^2/2)
  const float half = (t * e) * r;                                            // Phi(-|x|)
  const float phi = x >= 0.f ? 1.f - half : half;
  g = x * phi;
  d = phi + x * (e * 0.39894228040143267794f);
}
