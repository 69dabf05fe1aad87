// LayerNorm pieces shared by the token-parallel kernels (f32 and split paths).
// Reference: nn.LayerNorm(128) in models/model.py:740,748,772,784 (biased
// variance, eps inside the square root).
#pragma once
#include "ghm_common.h"

// Load one token row (row layout), LayerNorm it in place; returns stats.
__device__ __forceinline__ void ln_row(const float* __restrict__ row, const float* __restrict__ lnw,
                                       const float* __restrict__ lnb, int h, float eps, float* x,
                                       float& mean, float& rstd) {
  load64(row + 64 * h, x);
  ln_stats64(x, eps, mean, rstd);
  const float4* g4 = reinterpret_cast<const float4*>(lnw + 64 * h);
  const float4* b4 = reinterpret_cast<const float4*>(lnb + 64 * h);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float4 g = g4[q], b = b4[q];
    x[4 * q + 0] = (x[4 * q + 0] - mean) * rstd * g.x + b.x;
    x[4 * q + 1] = (x[4 * q + 1] - mean) * rstd * g.y + b.y;
    x[4 * q + 2] = (x[4 * q + 2] - mean) * rstd * g.z + b.z;
    x[4 * q + 3] = (x[4 * q + 3] - mean) * rstd * g.w + b.w;
  }
}

// LayerNorm backward for one token held in accumulator layout (feature
// f = 32*it + 8q + 4h + t for register 4q+t of tile it); dy = dL/d(LN output).
// Writes dH = dres + dx (float4 per quad) and, reduced over the wave's 32
// tokens, the (sum dy*xhat, sum dy) partials of dgamma/dbeta into red_g/red_b
// (LDS, indexed by feature).  gam: LN weight staged in LDS.
__device__ __forceinline__ void ln_bwd_acc(const f32x16* dy, const float* __restrict__ X,
                                           float2 st, const float* gam,
                                           const float* __restrict__ dres, float* __restrict__ dH,
                                           bool valid, int h, int j, float* red_g, float* red_b) {
  const float mean = st.x, rstd = st.y;
  float xh[64];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 32 * it + quad_off(q, h);
      const float4 xv = *reinterpret_cast<const float4*>(X + f);
      const float4 gv = lds4(gam + f);
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gs[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float xhat = (xs[t] - mean) * rstd;
        xh[16 * it + 4 * q + t] = xhat;
        const float dyg = dy[it][4 * q + t] * gs[t];
        s1 += dyg;
        s2 += dyg * xhat;
      }
    }
  }
  s1 += xhalf(s1);
  s2 += xhalf(s2);
  const float m1 = s1 * (1.f / GHM_D), m2 = s2 * (1.f / GHM_D);
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    float4 dr[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dr[q] = *reinterpret_cast<const float4*>(dres + 32 * it + quad_off(q, h));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 32 * it + quad_off(q, h);
      const float4 gv = lds4(gam + f);
      const float gs[4] = {gv.x, gv.y, gv.z, gv.w}, rs[4] = {dr[q].x, dr[q].y, dr[q].z, dr[q].w};
      float o[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float xhat = xh[16 * it + 4 * q + t];
        o[t] = rs[t] + rstd * (dy[it][4 * q + t] * gs[t] - m1 - xhat * m2);
      }
      if (valid) st4(dH + f, o[0], o[1], o[2], o[3]);
    }
  }
  // dgamma / dbeta partials over the wave's 32 tokens, 16 features at a time:
  // butterfly reduce-scatter, lane j ends with feature r = j >> 1 of the group
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    float vg[16], vb[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      vb[r] = valid ? dy[it][r] : 0.f;
      vg[r] = vb[r] * xh[16 * it + r];
    }
    const float sg = reduce_scatter16(vg, j);
    const float sb = reduce_scatter16(vb, j);
    if ((j & 1) == 0) {
      const int f = 32 * it + acc_row(j >> 1, h);
      red_g[f] = sg;
      red_b[f] = sb;
    }
  }
}

// Sum the 4 waves' LN partials (fixed order) and write the block's partial.
__device__ __forceinline__ void ln_partial_store(const float* red /*[2][4][128]*/, float* out) {
  const int f = threadIdx.x;
  if (f < GHM_D) {
    out[f] = (red[f] + red[GHM_D + f]) + (red[2 * GHM_D + f] + red[3 * GHM_D + f]);
    const float* rb = red + 4 * GHM_D;
    out[GHM_D + f] = (rb[f] + rb[GHM_D + f]) + (rb[2 * GHM_D + f] + rb[3 * GHM_D + f]);
  }
}

