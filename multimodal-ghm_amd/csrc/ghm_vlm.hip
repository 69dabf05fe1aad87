// Sequential VLM (next-word prediction, BASELINE config 5) on the device: the
// non-GEMM operators of AutoRegressiveTransformer (d = 256, T = 1 image + 80 text
// tokens), generic in the width D.  The VLM's plain projections (QKV, MLP, readout)
// are library GEMMs on the host side (models/vlm.py); everything between them —
// embedding, LayerNorm, masked double-residual attention, GELU, loss — runs here.
// Reference (src/ghmclip/):
//   generate_mask                 models/model.py:24-33
//   token_embeddings (sequential) models/model.py:274-293
//   layer loop                    models/model.py:301-347 (mask, 1/sqrt(d), softmax,
//                                 H += A V, A /= d, H += A V, LN, MLP)
//   readout                       models/model.py:397-401
//   ConditionalGuidedCELoss       models/model.py:1087-1098 (guide=False)
//   KLdiv                         models/model.py:1067-1078
#include "ghm_common.h"
#include "ghm_launch.h"

constexpr int VA_T = 96;       // padded sequence length of the attention kernels
constexpr int VA_TP = VA_T + 1;  // LDS pitch of the 96 x 96 probability tile
constexpr int VA_KC = 32;      // feature chunk of the score products
constexpr int VA_VC = 64;      // feature chunk of the value products

// H0[n, t, :] = e(n, t) + pos[t, :]: prefix token t < P gets the image feature
// feat[n, t, 0:V] (zero-padded to D, :281-286), text token t >= P the embedding
// tok_w[xt[n, t - P]] (:292).  onehot (optional) [n*T + t][V] = 1 at the text
// token's value (the deterministic token-embedding gradient is onehot^T dH0).
__global__ __launch_bounds__(256) void k_vlm_embed_fwd(const uint8_t* __restrict__ xt, const float* __restrict__ feat,
                                                       const float* __restrict__ tok_w, const float* __restrict__ pos,
                                                       float* __restrict__ H0, float* __restrict__ onehot, int64_t n_tok,
                                                       int T, int P, int V, int D) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int D4 = D / 4;
  if (idx >= n_tok * D4) return;
  const int q = static_cast<int>(idx % D4);
  const int64_t m = idx / D4;
  const int64_t n = m / T;
  const int t = static_cast<int>(m % T);
  const float4 p = *reinterpret_cast<const float4*>(pos + static_cast<int64_t>(t) * D + 4 * q);
  float e[4];
  if (t < P) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int d = 4 * q + k;
      e[k] = d < V ? feat[(n * P + t) * V + d] : 0.f;
    }
  } else {
    int x = xt[n * (T - P) + (t - P)];
    x = x < V ? x : V - 1;
    const float4 w = *reinterpret_cast<const float4*>(tok_w + static_cast<int64_t>(x) * D + 4 * q);
    e[0] = w.x; e[1] = w.y; e[2] = w.z; e[3] = w.w;
  }
  st4(H0 + m * D + 4 * q, e[0] + p.x, e[1] + p.y, e[2] + p.z, e[3] + p.w);
  if (onehot && q < V) {
    const int x = t < P ? -1 : static_cast<int>(xt[n * (T - P) + (t - P)]);
    onehot[m * V + q] = (x == q) ? 1.f : 0.f;
  }
}

// Joint VLM embedding (AutoRegressiveTransformer, sequential=False, model.py:221-232):
// prefix (image) token t < P gets i_w[it[n, t]], text token t >= P gets
// tok_w[xt[n, t - P]]; + positions.  onehot_t / onehot_i (may be NULL) [M][V]: the
// text / image tokens' one-hot rows (0 on the other kind), for the two embedding
// gradients.
__global__ __launch_bounds__(256) void k_vlm_embed_joint_fwd(const uint8_t* __restrict__ xt,
                                                             const uint8_t* __restrict__ it,
                                                             const float* __restrict__ i_w,
                                                             const float* __restrict__ tok_w,
                                                             const float* __restrict__ pos, float* __restrict__ H0,
                                                             float* __restrict__ onehot_t,
                                                             float* __restrict__ onehot_i, int64_t n_tok, int T,
                                                             int P, int V, int D) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int D4 = D / 4;
  if (idx >= n_tok * D4) return;
  const int q = static_cast<int>(idx % D4);
  const int64_t m = idx / D4;
  const int64_t n = m / T;
  const int t = static_cast<int>(m % T);
  const float4 p = *reinterpret_cast<const float4*>(pos + static_cast<int64_t>(t) * D + 4 * q);
  const bool pre = t < P;
  int x = pre ? it[n * P + t] : xt[n * (T - P) + (t - P)];
  x = x < V ? x : V - 1;
  const float4 w = *reinterpret_cast<const float4*>((pre ? i_w : tok_w) + static_cast<int64_t>(x) * D + 4 * q);
  st4(H0 + m * D + 4 * q, w.x + p.x, w.y + p.y, w.z + p.z, w.w + p.w);
  if (q < V) {
    if (onehot_t) onehot_t[m * V + q] = (!pre && x == q) ? 1.f : 0.f;
    if (onehot_i) onehot_i[m * V + q] = (pre && x == q) ? 1.f : 0.f;
  }
}

// ---------------------------------------------------------------------------
// Row LayerNorm, one wave per row (D = 64 * R), two-pass statistics like
// nn.LayerNorm (biased variance, eps inside the sqrt).
// ---------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(256) void k_ln_rows_fwd(const float* __restrict__ X, const float* __restrict__ w,
                                                     const float* __restrict__ b, float* __restrict__ Y,
                                                     float2* __restrict__ stats, int64_t M, float eps) {
  constexpr int D = 64 * R;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* x = X + row * D;
  float v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = x[lane + 64 * r];
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) s += v[r];
  s = sum32(s);
  s += xhalf(s);
  const float mean = s / static_cast<float>(D);
  float q = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float d = v[r] - mean;
    q += d * d;
  }
  q = sum32(q);
  q += xhalf(q);
  const float rstd = 1.f / sqrtf(q / static_cast<float>(D) + eps);
  if (lane == 0) stats[row] = make_float2(mean, rstd);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int c = lane + 64 * r;
    Y[row * D + c] = (v[r] - mean) * rstd * w[c] + b[c];
  }
}

// dX = dres + LN backward of dY (dres may alias dX); per-workgroup partials of
// dgamma = sum dY * xhat and dbeta = sum dY over the workgroup's rows in fixed
// order: part [n_blocks][2][D], n_blocks = ceil(M / (4 * LN_ROWS_PER_WAVE)).
// 4 rows per wave (648 workgroups at M = 10,368): the backward 11.0 -> 9.0 us
// against 8 (324 workgroups, 1.3 waves per SIMD), 2 no better (profiles/r5_rpw_ab.txt)
#ifndef GHM_LN_RPW
#define GHM_LN_RPW 4
#endif
constexpr int LN_ROWS_PER_WAVE = GHM_LN_RPW;
template <int R>
__global__ __launch_bounds__(256) void k_ln_rows_bwd(const float* __restrict__ dY, const float* __restrict__ X,
                                                     const float2* __restrict__ stats, const float* __restrict__ w,
                                                     const float* dres, float* dX, float* __restrict__ part,
                                                     int64_t M) {
  constexpr int D = 64 * R;
  __shared__ float red[4][2][D];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float gacc[R], bacc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) gacc[r] = bacc[r] = 0.f;
  // rows in batches of LN_BATCH whose loads are all issued before the first
  // row's reductions (one row at a time was load-latency bound: 18 us at M = 10,368)
  constexpr int LN_BATCH = (R <= 4 ? 4 : 2) < LN_ROWS_PER_WAVE ? (R <= 4 ? 4 : 2) : LN_ROWS_PER_WAVE;
  for (int k0 = 0; k0 < LN_ROWS_PER_WAVE; k0 += LN_BATCH) {
    const int64_t row0 = (static_cast<int64_t>(blockIdx.x) * 4 + wv) * LN_ROWS_PER_WAVE + k0;
    if (row0 >= M) break;
    float dyv[LN_BATCH][R], xv[LN_BATCH][R], rv[LN_BATCH][R];
    float2 stv[LN_BATCH];
#pragma unroll
    for (int b = 0; b < LN_BATCH; ++b) {
      const int64_t row = row0 + b < M ? row0 + b : M - 1;  // clamped (unused past M)
      stv[b] = ld_stats_sys(stats, row);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int c = lane + 64 * r;
        dyv[b][r] = dY[row * D + c];
        xv[b][r] = X[row * D + c];
        rv[b][r] = dres[row * D + c];
      }
    }
#pragma unroll
    for (int b = 0; b < LN_BATCH; ++b) {
      const int64_t row = row0 + b;
      if (row >= M) break;
      const float2 st = stv[b];
      float xh[R], g[R];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int c = lane + 64 * r;
        const float dy = dyv[b][r];
        xh[r] = (xv[b][r] - st.x) * st.y;
        g[r] = dy * w[c];
        s1 += g[r];
        s2 += g[r] * xh[r];
        gacc[r] += dy * xh[r];
        bacc[r] += dy;
      }
      s1 = sum32(s1);
      s1 += xhalf(s1);
      s2 = sum32(s2);
      s2 += xhalf(s2);
      const float m1 = s1 / static_cast<float>(D), m2 = s2 / static_cast<float>(D);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int c = lane + 64 * r;
        const float d = st.y * (g[r] - m1 - xh[r] * m2);
        dX[row * D + c] = rv[b][r] + d;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    red[wv][0][lane + 64 * r] = gacc[r];
    red[wv][1][lane + 64 * r] = bacc[r];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * D; i += 256) {
    const int which = i / D, c = i % D;
    part[static_cast<int64_t>(blockIdx.x) * 2 * D + i] =
        (red[0][which][c] + red[1][which][c]) + (red[2][which][c] + red[3][which][c]);
  }
}

// The same two kernels for D = 256 J with one float4 per lane and 256-column block
// (lane owns columns 256 j + 4 lane .. + 3): a row moves in J 1 KB loads per
// tensor instead of 4 J 256-byte ones.  Same statistics (two-pass, biased
// variance), summed in a different order.  Measured at par with the scalar form
// (VLM: fwd 6.6 -> 6.8, bwd 11.4 -> 11.0 us, profiles/r5_lnv_ab.txt): the access
// width was not what bounds them; the backward's grid was (GHM_LN_RPW below).
template <int J>
__global__ __launch_bounds__(256) void k_ln_rows_fwd_v4(const float* __restrict__ X, const float* __restrict__ w,
                                                        const float* __restrict__ b, float* __restrict__ Y,
                                                        float2* __restrict__ stats, int64_t M, float eps) {
  constexpr int D = 256 * J;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float4 v[J];
#pragma unroll
  for (int j = 0; j < J; ++j) v[j] = *reinterpret_cast<const float4*>(X + row * D + 256 * j + 4 * lane);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  s = sum32(s);
  s += xhalf(s);
  const float mean = s / static_cast<float>(D);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const float a = v[j].x - mean, bb = v[j].y - mean, c = v[j].z - mean, d = v[j].w - mean;
    q += (a * a + bb * bb) + (c * c + d * d);
  }
  q = sum32(q);
  q += xhalf(q);
  const float rstd = 1.f / sqrtf(q / static_cast<float>(D) + eps);
  if (lane == 0) stats[row] = make_float2(mean, rstd);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int c = 256 * j + 4 * lane;
    const float4 wv = *reinterpret_cast<const float4*>(w + c), bv = *reinterpret_cast<const float4*>(b + c);
    st4(Y + row * D + c, (v[j].x - mean) * rstd * wv.x + bv.x, (v[j].y - mean) * rstd * wv.y + bv.y,
        (v[j].z - mean) * rstd * wv.z + bv.z, (v[j].w - mean) * rstd * wv.w + bv.w);
  }
}

template <int J>
__global__ __launch_bounds__(256) void k_ln_rows_bwd_v4(const float* __restrict__ dY, const float* __restrict__ X,
                                                        const float2* __restrict__ stats, const float* __restrict__ w,
                                                        const float* dres, float* dX, float* __restrict__ part,
                                                        int64_t M) {
  constexpr int D = 256 * J;
  __shared__ float4 red[4][2][D / 4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float4 gacc[J], bacc[J], wj[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    gacc[j] = bacc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    wj[j] = *reinterpret_cast<const float4*>(w + 256 * j + 4 * lane);
  }
  constexpr int LN_BATCH = LN_ROWS_PER_WAVE < 4 ? LN_ROWS_PER_WAVE : 4;
  for (int k0 = 0; k0 < LN_ROWS_PER_WAVE; k0 += LN_BATCH) {
    const int64_t row0 = (static_cast<int64_t>(blockIdx.x) * 4 + wv) * LN_ROWS_PER_WAVE + k0;
    if (row0 >= M) break;
    float4 dyv[LN_BATCH][J], xv[LN_BATCH][J], rv[LN_BATCH][J];
    float2 stv[LN_BATCH];
#pragma unroll
    for (int b = 0; b < LN_BATCH; ++b) {
      const int64_t row = row0 + b < M ? row0 + b : M - 1;  // clamped (unused past M)
      stv[b] = ld_stats_sys(stats, row);
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int64_t o = row * D + 256 * j + 4 * lane;
        dyv[b][j] = *reinterpret_cast<const float4*>(dY + o);
        xv[b][j] = *reinterpret_cast<const float4*>(X + o);
        rv[b][j] = *reinterpret_cast<const float4*>(dres + o);
      }
    }
#pragma unroll
    for (int b = 0; b < LN_BATCH; ++b) {
      const int64_t row = row0 + b;
      if (row >= M) break;
      const float2 st = stv[b];
      float xh[J][4], g[J][4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const float dy[4] = {dyv[b][j].x, dyv[b][j].y, dyv[b][j].z, dyv[b][j].w};
        const float xx[4] = {xv[b][j].x, xv[b][j].y, xv[b][j].z, xv[b][j].w};
        const float ww[4] = {wj[j].x, wj[j].y, wj[j].z, wj[j].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[j][e] = (xx[e] - st.x) * st.y;
          g[j][e] = dy[e] * ww[e];
          s1 += g[j][e];
          s2 += g[j][e] * xh[j][e];
        }
        gacc[j].x += dy[0] * xh[j][0]; gacc[j].y += dy[1] * xh[j][1];
        gacc[j].z += dy[2] * xh[j][2]; gacc[j].w += dy[3] * xh[j][3];
        bacc[j].x += dy[0]; bacc[j].y += dy[1]; bacc[j].z += dy[2]; bacc[j].w += dy[3];
      }
      s1 = sum32(s1);
      s1 += xhalf(s1);
      s2 = sum32(s2);
      s2 += xhalf(s2);
      const float m1 = s1 / static_cast<float>(D), m2 = s2 / static_cast<float>(D);
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const float4 r = rv[b][j];
        st4(dX + row * D + 256 * j + 4 * lane, r.x + st.y * (g[j][0] - m1 - xh[j][0] * m2),
            r.y + st.y * (g[j][1] - m1 - xh[j][1] * m2), r.z + st.y * (g[j][2] - m1 - xh[j][2] * m2),
            r.w + st.y * (g[j][3] - m1 - xh[j][3] * m2));
      }
    }
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    red[wv][0][64 * j + lane] = gacc[j];
    red[wv][1][64 * j + lane] = bacc[j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * D / 4; i += 256) {
    const int which = i / (D / 4), c4 = i % (D / 4);
    const float4 a = red[0][which][c4], b = red[1][which][c4], c = red[2][which][c4], d = red[3][which][c4];
    st4(part + static_cast<int64_t>(blockIdx.x) * 2 * D + which * D + 4 * c4, (a.x + b.x) + (c.x + d.x),
        (a.y + b.y) + (c.y + d.y), (a.z + b.z) + (c.z + d.z), (a.w + b.w) + (c.w + d.w));
  }
}

// GHM_LN_VEC = 0: the one-float-per-lane kernels for every D (A/B knob, read per call)
static bool ln_vec() {
  const char* e = getenv("GHM_LN_VEC");
  return !(e && atoi(e) == 0);
}

// ---------------------------------------------------------------------------
// Masked double-residual attention, one 256-thread workgroup per sequence.
// Thread (ty, tx) = (t >> 4, t & 15) owns rows 6ty..6ty+5 and columns
// 6tx..6tx+5 of the 96 x 96 score tile; feature chunks are staged in LDS.
// allowed(i, j): both in the prefix, or i a text token and j <= i (:24-33).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool va_allowed(int i, int j, int P) { return (i < P) ? (j < P) : (j <= i); }

// acc[6][6] += A[rows][c0:c0+D] . B[cols][c0:c0+D] over all D, both [T][ld] global
// row-major (rows >= T read as 0), through LDS chunks sa / sb [96][VA_KC + 1].
__device__ __forceinline__ void va_scores(const float* __restrict__ A, const float* __restrict__ Bm, int ld, int T,
                                          int D, float* sa, float* sb, float (&acc)[6][6]) {
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) acc[a][b] = 0.f;
  for (int c0 = 0; c0 < D; c0 += VA_KC) {
    for (int i = threadIdx.x; i < VA_T * VA_KC; i += 256) {
      const int r = i / VA_KC, c = i % VA_KC;
      sa[r * (VA_KC + 1) + c] = r < T ? A[static_cast<int64_t>(r) * ld + c0 + c] : 0.f;
      sb[r * (VA_KC + 1) + c] = r < T ? Bm[static_cast<int64_t>(r) * ld + c0 + c] : 0.f;
    }
    __syncthreads();
    for (int kk = 0; kk < VA_KC; ++kk) {
      float av[6], bv[6];
#pragma unroll
      for (int a = 0; a < 6; ++a) av[a] = sa[(6 * ty + a) * (VA_KC + 1) + kk];
#pragma unroll
      for (int b = 0; b < 6; ++b) bv[b] = sb[(6 * tx + b) * (VA_KC + 1) + kk];
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < 6; ++b) acc[a][b] = fmaf(av[a], bv[b], acc[a][b]);
    }
    __syncthreads();
  }
}

// out[r][c] = sum_j W(r, j) X[j][c] for the 96 x D output, W from the LDS tile
// sw (row-major [96][VA_TP], or transposed when TRANS), X [T][ld] global staged in
// chunks sx [96][VA_VC]; thread (ty, tx): rows 6ty.., columns 4tx.. of a chunk.
// Calls epi(r, c, value) for rows r < T.
template <bool TRANS, class Epi>
__device__ __forceinline__ void va_apply(const float* sw, const float* __restrict__ X, int ld, int T, int D,
                                         float* sx, Epi epi) {
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
  for (int c0 = 0; c0 < D; c0 += VA_VC) {
    for (int i = threadIdx.x; i < VA_T * VA_VC; i += 256) {
      const int r = i / VA_VC, c = i % VA_VC;
      sx[i] = r < T ? X[static_cast<int64_t>(r) * ld + c0 + c] : 0.f;
    }
    __syncthreads();
    float acc[6][4];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
    for (int j = 0; j < T; ++j) {
      float wv[6];
#pragma unroll
      for (int a = 0; a < 6; ++a) wv[a] = TRANS ? sw[j * VA_TP + 6 * ty + a] : sw[(6 * ty + a) * VA_TP + j];
      const float4 xv = *reinterpret_cast<const float4*>(sx + j * VA_VC + 4 * tx);
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        acc[a][0] = fmaf(wv[a], xv.x, acc[a][0]);
        acc[a][1] = fmaf(wv[a], xv.y, acc[a][1]);
        acc[a][2] = fmaf(wv[a], xv.z, acc[a][2]);
        acc[a][3] = fmaf(wv[a], xv.w, acc[a][3]);
      }
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const int r = 6 * ty + a;
      if (r < T) {
#pragma unroll
        for (int b = 0; b < 4; ++b) epi(r, c0 + 4 * tx + b, acc[a][b]);
      }
    }
    __syncthreads();
  }
}

// Hmid = H + A V + (A / D) V = (H + O) + O / D, A = softmax((Q K^T + mask) / scale_div);
// P [n][96][96] saved (rows >= T and masked / padded keys 0).
__global__ __launch_bounds__(256) void k_vlm_attn_fwd(const float* __restrict__ q, const float* __restrict__ k,
                                                      const float* __restrict__ v, const float* __restrict__ H,
                                                      float* __restrict__ Hmid, float* __restrict__ Pg, int T, int D,
                                                      int P, float scale_div, float dbl) {
  __shared__ float sp[VA_T * VA_TP];
  __shared__ float stage[2 * VA_T * (VA_KC + 1)];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
  float acc[6][6];
  va_scores(q + base * D, k + base * D, D, T, D, stage, stage + VA_T * (VA_KC + 1), acc);
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int i = 6 * ty + a, j = 6 * tx + b;
      // (Q K^T + mask) / scale_div, mask = -inf where not allowed (:329-336)
      sp[i * VA_TP + j] = (i < T && j < T && va_allowed(i, j, P)) ? acc[a][b] / scale_div : -INFINITY;
    }
  __syncthreads();
  {  // row softmax: wave w takes rows w, w+4, ...; lanes over keys
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x >> 6; i < VA_T; i += 4) {
      float* row = sp + i * VA_TP;
      float* prow = Pg + (static_cast<int64_t>(blockIdx.x) * VA_T + i) * VA_T;
      if (i >= T) {
        for (int j = lane; j < VA_T; j += 64) {
          row[j] = 0.f;
          prow[j] = 0.f;
        }
        continue;
      }
      const float x0 = row[lane], x1 = lane + 64 < VA_T ? row[lane + 64] : -INFINITY;
      float mx = fmaxf(x0, x1);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      const float e0 = expf(x0 - mx), e1 = expf(x1 - mx);
      float sm = e0 + e1;
      sm = sum32(sm);
      sm += xhalf(sm);
      const float p0 = e0 / sm, p1 = e1 / sm;
      row[lane] = p0;
      prow[lane] = p0;
      if (lane + 64 < VA_T) {
        row[lane + 64] = p1;
        prow[lane + 64] = p1;
      }
    }
  }
  __syncthreads();
  const float* vs = v + base * D;
  const float* hs = H + base * D;
  float* os = Hmid + base * D;
  va_apply<false>(sp, vs, D, T, D, stage, [&](int r, int c, float o) {
    const int64_t i = static_cast<int64_t>(r) * D + c;
    os[i] = (hs[i] + o) + o * dbl;  // :338-341
  });
}

// Backward of k_vlm_attn_fwd given dHmid (= dL/dH after attention; the residual
// path dH += dHmid is the caller's):
//   dV = A^T dHmid (1 + 1/D);  dA = (dHmid V^T)(1 + 1/D);
//   dS = A o (dA - rowsum(dA o A)) / scale_div;  dQ = dS K;  dK = dS^T Q.
__global__ __launch_bounds__(256) void k_vlm_attn_bwd(const float* __restrict__ q, const float* __restrict__ k,
                                                      const float* __restrict__ v, const float* __restrict__ Pg,
                                                      const float* __restrict__ dHmid, float* __restrict__ dq,
                                                      float* __restrict__ dk, float* __restrict__ dv, int T, int D,
                                                      float scale_div, float dbl) {
  __shared__ float sp[VA_T * VA_TP];
  __shared__ float stage[2 * VA_T * (VA_KC + 1)];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
  const float* pg = Pg + static_cast<int64_t>(blockIdx.x) * VA_T * VA_T;
  for (int i = threadIdx.x; i < VA_T * VA_T; i += 256) sp[(i / VA_T) * VA_TP + (i % VA_T)] = pg[i];
  __syncthreads();
  const float* dh = dHmid + base * D;
  float* dvs = dv + base * D;
  // dV[j][c] = sum_i P[i][j] dH[i][c] (+ the A/D branch)
  va_apply<true>(sp, dh, D, T, D, stage, [&](int r, int c, float o) {
    dvs[static_cast<int64_t>(r) * D + c] = o + o * dbl;
  });
  float g[6][6];
  va_scores(dh, v + base * D, D, T, D, stage, stage + VA_T * (VA_KC + 1), g);
  // rowsum(dA o P) per query row: 16 column-group partials per row through LDS
  float* rs = stage;  // [96][16]
  float pv[6][6];
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float s = 0.f;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      pv[a][b] = sp[(6 * ty + a) * VA_TP + 6 * tx + b];
      g[a][b] = g[a][b] + g[a][b] * dbl;
      s += g[a][b] * pv[a][b];
    }
    rs[(6 * ty + a) * 16 + tx] = s;
  }
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    const int i = 6 * ty + a;
    float s = 0.f;
    for (int u = 0; u < 16; ++u) s += rs[i * 16 + u];
#pragma unroll
    for (int b = 0; b < 6; ++b) sp[i * VA_TP + 6 * tx + b] = pv[a][b] * (g[a][b] - s) / scale_div;
  }
  __syncthreads();
  float* dqs = dq + base * D;
  float* dks = dk + base * D;
  va_apply<false>(sp, k + base * D, D, T, D, stage, [&](int r, int c, float o) {
    dqs[static_cast<int64_t>(r) * D + c] = o;
  });
  va_apply<true>(sp, q + base * D, D, T, D, stage, [&](int r, int c, float o) {
    dks[static_cast<int64_t>(r) * D + c] = o;
  });
}

// ---------------------------------------------------------------------------
// Elementwise: G = GELU(U), Dg = GELU'(U) (exact erf form, as nn.GELU and its
// backward); out = a * b; out = a + b.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gelu_fwd(const float* __restrict__ U, float* __restrict__ G,
                                                  float* __restrict__ Dg, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  float g, d;
  gelu_and_grad(U[i], g, d);
  G[i] = g;
  Dg[i] = d;
}

// (out may alias a or b: no __restrict__)
__global__ __launch_bounds__(256) void k_mul(const float* a, const float* b, float* out, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) out[i] = a[i] * b[i];
}

__global__ __launch_bounds__(256) void k_add(const float* a, const float* b, float* out, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

// ---------------------------------------------------------------------------
// Next-token cross entropy and the KL "Compare" over the text rows t >= P of
// logits [n][T][V] (targets [n][T - P], post [n][T - P][V]):
//   loss = mean over rows of (lse - logit[target]) (per-sample means of equal
//   length averaged = the mean over all rows, :1092-1098);
//   compare = sum_rows sum_v p (log p - log_softmax) / rows (batchmean, p = 0 -> 0);
//   dlogits = (softmax - onehot) / rows on text rows, 0 on prefix rows.
// Two launches, fixed reduction order (k_ce_kl_rows / k_ce_kl_final below).
// ---------------------------------------------------------------------------
constexpr int CE_THREADS = 256;
constexpr int CE_ROWS_PER_BLOCK = 256;  // text rows per workgroup (one per thread)

// Stage 1: each workgroup takes CE_ROWS_PER_BLOCK consecutive text rows (one row
// per thread in turn), writes their dlogits and one (loss, KL) partial per
// workgroup, reduced in a fixed tree; stage 2 sums the partials in order.  (The
// one-workgroup version took 141 us at 10,240 rows.)
__global__ __launch_bounds__(CE_THREADS) void k_ce_kl_rows(const float* __restrict__ logits,
                                                           const uint8_t* __restrict__ targets,
                                                           const float* __restrict__ post,
                                                           float* __restrict__ dlogits, float* __restrict__ part,
                                                           int N, int T, int P, int V) {
  __shared__ float red[2][CE_THREADS];
  const int64_t rows = static_cast<int64_t>(N) * (T - P);
  const float inv = 1.f / static_cast<float>(rows);
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * CE_ROWS_PER_BLOCK;
  const int64_t r1 = r0 + CE_ROWS_PER_BLOCK < rows ? r0 + CE_ROWS_PER_BLOCK : rows;
  float sl = 0.f, sc = 0.f;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += CE_THREADS) {
    const int64_t n = r / (T - P);
    const int t = static_cast<int>(r % (T - P)) + P;
    const float* z = logits + (n * T + t) * V;
    float mx = z[0];
    for (int c = 1; c < V; ++c) mx = fmaxf(mx, z[c]);
    float se = 0.f;
    for (int c = 0; c < V; ++c) se += expf(z[c] - mx);
    const float lse = mx + logf(se);
    const int y = targets[r];
    sl += lse - z[y];
    if (post) {
      const float* pp = post + r * V;
      float kl = 0.f;
      for (int c = 0; c < V; ++c)
        if (pp[c] > 0.f) kl += pp[c] * (logf(pp[c]) - (z[c] - lse));
      sc += kl;
    }
    if (dlogits) {
      float* dz = dlogits + (n * T + t) * V;
      for (int c = 0; c < V; ++c) dz[c] = (expf(z[c] - lse) - (c == y ? 1.f : 0.f)) * inv;
    }
  }
  red[0][threadIdx.x] = sl;
  red[1][threadIdx.x] = sc;
  __syncthreads();
  for (int s = CE_THREADS / 2; s >= 1; s >>= 1) {
    if (threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = red[0][0];
    part[2 * blockIdx.x + 1] = red[1][0];
  }
  if (dlogits && P > 0) {  // prefix rows carry no loss: this workgroup's share of them
    const int64_t nz = static_cast<int64_t>(N) * P * V;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * CE_THREADS + threadIdx.x; i < nz;
         i += static_cast<int64_t>(gridDim.x) * CE_THREADS) {
      const int64_t n = i / (P * V), rem = i % (P * V);
      dlogits[n * T * V + rem] = 0.f;
    }
  }
}

__global__ __launch_bounds__(64) void k_ce_kl_final(const float* __restrict__ part, int nblk, int64_t rows,
                                                    float* __restrict__ loss_out, float* __restrict__ hist,
                                                    float* __restrict__ chist, const int32_t* __restrict__ step) {
  if (threadIdx.x != 0) return;
  const float inv = 1.f / static_cast<float>(rows);
  float l = 0.f, c = 0.f;
  for (int b = 0; b < nblk; ++b) {
    l += part[2 * b];
    c += part[2 * b + 1];
  }
  l *= inv;
  c *= inv;
  loss_out[0] = l;
  loss_out[1] = c;
  if (hist && step) hist[*step] = l;
  if (chist && step) chist[*step] = c;
}

// ---------------------------------------------------------------------------
// C-ABI launchers
// ---------------------------------------------------------------------------
extern "C" int ghm_vlm_embed_fwd(const uint8_t* xt, const float* feat, const float* tok_w, const float* pos_w,
                                 float* H0, float* onehot, int64_t n_seq, int T, int P, int V, int D, void* stream) {
  GHM_CHECK(xt && feat && tok_w && pos_w && H0, "null pointer");
  GHM_CHECK(n_seq >= 1 && T > P && P >= 1 && V >= 1 && V <= D && D % 4 == 0 && D >= 4 * V, "shape");
  const int64_t n = n_seq * T * (D / 4);
  hipLaunchKernelGGL(k_vlm_embed_fwd, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, ghm_stream(stream),
                     xt, feat, tok_w, pos_w, H0, onehot, n_seq * T, T, P, V, D);
  return ghm_launch_status();
}

extern "C" int ghm_vlm_embed_joint_fwd(const uint8_t* xt, const uint8_t* it, const float* i_w, const float* tok_w,
                                       const float* pos_w, float* H0, float* onehot_t, float* onehot_i, int64_t n_seq,
                                       int T, int P, int V, int D, void* stream) {
  GHM_CHECK(xt && it && i_w && tok_w && pos_w && H0, "null pointer");
  GHM_CHECK(n_seq >= 1 && T > P && P >= 1 && V >= 1 && D % 4 == 0 && D >= 4 * V, "shape");
  const int64_t n = n_seq * T * (D / 4);
  hipLaunchKernelGGL(k_vlm_embed_joint_fwd, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     ghm_stream(stream), xt, it, i_w, tok_w, pos_w, H0, onehot_t, onehot_i, n_seq * T, T, P, V, D);
  return ghm_launch_status();
}

extern "C" int ghm_ln_rows_fwd(const float* X, const float* w, const float* b, float* Y, float* stats, int64_t M,
                               int D, float eps, void* stream) {
  GHM_CHECK(X && w && b && Y && stats, "null pointer");
  GHM_CHECK(M >= 1 && (D == 64 || D == 128 || D == 256 || D == 512), "shape (D in {64, 128, 256, 512})");
  const dim3 g(static_cast<unsigned>((M + 3) / 4));
  float2* st = reinterpret_cast<float2*>(stats);
  hipStream_t s = ghm_stream(stream);
  if (D == 64) hipLaunchKernelGGL(k_ln_rows_fwd<1>, g, dim3(256), 0, s, X, w, b, Y, st, M, eps);
  else if (D == 128) hipLaunchKernelGGL(k_ln_rows_fwd<2>, g, dim3(256), 0, s, X, w, b, Y, st, M, eps);
  else if (ln_vec() && D == 256) hipLaunchKernelGGL(k_ln_rows_fwd_v4<1>, g, dim3(256), 0, s, X, w, b, Y, st, M, eps);
  else if (ln_vec()) hipLaunchKernelGGL(k_ln_rows_fwd_v4<2>, g, dim3(256), 0, s, X, w, b, Y, st, M, eps);
  else if (D == 256) hipLaunchKernelGGL(k_ln_rows_fwd<4>, g, dim3(256), 0, s, X, w, b, Y, st, M, eps);
  else hipLaunchKernelGGL(k_ln_rows_fwd<8>, g, dim3(256), 0, s, X, w, b, Y, st, M, eps);
  return ghm_launch_status();
}

extern "C" int64_t ghm_ln_rows_blocks(int64_t M) { return (M + 4 * LN_ROWS_PER_WAVE - 1) / (4 * LN_ROWS_PER_WAVE); }

extern "C" int ghm_ln_rows_bwd(const float* dY, const float* X, const float* stats, const float* w, const float* dres,
                               float* dX, float* part, int64_t M, int D, void* stream) {
  GHM_CHECK(dY && X && stats && w && dres && dX && part, "null pointer");
  GHM_CHECK(M < (int64_t(1) << 28), "stats byte offsets must fit 31 bits (M < 2^28 tokens)");
  GHM_CHECK(M >= 1 && (D == 64 || D == 128 || D == 256 || D == 512), "shape (D in {64, 128, 256, 512})");
  const dim3 g(static_cast<unsigned>(ghm_ln_rows_blocks(M)));
  const float2* st = reinterpret_cast<const float2*>(stats);
  hipStream_t s = ghm_stream(stream);
  if (D == 64) hipLaunchKernelGGL(k_ln_rows_bwd<1>, g, dim3(256), 0, s, dY, X, st, w, dres, dX, part, M);
  else if (D == 128) hipLaunchKernelGGL(k_ln_rows_bwd<2>, g, dim3(256), 0, s, dY, X, st, w, dres, dX, part, M);
  else if (ln_vec() && D == 256)
    hipLaunchKernelGGL(k_ln_rows_bwd_v4<1>, g, dim3(256), 0, s, dY, X, st, w, dres, dX, part, M);
  else if (ln_vec()) hipLaunchKernelGGL(k_ln_rows_bwd_v4<2>, g, dim3(256), 0, s, dY, X, st, w, dres, dX, part, M);
  else if (D == 256) hipLaunchKernelGGL(k_ln_rows_bwd<4>, g, dim3(256), 0, s, dY, X, st, w, dres, dX, part, M);
  else hipLaunchKernelGGL(k_ln_rows_bwd<8>, g, dim3(256), 0, s, dY, X, st, w, dres, dX, part, M);
  return ghm_launch_status();
}

extern "C" int ghm_vlm_attn_fwd(const float* q, const float* k, const float* v, const float* H, float* H_mid, float* P,
                                int64_t n_seq, int T, int D, int n_prefix, float scale_div, void* stream) {
  GHM_CHECK(q && k && v && H && H_mid && P, "null pointer");
  GHM_CHECK(n_seq >= 1 && T >= 2 && T <= VA_T && D % VA_VC == 0 && D >= VA_VC && n_prefix >= 1 && n_prefix < T,
            "shape (T <= 96, D % 64 == 0)");
  hipLaunchKernelGGL(k_vlm_attn_fwd, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, ghm_stream(stream), q, k, v, H,
                     H_mid, P, T, D, n_prefix, scale_div, 1.f / static_cast<float>(D));
  return ghm_launch_status();
}

extern "C" int ghm_vlm_attn_bwd(const float* q, const float* k, const float* v, const float* P, const float* dH_mid,
                                float* dq, float* dk, float* dv, int64_t n_seq, int T, int D, float scale_div,
                                void* stream) {
  GHM_CHECK(q && k && v && P && dH_mid && dq && dk && dv, "null pointer");
  GHM_CHECK(n_seq >= 1 && T >= 2 && T <= VA_T && D % VA_VC == 0 && D >= VA_VC, "shape (T <= 96, D % 64 == 0)");
  hipLaunchKernelGGL(k_vlm_attn_bwd, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, ghm_stream(stream), q, k, v, P,
                     dH_mid, dq, dk, dv, T, D, scale_div, 1.f / static_cast<float>(D));
  return ghm_launch_status();
}

extern "C" int ghm_gelu_fwd(const float* U, float* G, float* Dg, int64_t n, void* stream) {
  GHM_CHECK(U && G && Dg && n >= 1, "bad arguments");
  hipLaunchKernelGGL(k_gelu_fwd, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, ghm_stream(stream), U, G,
                     Dg, n);
  return ghm_launch_status();
}

extern "C" int ghm_mul(const float* a, const float* b, float* out, int64_t n, void* stream) {
  GHM_CHECK(a && b && out && n >= 1, "bad arguments");
  hipLaunchKernelGGL(k_mul, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, ghm_stream(stream), a, b, out,
                     n);
  return ghm_launch_status();
}

extern "C" int ghm_add(const float* a, const float* b, float* out, int64_t n, void* stream) {
  GHM_CHECK(a && b && out && n >= 1, "bad arguments");
  hipLaunchKernelGGL(k_add, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, ghm_stream(stream), a, b, out,
                     n);
  return ghm_launch_status();
}

extern "C" int64_t ghm_ce_kl_out_elems(int64_t n_seq, int T, int n_prefix) {
  const int64_t rows = n_seq * (T - n_prefix);
  return 2 + 2 * ((rows + CE_ROWS_PER_BLOCK - 1) / CE_ROWS_PER_BLOCK);
}

extern "C" int ghm_ce_kl(const float* logits, const uint8_t* targets, const float* post, float* dlogits,
                         float* loss_out, float* hist, float* chist, const int32_t* step, int64_t n_seq, int T,
                         int n_prefix, int V, void* stream) {
  GHM_CHECK(logits && targets && loss_out, "null pointer");
  GHM_CHECK(n_seq >= 1 && n_seq <= (1 << 24) && T > n_prefix && n_prefix >= 0 && V >= 2, "shape");
  const int64_t rows = n_seq * (T - n_prefix);
  const int nblk = static_cast<int>((rows + CE_ROWS_PER_BLOCK - 1) / CE_ROWS_PER_BLOCK);
  // partials: loss_out[2 .. 2 + 2 nblk) (the caller's buffer holds ghm_ce_kl_out_elems floats)
  float* part = loss_out + 2;
  hipStream_t s = ghm_stream(stream);
  hipLaunchKernelGGL(k_ce_kl_rows, dim3(static_cast<unsigned>(nblk)), dim3(CE_THREADS), 0, s, logits, targets, post,
                     dlogits, part, static_cast<int>(n_seq), T, n_prefix, V);
  hipLaunchKernelGGL(k_ce_kl_final, dim3(1), dim3(64), 0, s, part, nblk, rows, loss_out, hist, chist, step);
  return ghm_launch_status();
}
