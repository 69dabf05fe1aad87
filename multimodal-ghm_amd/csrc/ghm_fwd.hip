// Forward kernels of the GHM CLIP encoder step (gfx950, fp32 via exact-f32 MFMA).
// Reference semantics: src/ghmclip/models/model.py:760-808 (EncoderTransformer.forward)
// and :877-907 (GuidedClipLoss, guide=False).  See ghm_common.h for the
// "tokens on lanes" register layout shared by all token-parallel kernels.
#include "ghm_common.h"
#include "ghm_ln.h"

// ---------------------------------------------------------------------------
// H0[m] = tok_w[tokens[m]] + pos_w[m % T]                      (model.py:764-765)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_embed_fwd(const uint8_t* __restrict__ tok,
                                                   const float* __restrict__ tok_w,
                                                   const float* __restrict__ pos_w,
                                                   float* __restrict__ H, int64_t M, int T, int V) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= M * 32) return;
  const int64_t m = idx >> 5;
  const int c4 = static_cast<int>(idx & 31);
  const int t = static_cast<int>(m % T);
  int v = tok[m];
  v = v < V ? v : V - 1;  // host validates; never read out of the table
  const float4 a = reinterpret_cast<const float4*>(tok_w + v * GHM_D)[c4];
  const float4 b = reinterpret_cast<const float4*>(pos_w + t * GHM_D)[c4];
  reinterpret_cast<float4*>(H + m * GHM_D)[c4] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// Y^T tile (32 out features x 32 tokens) = W[o0:o0+32, :] . X^T, X in row layout,
// W rows staged in LDS ([32][PW], PW = 132: the float4 reads of 16 lanes with
// distinct rows hit 16 distinct 4-bank groups).  A operand: lane (i=j, h) reads
// W[o0 + j][64h + s]; B operand: x[s].
constexpr int PW = 132;
__device__ __forceinline__ f32x16 proj_tile_lds(const float* wl, const float* x) {
  f32x16 acc = zero16();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float4 w = lds4(wl + 4 * q);
    acc = mfma32(w.x, x[4 * q + 0], acc);
    acc = mfma32(w.y, x[4 * q + 1], acc);
    acc = mfma32(w.z, x[4 * q + 2], acc);
    acc = mfma32(w.w, x[4 * q + 3], acc);
  }
  return acc;
}

// ---------------------------------------------------------------------------
// LN1 + Q/K/V projections                                       (model.py:772-775)
// one wave = 32 tokens, 4 waves per workgroup; the 12 weight tiles (3 matrices
// x 4 blocks of 32 output rows) stream through a double-buffered LDS ring, so
// each weight byte is read from L2 once per 128 tokens.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void k_ln_qkv_fwd(
    const float* __restrict__ H, const float* __restrict__ lnw, const float* __restrict__ lnb,
    const float* __restrict__ Wq, const float* __restrict__ Wk, const float* __restrict__ Wv,
    float* __restrict__ qkv, float2* __restrict__ stats, int64_t M, float eps) {
  __shared__ __attribute__((aligned(16))) float sw[2][32 * PW];
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t m0 = (static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6)) * 32;
  const bool active = m0 < M;  // inactive waves still stage tiles and join barriers
  const int64_t m = m0 + j;
  const bool valid = m < M;
  const int64_t mc = valid ? m : M - 1;
  float x[64], mean = 0.f, rstd = 0.f;
  if (active) {
    ln_row(H + mc * GHM_D, lnw, lnb, h, eps, x, mean, rstd);
    if (h == 0 && valid) stats[m] = make_float2(mean, rstd);
  }
  float4 st[stage_n<32, GHM_D>()];
  stage_load<32, GHM_D>(st, Wq, GHM_D);
  stage_store<32, GHM_D, PW>(st, sw[0]);
  __syncthreads();
#pragma unroll 1
  for (int b = 0; b < 12; ++b) {  // b = mat * 4 + output block
    const int cur = b & 1;
    {  // prefetch tile b+1 (the last iteration re-stages tile 11 into the idle buffer)
      const int nb = b + 1 < 12 ? b + 1 : 11;
      const float* Wn = nb < 4 ? Wq : (nb < 8 ? Wk : Wv);
      stage_load<32, GHM_D>(st, Wn + (nb & 3) * 32 * GHM_D, GHM_D);
    }
    if (active) {
      const f32x16 acc = proj_tile_lds(sw[cur] + j * PW + 64 * h, x);
      if (valid) {
        float* o = qkv + m * (3 * GHM_D) + (b >> 2) * GHM_D + (b & 3) * 32;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          st4(o + quad_off(q, h), acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
      }
    }
    stage_store<32, GHM_D, PW>(st, sw[cur ^ 1]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Single-head full-width softmax attention + residual           (model.py:778-782)
// one workgroup = one sequence; wave w = query block [32w, 32w+32).
// S^T = K Q^T keeps the query on the lane, so the softmax row lives in the
// lane's registers (+ one lane-pair exchange) and the probabilities are the B
// operand of O^T = V^T P^T without leaving registers.  K (two halves of the
// feature dim) and V (four 32-column blocks) pass through one LDS buffer
// shared by the workgroup's waves.  P is written dense and padded,
// [seq][96][96] (float4 per quad, unconditional; padded keys and padded
// query rows hold 0).
// ---------------------------------------------------------------------------
constexpr int AT_P = 96;          // padded sequence length of the P / dS layouts
constexpr int AK_PITCH = 68;      // K half-chunk row: [h][32] + 4 pad -> conflict-free float4
__device__ __forceinline__ int kchunk_elems(int tp) { return tp * AK_PITCH; }

// stage K[:, 64h + 32c + t] (h = 0,1; t < 32) of the sequence as [key][h][32]
template <int NKT>
__device__ __forceinline__ void stage_k_half(const float* __restrict__ seq, int T, int c, int col0, float* sk) {
  // K/V[:, 64h + 32c + t] (h = 0,1; t < 32) of the sequence as [key][h][32] (pitch AK_PITCH);
  // all global loads are issued before the first LDS write
  constexpr int NT = NKT * 64, NIT = NKT * 32 * 16 / NT;
  float4 v[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int idx = threadIdx.x + NT * k;
    const int key = idx >> 4, hh = (idx >> 3) & 1, q4 = idx & 7;
    const int kc = key < T ? key : T - 1;
    v[k] = *reinterpret_cast<const float4*>(seq + static_cast<int64_t>(kc) * (3 * GHM_D) + col0 + 64 * hh +
                                            32 * c + 4 * q4);
  }
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int idx = threadIdx.x + NT * k;
    const int key = idx >> 4, hh = (idx >> 3) & 1, q4 = idx & 7;
    *reinterpret_cast<float4*>(sk + key * AK_PITCH + 32 * hh + 4 * q4) = v[k];
  }
}

template <int NKT>
__device__ __forceinline__ void stage_cols32(const float* __restrict__ base_row, int ld, int T, int col,
                                             float* sv) {
  // X[:, col + t] (t < 32) of the sequence as [row][32]; rows >= T clamp
  constexpr int NT = NKT * 64, NIT = NKT * 32 * 8 / NT;
  float4 v[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int idx = threadIdx.x + NT * k;
    const int row = idx >> 3, q4 = idx & 7;
    const int rc = row < T ? row : T - 1;
    v[k] = *reinterpret_cast<const float4*>(base_row + static_cast<int64_t>(rc) * ld + col + 4 * q4);
  }
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int idx = threadIdx.x + NT * k;
    *reinterpret_cast<float4*>(sv + (idx >> 3) * 32 + 4 * (idx & 7)) = v[k];
  }
}

// ACT (model.py:121-130, applied at :781): softmax, or the elementwise relu / gelu
// of the scaled score (keys past T and padded queries 0; gelu also stores GELU'
// of the score in Pd, P's layout, for the backward)
template <int NKT, int ACT = ACT_SOFTMAX>
__global__ __launch_bounds__(NKT * 64, 2) void k_attn_fwd(const float* __restrict__ qkv,
                                                          const float* __restrict__ H,
                                                          float* __restrict__ Hmid,
                                                          float* __restrict__ P, int T,
                                                          float scale_div, float* __restrict__ Pd = nullptr) {
  constexpr int TP = NKT * 32;
  __shared__ __attribute__((aligned(16))) float sbuf[TP * AK_PITCH];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const float* seq = qkv + base * (3 * GHM_D);
  const int q = 32 * w + j;
  const bool qv = q < T;
  const int qc = qv ? q : T - 1;
  float xq[64];
  load64(seq + static_cast<int64_t>(qc) * (3 * GHM_D) + 64 * h, xq);  // Q[q][64h + s]
  f32x16 s[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) s[kt] = zero16();
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    stage_k_half<NKT>(seq, T, c, GHM_D, sbuf);
    __syncthreads();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const float* kr = sbuf + (32 * kt + j) * AK_PITCH + 32 * h;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 kv = lds4(kr + 4 * i);
        s[kt] = mfma32(kv.x, xq[32 * c + 4 * i + 0], s[kt]);
        s[kt] = mfma32(kv.y, xq[32 * c + 4 * i + 1], s[kt]);
        s[kt] = mfma32(kv.z, xq[32 * c + 4 * i + 2], s[kt]);
        s[kt] = mfma32(kv.w, xq[32 * c + 4 * i + 3], s[kt]);
      }
    }
    __syncthreads();
  }
  // rows of padded queries (q >= T) are stored as 0: the key-block backward
  // kernel sums P over all 96 rows
  float inv;
  if (ACT == ACT_SOFTMAX) {  // softmax over keys for query q (= this lane's column)
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + acc_row(r, h);
        const float v = key < T ? s[kt][r] / scale_div : -INFINITY;
        s[kt][r] = v;
        mx = fmaxf(mx, v);
      }
    }
    mx = fmaxf(mx, xhalf(mx));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = expf(s[kt][r] - mx);
        s[kt][r] = e;
        sum += e;
      }
    }
    sum += xhalf(sum);
    inv = qv ? 1.f / sum : 0.f;
  } else {
    inv = 1.f;
    float* drow = ACT == ACT_GELU ? Pd + (static_cast<int64_t>(blockIdx.x) * AT_P + q) * AT_P : nullptr;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      float dv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + acc_row(r, h);
        const float x = s[kt][r] / scale_div;
        float a, d = 0.f;
        if (ACT == ACT_RELU)
          a = fmaxf(x, 0.f);
        else
          gelu_and_grad(x, a, d);
        const bool ok = key < T && qv;
        s[kt][r] = ok ? a : 0.f;
        dv[r] = ok ? d : 0.f;
      }
      if (ACT == ACT_GELU) {
#pragma unroll
        for (int qd = 0; qd < 4; ++qd)
          st4(drow + 32 * kt + quad_off(qd, h), dv[4 * qd], dv[4 * qd + 1], dv[4 * qd + 2], dv[4 * qd + 3]);
      }
    }
  }
  float* prow = P + (static_cast<int64_t>(blockIdx.x) * AT_P + q) * AT_P;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kt][r] *= inv;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
      st4(prow + 32 * kt + quad_off(qd, h), s[kt][4 * qd], s[kt][4 * qd + 1], s[kt][4 * qd + 2], s[kt][4 * qd + 3]);
  }
  // O^T[d][q] = sum_key V[key][d] P[q][key], V block [key][32] in LDS
#pragma unroll 1
  for (int dt = 0; dt < 4; ++dt) {
    stage_cols32<NKT>(seq, 3 * GHM_D, T, 2 * GHM_D + 32 * dt, sbuf);
    __syncthreads();
    f32x16 acc = zero16();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc = mfma32(sbuf[(32 * kt + acc_row(r, h)) * 32 + j], s[kt][r], acc);
    }
    __syncthreads();
    if (qv) {
      const int64_t row = (base + q) * GHM_D + 32 * dt;
      float4 hv[4];
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) hv[qd] = *reinterpret_cast<const float4*>(H + row + quad_off(qd, h));
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        st4(Hmid + row + quad_off(qd, h), hv[qd].x + acc[4 * qd], hv[qd].y + acc[4 * qd + 1],
            hv[qd].z + acc[4 * qd + 2], hv[qd].w + acc[4 * qd + 3]);
    }
  }
}

// ---------------------------------------------------------------------------
// LN2 + MLP (128 -> 512 -> GELU -> 128) + residual             (model.py:784-788)
// The 512-wide hidden activation never leaves registers: each 32-unit chunk of
// U^T is GELU'd in place and is immediately the B operand of the down product.
// Per chunk the workgroup stages W1[32c:32c+32, :] ([32][132]) and
// W2[:, 32c:32c+32] ([128][36]: float4 reads conflict-free) in a double-buffered
// LDS ring.  G = GELU(U) and D = GELU'(U) are stored for the backward pass
// (one erf evaluation serves both; the backward needs no transcendentals).
// SAVE = false (G = Dg = null): nothing stored for the backward -- the "f32fwd"
// mode, whose split-bf16 backward recomputes U (k_mlp_bwd_rc_x3).
// ---------------------------------------------------------------------------
constexpr int PW2 = 36;
template <bool SAVE>
__global__ __launch_bounds__(256, 2) void k_ln_mlp_fwd(
    const float* __restrict__ Hmid, const float* __restrict__ lnw, const float* __restrict__ lnb,
    const float* __restrict__ W1, const float* __restrict__ b1, const float* __restrict__ W2,
    const float* __restrict__ b2, float* __restrict__ Hout, float* __restrict__ G,
    float* __restrict__ Dg, float2* __restrict__ stats, int64_t M, float eps) {
  __shared__ __attribute__((aligned(16))) float s1[2][32 * PW];
  __shared__ __attribute__((aligned(16))) float s2[2][GHM_D * PW2];
  __shared__ __attribute__((aligned(16))) float sb1[GHM_F];
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t m0 = (static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6)) * 32;
  const bool active = m0 < M;
  const int64_t m = m0 + j;
  const bool valid = m < M;
  const int64_t mc = valid ? m : M - 1;
  for (int i = threadIdx.x; i < GHM_F; i += 256) sb1[i] = b1[i];
  float x[64], mean = 0.f, rstd = 0.f;
  if (active) {
    ln_row(Hmid + mc * GHM_D, lnw, lnb, h, eps, x, mean, rstd);
    if (h == 0 && valid) stats[m] = make_float2(mean, rstd);
  }
  f32x16 y[4];
#pragma unroll
  for (int ot = 0; ot < 4; ++ot) y[ot] = zero16();
  float4 st1[stage_n<32, GHM_D>()], st2[stage_n<GHM_D, 32>()];
  stage_load<32, GHM_D>(st1, W1, GHM_D);
  stage_load<GHM_D, 32>(st2, W2, GHM_F);
  stage_store<32, GHM_D, PW>(st1, s1[0]);
  stage_store<GHM_D, 32, PW2>(st2, s2[0]);
  __syncthreads();
#pragma unroll 1
  for (int c = 0; c < GHM_F / 32; ++c) {
    const int cur = c & 1;
    {
      const int nc = c + 1 < GHM_F / 32 ? c + 1 : c;
      stage_load<32, GHM_D>(st1, W1 + static_cast<size_t>(nc) * 32 * GHM_D, GHM_D);
      stage_load<GHM_D, 32>(st2, W2 + nc * 32, GHM_F);
    }
    if (active) {
      const f32x16 u = proj_tile_lds(s1[cur] + j * PW + 64 * h, x);
      float g[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bb = lds4(sb1 + 32 * c + quad_off(q, h));
        g[4 * q + 0] = u[4 * q + 0] + bb.x;
        g[4 * q + 1] = u[4 * q + 1] + bb.y;
        g[4 * q + 2] = u[4 * q + 2] + bb.z;
        g[4 * q + 3] = u[4 * q + 3] + bb.w;
      }
      float dg[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) gelu_and_grad(g[r], g[r], dg[r]);
      if (SAVE && valid) {  // G = GELU(U) for dW2, D = GELU'(U) for the backward
        float* grow = G + m * GHM_F + 32 * c;
        float* drow = Dg + m * GHM_F + 32 * c;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          st4(grow + quad_off(q, h), g[4 * q], g[4 * q + 1], g[4 * q + 2], g[4 * q + 3]);
          st4(drow + quad_off(q, h), dg[4 * q], dg[4 * q + 1], dg[4 * q + 2], dg[4 * q + 3]);
        }
      }
#pragma unroll
      for (int ot = 0; ot < 4; ++ot) {
        // A operand: W2[32ot + j][32c + 8q + 4h + t] = s2[(32ot + j) * PW2 + 8q + 4h + t]
        const float* w2 = s2[cur] + (32 * ot + j) * PW2 + 4 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 w = lds4(w2 + 8 * q);
          y[ot] = mfma32(w.x, g[4 * q + 0], y[ot]);
          y[ot] = mfma32(w.y, g[4 * q + 1], y[ot]);
          y[ot] = mfma32(w.z, g[4 * q + 2], y[ot]);
          y[ot] = mfma32(w.w, g[4 * q + 3], y[ot]);
        }
      }
    }
    stage_store<32, GHM_D, PW>(st1, s1[cur ^ 1]);
    stage_store<GHM_D, 32, PW2>(st2, s2[cur ^ 1]);
    __syncthreads();
  }
  if (active && valid) {
#pragma unroll
    for (int ot = 0; ot < 4; ++ot) {
      float4 hv[4], bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        hv[q] = *reinterpret_cast<const float4*>(Hmid + m * GHM_D + 32 * ot + quad_off(q, h));
        bv[q] = *reinterpret_cast<const float4*>(b2 + 32 * ot + quad_off(q, h));
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st4(Hout + m * GHM_D + 32 * ot + quad_off(q, h), hv[q].x + (y[ot][4 * q] + bv[q].x),
            hv[q].y + (y[ot][4 * q + 1] + bv[q].y), hv[q].z + (y[ot][4 * q + 2] + bv[q].z),
            hv[q].w + (y[ot][4 * q + 3] + bv[q].w));
    }
  }
}

// ---------------------------------------------------------------------------
// Readout: Linear(D->C) over every token, then Linear(T->1) over the token axis
// (model.py:802-805): emb[c] = sum_t w_out[t] (H[t] . W_ro[c] + b_ro[c]) + b_out.
// Both maps are linear, so the kernel forms the token-weighted row sum
// hbar = sum_t w_out[t] H[t] first and then emb[c] = hbar . W_ro[c] +
// S_w b_ro[c] + b_out (S_w = sum_t w_out[t]): one pass over H at HBM rate
// instead of a 10-wide dot product per token.  One 256-thread workgroup per
// sequence: wave w takes tokens w, w + 4, ...; lane l holds features 2l, 2l + 1
// (one coalesced 512-B row per wave instruction); the four wave sums are added
// in a fixed order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int NC>
__global__ __launch_bounds__(256) void k_readout_fwd(const float* __restrict__ H,
                                                     const float* __restrict__ Wro,
                                                     const float* __restrict__ bro,
                                                     const float* __restrict__ wout,
                                                     const float* __restrict__ bout,
                                                     float* __restrict__ emb, int T) {
  __shared__ float2 red[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, n = blockIdx.x;
  const float2* Hs = reinterpret_cast<const float2*>(H + static_cast<int64_t>(n) * T * GHM_D) + lane;
  float2 hb = make_float2(0.f, 0.f);
  int t = w;
  for (; t + 12 < T; t += 16) {  // four rows in flight per wave
    float2 h[4];
    float wt[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      h[u] = Hs[(t + 4 * u) * (GHM_D / 2)];
      wt[u] = wout[t + 4 * u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      hb.x += wt[u] * h[u].x;
      hb.y += wt[u] * h[u].y;
    }
  }
  for (; t < T; t += 4) {
    const float2 h = Hs[t * (GHM_D / 2)];
    const float wt = wout[t];
    hb.x += wt * h.x;
    hb.y += wt * h.y;
  }
  red[w][lane] = hb;
  __syncthreads();
  if (w != 0) return;
  float2 hbar;
  hbar.x = (red[0][lane].x + red[1][lane].x) + (red[2][lane].x + red[3][lane].x);
  hbar.y = (red[0][lane].y + red[1][lane].y) + (red[2][lane].y + red[3][lane].y);
  float sw = 0.f;
  for (int k = lane; k < T; k += 64) sw += wout[k];
  sw = wave_sum(sw);
  const float2* W2 = reinterpret_cast<const float2*>(Wro) + lane;
  float mine = 0.f;  // lane c < NC keeps emb[c]
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const float2 wv = W2[c * (GHM_D / 2)];
    const float d = wave_sum(hbar.x * wv.x + hbar.y * wv.y);
    if (lane == c) mine = d;
  }
  if (lane < NC) emb[static_cast<int64_t>(n) * NC + lane] = mine + sw * bro[lane] + bout[0];
}

// ---------------------------------------------------------------------------
// K-way symmetric CLIP loss + gradient, one workgroup        (model.py:877-907)
// Rows are blocks b = 0..K of B rows; row i of block 0 (text) / 1 (image) is
// scored against its matched partner and row i of blocks 2..K.  exp() is
// unshifted, exactly as the reference.  The (K+1) B x C embeddings of both
// towers are first staged into LDS with coalesced loads (the round-2 kernel
// read them row by row from HBM in a chain of dependent loads: 25 us per step
// on one workgroup while the rest of the GPU idled); thread t < B then scores
// direction 1 of row t, thread B + t direction 2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float dotc(const float* a, const float* b, int C) {
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += a[c] * b[c];
  return s;
}

// direction of row i: the matched pair (tm, im) scored against the negatives
// ng(k) = row i of block k (k = 2..K) of the other tower; writes the gradients
// of tm, im and the negatives; returns -log(Sm / (Sm + Sn))
__device__ __forceinline__ float clip_dir(const float* tm, const float* im, const float* neg, int B, int K, int C,
                                          float invB, float* dtm, float* dim, float* dneg, bool neg_is_text) {
  const float* self = neg_is_text ? im : tm;  // the row the negatives are scored against
  const float Sm = expf(dotc(tm, im, C));
  float Sn = 0.f;
  for (int k = 2; k <= K; ++k) Sn += expf(dotc(neg + static_cast<int64_t>(k) * B * C, self, C));
  const float den = Sm + Sn;
  const float ga = -(Sn / den) * invB;
  float* dself = neg_is_text ? dim : dtm;
  for (int c = 0; c < C; ++c) { dtm[c] = ga * im[c]; dim[c] = ga * tm[c]; }
  for (int k = 2; k <= K; ++k) {
    const float* nk = neg + static_cast<int64_t>(k) * B * C;
    const float gb = (expf(dotc(nk, self, C)) / den) * invB;
    float* dnk = dneg + static_cast<int64_t>(k) * B * C;
    for (int c = 0; c < C; ++c) { dnk[c] = gb * self[c]; dself[c] += gb * nk[c]; }
  }
  return -logf(Sm / (Sm + Sn));
}

// the loss term of a direction only (clip_dir without the gradient writes)
__device__ __forceinline__ float clip_dir_value(const float* tm, const float* im, const float* neg, int B, int K,
                                                int C, bool neg_is_text) {
  const float* self = neg_is_text ? im : tm;
  const float Sm = expf(dotc(tm, im, C));
  float Sn = 0.f;
  for (int k = 2; k <= K; ++k) Sn += expf(dotc(neg + static_cast<int64_t>(k) * B * C, self, C));
  return -logf(Sm / (Sm + Sn));
}

// GRAD = false: the loss value only (the trainer's readout backward recomputes
// each row's gradient itself: ghm_readout_bwd_clip)
template <bool STAGE, bool GRAD = true>
__global__ __launch_bounds__(1024) void k_clip_loss(const float* __restrict__ te, const float* __restrict__ ie,
                                                    float* __restrict__ dte, float* __restrict__ die,
                                                    float* __restrict__ loss_out, float* __restrict__ hist,
                                                    const int32_t* __restrict__ step, int B, int K, int C) {
  extern __shared__ float sm[];  // STAGE: [te | ie], (K+1) B C floats each
  __shared__ float red[16];
  const int n = (K + 1) * B * C;
  const float* T = te;
  const float* I = ie;
  if (STAGE) {
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
      sm[e] = te[e];
      sm[n + e] = ie[e];
    }
    __syncthreads();
    T = sm;
    I = sm + n;
  }
  const float invB = 1.f / static_cast<float>(B);
  float acc = 0.f;
  for (int r = threadIdx.x; r < 2 * B; r += blockDim.x) {
    const int i = r < B ? r : r - B;
    if (r < B) {  // direction 1: image i of block 0 vs text i of block 0 and of blocks 2..K
      const int64_t o = static_cast<int64_t>(i) * C;
      acc += GRAD ? clip_dir(T + o, I + o, T + o, B, K, C, invB, dte + o, die + o, dte + o, true)
                  : clip_dir_value(T + o, I + o, T + o, B, K, C, true);
    } else {      // direction 2: text i of block 1 vs image i of block 1 and of blocks 2..K
      const int64_t o = (static_cast<int64_t>(B) + i) * C, on = static_cast<int64_t>(i) * C;
      acc += GRAD ? clip_dir(T + o, I + o, I + on, B, K, C, invB, dte + o, die + o, die + on, false)
                  : clip_dir_value(T + o, I + o, I + on, B, K, C, false);
    }
  }
  // deterministic block reduction
  acc = sum32(acc);
  acc += __shfl_xor(acc, 32, 64);
  const int nw = (blockDim.x + 63) / 64;
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < nw; ++w) tot += red[w];
    const float loss = tot * invB;
    loss_out[0] = loss;
    loss_out[1] = loss;
    if (hist) hist[*step] = loss;
  }
}

// ---------------------------------------------------------------------------
// C-ABI launchers
// ---------------------------------------------------------------------------
#include "ghm_launch.h"

extern "C" int ghm_embed_fwd(const uint8_t* tokens, const float* tok_w, const float* pos_w,
                             float* H0, int64_t n_seq, int T, int V, int D, void* stream) {
  GHM_CHECK(tokens && tok_w && pos_w && H0, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && V >= 1 && n_seq >= 1, "shape");
  const int64_t M = n_seq * T;
  const int64_t n = M * 32;
  hipLaunchKernelGGL(k_embed_fwd, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     ghm_stream(stream), tokens, tok_w, pos_w, H0, M, T, V);
  return ghm_launch_status();
}

extern "C" int ghm_ln_qkv_fwd(const float* H, const float* ln_w, const float* ln_b,
                              const float* Wq, const float* Wk, const float* Wv, float* qkv,
                              float* stats, int64_t M, int D, float eps, void* stream) {
  GHM_CHECK(H && ln_w && ln_b && Wq && Wk && Wv && qkv && stats, "null pointer");
  GHM_CHECK(D == GHM_D && M >= 1, "shape");
  hipLaunchKernelGGL(k_ln_qkv_fwd, dim3(static_cast<unsigned>(ghm_token_blocks(M))), dim3(256), 0,
                     ghm_stream(stream), H, ln_w, ln_b, Wq, Wk, Wv, qkv,
                     reinterpret_cast<float2*>(stats), M, eps);
  return ghm_launch_status();
}

template <int ACT>
static void attn_fwd_launch(const float* qkv, const float* H, float* H_mid, float* P, float* Pd, int64_t n_seq,
                            int T, float scale_div, hipStream_t s) {
  const unsigned g = static_cast<unsigned>(n_seq);
  if (T <= 32)
    hipLaunchKernelGGL((k_attn_fwd<1, ACT>), dim3(g), dim3(64), 0, s, qkv, H, H_mid, P, T, scale_div, Pd);
  else if (T <= 64)
    hipLaunchKernelGGL((k_attn_fwd<2, ACT>), dim3(g), dim3(128), 0, s, qkv, H, H_mid, P, T, scale_div, Pd);
  else
    hipLaunchKernelGGL((k_attn_fwd<3, ACT>), dim3(g), dim3(192), 0, s, qkv, H, H_mid, P, T, scale_div, Pd);
}

extern "C" int ghm_attn_fwd(const float* qkv, const float* H, float* H_mid, float* P,
                            int64_t n_seq, int T, int D, float scale_div, void* stream) {
  GHM_CHECK(qkv && H && H_mid && P, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96, D == 128)");
  attn_fwd_launch<ACT_SOFTMAX>(qkv, H, H_mid, P, nullptr, n_seq, T, scale_div, ghm_stream(stream));
  return ghm_launch_status();
}

extern "C" int ghm_attn_fwd_act(const float* qkv, const float* H, float* H_mid, float* P, float* Pd, int64_t n_seq,
                                int T, int D, float scale_div, int act, void* stream) {
  GHM_CHECK(qkv && H && H_mid && P && (act != ACT_GELU || Pd), "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96, D == 128)");
  GHM_CHECK(act >= ACT_SOFTMAX && act <= ACT_GELU, "act: 0 softmax, 1 relu, 2 gelu");
  hipStream_t s = ghm_stream(stream);
  if (act == ACT_SOFTMAX)
    attn_fwd_launch<ACT_SOFTMAX>(qkv, H, H_mid, P, Pd, n_seq, T, scale_div, s);
  else if (act == ACT_RELU)
    attn_fwd_launch<ACT_RELU>(qkv, H, H_mid, P, Pd, n_seq, T, scale_div, s);
  else
    attn_fwd_launch<ACT_GELU>(qkv, H, H_mid, P, Pd, n_seq, T, scale_div, s);
  return ghm_launch_status();
}

extern "C" int ghm_ln_mlp_fwd(const float* H_mid, const float* ln_w, const float* ln_b,
                              const float* W1, const float* b1, const float* W2, const float* b2,
                              float* H_out, float* G, float* Dg, float* stats, int64_t M, int D, int F,
                              float eps, void* stream) {
  GHM_CHECK(H_mid && ln_w && ln_b && W1 && b1 && W2 && b2 && H_out && stats, "null pointer");
  GHM_CHECK((G != nullptr) == (Dg != nullptr), "G and Dg: both saved or neither");
  GHM_CHECK(D == GHM_D && F == GHM_F && M >= 1, "shape (D == 128, F == 512)");
  const dim3 grid(static_cast<unsigned>(ghm_token_blocks(M)));
  if (G)
    hipLaunchKernelGGL(k_ln_mlp_fwd<true>, grid, dim3(256), 0, ghm_stream(stream), H_mid, ln_w, ln_b, W1, b1, W2, b2,
                       H_out, G, Dg, reinterpret_cast<float2*>(stats), M, eps);
  else
    hipLaunchKernelGGL(k_ln_mlp_fwd<false>, grid, dim3(256), 0, ghm_stream(stream), H_mid, ln_w, ln_b, W1, b1, W2,
                       b2, H_out, G, Dg, reinterpret_cast<float2*>(stats), M, eps);
  return ghm_launch_status();
}

extern "C" int ghm_readout_fwd(const float* H, const float* W_ro, const float* b_ro,
                               const float* w_out, const float* b_out, float* emb, int64_t n_seq,
                               int T, int D, int C, void* stream) {
  GHM_CHECK(H && W_ro && b_ro && w_out && b_out && emb, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96)");
  GHM_CHECK(C == 10, "readout kernels are built for num_class == 10 (the GHM vocabulary)");
  hipLaunchKernelGGL(k_readout_fwd<10>, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0,
                     ghm_stream(stream), H, W_ro, b_ro, w_out, b_out, emb, T);
  return ghm_launch_status();
}

extern "C" int ghm_clip_loss(const float* t_emb, const float* i_emb, float* dt_emb, float* di_emb,
                             float* loss_out, float* hist, const int32_t* step, int B, int K, int C,
                             void* stream) {
  GHM_CHECK(t_emb && i_emb && loss_out, "null pointer");
  GHM_CHECK((dt_emb == nullptr) == (di_emb == nullptr), "both gradients or neither (value only)");
  GHM_CHECK(!hist || step, "hist needs step");
  GHM_CHECK(B >= 1 && K >= 2 && C >= 1, "shape");
  const int threads = 2 * B >= 1024 ? 1024 : ((2 * B + 63) / 64) * 64;
  const size_t lds = 2 * static_cast<size_t>(K + 1) * B * C * sizeof(float);
  hipStream_t s = ghm_stream(stream);
  if (!dt_emb)
    hipLaunchKernelGGL((k_clip_loss<false, false>), dim3(1), dim3(threads), 0, s, t_emb, i_emb, dt_emb, di_emb,
                       loss_out, hist, step, B, K, C);
  else if (lds <= 64 * 1024)
    hipLaunchKernelGGL(k_clip_loss<true>, dim3(1), dim3(threads), lds, s, t_emb, i_emb, dt_emb, di_emb, loss_out,
                       hist, step, B, K, C);
  else
    hipLaunchKernelGGL(k_clip_loss<false>, dim3(1), dim3(threads), 0, s, t_emb, i_emb, dt_emb, di_emb, loss_out,
                       hist, step, B, K, C);
  return ghm_launch_status();
}
