// Backward kernels of the GHM CLIP encoder step (the autograd of
// src/ghmclip/training/train_CLIP.py:158 through models/model.py:760-808).
// Parameter gradients are produced deterministically: per-block partials in a
// fixed layout, summed in a fixed order by ghm_reduce_partials (no atomics).
#include "ghm_common.h"
#include "ghm_ln.h"
#include "ghm_launch.h"

// ---------------------------------------------------------------------------
// MLP + LN2 backward, one wave = 32 tokens                    (model.py:784-788)
//   dG^T = W2^T dY^T (per 32-unit chunk), dU = dG * GELU'(U) (stored),
//   dX2^T += W1^T dU^T (accumulated in registers), then LN2 backward.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void k_mlp_bwd(
    const float* __restrict__ dHout, const float* __restrict__ Hmid, const float2* __restrict__ stats,
    const float* __restrict__ lnw, const float* __restrict__ W1, const float* __restrict__ W2,
    const float* __restrict__ U, float* __restrict__ dU, float* __restrict__ dHmid,
    float* __restrict__ part_ln, int64_t M) {
  // U here is D = GELU'(pre-activation), written by k_ln_mlp_fwd.
  // per 32-unit chunk c: W2[:, 32c:32c+32] as [o][32] and W1[32c:32c+32, :] as [32][in]
  // in a double-buffered LDS ring; every MFMA A operand is a conflict-free ds_read_b32
  __shared__ __attribute__((aligned(16))) float s2[2][GHM_D * 32];
  __shared__ __attribute__((aligned(16))) float s1[2][32 * GHM_D];
  __shared__ float red[2 * 4 * GHM_D];
  __shared__ __attribute__((aligned(16))) float gam[GHM_D];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t m0 = (static_cast<int64_t>(blockIdx.x) * 4 + wave) * 32;
  const bool active = m0 < M;  // inactive waves still stage tiles and join barriers
  for (int i = threadIdx.x; i < 2 * 4 * GHM_D; i += 256) red[i] = 0.f;
  if (threadIdx.x < GHM_D) gam[threadIdx.x] = lnw[threadIdx.x];
  const int64_t m = m0 + j;
  const bool valid = active && m < M;
  const int64_t mc = m < M ? m : M - 1;
  f32x16 dx[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) dx[it] = zero16();
  float dy[64];
  if (active) load64(dHout + mc * GHM_D + 64 * h, dy);  // dY[token][o = 64h + s]
  float4 st2[stage_n<GHM_D, 32>()], st1[stage_n<32, GHM_D>()];
  stage_load<GHM_D, 32>(st2, W2, GHM_F);
  stage_load<32, GHM_D>(st1, W1, GHM_D);
  // U of the current chunk, prefetched one chunk ahead (row-scattered loads whose
  // latency would otherwise sit between the dG and dX MFMA chains)
  float4 un[4];
  const float* urow = U + mc * GHM_F;
#pragma unroll
  for (int q = 0; q < 4; ++q) un[q] = *reinterpret_cast<const float4*>(urow + quad_off(q, h));
  stage_store<GHM_D, 32, 32>(st2, s2[0]);
  stage_store<32, GHM_D, GHM_D>(st1, s1[0]);
  __syncthreads();
#pragma unroll 1
  for (int c = 0; c < GHM_F / 32; ++c) {
    const int cur = c & 1;
    float uc[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uc[4 * q] = un[q].x; uc[4 * q + 1] = un[q].y; uc[4 * q + 2] = un[q].z; uc[4 * q + 3] = un[q].w;
    }
    {
      const int nc = c + 1 < GHM_F / 32 ? c + 1 : c;
      stage_load<GHM_D, 32>(st2, W2 + nc * 32, GHM_F);
      stage_load<32, GHM_D>(st1, W1 + static_cast<size_t>(nc) * 32 * GHM_D, GHM_D);
#pragma unroll
      for (int q = 0; q < 4; ++q) un[q] = *reinterpret_cast<const float4*>(urow + 32 * nc + quad_off(q, h));
    }
    if (active) {
      // dG^T[hid][token] = sum_o W2[o][hid] dY[token][o]
      const float* w2 = s2[cur] + 64 * h * 32 + j;
      f32x16 g = zero16();
#pragma unroll
      for (int s = 0; s < 64; ++s) g = mfma32(w2[s * 32], dy[s], g);
      float du[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) du[r] = g[r] * uc[r];
      if (valid) {
        float* drow = dU + m * GHM_F + 32 * c;
#pragma unroll
        for (int q = 0; q < 4; ++q) st4(drow + quad_off(q, h), du[4 * q], du[4 * q + 1], du[4 * q + 2], du[4 * q + 3]);
      }
      // dX2^T[in][token] += sum_hid W1[hid][in] dU[token][hid]
      const float* w1 = s1[cur] + j;
#pragma unroll
      for (int it = 0; it < 4; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) dx[it] = mfma32(w1[acc_row(r, h) * GHM_D + 32 * it], du[r], dx[it]);
      }
    }
    stage_store<GHM_D, 32, 32>(st2, s2[cur ^ 1]);
    stage_store<32, GHM_D, GHM_D>(st1, s1[cur ^ 1]);
    __syncthreads();
  }
  if (active)
    ln_bwd_acc(dx, Hmid + mc * GHM_D, ld_stats_sys(stats, mc), gam, dHout + mc * GHM_D, dHmid + mc * GHM_D, valid, h, j,
               red + wave * GHM_D, red + 4 * GHM_D + wave * GHM_D);
  __syncthreads();
  ln_partial_store(red, part_ln + static_cast<int64_t>(blockIdx.x) * 2 * GHM_D);
}

// ---------------------------------------------------------------------------
// QKV + LN1 backward, one wave = 32 tokens                    (model.py:772-775)
//   dX1^T = Wq^T dQ^T + Wk^T dK^T + Wv^T dV^T, then LN1 backward + residual.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void k_qkv_bwd(
    const float* __restrict__ dqkv, const float* __restrict__ H, const float2* __restrict__ stats,
    const float* __restrict__ lnw, const float* __restrict__ Wq, const float* __restrict__ Wk,
    const float* __restrict__ Wv, const float* __restrict__ dHmid, float* __restrict__ dH,
    float* __restrict__ part_ln, int64_t M) {
  // tile b = mat*4 + it: W_mat[:, 32it:32it+32] as [o][32] in a double-buffered LDS ring
  __shared__ __attribute__((aligned(16))) float sw[2][GHM_D * 32];
  __shared__ float red[2 * 4 * GHM_D];
  __shared__ __attribute__((aligned(16))) float gam[GHM_D];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t m0 = (static_cast<int64_t>(blockIdx.x) * 4 + wave) * 32;
  const bool active = m0 < M;
  for (int i = threadIdx.x; i < 2 * 4 * GHM_D; i += 256) red[i] = 0.f;
  if (threadIdx.x < GHM_D) gam[threadIdx.x] = lnw[threadIdx.x];
  const int64_t m = m0 + j;
  const bool valid = active && m < M;
  const int64_t mc = m < M ? m : M - 1;
  f32x16 dx[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) dx[it] = zero16();
  float4 st[stage_n<GHM_D, 32>()];
  stage_load<GHM_D, 32>(st, Wq, GHM_D);
  stage_store<GHM_D, 32, 32>(st, sw[0]);
  __syncthreads();
#pragma unroll 1
  for (int mat = 0; mat < 3; ++mat) {
    float g[64];
    if (active) load64(dqkv + mc * (3 * GHM_D) + mat * GHM_D + 64 * h, g);  // dQ[token][o = 64h + s]
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int b = mat * 4 + it, cur = b & 1;
      {
        const int nb = b + 1 < 12 ? b + 1 : 11;
        const float* Wn = nb < 4 ? Wq : (nb < 8 ? Wk : Wv);
        stage_load<GHM_D, 32>(st, Wn + (nb & 3) * 32, GHM_D);
      }
      if (active) {
        const float* w = sw[cur] + 64 * h * 32 + j;
#pragma unroll
        for (int s = 0; s < 64; ++s) dx[it] = mfma32(w[s * 32], g[s], dx[it]);
      }
      stage_store<GHM_D, 32, 32>(st, sw[cur ^ 1]);
      __syncthreads();
    }
  }
  if (active)
    ln_bwd_acc(dx, H + mc * GHM_D, ld_stats_sys(stats, mc), gam, dHmid + mc * GHM_D, dH + mc * GHM_D, valid, h, j,
               red + wave * GHM_D, red + 4 * GHM_D + wave * GHM_D);
  __syncthreads();
  ln_partial_store(red, part_ln + static_cast<int64_t>(blockIdx.x) * 2 * GHM_D);
}

// ---------------------------------------------------------------------------
// Attention backward                                            (model.py:778-782)
// kernel 1 (workgroup = sequence, wave = query block): dP^T = V dO^T,
//   dS = P (dP - rowsum(P dP)) / c, dQ^T = K^T dS^T; dS written dense/padded
//   like P.  V (feature halves) and K (column blocks) staged in LDS.
// kernel 2 (workgroup = sequence, wave = key block): dV^T = dO^T P and
//   dK^T = Q^T dS, summing over queries; P and dS are read with the key on the
//   lane (coalesced 128-B rows), dO and Q column blocks staged in LDS.
// ---------------------------------------------------------------------------
constexpr int AT_P = 96;
constexpr int AK_PITCH = 68;

template <int NKT>
__device__ __forceinline__ void stage_k_half_b(const float* __restrict__ seq, int T, int c, int col0, float* sk) {
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
__device__ __forceinline__ void stage_cols32_b(const float* __restrict__ base_row, int ld, int T, int col,
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

// ACT: dS = P (dP - rowsum(P dP)) / scale (softmax), [P > 0] dP / scale (relu),
// GELU'(s) dP / scale (gelu, GELU' from the forward's Pd)
template <int NKT, int ACT = ACT_SOFTMAX>
__global__ __launch_bounds__(NKT * 64, 2) void k_attn_bwd_q(const float* __restrict__ qkv,
                                                            const float* __restrict__ P,
                                                            const float* __restrict__ dHmid,
                                                            float* __restrict__ dS_out,
                                                            float* __restrict__ dqkv, int T,
                                                            float scale_div, const float* __restrict__ Pd = nullptr) {
  constexpr int TP = NKT * 32;
  __shared__ __attribute__((aligned(16))) float sbuf[TP * AK_PITCH];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const float* seq = qkv + base * (3 * GHM_D);
  const int q = 32 * w + j;
  const bool qv = q < T;
  const int qc = qv ? q : T - 1;
  float go[64];
  load64(dHmid + (base + qc) * GHM_D + 64 * h, go);  // dO[q][64h + s]
  f32x16 dp[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) dp[kt] = zero16();
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    stage_k_half_b<NKT>(seq, T, c, 2 * GHM_D, sbuf);  // V halves
    __syncthreads();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const float* vr = sbuf + (32 * kt + j) * AK_PITCH + 32 * h;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 v = lds4(vr + 4 * i);
        dp[kt] = mfma32(v.x, go[32 * c + 4 * i + 0], dp[kt]);
        dp[kt] = mfma32(v.y, go[32 * c + 4 * i + 1], dp[kt]);
        dp[kt] = mfma32(v.z, go[32 * c + 4 * i + 2], dp[kt]);
        dp[kt] = mfma32(v.w, go[32 * c + 4 * i + 3], dp[kt]);
      }
    }
    __syncthreads();
  }
  // P rows (dense, padded keys are 0); queries >= T contribute nothing
  const int64_t poff = (static_cast<int64_t>(blockIdx.x) * AT_P + q) * AT_P;
  const float* prow = (ACT == ACT_GELU ? Pd : P) + poff;  // gelu: the factor is GELU'(s)
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
    if (ACT == ACT_SOFTMAX) {
#pragma unroll
      for (int r = 0; r < 16; ++r) delta += p[kt][r] * dp[kt][r];
    }
  }
  if (ACT == ACT_SOFTMAX) delta += xhalf(delta);
  float* srow = dS_out + poff;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (ACT == ACT_SOFTMAX)
        dp[kt][r] = (p[kt][r] * (dp[kt][r] - delta)) / scale_div;
      else if (ACT == ACT_RELU)
        dp[kt][r] = (p[kt][r] > 0.f ? dp[kt][r] : 0.f) / scale_div;
      else
        dp[kt][r] = (p[kt][r] * dp[kt][r]) / scale_div;
    }
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
      st4(srow + 32 * kt + quad_off(qd, h), dp[kt][4 * qd], dp[kt][4 * qd + 1], dp[kt][4 * qd + 2],
          dp[kt][4 * qd + 3]);
  }
  // dQ^T[d][q] = sum_key K[key][d] dS[q][key], K column block [key][32] in LDS
#pragma unroll 1
  for (int dt = 0; dt < 4; ++dt) {
    stage_cols32_b<NKT>(seq, 3 * GHM_D, T, GHM_D + 32 * dt, sbuf);
    __syncthreads();
    f32x16 acc = zero16();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc = mfma32(sbuf[(32 * kt + acc_row(r, h)) * 32 + j], dp[kt][r], acc);
    }
    __syncthreads();
    if (qv) {
      float* o = dqkv + (base + q) * (3 * GHM_D) + 32 * dt;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        st4(o + quad_off(qd, h), acc[4 * qd], acc[4 * qd + 1], acc[4 * qd + 2], acc[4 * qd + 3]);
    }
  }
}

template <int NKT>
__global__ __launch_bounds__(NKT * 64, 2) void k_attn_bwd_kv(const float* __restrict__ qkv,
                                                             const float* __restrict__ P,
                                                             const float* __restrict__ dS,
                                                             const float* __restrict__ dHmid,
                                                             float* __restrict__ dqkv, int T) {
  constexpr int TP = NKT * 32;
  __shared__ __attribute__((aligned(16))) float sdo[TP * 32];
  __shared__ __attribute__((aligned(16))) float sq[TP * 32];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const int key = 32 * w + j;
  const bool kv = key < T;
  // this lane's column of P and dS (queries 2st + h), loaded once and reused by
  // all four column blocks; rows >= T of P / dS are 0
  const float* pc = P + static_cast<int64_t>(blockIdx.x) * AT_P * AT_P + key;
  const float* sc = dS + static_cast<int64_t>(blockIdx.x) * AT_P * AT_P + key;
  float pb[TP / 2], sb[TP / 2];
#pragma unroll
  for (int st = 0; st < TP / 2; ++st) {
    pb[st] = pc[(2 * st + h) * AT_P];
    sb[st] = sc[(2 * st + h) * AT_P];
  }
#pragma unroll 1
  for (int dt = 0; dt < 4; ++dt) {
    stage_cols32_b<NKT>(dHmid + base * GHM_D, GHM_D, T, 32 * dt, sdo);
    stage_cols32_b<NKT>(qkv + base * (3 * GHM_D), 3 * GHM_D, T, 32 * dt, sq);
    __syncthreads();
    f32x16 aV = zero16(), aK = zero16();
#pragma unroll
    for (int st = 0; st < TP / 2; ++st) {
      const int qq = 2 * st + h;
      aV = mfma32(sdo[qq * 32 + j], pb[st], aV);
      aK = mfma32(sq[qq * 32 + j], sb[st], aK);
    }
    __syncthreads();
    if (kv) {
      float* o = dqkv + (base + key) * (3 * GHM_D) + 32 * dt;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        st4(o + 2 * GHM_D + quad_off(qd, h), aV[4 * qd], aV[4 * qd + 1], aV[4 * qd + 2], aV[4 * qd + 3]);
        st4(o + GHM_D + quad_off(qd, h), aK[4 * qd], aK[4 * qd + 1], aK[4 * qd + 2], aK[4 * qd + 3]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Split-K weight gradient: part[z][a][b] = sum_{m in chunk z} A[m][a] op(B)[m][b]
// MFMA k-dimension = tokens (k-slot h = token parity).  The workgroup covers a
// 128 x 128 output tile (4 waves as 2x2, 64x64 each); per 32-token k-step the A
// and op(B) tiles ([32][128] each, op applied once while staging) pass through a
// double-buffered LDS ring.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256, 2) void k_wgrad(const float* __restrict__ A, int lda,
                                                  const float* __restrict__ Bs, int ldb,
                                                  const float2* __restrict__ stats,
                                                  const float* __restrict__ lnw,
                                                  const float* __restrict__ lnb,
                                                  float* __restrict__ part,
                                                  float* __restrict__ bias_part, int64_t M,
                                                  int tok_per_split, int Acols, int Bcols) {
  constexpr int KT = 32, PT = 128;
  __shared__ __attribute__((aligned(16))) float sA[2][KT * PT];
  __shared__ __attribute__((aligned(16))) float sB[2][KT * PT];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int wa = (wave >> 1) * 64, wb = (wave & 1) * 64;
  const int a_blk = blockIdx.x * 128, b_blk = blockIdx.y * 128;
  const int64_t m_begin = static_cast<int64_t>(blockIdx.z) * tok_per_split;
  int64_t m_end = m_begin + tok_per_split;
  if (m_end > M) m_end = M;
  const int nsteps = static_cast<int>((m_end - m_begin + KT - 1) / KT);
  // per-thread column constants of the B transform (columns 4*c4 .. +3 of the tile)
  float4 gcol = make_float4(1.f, 1.f, 1.f, 1.f), ecol = make_float4(0.f, 0.f, 0.f, 0.f);
  const int c4 = threadIdx.x & 31;
  if (MODE == 2) {
    gcol = *reinterpret_cast<const float4*>(lnw + b_blk + 4 * c4);
    ecol = *reinterpret_cast<const float4*>(lnb + b_blk + 4 * c4);
  }
  float4 va[4], vb[4];
  float2 vs[4];
  auto load = [&](int step) {
    const int64_t mb = m_begin + static_cast<int64_t>(step) * KT;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = (threadIdx.x >> 5) + 8 * k;
      const int64_t mt = mb + r;
      const bool ok = mt < m_end;
      const int64_t mcl = ok ? mt : m_begin;
      va[k] = *reinterpret_cast<const float4*>(A + mcl * lda + a_blk + 4 * c4);
      vb[k] = *reinterpret_cast<const float4*>(Bs + mcl * ldb + b_blk + 4 * c4);
      if (!ok) va[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (MODE == 2) vs[k] = ld_stats_sys(stats, mcl);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = (threadIdx.x >> 5) + 8 * k;
      float4 b = vb[k];
      if (MODE == 1) {
        b = make_float4(gelu_f(b.x), gelu_f(b.y), gelu_f(b.z), gelu_f(b.w));
      } else if (MODE == 2) {
        const float mu = vs[k].x, rs = vs[k].y;
        b = make_float4((b.x - mu) * rs * gcol.x + ecol.x, (b.y - mu) * rs * gcol.y + ecol.y,
                        (b.z - mu) * rs * gcol.z + ecol.z, (b.w - mu) * rs * gcol.w + ecol.w);
      }
      *reinterpret_cast<float4*>(sA[buf] + r * PT + 4 * c4) = va[k];
      *reinterpret_cast<float4*>(sB[buf] + r * PT + 4 * c4) = b;
    }
  };
  f32x16 acc00 = zero16(), acc01 = zero16(), acc10 = zero16(), acc11 = zero16();
  float bs0 = 0.f, bs1 = 0.f;
  load(0);
  store(0);
  __syncthreads();
#pragma unroll 1
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st & 1;
    load(st + 1 < nsteps ? st + 1 : st);
    const float* pa = sA[cur] + h * PT + wa + j;
    const float* pb = sB[cur] + h * PT + wb + j;
#pragma unroll
    for (int s = 0; s < KT / 2; ++s) {
      const float a0 = pa[2 * s * PT], a1 = pa[2 * s * PT + 32];
      const float b0 = pb[2 * s * PT], b1 = pb[2 * s * PT + 32];
      acc00 = mfma32(a0, b0, acc00);
      acc01 = mfma32(a0, b1, acc01);
      acc10 = mfma32(a1, b0, acc10);
      acc11 = mfma32(a1, b1, acc11);
      bs0 += a0;
      bs1 += a1;
    }
    store(cur ^ 1);
    __syncthreads();
  }
  float* pz = part + static_cast<int64_t>(blockIdx.z) * Acols * Bcols;
  const int a_base = a_blk + wa, b_base = b_blk + wb;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t ra = a_base + acc_row(r, h);
    pz[ra * Bcols + b_base + j] = acc00[r];
    pz[ra * Bcols + b_base + 32 + j] = acc01[r];
    pz[(ra + 32) * Bcols + b_base + j] = acc10[r];
    pz[(ra + 32) * Bcols + b_base + 32 + j] = acc11[r];
  }
  if (bias_part && blockIdx.y == 0 && (wave & 1) == 0) {
    bs0 += xhalf(bs0);
    bs1 += xhalf(bs1);
    if (h == 0) {
      float* bz = bias_part + static_cast<int64_t>(blockIdx.z) * Acols;
      bz[a_base + j] = bs0;
      bz[a_base + 32 + j] = bs1;
    }
  }
}

// ---------------------------------------------------------------------------
// Readout backward, one workgroup per sequence                 (model.py:802-805)
// With de = d(loss)/d(emb) of the sequence and u = W_ro^T de (a 128-vector):
//   dH[t]         = w_out[t] u                    (rank one per sequence)
//   part_wout[t]  = H[t] . u + de . b_ro          (d/dw_out[t])
//   part_wro[c]   = de[c] hbar,  hbar = sum_t w_out[t] H[t]
//   part_bro[c]   = de[c] S_w,   part_bout = sum_c de[c]
// so H is read once and dH written once (the partials are reduced over the
// sequences by ghm_reduce_batch, as before).  Wave w takes tokens w, w + 4, ...;
// lane l holds features 2l, 2l + 1; the token dot products are wave sums and
// the four waves' hbar are added in a fixed order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// d(CLIP loss)/d(emb) of row n of one tower, recomputed from the loss terms that
// touch it (model.py:877-907): rows are blocks b = 0..K of B rows, and row n =
// b B + i belongs to group i only.  Text rows of blocks 0 and >= 2 and image row
// i of block 0 get their gradient from direction 1 (image i of block 0 scored
// against text i of blocks 0, 2..K), the others from direction 2 (text i of block
// 1 against image i of blocks 1, 2..K).  Same arithmetic, in the same order, as
// clip_dir (ghm_fwd.hip), so the values equal k_clip_loss's bit for bit.
template <int NC>
__device__ __forceinline__ void clip_row_grad(const float* __restrict__ te, const float* __restrict__ ie, int tower,
                                              int n, int B, int K, float* de) {
  const int b = n / B, i = n - b * B;
  const bool dir1 = tower == 0 ? b != 1 : b == 0;
  // direction 1: tm = text i of block 0, im = image i of block 0, negatives = text
  // rows, self = im; direction 2: tm / im of block 1, negatives = image rows, self = tm
  const int64_t om = static_cast<int64_t>(dir1 ? i : B + i) * NC;
  const float* tm = te + om;
  const float* im = ie + om;
  const float* neg = dir1 ? te : ie;
  const float* self = dir1 ? im : tm;
  auto dot = [&](const float* a, const float* c) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) s += a[k] * c[k];
    return s;
  };
  const float invB = 1.f / static_cast<float>(B);
  const float Sm = expf(dot(tm, im));
  float Sn = 0.f;
  for (int k = 2; k <= K; ++k) Sn += expf(dot(neg + (static_cast<int64_t>(k) * B + i) * NC, self));
  const float den = Sm + Sn;
  const float ga = -(Sn / den) * invB;
  if (b >= 2) {  // a negative row: gb_b * self
    const float gb = (expf(dot(neg + (static_cast<int64_t>(b) * B + i) * NC, self)) / den) * invB;
#pragma unroll
    for (int c = 0; c < NC; ++c) de[c] = gb * self[c];
    return;
  }
  // a matched row: ga * (the other tower's matched row), plus (for the row the
  // negatives were scored against) sum_k gb_k * negative k, k ascending
  const float* other = tower == 0 ? im : tm;
#pragma unroll
  for (int c = 0; c < NC; ++c) de[c] = ga * other[c];
  const bool is_self = (tower == 0) != dir1;  // text row of block 1 (dir 2) / image row of block 0 (dir 1)
  if (is_self) {
    for (int k = 2; k <= K; ++k) {
      const float* nk = neg + (static_cast<int64_t>(k) * B + i) * NC;
      const float gb = (expf(dot(nk, self)) / den) * invB;
#pragma unroll
      for (int c = 0; c < NC; ++c) de[c] += gb * nk[c];
    }
  }
}

// One tower's rows of the loss gradient, one thread per row (a few-microsecond
// kernel ahead of that tower's readout backward: computing the row inside each
// readout-backward workgroup put its latency chain in front of every round of
// the 640 workgroups, 14 -> 28 us)
template <int NC>
__global__ __launch_bounds__(64) void k_clip_grad_rows(const float* __restrict__ te, const float* __restrict__ ie,
                                                       int tower, int B, int K, float* __restrict__ demb) {
  const int n = blockIdx.x * 64 + threadIdx.x;
  if (n >= (K + 1) * B) return;
  float de[NC];
  clip_row_grad<NC>(te, ie, tower, n, B, K, de);
#pragma unroll
  for (int c = 0; c < NC; ++c) demb[static_cast<int64_t>(n) * NC + c] = de[c];
}

template <int NC>
__global__ __launch_bounds__(256) void k_readout_bwd(
    const float* __restrict__ H, const float* __restrict__ Wro, const float* __restrict__ bro,
    const float* __restrict__ wout, const float* __restrict__ demb, float* __restrict__ dH,
    float* __restrict__ part_wro, float* __restrict__ part_bro, float* __restrict__ part_wout,
    float* __restrict__ part_bout, int T) {
  __shared__ float2 red[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, n = blockIdx.x;
  const int64_t base = static_cast<int64_t>(n) * T;
  float de[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) de[c] = demb[static_cast<int64_t>(n) * NC + c];
  float2 u = make_float2(0.f, 0.f);
  float bdot = 0.f;
  {
    const float2* W2 = reinterpret_cast<const float2*>(Wro) + lane;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float2 wv = W2[c * (GHM_D / 2)];
      u.x += de[c] * wv.x;
      u.y += de[c] * wv.y;
      bdot += de[c] * bro[c];
    }
  }
  const float2* Hs = reinterpret_cast<const float2*>(H + base * GHM_D) + lane;
  float2* dHs = reinterpret_cast<float2*>(dH + base * GHM_D) + lane;
  float2 hb = make_float2(0.f, 0.f);
  int t = w;
  for (; t + 4 < T; t += 8) {  // two rows in flight per wave
    const float2 h0 = Hs[t * (GHM_D / 2)], h1 = Hs[(t + 4) * (GHM_D / 2)];
    const float w0 = wout[t], w1 = wout[t + 4];
    dHs[t * (GHM_D / 2)] = make_float2(w0 * u.x, w0 * u.y);
    dHs[(t + 4) * (GHM_D / 2)] = make_float2(w1 * u.x, w1 * u.y);
    hb.x += w0 * h0.x;
    hb.y += w0 * h0.y;
    hb.x += w1 * h1.x;
    hb.y += w1 * h1.y;
    const float d0 = wave_sum64(h0.x * u.x + h0.y * u.y), d1 = wave_sum64(h1.x * u.x + h1.y * u.y);
    if (lane == 0) {
      part_wout[base + t] = d0 + bdot;
      part_wout[base + t + 4] = d1 + bdot;
    }
  }
  for (; t < T; t += 4) {
    const float2 h0 = Hs[t * (GHM_D / 2)];
    const float w0 = wout[t];
    dHs[t * (GHM_D / 2)] = make_float2(w0 * u.x, w0 * u.y);
    hb.x += w0 * h0.x;
    hb.y += w0 * h0.y;
    const float d0 = wave_sum64(h0.x * u.x + h0.y * u.y);
    if (lane == 0) part_wout[base + t] = d0 + bdot;
  }
  red[w][lane] = hb;
  __syncthreads();
  if (w != 0) return;
  float2 hbar;
  hbar.x = (red[0][lane].x + red[1][lane].x) + (red[2][lane].x + red[3][lane].x);
  hbar.y = (red[0][lane].y + red[1][lane].y) + (red[2][lane].y + red[3][lane].y);
  float2* pw = reinterpret_cast<float2*>(part_wro + static_cast<int64_t>(n) * NC * GHM_D) + lane;
#pragma unroll
  for (int c = 0; c < NC; ++c) pw[c * (GHM_D / 2)] = make_float2(de[c] * hbar.x, de[c] * hbar.y);
  float sw = 0.f;
  for (int k = lane; k < T; k += 64) sw += wout[k];
  sw = wave_sum64(sw);
  if (lane < NC) {
    float dl = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) dl = lane == c ? de[c] : dl;
    part_bro[static_cast<int64_t>(n) * NC + lane] = dl * sw;
  }
  if (lane == 0) {
    float sbo = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) sbo += de[c];
    part_bout[n] = sbo;
  }
}

// ---------------------------------------------------------------------------
// Embedding gradients in one pass over dH_0 [n_seq][T][128]   (model.py:764-765)
//   tok_grad[v] = sum over (n, t) with token v of dH_0[n][t],
//   pos_grad[t] = sum over n of dH_0[n][t].
// Workgroup (t, s): position t of the sequences of split s, 32 lanes (float4)
// per row, 8 rows at a time (4 in flight per thread); every thread sums its rows
// in sequence order into the position sum and, through a 0/1 fused multiply-add
// (exact), into the sum of the row's token; the 8 row slots combine in order
// through LDS.  Partials: tokens [s T + t][V][128] then positions [s][T][128];
// the caller reduces them over their leading index (ghm_reduce_batch jobs of
// S T and S splits: the trainer's final partial-reduction launch), so the
// gradients cost one pass over dH_0 and no launch of their own.  Replaces two
// column-sum passes over dH_0 (token ids, then positions: 4 launches, ~50 us of
// the step's serial tail).
// ---------------------------------------------------------------------------
constexpr int EMB_SPLIT = 4;
template <int V>
__global__ __launch_bounds__(256) void k_embed_grad_part(const float* __restrict__ dH, const uint8_t* __restrict__ tok,
                                                         int n_seq, int T, float* __restrict__ part) {
  __shared__ float4 red[8][V + 1][32];
  const int t = blockIdx.x, sp = blockIdx.y, slot = threadIdx.x >> 5, c4 = threadIdx.x & 31;
  const int n0 = static_cast<int>((static_cast<int64_t>(n_seq) * sp) / EMB_SPLIT);
  const int n1 = static_cast<int>((static_cast<int64_t>(n_seq) * (sp + 1)) / EMB_SPLIT);
  float4 pos = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int nb = n0 + slot; nb < n1; nb += 32) {  // 4 rows in flight, summed in sequence order
    float4 x[4];
    int tv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = nb + 8 * u;
      const int nc = n < n1 ? n : nb;  // rows past the split re-read row nb with token -1 (no class)
      const int64_t row = static_cast<int64_t>(nc) * T + t;
      x[u] = reinterpret_cast<const float4*>(dH + row * GHM_D)[c4];
      tv[u] = n < n1 ? static_cast<int>(tok[row]) : -1;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float pw = tv[u] >= 0 ? 1.f : 0.f;
      pos.x = fmaf(x[u].x, pw, pos.x); pos.y = fmaf(x[u].y, pw, pos.y);
      pos.z = fmaf(x[u].z, pw, pos.z); pos.w = fmaf(x[u].w, pw, pos.w);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float w = tv[u] == v ? 1.f : 0.f;  // acc + 1 * x = acc + x, acc + 0 * x = acc: exact
        acc[v].x = fmaf(x[u].x, w, acc[v].x);
        acc[v].y = fmaf(x[u].y, w, acc[v].y);
        acc[v].z = fmaf(x[u].z, w, acc[v].z);
        acc[v].w = fmaf(x[u].w, w, acc[v].w);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) red[slot][v][c4] = acc[v];
  red[slot][V][c4] = pos;
  __syncthreads();
  // thread (k, c4), k < V + 1 (the 8 row slots in order): token rows, then the position row
  float4* ptok = reinterpret_cast<float4*>(part) + (static_cast<int64_t>(sp) * T + t) * V * 32;
  float4* ppos = reinterpret_cast<float4*>(part) + static_cast<int64_t>(EMB_SPLIT) * T * V * 32 +
                 (static_cast<int64_t>(sp) * T + t) * 32;
  for (int e = threadIdx.x; e < (V + 1) * 32; e += 256) {
    const int k = e >> 5, c = e & 31;
    float4 a = red[0][k][c];
#pragma unroll
    for (int q = 1; q < 8; ++q) {
      const float4 b = red[q][k][c];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    (k < V ? ptok[k * 32 + c] : ppos[c]) = a;
  }
}

// ---------------------------------------------------------------------------
// Deterministic partial reductions, several jobs per launch.  Wide, shallow jobs
// (the weight-gradient partials): thread = one output, its splits summed in 8
// interleaved partial sums and a balanced tree, 256 outputs per block.  The others (LayerNorm / readout /
// embedding partials: up to 10 K outputs over hundreds of splits): 16
// outputs x 16 split groups per block, group g summing splits g, g+16, ... in
// order and the 16 group sums added in order.  Either way a fixed summation
// order independent of timing.  Block b serves the job whose block range
// contains b.
// ---------------------------------------------------------------------------
#define GHM_MAX_JOBS 32  // 32 x 96-B jobs + block table: 3.3 KB of kernel arguments
// a job takes one thread per output when it is wide and shallow (the split-K
// weight partials: 49 K - 66 K outputs x 64 - 85 splits)
__host__ __device__ __forceinline__ bool red_wide(int64_t n, int n_split) { return n >= 8192 && n_split <= 256; }
struct ReduceJobs {
  ghm_reduce_job job[GHM_MAX_JOBS];
  int64_t blk_end[GHM_MAX_JOBS];  // cumulative block counts
  int n_jobs;
};

__device__ __forceinline__ void red_store(const ghm_reduce_job& jb, int64_t i, float t) {
  int d = 0;
  while (d + 1 < jb.n_seg && i >= jb.off[d + 1]) ++d;
  jb.dst[d][i - jb.off[d]] = t;
}

__global__ __launch_bounds__(256) void k_reduce(ReduceJobs J) {
  __shared__ float red[16][17];
  int q = 0;
  while (q + 1 < J.n_jobs && static_cast<int64_t>(blockIdx.x) >= J.blk_end[q]) ++q;
  const ghm_reduce_job& jb = J.job[q];
  const int64_t blk = static_cast<int64_t>(blockIdx.x) - (q ? J.blk_end[q - 1] : 0);
  const int64_t n = jb.n;
  if (red_wide(n, jb.n_split)) {
    const int64_t i = blk * 256 + threadIdx.x;
    if (i >= n) return;
    // 8 interleaved partial sums (split k goes to sum k % 8), combined as a
    // balanced tree: as accurate as the round-1 16-group tree, more loads in flight
    const float* p = jb.part + i;
    float a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = 0.f;
    int k = 0;
    // 32 loads in flight per round trip (the launch is latency-bound: 8 per trip
    // took 64-85 splits / 8 serial trips); the sums keep their order (split k
    // into a[k % 8], k ascending), so the result is unchanged bit for bit
    for (; k + 32 <= jb.n_split; k += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = p[static_cast<int64_t>(k + u) * n];
#pragma unroll
      for (int u = 0; u < 32; ++u) a[u & 7] += v[u];
    }
    for (; k + 8 <= jb.n_split; k += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[static_cast<int64_t>(k + u) * n];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += v[u];
    }
    for (int u = 0; k < jb.n_split; ++k, ++u) a[u] += p[static_cast<int64_t>(k) * n];
    red_store(jb, i, ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7])));
    return;
  }
  const int e = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t i = blk * 16 + e;
  float s = 0.f;
  if (i < n) {
#pragma unroll 8
    for (int k = g; k < jb.n_split; k += 16) s += jb.part[static_cast<int64_t>(k) * n + i];
  }
  red[g][e] = s;
  __syncthreads();
  if (g == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][e];
    red_store(jb, i, t);
  }
}

// ---------------------------------------------------------------------------
// C-ABI launchers
// ---------------------------------------------------------------------------
extern "C" int ghm_readout_bwd(const float* H, const float* W_ro, const float* b_ro,
                               const float* w_out, const float* d_emb, float* dH, float* part_wro,
                               float* part_bro, float* part_wout, float* part_bout, int64_t n_seq,
                               int T, int D, int C, void* stream) {
  GHM_CHECK(H && W_ro && b_ro && w_out && d_emb && dH && part_wro && part_bro && part_wout && part_bout,
            "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96)");
  GHM_CHECK(C == 10, "readout kernels are built for num_class == 10 (the GHM vocabulary)");
  hipLaunchKernelGGL(k_readout_bwd<10>, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, ghm_stream(stream),
                     H, W_ro, b_ro, w_out, d_emb, dH, part_wro, part_bro, part_wout, part_bout, T);
  return ghm_launch_status();
}

extern "C" int ghm_readout_bwd_clip(const float* H, const float* W_ro, const float* b_ro, const float* w_out,
                                    const float* t_emb, const float* i_emb, int tower, int B, int K, float* d_emb,
                                    float* dH, float* part_wro, float* part_bro, float* part_wout, float* part_bout,
                                    int64_t n_seq, int T, int D, int C, void* stream) {
  GHM_CHECK(H && W_ro && b_ro && w_out && t_emb && i_emb && d_emb && dH && part_wro && part_bro && part_wout &&
                part_bout, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96)");
  GHM_CHECK(C == 10, "readout kernels are built for num_class == 10 (the GHM vocabulary)");
  GHM_CHECK(tower == 0 || tower == 1, "tower 0 (text) or 1 (image)");
  GHM_CHECK(B >= 1 && K >= 2 && n_seq == static_cast<int64_t>(K + 1) * B, "n_seq must be (K + 1) B");
  hipStream_t s = ghm_stream(stream);
  hipLaunchKernelGGL(k_clip_grad_rows<10>, dim3(static_cast<unsigned>((n_seq + 63) / 64)), dim3(64), 0, s, t_emb,
                     i_emb, tower, B, K, d_emb);
  hipLaunchKernelGGL(k_readout_bwd<10>, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, s, H, W_ro, b_ro, w_out,
                     d_emb, dH, part_wro, part_bro, part_wout, part_bout, T);
  return ghm_launch_status();
}

extern "C" int ghm_embed_bwd_splits(void) { return EMB_SPLIT; }

extern "C" int64_t ghm_embed_bwd_part_elems(int T, int V) {
  return static_cast<int64_t>(EMB_SPLIT) * T * (V + 1) * GHM_D;
}

extern "C" int ghm_embed_bwd_part(const float* dH0, const uint8_t* tokens, int64_t n_seq, int T, int V, int D,
                                  float* part, void* stream) {
  GHM_CHECK(dH0 && tokens && part, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && n_seq >= 1 && n_seq < (int64_t(1) << 30), "shape (D == 128)");
  GHM_CHECK(V == 10, "token embedding gradients are built for the 10-value GHM vocabulary");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(dH0) | reinterpret_cast<uintptr_t>(part)) & 15) == 0, "16-byte aligned");
  hipLaunchKernelGGL(k_embed_grad_part<10>, dim3(static_cast<unsigned>(T), EMB_SPLIT), dim3(256), 0,
                     ghm_stream(stream), dH0, tokens, static_cast<int>(n_seq), T, part);
  return ghm_launch_status();
}

extern "C" int ghm_mlp_bwd(const float* dH_out, const float* H_mid, const float* stats,
                           const float* ln_w, const float* W1, const float* W2, const float* U,
                           float* dU, float* dH_mid, float* part_ln, int64_t M, int D, int F,
                           void* stream) {
  GHM_CHECK(dH_out && H_mid && stats && ln_w && W1 && W2 && U && dU && dH_mid && part_ln, "null pointer");
  GHM_CHECK(M < (int64_t(1) << 28), "stats byte offsets must fit 31 bits (M < 2^28 tokens)");
  GHM_CHECK(D == GHM_D && F == GHM_F && M >= 1, "shape (D == 128, F == 512)");
  hipLaunchKernelGGL(k_mlp_bwd, dim3(static_cast<unsigned>(ghm_token_blocks(M))), dim3(256), 0,
                     ghm_stream(stream), dH_out, H_mid, reinterpret_cast<const float2*>(stats), ln_w, W1,
                     W2, U, dU, dH_mid, part_ln, M);
  return ghm_launch_status();
}

template <int ACT>
static void attn_bwd_launch(const float* qkv, const float* P, const float* Pd, const float* dH_mid, float* dS,
                            float* dqkv, int64_t n_seq, int T, float scale_div, hipStream_t s) {
  const unsigned g = static_cast<unsigned>(n_seq);
  if (T <= 32) {
    hipLaunchKernelGGL((k_attn_bwd_q<1, ACT>), dim3(g), dim3(64), 0, s, qkv, P, dH_mid, dS, dqkv, T, scale_div, Pd);
    hipLaunchKernelGGL(k_attn_bwd_kv<1>, dim3(g), dim3(64), 0, s, qkv, P, dS, dH_mid, dqkv, T);
  } else if (T <= 64) {
    hipLaunchKernelGGL((k_attn_bwd_q<2, ACT>), dim3(g), dim3(128), 0, s, qkv, P, dH_mid, dS, dqkv, T, scale_div, Pd);
    hipLaunchKernelGGL(k_attn_bwd_kv<2>, dim3(g), dim3(128), 0, s, qkv, P, dS, dH_mid, dqkv, T);
  } else {
    hipLaunchKernelGGL((k_attn_bwd_q<3, ACT>), dim3(g), dim3(192), 0, s, qkv, P, dH_mid, dS, dqkv, T, scale_div, Pd);
    hipLaunchKernelGGL(k_attn_bwd_kv<3>, dim3(g), dim3(192), 0, s, qkv, P, dS, dH_mid, dqkv, T);
  }
}

extern "C" int ghm_attn_bwd(const float* qkv, const float* P, const float* dH_mid, float* dS, float* dqkv,
                            int64_t n_seq, int T, int D, float scale_div, void* stream) {
  GHM_CHECK(qkv && P && dH_mid && dS && dqkv, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96, D == 128)");
  attn_bwd_launch<ACT_SOFTMAX>(qkv, P, nullptr, dH_mid, dS, dqkv, n_seq, T, scale_div, ghm_stream(stream));
  return ghm_launch_status();
}

extern "C" int ghm_attn_bwd_act(const float* qkv, const float* P, const float* Pd, const float* dH_mid, float* dS,
                                float* dqkv, int64_t n_seq, int T, int D, float scale_div, int act, void* stream) {
  GHM_CHECK(qkv && P && dH_mid && dS && dqkv && (act != ACT_GELU || Pd), "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96, D == 128)");
  GHM_CHECK(act >= ACT_SOFTMAX && act <= ACT_GELU, "act: 0 softmax, 1 relu, 2 gelu");
  hipStream_t s = ghm_stream(stream);
  if (act == ACT_SOFTMAX)
    attn_bwd_launch<ACT_SOFTMAX>(qkv, P, Pd, dH_mid, dS, dqkv, n_seq, T, scale_div, s);
  else if (act == ACT_RELU)
    attn_bwd_launch<ACT_RELU>(qkv, P, Pd, dH_mid, dS, dqkv, n_seq, T, scale_div, s);
  else
    attn_bwd_launch<ACT_GELU>(qkv, P, Pd, dH_mid, dS, dqkv, n_seq, T, scale_div, s);
  return ghm_launch_status();
}

extern "C" int ghm_qkv_bwd(const float* dqkv, const float* H, const float* stats, const float* ln_w,
                           const float* Wq, const float* Wk, const float* Wv, const float* dH_mid,
                           float* dH, float* part_ln, int64_t M, int D, void* stream) {
  GHM_CHECK(dqkv && H && stats && ln_w && Wq && Wk && Wv && dH_mid && dH && part_ln, "null pointer");
  GHM_CHECK(M < (int64_t(1) << 28), "stats byte offsets must fit 31 bits (M < 2^28 tokens)");
  GHM_CHECK(D == GHM_D && M >= 1, "shape");
  hipLaunchKernelGGL(k_qkv_bwd, dim3(static_cast<unsigned>(ghm_token_blocks(M))), dim3(256), 0,
                     ghm_stream(stream), dqkv, H, reinterpret_cast<const float2*>(stats), ln_w, Wq, Wk, Wv,
                     dH_mid, dH, part_ln, M);
  return ghm_launch_status();
}

extern "C" int ghm_wgrad(const float* A, int lda, int A_cols, const float* B, int ldb, int B_cols,
                         int b_mode, const float* stats, const float* ln_w, const float* ln_b,
                         float* part, float* bias_part, int64_t M, int tok_per_split, void* stream) {
  GHM_CHECK(A && B && part, "null pointer");
  GHM_CHECK(M < (int64_t(1) << 28), "stats byte offsets must fit 31 bits (M < 2^28 tokens)");
  GHM_CHECK(A_cols > 0 && B_cols > 0 && A_cols % 128 == 0 && B_cols % 128 == 0, "A_cols/B_cols % 128");
  GHM_CHECK(lda >= A_cols && ldb >= B_cols && M >= 1, "shape");
  GHM_CHECK(tok_per_split > 0 && tok_per_split % 32 == 0, "tok_per_split must be a positive multiple of 32");
  GHM_CHECK(b_mode >= 0 && b_mode <= 2, "b_mode");
  GHM_CHECK(b_mode != 2 || (stats && ln_w && ln_b), "layernorm mode needs stats/ln_w/ln_b");
  const int64_t nsplit = (M + tok_per_split - 1) / tok_per_split;
  GHM_CHECK(nsplit <= 65535, "too many splits");
  dim3 grid(A_cols / 128, B_cols / 128, static_cast<unsigned>(nsplit));
  hipStream_t s = ghm_stream(stream);
  const float2* st = reinterpret_cast<const float2*>(stats);
  if (b_mode == 0)
    hipLaunchKernelGGL(k_wgrad<0>, grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part, bias_part, M,
                       tok_per_split, A_cols, B_cols);
  else if (b_mode == 1)
    hipLaunchKernelGGL(k_wgrad<1>, grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part, bias_part, M,
                       tok_per_split, A_cols, B_cols);
  else
    hipLaunchKernelGGL(k_wgrad<2>, grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part, bias_part, M,
                       tok_per_split, A_cols, B_cols);
  return ghm_launch_status();
}

static int validate_job(const ghm_reduce_job& j) {
  GHM_CHECK(j.part, "null partials");
  GHM_CHECK(j.n_split >= 1 && j.n >= 1 && j.n_seg >= 1 && j.n_seg <= 4, "job shape");
  GHM_CHECK(j.off[0] == 0 && j.off[j.n_seg] == j.n, "segment offsets");
  for (int k = 0; k < j.n_seg; ++k) GHM_CHECK(j.dst[k] && j.off[k] <= j.off[k + 1], "segment");
  return 0;
}

extern "C" int ghm_reduce_batch(const ghm_reduce_job* jobs, int n_jobs, void* stream) {
  GHM_CHECK(jobs && n_jobs >= 1 && n_jobs <= GHM_MAX_JOBS, "1..32 jobs");
  ReduceJobs J;
  J.n_jobs = n_jobs;
  int64_t blocks = 0;
  for (int q = 0; q < GHM_MAX_JOBS; ++q) {
    if (q < n_jobs) {
      const int rc = validate_job(jobs[q]);
      if (rc) return rc;
      J.job[q] = jobs[q];
      blocks += red_wide(jobs[q].n, jobs[q].n_split) ? (jobs[q].n + 255) / 256 : (jobs[q].n + 15) / 16;
    } else {
      J.job[q] = jobs[n_jobs - 1];
    }
    J.blk_end[q] = blocks;
  }
  hipLaunchKernelGGL(k_reduce, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, ghm_stream(stream), J);
  return ghm_launch_status();
}

extern "C" int ghm_reduce_partials(const float* part, int n_split, int64_t n, int n_seg,
                                   float* const* dst, const int64_t* off, void* stream) {
  GHM_CHECK(dst && off, "null pointer");
  GHM_CHECK(n_seg >= 1 && n_seg <= 4, "segments");
  ghm_reduce_job j;
  j.part = part;
  j.n_split = n_split;
  j.n = n;
  j.n_seg = n_seg;
  for (int k = 0; k < 4; ++k) j.dst[k] = k < n_seg ? dst[k] : nullptr;
  for (int k = 0; k < 5; ++k) j.off[k] = k <= n_seg ? off[k] : n;
  return ghm_reduce_batch(&j, 1, stream);
}
