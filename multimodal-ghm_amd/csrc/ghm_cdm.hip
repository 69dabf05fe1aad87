// Sequential conditional denoising (CDM, BASELINE config 4) on the device: the
// parts of ConditionalDenoiseEncoderTransformer that differ from the CLIP encoder
// (the layer stack reuses the LN+QKV / attention / LN+MLP kernels unchanged at
// T = 82 tokens), its loss, and the exact BP_DNS posterior the reference logs as
// "Compare".
// Reference (src/ghmclip/):
//   token_embeddings (sequential)  models/model.py:404-423
//   embedding + positions          models/model.py:430-437
//   readout                        models/model.py:527-531   (_read_out: Linear(d, 1))
//   loss                           models/model.py:997-998, :1152-1160 (sum of squares per sample, mean)
//   BP_CLS root message            data/data_random_GHM.py:185-208
//   BP_DNS                         data/data_random_GHM.py:467-523
//   sampler glue                   data/data_random_GHM.py:854-884
#include "ghm_common.h"
#include "ghm_launch.h"

constexpr int DNS_MAXV = 16;
constexpr int DNS_MAXNODES = 128;  // non-root nodes of the image tree (81 + 27 + 9 + 3 = 120)
constexpr int DNS_MAXLEAF = 96;

// H0[n, t, :] = e(n, t) + pos[t, :] with
//   t <  T_img: e[d] = -((d - z[n, t])^2) / 2 for d < V, else 0   (:412-416)
//   t >= T_img: e[d] = cond[n, t - T_img, d] for d < V, else 0   (:418-423)
// One thread per 4 features of a token (float4 in / out).
__global__ __launch_bounds__(256) void k_cdm_embed_fwd(const float* __restrict__ z, const float* __restrict__ cond,
                                                       int cond_ld, const float* __restrict__ pos,
                                                       float* __restrict__ H0, int64_t n_tok, int T, int T_img,
                                                       int V) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (idx >= n_tok * (GHM_D / 4)) return;
  const int q = static_cast<int>(idx & 31);
  const int64_t m = idx >> 5;
  const int64_t n = m / T;
  const int t = static_cast<int>(m % T);
  const float4 p = *reinterpret_cast<const float4*>(pos + static_cast<int64_t>(t) * GHM_D + 4 * q);
  float e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int d = 4 * q + k;
    float v = 0.f;
    if (d < V) {
      if (t < T_img) {
        const float x = static_cast<float>(d) - z[n * T_img + t];
        v = -(x * x) * 0.5f;
      } else {
        v = cond[(n * (T - T_img) + (t - T_img)) * cond_ld + d];
      }
    }
    e[k] = v;
  }
  st4(H0 + m * GHM_D + 4 * q, e[0] + p.x, e[1] + p.y, e[2] + p.z, e[3] + p.w);
}

// Joint CDM embedding (ConditionalDenoiseEncoderTransformer, sequential=False,
// model.py:408-423, :437): image token t < T_img gets -(d - z)^2 / 2 in d < V,
// text token t >= T_img gets the full row t_emb[tok[n, t - T_img]]; + positions.
__global__ __launch_bounds__(256) void k_cdm_embed_joint_fwd(const float* __restrict__ z,
                                                             const uint8_t* __restrict__ tok,
                                                             const float* __restrict__ t_emb,
                                                             const float* __restrict__ pos, float* __restrict__ H0,
                                                             int64_t n_tok, int T, int T_img, int V) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (idx >= n_tok * (GHM_D / 4)) return;
  const int q = static_cast<int>(idx & 31);
  const int64_t m = idx >> 5;
  const int64_t n = m / T;
  const int t = static_cast<int>(m % T);
  const float4 p = *reinterpret_cast<const float4*>(pos + static_cast<int64_t>(t) * GHM_D + 4 * q);
  float4 e;
  if (t < T_img) {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int d = 4 * q + k;
      const float x = static_cast<float>(d) - z[n * T_img + t];
      v[k] = d < V ? -(x * x) * 0.5f : 0.f;
    }
    e = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    const int c = tok[n * (T - T_img) + (t - T_img)];
    e = *reinterpret_cast<const float4*>(t_emb + static_cast<int64_t>(c) * GHM_D + 4 * q);
  }
  st4(H0 + m * GHM_D + 4 * q, e.x + p.x, e.y + p.y, e.z + p.z, e.w + p.w);
}

// --------------------------------------------------------------------------
// Exact BP on the device, f64 like the reference's numpy.  One 64-thread
// workgroup per sample: the text tree's BP_CLS root message (:185-208), then
// BP_DNS of the image tree with that message as external evidence (:467-523).
// Node k of depth d uses the translation-invariant matrix of child slot k % C.
// trans: [L][C][V][V] (row = parent value, column = child value).
// --------------------------------------------------------------------------
__device__ __forceinline__ void bp_shift(double* m, int nodes, int V, int tid) {
  for (int node = tid; node < nodes; node += 64) {
    double mx = m[node * V];
    for (int v = 1; v < V; ++v) mx = fmax(mx, m[node * V + v]);
    for (int v = 0; v < V; ++v) m[node * V + v] -= mx;
  }
}

// Guided-CDM targets (data_random_GHM.py:563-592 reads them off the tree): the
// image tree's hd / qd / bu messages as f32 planes [n][3][n_nodes][V]; node
// index = depth-d breadth-first order starting at off[d], root last.  The root
// has hd and bu only (plane 1 of the root is never read).
__device__ __forceinline__ void dns_emit(float* msgs, int n, int n_nodes, int plane, int node0, const double* src,
                                         int cnt, int V, int tid) {
  if (!msgs) return;
  float* o = msgs + ((static_cast<int64_t>(n) * 3 + plane) * n_nodes + node0) * V;
  for (int e = tid; e < cnt * V; e += 64) o[e] = static_cast<float>(src[e]);
}

__global__ __launch_bounds__(64) void k_bp_dns(const double* __restrict__ t_trans, const double* __restrict__ i_trans,
                                               const uint8_t* __restrict__ t_tok, const double* __restrict__ z,
                                               double sigma, float* __restrict__ post, float* __restrict__ z32,
                                               float* __restrict__ msgs, int n_nodes,
                                               int Lt, int Ct, int Tt, int Li, int Ci, int Ti, int V,
                                               int per_edge) {
  const int pe_t = per_edge & 1, pe_i = (per_edge >> 1) & 1;
  __shared__ double hd[DNS_MAXNODES * DNS_MAXV];
  __shared__ double qd[DNS_MAXNODES * DNS_MAXV];
  __shared__ double bu_a[DNS_MAXLEAF * DNS_MAXV];
  __shared__ double bu_b[DNS_MAXLEAF * DNS_MAXV];
  __shared__ double ext[DNS_MAXV];
  const int n = blockIdx.x, tid = threadIdx.x;

  // ---- text tree: BP_CLS messages up to the root (cur/nxt ping-pong in hd/qd)
  {
    const uint8_t* x = t_tok + static_cast<int64_t>(n) * Tt;
    double* cur = hd;
    double* nxt = qd;
    int nodes = Tt / Ct;
    for (int e = tid; e < nodes * V; e += 64) {
      const int node = e / V, v = e % V;
      double s = 0.0;
      for (int c = 0; c < Ct; ++c) {
        int xv = x[node * Ct + c];
        xv = xv < V ? xv : V - 1;
        s += log(bp_edge(t_trans, Lt - 1, node * Ct + c, Ct, V, pe_t)[v * V + xv]);
      }
      cur[e] = s;
    }
    __syncthreads();
    bp_shift(cur, nodes, V, tid);
    __syncthreads();
    for (int d = Lt - 1; d > 0; --d) {
      const int np = nodes / Ct;
      for (int e = tid; e < np * V; e += 64) {
        const int node = e / V, v = e % V;
        double s = 0.0;
        for (int c = 0; c < Ct; ++c) {
          const double* tr = bp_edge(t_trans, d - 1, node * Ct + c, Ct, V, pe_t) + v * V;
          const double* ch = cur + (node * Ct + c) * V;
          double a = 0.0;
          for (int u = 0; u < V; ++u) a += tr[u] * exp(ch[u]);
          s += log(a);
        }
        nxt[e] = s;
      }
      __syncthreads();
      bp_shift(nxt, np, V, tid);
      __syncthreads();
      double* tmp = cur;
      cur = nxt;
      nxt = tmp;
      nodes = np;
    }
    if (tid < V) ext[tid] = cur[tid];  // root hd_message (max-shifted)
    __syncthreads();
  }

  // ---- image tree: BP_DNS.  Level offsets: depth d (1..Li) starts at off[d].
  int off[8];
  {
    int o = 0, w = Ci;
    for (int d = 1; d <= Li; ++d) {
      off[d] = o;
      o += w;
      w *= Ci;
    }
  }
  const double* zn = z + static_cast<int64_t>(n) * Ti;
  const double s2 = sigma * sigma;
  // leaves: hd = -0.5 (z - v)^2 / sigma^2, qd = log(T_slot @ exp(hd))   (:481-486)
  for (int e = tid; e < Ti * V; e += 64) {
    const int leaf = e / V, v = e % V;
    const double dz = zn[leaf] - static_cast<double>(v);
    hd[(off[Li] + leaf) * V + v] = -0.5 * (dz * dz) / s2;
  }
  for (int leaf = tid; leaf < Ti; leaf += 64) z32[static_cast<int64_t>(n) * Ti + leaf] = static_cast<float>(zn[leaf]);
  __syncthreads();
  dns_emit(msgs, n, n_nodes, 0, off[Li], hd + off[Li] * V, Ti, V, tid);  // leaf hd (not max-shifted, :483)
  // downward pass, leaves -> root (:489-495): qd of depth d from its hd, then
  // hd of depth d-1 = sum of the children's qd (slot order), max-shifted
  for (int d = Li, cnt = Ti; d >= 1; --d, cnt /= Ci) {
    for (int e = tid; e < cnt * V; e += 64) {
      const int node = e / V, v = e % V;
      const double* tr = bp_edge(i_trans, d - 1, node, Ci, V, pe_i) + v * V;
      const double* h = hd + (off[d] + node) * V;
      double a = 0.0;
      for (int u = 0; u < V; ++u) a += tr[u] * exp(h[u]);
      qd[(off[d] + node) * V + v] = log(a);
    }
    __syncthreads();
    dns_emit(msgs, n, n_nodes, 1, off[d], qd + off[d] * V, cnt, V, tid);
    if (d == 1) break;
    const int np = cnt / Ci;
    for (int e = tid; e < np * V; e += 64) {
      const int node = e / V, v = e % V;
      double s = 0.0;
      for (int c = 0; c < Ci; ++c) s += qd[(off[d] + node * Ci + c) * V + v];
      hd[(off[d - 1] + node) * V + v] = s;
    }
    __syncthreads();
    bp_shift(hd + off[d - 1] * V, np, V, tid);
    __syncthreads();
    dns_emit(msgs, n, n_nodes, 0, off[d - 1], hd + off[d - 1] * V, np, V, tid);
  }
  // root: hd = sum of the children's qd, max shift, bu = hd + external (:499-504)
  double* bu = bu_a;
  double* bn = bu_b;
  if (tid == 0) {
    double r[DNS_MAXV];
    double mx = -1e300;
    for (int v = 0; v < V; ++v) {
      double s = 0.0;
      for (int c = 0; c < Ci; ++c) s += qd[(off[1] + c) * V + v];
      r[v] = s;
      mx = fmax(mx, s);
    }
    for (int v = 0; v < V; ++v) bu[v] = (r[v] - mx) + ext[v];
    if (msgs) {
      float* o = msgs + static_cast<int64_t>(n) * 3 * n_nodes * V;
      for (int v = 0; v < V; ++v) {
        // root hd: the reference's `bu_message = hd_message; bu_message += external`
        // (data_random_GHM.py:501-504) adds in place to the shared numpy array, so
        // the root's hd guide target is its bu message as well
        o[(n_nodes - 1) * V + v] = static_cast<float>(bu[v]);
        o[(2 * n_nodes + n_nodes - 1) * V + v] = static_cast<float>(bu[v]);          // root bu
      }
    }
  }
  __syncthreads();
  // upward pass, root -> leaves (:507-512)
  int nodes = 1;
  for (int d = 1; d <= Li; ++d) {
    nodes *= Ci;
    for (int e = tid; e < nodes * V; e += 64) {
      const int node = e / V, v = e % V;
      const double* tr = bp_edge(i_trans, d - 1, node, Ci, V, pe_i) + v;  // column v
      const double* par = bu + (node / Ci) * V;
      const double* q = qd + (off[d] + node) * V;
      double a = 0.0;
      for (int u = 0; u < V; ++u) a += tr[u * V] * exp(par[u] - q[u]);
      bn[node * V + v] = hd[(off[d] + node) * V + v] + log(a);
    }
    __syncthreads();
    bp_shift(bn, nodes, V, tid);
    __syncthreads();
    dns_emit(msgs, n, n_nodes, 2, off[d], bn, nodes, V, tid);
    double* tmp = bu;
    bu = bn;
    bn = tmp;
  }
  // posterior means sum_v v exp(bu) / sum_v exp(bu)   (:514-518)
  for (int leaf = tid; leaf < Ti; leaf += 64) {
    double num = 0.0, den = 0.0;
    for (int v = 0; v < V; ++v) {
      const double w = exp(bu[leaf * V + v]);
      num += static_cast<double>(v) * w;
      den += w;
    }
    post[static_cast<int64_t>(n) * Ti + leaf] = static_cast<float>(num / den);
  }
}

// pred[n, t] = H[n, t, :] . w + b for t < T_img (:527-531).  One wave per token,
// lane = 2 features (coalesced 512-B rows), fixed shuffle tree.
__global__ __launch_bounds__(256) void k_cdm_readout_fwd(const float* __restrict__ H, const float* __restrict__ w,
                                                         const float* __restrict__ b, float* __restrict__ pred,
                                                         int64_t n_pred, int T, int T_img) {
  const int lane = threadIdx.x & 63;
  const int64_t k = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (k >= n_pred) return;
  const int64_t n = k / T_img;
  const int t = static_cast<int>(k % T_img);
  const float2 h = *reinterpret_cast<const float2*>(H + (n * T + t) * GHM_D + 2 * lane);
  const float2 ww = *reinterpret_cast<const float2*>(w + 2 * lane);
  float s = h.x * ww.x + h.y * ww.y;
  s = sum32(s);
  s += xhalf(s);
  if (lane == 0) pred[k] = s + b[0];
}

// Sum-of-squares loss of the CDM (ConditionalGuidedLsLoss guide=False, LsLoss):
//   loss = mean_n sum_t (pred - target)^2, compare = the same against the BP
//   posterior means; dpred = 2 (pred - target) / N.  One 1024-thread workgroup:
//   wave w takes rows w, w+16, ... (lanes over tokens, coalesced), each row sum a
//   fixed shuffle tree, rows accumulated in order per wave, waves in fixed order
//   (deterministic).  loss_out[0] <- loss, loss_out[1] <- compare; hist /
//   chist[*step] likewise.
constexpr int LS_WAVES = 16;
__global__ __launch_bounds__(64 * LS_WAVES) void k_ls_loss(const float* __restrict__ pred,
                                                           const uint8_t* __restrict__ target,
                                                           const float* __restrict__ post, float* __restrict__ dpred,
                                                           float* __restrict__ loss_out, float* __restrict__ hist,
                                                           float* __restrict__ chist,
                                                           const int32_t* __restrict__ step, int N, int Tp) {
  __shared__ float red[2][LS_WAVES];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float inv2 = 2.f / static_cast<float>(N);
  float sl = 0.f, sc = 0.f;
  for (int n = w; n < N; n += LS_WAVES) {
    float rl = 0.f, rc = 0.f;
    for (int t = lane; t < Tp; t += 64) {
      const int64_t i = static_cast<int64_t>(n) * Tp + t;
      const float p = pred[i];
      const float r = p - static_cast<float>(target[i]);
      rl += r * r;
      if (dpred) dpred[i] = inv2 * r;
      if (post) {
        const float c = p - post[i];
        rc += c * c;
      }
    }
    rl = sum32(rl);
    rl += xhalf(rl);
    rc = sum32(rc);
    rc += xhalf(rc);
    sl += rl;
    sc += rc;
  }
  if (lane == 0) {
    red[0][w] = sl;
    red[1][w] = sc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float l = 0.f, c = 0.f;
    for (int k = 0; k < LS_WAVES; ++k) {
      l += red[0][k];
      c += red[1][k];
    }
    l /= static_cast<float>(N);
    c /= static_cast<float>(N);
    loss_out[0] = l;
    loss_out[1] = c;
    if (hist && step) hist[*step] = l;
    if (chist && step) chist[*step] = c;
  }
}

// Readout backward, one 256-thread workgroup per sequence (wave w takes tokens
// w, w+4, ...; lane = 2 features):
//   dH[n, t, :] = dpred[n, t] * w for t < T_img, 0 for the conditioning tokens
//   part_w[n, :] = sum_t dpred[n, t] H[n, t, :],  part_b[n] = sum_t dpred[n, t]
__global__ __launch_bounds__(256) void k_cdm_readout_bwd(const float* __restrict__ H, const float* __restrict__ w,
                                                         const float* __restrict__ dpred, float* __restrict__ dH,
                                                         float* __restrict__ part_w, float* __restrict__ part_b,
                                                         int T, int T_img) {
  __shared__ float2 red[4][64];
  const int n = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float2 ww = *reinterpret_cast<const float2*>(w + 2 * lane);
  float2 acc = make_float2(0.f, 0.f);
  for (int t = wv; t < T; t += 4) {
    const int64_t row = (static_cast<int64_t>(n) * T + t) * GHM_D + 2 * lane;
    float2 o = make_float2(0.f, 0.f);
    if (t < T_img) {
      const float dp = dpred[static_cast<int64_t>(n) * T_img + t];
      const float2 h = *reinterpret_cast<const float2*>(H + row);
      acc.x += dp * h.x;
      acc.y += dp * h.y;
      o = make_float2(dp * ww.x, dp * ww.y);
    }
    *reinterpret_cast<float2*>(dH + row) = o;
  }
  red[wv][lane] = acc;
  __syncthreads();
  if (wv == 0) {
    const float2 a = red[0][lane], b = red[1][lane], c = red[2][lane], d = red[3][lane];
    *reinterpret_cast<float2*>(part_w + static_cast<int64_t>(n) * GHM_D + 2 * lane) =
        make_float2((a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y));
  }
  if (threadIdx.x == 64) {
    float s = 0.f;
    for (int t = 0; t < T_img; ++t) s += dpred[static_cast<int64_t>(n) * T_img + t];
    part_b[n] = s;
  }
}

// ---------------------------------------------------------------------------
// C-ABI launchers
// ---------------------------------------------------------------------------
extern "C" int ghm_cdm_embed_fwd(const float* z, const float* cond, int cond_ld, const float* pos_w, float* H0,
                                 int64_t n_seq, int T, int T_img, int V, int D, void* stream) {
  GHM_CHECK(z && pos_w && H0 && (cond || T == T_img), "null pointer");
  GHM_CHECK(D == GHM_D && T >= T_img && T_img >= 1 && T <= GHM_MAXT && V >= 1 && V <= GHM_D && n_seq >= 1,
            "shape (D == 128, T_img <= T <= 96)");
  GHM_CHECK(T == T_img || cond_ld >= V, "cond_ld");
  const int64_t n = n_seq * T * (GHM_D / 4);
  hipLaunchKernelGGL(k_cdm_embed_fwd, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, ghm_stream(stream),
                     z, cond, cond_ld, pos_w, H0, n_seq * T, T, T_img, V);
  return ghm_launch_status();
}

extern "C" int ghm_cdm_embed_joint_fwd(const float* z, const uint8_t* tok, const float* t_emb, const float* pos_w,
                                       float* H0, int64_t n_seq, int T, int T_img, int V, int D, void* stream) {
  GHM_CHECK(z && tok && t_emb && pos_w && H0, "null pointer");
  GHM_CHECK(D == GHM_D && T > T_img && T_img >= 1 && T <= 192 && V >= 1 && V <= 16 && n_seq >= 1,
            "shape (D == 128, T_img < T <= 192, V <= 16)");
  const int64_t n = n_seq * T * (GHM_D / 4);
  hipLaunchKernelGGL(k_cdm_embed_joint_fwd, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     ghm_stream(stream), z, tok, t_emb, pos_w, H0, n_seq * T, T, T_img, V);
  return ghm_launch_status();
}

static int tree_leaves(int L, int C) {
  int T = 1;
  for (int d = 0; d < L; ++d) T *= C;
  return T;
}

static int bp_dns_launch(const double* t_trans, const double* i_trans, const uint8_t* t_tokens, const double* z,
                         double sigma, float* post, float* z32, float* msgs, int64_t n_seq, int L_t, int C_t, int L_i,
                         int C_i, int V, int per_edge, void* stream) {
  GHM_CHECK(t_trans && i_trans && t_tokens && z && post && z32, "null pointer");
  GHM_CHECK(L_t >= 1 && C_t >= 2 && L_i >= 1 && L_i <= 6 && C_i >= 2 && V >= 2 && V <= DNS_MAXV && n_seq >= 1 &&
                sigma > 0.0,
            "shape");
  const int Tt = tree_leaves(L_t, C_t), Ti = tree_leaves(L_i, C_i);
  int nonroot = 0;
  for (int d = 1, w = C_i; d <= L_i; ++d, w *= C_i) nonroot += w;
  GHM_CHECK(Tt <= DNS_MAXLEAF && Tt / C_t <= DNS_MAXLEAF && Ti <= DNS_MAXLEAF && nonroot <= DNS_MAXNODES,
            "tree too large (leaves <= 96)");
  hipLaunchKernelGGL(k_bp_dns, dim3(static_cast<unsigned>(n_seq)), dim3(64), 0, ghm_stream(stream), t_trans, i_trans,
                     t_tokens, z, sigma, post, z32, msgs, nonroot + 1, L_t, C_t, Tt, L_i, C_i, Ti, V, per_edge);
  return ghm_launch_status();
}

extern "C" int ghm_bp_dns(const double* t_trans, const double* i_trans, const uint8_t* t_tokens, const double* z,
                          double sigma, float* post, float* z32, int64_t n_seq, int L_t, int C_t, int L_i, int C_i,
                          int V, int per_edge, void* stream) {
  return bp_dns_launch(t_trans, i_trans, t_tokens, z, sigma, post, z32, nullptr, n_seq, L_t, C_t, L_i, C_i, V,
                       per_edge, stream);
}

extern "C" int ghm_bp_dns_msgs(const double* t_trans, const double* i_trans, const uint8_t* t_tokens,
                               const double* z, double sigma, float* post, float* z32, float* msgs, int64_t n_seq,
                               int L_t, int C_t, int L_i, int C_i, int V, int per_edge, void* stream) {
  GHM_CHECK(msgs, "null pointer");
  return bp_dns_launch(t_trans, i_trans, t_tokens, z, sigma, post, z32, msgs, n_seq, L_t, C_t, L_i, C_i, V,
                       per_edge, stream);
}

extern "C" int ghm_cdm_readout_fwd(const float* H, const float* w_ro, const float* b_ro, float* pred, int64_t n_seq,
                                   int T, int T_img, int D, void* stream) {
  GHM_CHECK(H && w_ro && b_ro && pred, "null pointer");
  GHM_CHECK(D == GHM_D && T >= T_img && T_img >= 1 && n_seq >= 1, "shape (D == 128)");
  const int64_t np = n_seq * T_img;
  hipLaunchKernelGGL(k_cdm_readout_fwd, dim3(static_cast<unsigned>((np + 3) / 4)), dim3(256), 0, ghm_stream(stream),
                     H, w_ro, b_ro, pred, np, T, T_img);
  return ghm_launch_status();
}

extern "C" int ghm_ls_loss(const float* pred, const uint8_t* target, const float* post, float* dpred,
                           float* loss_out, float* hist, float* chist, const int32_t* step, int64_t n_seq, int T_img,
                           void* stream) {
  GHM_CHECK(pred && target && loss_out, "null pointer");
  GHM_CHECK(n_seq >= 1 && n_seq <= (1 << 30) && T_img >= 1, "shape");
  hipLaunchKernelGGL(k_ls_loss, dim3(1), dim3(64 * LS_WAVES), 0, ghm_stream(stream), pred, target, post, dpred,
                     loss_out, hist, chist, step, static_cast<int>(n_seq), T_img);
  return ghm_launch_status();
}

extern "C" int ghm_cdm_readout_bwd(const float* H, const float* w_ro, const float* dpred, float* dH, float* part_w,
                                   float* part_b, int64_t n_seq, int T, int T_img, int D, void* stream) {
  GHM_CHECK(H && w_ro && dpred && dH && part_w && part_b, "null pointer");
  GHM_CHECK(D == GHM_D && T >= T_img && T_img >= 1 && n_seq >= 1, "shape (D == 128)");
  hipLaunchKernelGGL(k_cdm_readout_bwd, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, ghm_stream(stream), H, w_ro,
                     dpred, dH, part_w, part_b, T, T_img);
  return ghm_launch_status();
}
