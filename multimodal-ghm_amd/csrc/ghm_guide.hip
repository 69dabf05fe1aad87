// Guided CLIP (clip_guide=True) on the device: exact BP_CLS messages of the GHM
// trees behind each sequence, and the layer-wise Frobenius penalty that pulls a
// guided layer's first V hidden features toward them.
// Reference: src/ghmclip/data/data_random_GHM.py:185-221 (GHMTree.BP_CLS),
// :526-549 (guided_info), models/model.py:790-800 (guided layers: H[:, :, 0:V]
// after each flagged layer) and :909-924 (GuidedClipLoss guide branch).
#include "ghm_common.h"
#include "ghm_launch.h"

constexpr int BP_MAXV = 16;
constexpr int BP_MAXN = 32;  // nodes at depth L-1 (T / C <= 96 / 3)

// One 64-thread workgroup per sequence, f64 arithmetic like the reference's
// numpy.  Messages are log-domain and max-shifted per node (:196, :208).
// trans: [L][C][V][V] (parent value v, child value u) of the translation-
// invariant templates; msgs: [N][n_total][V] f32, levels in guided-target order
// (depth L-1 first, root last), nodes in breadth-first order within a level.
__global__ __launch_bounds__(64) void k_bp_cls(const double* __restrict__ trans, const uint8_t* __restrict__ tok,
                                               float* __restrict__ msgs, int L, int C, int V, int T,
                                               int n_total, int per_edge) {
  __shared__ double cur[BP_MAXN * BP_MAXV];
  __shared__ double nxt[BP_MAXN * BP_MAXV];
  const int n = blockIdx.x, tid = threadIdx.x;
  const uint8_t* x = tok + static_cast<int64_t>(n) * T;
  float* out = msgs + static_cast<int64_t>(n) * n_total * V;
  int nodes = T / C;
  // depth L-1: sum_c log T_{L-1,c}[v][x_child]                        (:191-195)
  for (int e = tid; e < nodes * V; e += 64) {
    const int node = e / V, v = e % V;
    double s = 0.0;
    for (int c = 0; c < C; ++c) {
      int xv = x[node * C + c];
      xv = xv < V ? xv : V - 1;
      s += log(bp_edge(trans, L - 1, node * C + c, C, V, per_edge)[v * V + xv]);
    }
    cur[e] = s;
  }
  __syncthreads();
  int off = 0;
  for (int d = L - 1;; --d) {
    // max shift per node (:196 / :208) and emit the level
    for (int node = tid; node < nodes; node += 64) {
      double mx = cur[node * V];
      for (int v = 1; v < V; ++v) mx = fmax(mx, cur[node * V + v]);
      for (int v = 0; v < V; ++v) {
        cur[node * V + v] -= mx;
        out[(off + node) * V + v] = static_cast<float>(cur[node * V + v]);
      }
    }
    __syncthreads();
    off += nodes;
    if (d == 0) break;
    // depth d-1: sum_c log(T_{d-1,c} @ exp(child message))              (:201-207)
    const int np = nodes / C;
    for (int e = tid; e < np * V; e += 64) {
      const int node = e / V, v = e % V;
      double s = 0.0;
      for (int c = 0; c < C; ++c) {
        const double* tr = bp_edge(trans, d - 1, node * C + c, C, V, per_edge) + v * V;
        const double* ch = cur + (node * C + c) * V;
        double a = 0.0;
        for (int u = 0; u < V; ++u) a += tr[u] * exp(ch[u]);
        s += log(a);
      }
      nxt[e] = s;
    }
    __syncthreads();
    for (int e = tid; e < np * V; e += 64) cur[e] = nxt[e];
    __syncthreads();
    nodes = np;
  }
}

// Per-sequence penalty partial of one guided layer:
//   part[n] = sum_{t<T, c<V} (H[n, t, c] - msg[n][lvl_off + t / ext][c])^2
// One 128-thread workgroup per sequence, thread = token, fixed reduction tree.
__global__ __launch_bounds__(128) void k_guide_fwd(const float* __restrict__ H, const float* __restrict__ msgs,
                                                   float* __restrict__ part, int T, int V, int n_total,
                                                   int lvl_off, int ext) {
  __shared__ float red[2];
  const int n = blockIdx.x, t = threadIdx.x;
  float s = 0.f;
  if (t < T) {
    const float* h = H + (static_cast<int64_t>(n) * T + t) * GHM_D;
    const float* m = msgs + (static_cast<int64_t>(n) * n_total + lvl_off + t / ext) * V;
    for (int c = 0; c < V; ++c) {
      const float dd = h[c] - m[c];
      s += dd * dd;
    }
  }
  s = sum32(s);
  s += __shfl_xor(s, 32, 64);
  if ((t & 63) == 0) red[t >> 6] = s;
  __syncthreads();
  if (t == 0) part[n] = red[0] + red[1];
}

// dH[n, t, c] += scale * (H[n, t, c] - msg[...][c]) for c < V   (scale = 2 penalty / N)
__global__ __launch_bounds__(256) void k_guide_bwd(const float* __restrict__ H, const float* __restrict__ msgs,
                                                   float* __restrict__ dH, int64_t M, int T, int V, int n_total,
                                                   int lvl_off, int ext, float scale) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= M * V) return;
  const int64_t m = i / V;
  const int c = static_cast<int>(i % V);
  const int64_t n = m / T;
  const int t = static_cast<int>(m % T);
  const float target = msgs[(n * n_total + lvl_off + t / ext) * V + c];
  dH[m * GHM_D + c] += scale * (H[m * GHM_D + c] - target);
}

// ploss = loss_nop + penalty * mean_n sum_k part[k][n]; also the logged
// penalty value mean / penalty (GuidedClipLoss returns loss3.mean()/penalty).
// loss_io[0] holds loss_nop on entry; loss_io[1] <- ploss, loss_io[2] <- pen.
// If phist is non-NULL: phist[*step] = ploss.  One 256-thread workgroup.
__global__ __launch_bounds__(256) void k_guide_total(const float* __restrict__ part, int n_parts, int N,
                                                     float penalty, float* __restrict__ loss_io,
                                                     float* __restrict__ phist, const int32_t* __restrict__ step) {
  __shared__ float red[4];
  float s = 0.f;
  for (int n = threadIdx.x; n < N; n += 256) {
    float r = 0.f;
    for (int k = 0; k < n_parts; ++k) r += part[static_cast<int64_t>(k) * N + n];
    s += r;
  }
  s = sum32(s);
  s += __shfl_xor(s, 32, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float mean = penalty * (((red[0] + red[1]) + (red[2] + red[3])) / static_cast<float>(N));
    const float ploss = loss_io[0] + mean;
    loss_io[1] = ploss;
    loss_io[2] = mean / penalty;
    if (phist) phist[*step] = ploss;
  }
}

// ---------------------------------------------------------------------------
// C-ABI launchers
// ---------------------------------------------------------------------------
extern "C" int ghm_bp_cls(const double* trans, const uint8_t* tokens, float* msgs, int64_t n_seq, int L, int C,
                          int V, int per_edge, void* stream) {
  GHM_CHECK(trans && tokens && msgs, "null pointer");
  GHM_CHECK(L >= 1 && C >= 2 && V >= 2 && V <= BP_MAXV && n_seq >= 1, "shape");
  int T = 1, n_total = 0;
  for (int d = 0; d < L; ++d) {
    n_total += T;
    T *= C;
  }
  GHM_CHECK(T <= GHM_MAXT && T / C <= BP_MAXN, "tree too large (leaves <= 96)");
  hipLaunchKernelGGL(k_bp_cls, dim3(static_cast<unsigned>(n_seq)), dim3(64), 0, ghm_stream(stream), trans, tokens,
                     msgs, L, C, V, T, n_total, per_edge);
  return ghm_launch_status();
}

static int guide_level(int L, int C, int level, int& off, int& ext, int& n_total, int& T) {
  T = 1;
  n_total = 0;
  for (int d = 0; d < L; ++d) {
    n_total += T;
    T *= C;
  }
  off = 0;
  int nodes = T / C;
  ext = C;
  for (int k = 0; k < level; ++k) {
    off += nodes;
    nodes /= C;
    ext *= C;
  }
  return 0;
}

extern "C" int ghm_guide_fwd(const float* H, const float* msgs, float* part, int64_t n_seq, int L, int C, int V,
                             int level, void* stream) {
  GHM_CHECK(H && msgs && part, "null pointer");
  GHM_CHECK(level >= 0 && level < L && V >= 1 && V <= GHM_D && n_seq >= 1, "shape");
  int off, ext, n_total, T;
  guide_level(L, C, level, off, ext, n_total, T);
  GHM_CHECK(T <= 128, "sequence too long");
  hipLaunchKernelGGL(k_guide_fwd, dim3(static_cast<unsigned>(n_seq)), dim3(128), 0, ghm_stream(stream), H, msgs,
                     part, T, V, n_total, off, ext);
  return ghm_launch_status();
}

extern "C" int ghm_guide_bwd(const float* H, const float* msgs, float* dH, int64_t n_seq, int L, int C, int V,
                             int level, float scale, void* stream) {
  GHM_CHECK(H && msgs && dH, "null pointer");
  GHM_CHECK(level >= 0 && level < L && V >= 1 && V <= GHM_D && n_seq >= 1, "shape");
  int off, ext, n_total, T;
  guide_level(L, C, level, off, ext, n_total, T);
  const int64_t M = n_seq * T;
  hipLaunchKernelGGL(k_guide_bwd, dim3(static_cast<unsigned>((M * V + 255) / 256)), dim3(256), 0,
                     ghm_stream(stream), H, msgs, dH, M, T, V, n_total, off, ext, scale);
  return ghm_launch_status();
}

extern "C" int ghm_guide_total(const float* part, int n_parts, int64_t n_seq, float penalty, float* loss_io,
                               float* phist, const int32_t* step, void* stream) {
  GHM_CHECK(part && loss_io, "null pointer");
  GHM_CHECK(!phist || step, "phist needs step");
  GHM_CHECK(n_parts >= 1 && n_seq >= 1 && penalty > 0.f, "shape");
  hipLaunchKernelGGL(k_guide_total, dim3(1), dim3(256), 0, ghm_stream(stream), part, n_parts,
                     static_cast<int>(n_seq), penalty, loss_io, phist, step);
  return ghm_launch_status();
}

// ---------------------------------------------------------------------------
// Guided joint CDM (train_CDNS.py --guide=True, exp_cdm_guidedTF.sh): each
// guided output is a V-column block of H_{l+1} over a token range (model.py:
// 502-527), compared with a BP message that one tree node repeats over `ext`
// consecutive tokens (data_random_GHM.py:551-592).  One block:
//   target(n, t, c) = msgs[n * msg_stride + moff + (t / ext) * V + c]
//   part[n]         = sum_{t < ntok, c < V} (H[n, tok0 + t, col + c] - target)^2
//   dH[n, tok0 + t, col + c] += scale * (H[...] - target)          (bwd)
// Blocks that share columns (model.py:513-517 reads q and u from the same
// slice on the first upward layer) are applied one after another on the stream.
// ---------------------------------------------------------------------------
struct GuideBlk {
  int T, tok0, ntok, col, ext, V;
  int64_t msg_stride, moff;
  int ld;  // row pitch of H (the model width: 128 for the encoder / CDM, 256 for the VLM)
};

__global__ __launch_bounds__(256) void k_guide_blk_fwd(const float* __restrict__ H, const float* __restrict__ msgs,
                                                       float* __restrict__ part, GuideBlk b) {
  __shared__ float red[4];
  const int n = blockIdx.x;
  const float* h = H + (static_cast<int64_t>(n) * b.T + b.tok0) * b.ld + b.col;
  const float* m = msgs + static_cast<int64_t>(n) * b.msg_stride + b.moff;
  float s = 0.f;
  for (int e = threadIdx.x; e < b.ntok * b.V; e += 256) {
    const int t = e / b.V, c = e - t * b.V;
    const float dd = h[static_cast<int64_t>(t) * b.ld + c] - m[(t / b.ext) * b.V + c];
    s += dd * dd;
  }
  s = sum32(s);
  s += __shfl_xor(s, 32, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[n] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void k_guide_blk_bwd(const float* __restrict__ H, const float* __restrict__ msgs,
                                                       float* __restrict__ dH, int64_t total, GuideBlk b,
                                                       float scale) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t per = static_cast<int64_t>(b.ntok) * b.V;
  const int64_t n = i / per;
  const int r = static_cast<int>(i - n * per);
  const int t = r / b.V, c = r - t * b.V;
  const int64_t at = (n * b.T + b.tok0 + t) * b.ld + b.col + c;
  const float target = msgs[n * b.msg_stride + b.moff + (t / b.ext) * b.V + c];
  dH[at] += scale * (H[at] - target);
}

static int guide_blk_check(GuideBlk& b, int T, int tok0, int ntok, int col, int64_t msg_stride, int64_t moff,
                           int ext, int V, int64_t n_seq, int ld = GHM_D) {
  b = GuideBlk{T, tok0, ntok, col, ext, V, msg_stride, moff, ld};
  if (!(n_seq >= 1 && T >= 1 && tok0 >= 0 && ntok >= 1 && tok0 + ntok <= T && V >= 1 && col >= 0 && ld >= 1 &&
        col + V <= ld && ext >= 1 && moff >= 0 && moff + static_cast<int64_t>((ntok - 1) / ext + 1) * V <= msg_stride))
    return -1;
  return 0;
}

extern "C" int ghm_guide_blk_fwd(const float* H, int T, int tok0, int ntok, int col, const float* msgs,
                                 int64_t msg_stride, int64_t moff, int ext, int V, float* part, int64_t n_seq,
                                 void* stream) {
  GHM_CHECK(H && msgs && part, "null pointer");
  GuideBlk b;
  GHM_CHECK(guide_blk_check(b, T, tok0, ntok, col, msg_stride, moff, ext, V, n_seq) == 0, "guide block shape");
  hipLaunchKernelGGL(k_guide_blk_fwd, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, ghm_stream(stream), H, msgs,
                     part, b);
  return ghm_launch_status();
}

extern "C" int ghm_guide_blk_bwd(const float* H, int T, int tok0, int ntok, int col, const float* msgs,
                                 int64_t msg_stride, int64_t moff, int ext, int V, float* dH, float scale,
                                 int64_t n_seq, void* stream) {
  GHM_CHECK(H && msgs && dH, "null pointer");
  GuideBlk b;
  GHM_CHECK(guide_blk_check(b, T, tok0, ntok, col, msg_stride, moff, ext, V, n_seq) == 0, "guide block shape");
  const int64_t total = n_seq * ntok * V;
  hipLaunchKernelGGL(k_guide_blk_bwd, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0,
                     ghm_stream(stream), H, msgs, dH, total, b, scale);
  return ghm_launch_status();
}

// One launch for a list of guided blocks (the 26 blocks of the guided joint CDM
// cost one launch each otherwise).  One workgroup per sequence walks the blocks
// in list order with a barrier between them, so blocks that share columns of dH
// are applied one after another exactly as the per-block launches do.
// fwd: part[k * n_seq + n] for block k;  bwd: dH (shared by every block) +=.
constexpr int GUIDE_MAXBLK = 32;
struct GuideBlkSet {
  const float* H[GUIDE_MAXBLK];
  const float* msgs[GUIDE_MAXBLK];
  GuideBlk b[GUIDE_MAXBLK];
  int nb;
};

__global__ __launch_bounds__(256) void k_guide_blks_fwd(GuideBlkSet set, float* __restrict__ part, int n_seq) {
  __shared__ float red[4];
  const int n = blockIdx.x;
  for (int k = 0; k < set.nb; ++k) {
    const GuideBlk& b = set.b[k];
    const float* h = set.H[k] + (static_cast<int64_t>(n) * b.T + b.tok0) * b.ld + b.col;
    const float* m = set.msgs[k] + static_cast<int64_t>(n) * b.msg_stride + b.moff;
    float s = 0.f;
    for (int e = threadIdx.x; e < b.ntok * b.V; e += 256) {
      const int t = e / b.V, c = e - t * b.V;
      const float dd = h[static_cast<int64_t>(t) * b.ld + c] - m[(t / b.ext) * b.V + c];
      s += dd * dd;
    }
    s = sum32(s);
    s += __shfl_xor(s, 32, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[static_cast<int64_t>(k) * n_seq + n] = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_guide_blks_bwd(GuideBlkSet set, float* __restrict__ dH, float scale) {
  const int n = blockIdx.x;
  for (int k = 0; k < set.nb; ++k) {
    const GuideBlk& b = set.b[k];
    const float* m = set.msgs[k] + static_cast<int64_t>(n) * b.msg_stride + b.moff;
    const int64_t base = (static_cast<int64_t>(n) * b.T + b.tok0) * b.ld + b.col;
    for (int e = threadIdx.x; e < b.ntok * b.V; e += 256) {
      const int t = e / b.V, c = e - t * b.V;
      const int64_t at = base + static_cast<int64_t>(t) * b.ld + c;
      dH[at] += scale * (set.H[k][at] - m[(t / b.ext) * b.V + c]);
    }
    __syncthreads();
  }
}

// desc[k*6 ..] = {T, tok0, ntok, col, ext, V}, desc64[k*2 ..] = {msg_stride, moff}
static int guide_blks_set(GuideBlkSet& set, const float* const* H, const float* const* msgs, const int32_t* desc,
                          const int64_t* desc64, int nb, int64_t n_seq, int ld = GHM_D) {
  if (!(H && msgs && desc && desc64 && nb >= 1 && nb <= GUIDE_MAXBLK)) return -1;
  set.nb = nb;
  for (int k = 0; k < nb; ++k) {
    const int32_t* d = desc + 6 * k;
    if (!H[k] || !msgs[k]) return -1;
    if (guide_blk_check(set.b[k], d[0], d[1], d[2], d[3], desc64[2 * k], desc64[2 * k + 1], d[4], d[5], n_seq, ld))
      return -1;
    set.H[k] = H[k];
    set.msgs[k] = msgs[k];
  }
  return 0;
}

extern "C" int ghm_guide_blks_fwd(const float* const* H, const float* const* msgs, const int32_t* desc,
                                  const int64_t* desc64, int nb, float* part, int64_t n_seq, void* stream) {
  GHM_CHECK(part, "null pointer");
  GuideBlkSet set;
  GHM_CHECK(guide_blks_set(set, H, msgs, desc, desc64, nb, n_seq) == 0, "guide block list");
  hipLaunchKernelGGL(k_guide_blks_fwd, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, ghm_stream(stream), set,
                     part, static_cast<int>(n_seq));
  return ghm_launch_status();
}

extern "C" int ghm_guide_blks_bwd(const float* const* H, const float* const* msgs, const int32_t* desc,
                                  const int64_t* desc64, int nb, float* dH, float scale, int64_t n_seq,
                                  void* stream) {
  GHM_CHECK(dH, "null pointer");
  GuideBlkSet set;
  GHM_CHECK(guide_blks_set(set, H, msgs, desc, desc64, nb, n_seq) == 0, "guide block list");
  hipLaunchKernelGGL(k_guide_blks_bwd, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, ghm_stream(stream), set,
                     dH, scale);
  return ghm_launch_status();
}

// The same block lists for a residual stream of row pitch D (the guided joint VLM,
// D = 256: train_NWP.py --guide=True, model.py:303-331, 1122-1149)
extern "C" int ghm_guide_blks_fwd_d(const float* const* H, const float* const* msgs, const int32_t* desc,
                                    const int64_t* desc64, int nb, int D, float* part, int64_t n_seq, void* stream) {
  GHM_CHECK(part, "null pointer");
  GuideBlkSet set;
  GHM_CHECK(guide_blks_set(set, H, msgs, desc, desc64, nb, n_seq, D) == 0, "guide block list");
  hipLaunchKernelGGL(k_guide_blks_fwd, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, ghm_stream(stream), set,
                     part, static_cast<int>(n_seq));
  return ghm_launch_status();
}

extern "C" int ghm_guide_blks_bwd_d(const float* const* H, const float* const* msgs, const int32_t* desc,
                                    const int64_t* desc64, int nb, int D, float* dH, float scale, int64_t n_seq,
                                    void* stream) {
  GHM_CHECK(dH, "null pointer");
  GuideBlkSet set;
  GHM_CHECK(guide_blks_set(set, H, msgs, desc, desc64, nb, n_seq, D) == 0, "guide block list");
  hipLaunchKernelGGL(k_guide_blks_bwd, dim3(static_cast<unsigned>(n_seq)), dim3(256), 0, ghm_stream(stream), set,
                     dH, scale);
  return ghm_launch_status();
}

extern "C" int ghm_guide_max_blocks(void) { return GUIDE_MAXBLK; }

// ---------------------------------------------------------------------------
// Dense-target helpers for the module API (GuidedClipLoss(guide=True) on the
// guided-layer tensors EncoderTransformer.forward returns)
// ---------------------------------------------------------------------------
// out[r] = sum_{e<E} (a[r*E+e] - b[r*E+e])^2, one 256-thread workgroup per row
__global__ __launch_bounds__(256) void k_sqdiff_rows(const float* __restrict__ a, const float* __restrict__ b,
                                                     float* __restrict__ out, int64_t E) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  float s = 0.f;
  for (int64_t e = threadIdx.x; e < E; e += 256) {
    const float d = a[r * E + e] - b[r * E + e];
    s += d * d;
  }
  s = sum32(s);
  s += __shfl_xor(s, 32, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[r] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out[i] = scale[0] * alpha * (a[i] - b[i])   (scale: device scalar, e.g. the upstream gradient)
__global__ __launch_bounds__(256) void k_scaled_diff(const float* __restrict__ a, const float* __restrict__ b,
                                                     const float* __restrict__ scale, float alpha,
                                                     float* __restrict__ out, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) out[i] = (scale[0] * alpha) * (a[i] - b[i]);
}

// dst[m*128 + c] += src[m*V + c], c < V: a guided layer's gradient into the residual stream
__global__ __launch_bounds__(256) void k_add_cols(float* __restrict__ dst, const float* __restrict__ src,
                                                  int64_t M, int V) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= M * V) return;
  const int64_t m = i / V;
  const int c = static_cast<int>(i % V);
  dst[m * GHM_D + c] += src[i];
}

extern "C" int ghm_sqdiff_rows(const float* a, const float* b, float* out, int64_t rows, int64_t row_len,
                               void* stream) {
  GHM_CHECK(a && b && out && rows >= 1 && row_len >= 1, "shape");
  hipLaunchKernelGGL(k_sqdiff_rows, dim3(static_cast<unsigned>(rows)), dim3(256), 0, ghm_stream(stream), a, b, out,
                     row_len);
  return ghm_launch_status();
}

extern "C" int ghm_scaled_diff(const float* a, const float* b, const float* scale, float alpha, float* out,
                               int64_t n, void* stream) {
  GHM_CHECK(a && b && scale && out && n >= 1, "shape");
  hipLaunchKernelGGL(k_scaled_diff, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, ghm_stream(stream),
                     a, b, scale, alpha, out, n);
  return ghm_launch_status();
}

extern "C" int ghm_add_cols(float* dst, const float* src, int64_t M, int V, void* stream) {
  GHM_CHECK(dst && src && M >= 1 && V >= 1 && V <= GHM_D, "shape");
  hipLaunchKernelGGL(k_add_cols, dim3(static_cast<unsigned>((M * V + 255) / 256)), dim3(256), 0, ghm_stream(stream),
                     dst, src, M, V);
  return ghm_launch_status();
}
