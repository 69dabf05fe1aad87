// Native host GHM sampler: numpy-legacy-compatible MT19937 stream + inverse-CDF
// tree sampling.  Behaviour follows the reference producers
//   ClipSampler.get_batch                src/ghmclip/data/data_random_GHM.py:753-784
//   ConditionalDenoiseSampler.get_batch  src/ghmclip/data/data_random_GHM.py:854-869
//   GHMTree.gen_values                   src/ghmclip/data/data_random_GHM.py:145-165
// The per-node Python loop of the reference becomes one pass per (layer, child
// slot) over a contiguous uint8 value plane; the RNG stream is consumed in the
// reference's exact order (BFS parent, child slot, batch element).
#include "../../include/ghm_sampler.h"

#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <vector>

namespace {

constexpr int kN = 624;
constexpr int kM = 397;

struct MT19937 {
  uint32_t key[kN];
  int pos = kN;

  void seed(uint32_t s) {  // numpy mt19937_seed == init_genrand
    for (int i = 0; i < kN; ++i) {
      key[i] = s;
      s = 1812433253u * (s ^ (s >> 30)) + static_cast<uint32_t>(i + 1);
    }
    pos = kN;
  }

  // One MT19937 twist, written so that the compiler vectorises it: within a
  // group of 4 words, key[kk + 1 .. kk + 4] are read before group kk writes
  // them (the only in-place overlap), which the explicit temporaries make plain.
  void generate() {
    constexpr uint32_t UP = 0x80000000u, LO = 0x7fffffffu, MAG = 0x9908b0dfu;
    int kk = 0;
    for (; kk + 4 <= kN - kM; kk += 4) {
      uint32_t y[4], r[4];
      for (int i = 0; i < 4; ++i) y[i] = (key[kk + i] & UP) | (key[kk + i + 1] & LO);
      for (int i = 0; i < 4; ++i) r[i] = key[kk + i + kM] ^ (y[i] >> 1) ^ ((0u - (y[i] & 1u)) & MAG);
      for (int i = 0; i < 4; ++i) key[kk + i] = r[i];
    }
    for (; kk < kN - kM; ++kk) {
      const uint32_t y = (key[kk] & UP) | (key[kk + 1] & LO);
      key[kk] = key[kk + kM] ^ (y >> 1) ^ ((0u - (y & 1u)) & MAG);
    }
    for (; kk + 4 <= kN - 1; kk += 4) {
      uint32_t y[4], r[4];
      for (int i = 0; i < 4; ++i) y[i] = (key[kk + i] & UP) | (key[kk + i + 1] & LO);
      for (int i = 0; i < 4; ++i) r[i] = key[kk + i + (kM - kN)] ^ (y[i] >> 1) ^ ((0u - (y[i] & 1u)) & MAG);
      for (int i = 0; i < 4; ++i) key[kk + i] = r[i];
    }
    static_assert((kN - 1 - (kN - kM)) % 4 == 0, "second twist range is whole groups of 4");
    const uint32_t y = (key[kN - 1] & UP) | (key[0] & LO);
    key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & MAG);
    pos = 0;
  }

  inline uint32_t next32() {
    if (pos == kN) generate();
    uint32_t y = key[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  static inline uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  // n consecutive next32() outputs: whole 624-word blocks are regenerated and
  // tempered in straight loops (vectorised), the partial ends word by word
  void fill(uint32_t* out, size_t n) {
    size_t i = 0;
    while (i < n && pos < kN) out[i++] = temper(key[pos++]);
    while (n - i >= static_cast<size_t>(kN)) {
      generate();
      for (int k = 0; k < kN; ++k) out[i + k] = temper(key[k]);
      i += kN;
      pos = kN;
    }
    while (i < n) out[i++] = next32();
  }

  inline double next_double() {  // numpy legacy random_sample
    const int32_t a = static_cast<int32_t>(next32() >> 5);
    const int32_t b = static_cast<int32_t>(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }

  // numpy legacy randint(0, V) for V-1 < 2^32: masked rejection sampling.
  inline uint32_t bounded(uint32_t rng) {
    if (rng == 0) return 0;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32() & mask)) > rng) {
    }
    return v;
  }
};

}  // namespace

// Fixed worker pool for the tree expansion (the MT stream itself is serial).
// Workers park on a condition variable between batches; run(f) calls f(w) for
// w = 0..n-1, w = 0 on the calling thread, and returns when all are done.
// Fork safety: a child process inherits the pool object but not its threads,
// so in any process other than the creating one run() calls f(0..n-1) serially
// on the calling thread (same results: the partition of the work is unchanged)
// and the destructor neither signals nor joins the absent workers.
class Pool {
 public:
  explicit Pool(int n) : n_(n < 1 ? 1 : n), pid_(getpid()) {
    for (int w = 1; w < n_; ++w) th_.emplace_back([this, w] { loop(w); });
  }
  ~Pool() {
    if (getpid() != pid_) {  // forked child: the workers do not exist here
      new std::vector<std::thread>(std::move(th_));  // leaked on purpose: never joined
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_; }
  void run(const std::function<void(int)>& f) {
    if (n_ == 1 || getpid() != pid_) {
      for (int w = 0; w < n_; ++w) f(w);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &f;
      left_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [this] { return left_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int w) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
      }
      (*f)(w);
      std::lock_guard<std::mutex> g(mu_);
      if (--left_ == 0) done_.notify_one();
    }
  }
  int n_;
  pid_t pid_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int left_ = 0;
  bool stop_ = false;
};

static int pool_threads() {
  const char* e = std::getenv("GHM_SAMPLER_THREADS");
  int n = e ? std::atoi(e) : 4;
  const int hw = static_cast<int>(std::thread::hardware_concurrency());
  if (hw > 0 && n > hw) n = hw;
  return n < 1 ? 1 : (n > 64 ? 64 : n);
}

// One tree shape: n_layer levels of n_child children; its n_runs non-root
// nodes in BFS order are also its edges (node k >= 1 hangs on edge k - 1, the
// reference's transition[layer][parent * n_child + child] in order), and
// cdf[edge][row][col] holds each edge's cumulative rows (translation-invariant
// trees repeat the per-child-slot templates; non-invariant trees, :80-85, give
// every edge its own matrix).
struct Tree {
  int n_layer = 0, n_child = 0, T = 0, n_runs = 0;
  std::vector<double> cdf;
};

struct ghm_sampler {
  int V, K;
  Tree tree[2];  // text, image
  MT19937 mt;
  int has_gauss = 0;  // numpy legacy Gaussian cache (RandomState state[3], state[4])
  double gauss = 0.0;
  std::vector<uint32_t> stream;  // raw u32 draws of the current batch's trees
  std::unique_ptr<Pool> pool;
};

// numpy legacy_gauss: polar Box-Muller on random_sample pairs, the second
// deviate cached for the next call (randn / normal consume this stream).
static double legacy_gauss(ghm_sampler* s) {
  if (s->has_gauss) {
    s->has_gauss = 0;
    const double g = s->gauss;
    s->gauss = 0.0;
    return g;
  }
  double x1, x2, r2;
  do {
    x1 = 2.0 * s->mt.next_double() - 1.0;
    x2 = 2.0 * s->mt.next_double() - 1.0;
    r2 = x1 * x1 + x2 * x2;
  } while (r2 >= 1.0 || r2 == 0.0);
  const double f = std::sqrt(-2.0 * std::log(r2) / r2);
  s->gauss = f * x1;
  s->has_gauss = 1;
  return f * x2;
}

// Tree shape; false if out of range (T <= 2^20 leaves)
static bool tree_shape(int n_layer, int n_child, Tree& t) {
  if (n_layer < 1 || n_child < 1) return false;
  long T = 1, runs = 0;
  for (int l = 0; l < n_layer; ++l) {
    T *= n_child;
    runs += T;
    if (T > (1 << 20)) return false;
  }
  t.n_layer = n_layer;
  t.n_child = n_child;
  t.T = static_cast<int>(T);
  t.n_runs = static_cast<int>(runs);
  return true;
}

// edge matrices [n_runs][V][V] -> cumulative rows (np.cumsum: sequential float64 adds)
static void build_cdf(const double* edges, int n_edges, int V, double* out) {
  for (int m = 0; m < n_edges; ++m) {
    for (int r = 0; r < V; ++r) {
      double acc = 0.0;
      for (int c = 0; c < V; ++c) {
        acc += edges[(static_cast<size_t>(m) * V + r) * V + c];
        out[(static_cast<size_t>(m) * V + r) * V + c] = acc;
      }
    }
  }
}

extern "C" ghm_sampler* ghm_sampler_create_edges(const double* t_edges, int t_layer, int t_child,
                                                 const double* i_edges, int i_layer, int i_child, int V, int K) {
  if (!t_edges || !i_edges || V < 1 || V > 255 || K < 2) return nullptr;
  ghm_sampler* s = new ghm_sampler();
  if (!tree_shape(t_layer, t_child, s->tree[0]) || !tree_shape(i_layer, i_child, s->tree[1])) {
    delete s;
    return nullptr;
  }
  s->V = V;
  s->K = K;
  const double* src[2] = {t_edges, i_edges};
  for (int k = 0; k < 2; ++k) {
    Tree& t = s->tree[k];
    t.cdf.resize(static_cast<size_t>(t.n_runs) * V * V);
    build_cdf(src[k], t.n_runs, V, t.cdf.data());
  }
  s->pool.reset(new Pool(pool_threads()));
  s->mt.seed(0);
  return s;
}

extern "C" ghm_sampler* ghm_sampler_create(const double* t_trans, const double* i_trans, int n_layer,
                                           int n_child, int V, int K) {
  if (!t_trans || !i_trans || V < 1 || V > 255) return nullptr;
  Tree shape;
  if (!tree_shape(n_layer, n_child, shape)) return nullptr;
  // expand the per-(layer, child slot) templates to every edge
  const size_t VV = static_cast<size_t>(V) * V;
  std::vector<double> te(shape.n_runs * VV), ie(shape.n_runs * VV);
  size_t e = 0;
  long width = 1;
  for (int l = 0; l < n_layer; ++l) {
    width *= n_child;
    for (long k = 0; k < width; ++k, ++e) {
      const size_t m = (static_cast<size_t>(l) * n_child + k % n_child) * VV;
      std::memcpy(te.data() + e * VV, t_trans + m, VV * sizeof(double));
      std::memcpy(ie.data() + e * VV, i_trans + m, VV * sizeof(double));
    }
  }
  return ghm_sampler_create_edges(te.data(), n_layer, n_child, ie.data(), n_layer, n_child, V, K);
}

extern "C" void ghm_sampler_destroy(ghm_sampler* s) { delete s; }

extern "C" int ghm_sampler_seed(ghm_sampler* s, uint32_t seed) {
  if (!s) return -1;
  s->mt.seed(seed);
  return 0;
}

extern "C" int ghm_sampler_set_state(ghm_sampler* s, const uint32_t* key, int pos) {
  if (!s || !key || pos < 0 || pos > kN) return -1;
  std::memcpy(s->mt.key, key, sizeof(s->mt.key));
  s->mt.pos = pos;
  return 0;
}

extern "C" int ghm_sampler_get_state(const ghm_sampler* s, uint32_t* key, int* pos) {
  if (!s || !key || !pos) return -1;
  std::memcpy(key, s->mt.key, sizeof(s->mt.key));
  *pos = s->mt.pos;
  return 0;
}

extern "C" int ghm_sampler_random_sample(ghm_sampler* s, double* out, int64_t n) {
  if (!s || (!out && n)) return -1;
  for (int64_t i = 0; i < n; ++i) out[i] = s->mt.next_double();
  return 0;
}

extern "C" int ghm_sampler_choice(ghm_sampler* s, int V, int64_t n, int64_t* out) {
  if (!s || V < 1 || (!out && n)) return -1;
  for (int64_t i = 0; i < n; ++i) out[i] = s->mt.bounded(static_cast<uint32_t>(V - 1));
  return 0;
}

// The reference draws a tree level by level: for each parent node (BFS) and
// child slot, ONE np.random.rand(rows) vector, i.e. a run of `rows` consecutive
// doubles (2 u32 each) per child node, in the child's BFS order
// (data_random_GHM.py:153-165).  The whole run of a tree is therefore a fixed
// slice of the stream once the roots are drawn: it is pulled serially here
// (0.6 M u32 for the default batch), and the inverse-CDF expansion of any set
// of rows runs in parallel (expand_rows), reading each row's draws at fixed
// offsets.  The result is bit-identical to the reference's draw.
static void pull_stream(ghm_sampler* s, size_t n_u32, uint32_t* out) { s->mt.fill(out, n_u32); }

static inline double to_double(uint32_t a, uint32_t b) {  // numpy legacy random_sample
  return (static_cast<int32_t>(a >> 5) * 67108864.0 + static_cast<int32_t>(b >> 6)) / 9007199254740992.0;
}

// Expand rows [r0, r1) of the rows listed in `sel` (indices into the batch of
// `rows` trees whose draws start at `draws`): values of every node in a
// [n_nodes][RB] scratch plane, leaves written row-major to out[i][T].
static void expand_rows(const ghm_sampler* s, const Tree& tr, const uint32_t* draws, int rows,
                        const uint8_t* root, const int* sel, int r0, int r1, uint8_t* out) {
  constexpr int RB = 32;
  const int V = s->V, C = tr.n_child, T = tr.T;
  const int n_nodes = tr.n_runs + 1;
  std::vector<uint8_t> val(static_cast<size_t>(n_nodes) * RB);
  for (int i0 = r0; i0 < r1; i0 += RB) {
    const int nb = (r1 - i0) < RB ? (r1 - i0) : RB;
    for (int i = 0; i < nb; ++i) val[i] = root[sel[i0 + i]];
    int first = 0, n_par = 1;  // BFS index of the level's first node, its width
    for (int layer = 0; layer < tr.n_layer; ++layer) {
      const int child0 = first + n_par;
      for (int p = 0; p < n_par; ++p) {
        const uint8_t* pv = val.data() + static_cast<size_t>(first + p) * RB;
        for (int c = 0; c < C; ++c) {
          const int node = child0 + p * C + c;
          const double* m = tr.cdf.data() + static_cast<size_t>(node - 1) * V * V;  // edge node - 1
          const uint32_t* run = draws + static_cast<size_t>(node - 1) * rows * 2;
          uint8_t* o = val.data() + static_cast<size_t>(node) * RB;
          for (int i = 0; i < nb; ++i) {
            const int b = sel[i0 + i];
            const double u = to_double(run[2 * b], run[2 * b + 1]);
            const double* row = m + static_cast<size_t>(pv[i]) * V;
            // (u < cdf).argmax(): the cdf is non-decreasing, so the first True is
            // the number of entries <= u; none True (count == V) gives 0
            int v = 0;
            for (int k = 0; k < V; ++k) v += row[k] <= u;
            o[i] = static_cast<uint8_t>(v == V ? 0 : v);
          }
        }
      }
      first = child0;
      n_par *= C;
    }
    for (int i = 0; i < nb; ++i) {
      uint8_t* dst = out + static_cast<size_t>(i0 + i) * T;
      for (int t = 0; t < T; ++t) dst[t] = val[static_cast<size_t>(first + t) * RB + i];
    }
  }
}

// Draw the text and image trees of `rows` sequences (roots given) and expand
// the selected rows of both in parallel.
static void draw_trees(ghm_sampler* s, int rows, const uint8_t* troot, const uint8_t* iroot, const int* sel,
                       int nsel, uint8_t* t_out, uint8_t* i_out) {
  const size_t t_tree = static_cast<size_t>(s->tree[0].n_runs) * rows * 2;
  const size_t i_tree = static_cast<size_t>(s->tree[1].n_runs) * rows * 2;
  s->stream.resize(t_tree + i_tree);
  pull_stream(s, t_tree + i_tree, s->stream.data());  // the text tree's runs, then the image tree's
  const uint32_t* ts = s->stream.data();
  const uint32_t* is = ts + t_tree;
  const int nw = s->pool->size();
  // 2 trees x row chunks of 32, dealt round-robin over the workers
  const int nch = (nsel + 31) / 32;
  s->pool->run([&](int w) {
    for (int k = w; k < 2 * nch; k += nw) {
      const int tree = k / nch, ch = k % nch;
      const int r0 = 32 * ch, r1 = (r0 + 32 < nsel) ? r0 + 32 : nsel;
      if (tree == 0)
        expand_rows(s, s->tree[0], ts, rows, troot, sel, r0, r1, t_out);
      else
        expand_rows(s, s->tree[1], is, rows, iroot, sel, r0, r1, i_out);
    }
  });
}

extern "C" int ghm_sampler_next_shard(ghm_sampler* s, int B, int lo, int n, uint8_t* t_leaves,
                                      uint8_t* i_leaves, uint8_t* t_root, uint8_t* i_root) {
  if (!s || B < 1 || lo < 0 || n < 1 || lo + n > B || !t_leaves || !i_leaves) return -1;
  const int K = s->K, V = s->V;
  const int rows = B * (K + 1);
  std::vector<uint8_t> tr(rows), ir(rows);
  for (int r = 0; r < rows; ++r) tr[r] = static_cast<uint8_t>(s->mt.bounded(V - 1));
  for (int r = 0; r < 2 * B; ++r) ir[r] = tr[r];
  for (int r = 2 * B; r < rows; ++r) ir[r] = static_cast<uint8_t>(s->mt.bounded(V - 1));
  std::vector<int> sel;
  sel.reserve(static_cast<size_t>(K + 1) * n);
  for (int k = 0; k <= K; ++k)
    for (int i = 0; i < n; ++i) sel.push_back(k * B + lo + i);
  draw_trees(s, rows, tr.data(), ir.data(), sel.data(), static_cast<int>(sel.size()), t_leaves, i_leaves);
  for (size_t i = 0; i < sel.size(); ++i) {
    if (t_root) t_root[i] = tr[sel[i]];
    if (i_root) i_root[i] = ir[sel[i]];
  }
  return 0;
}

extern "C" int ghm_sampler_next(ghm_sampler* s, int B, uint8_t* t_leaves, uint8_t* i_leaves,
                                uint8_t* t_root, uint8_t* i_root) {
  return ghm_sampler_next_shard(s, B, 0, B, t_leaves, i_leaves, t_root, i_root);
}

extern "C" int ghm_sampler_set_gauss(ghm_sampler* s, int has_gauss, double gauss) {
  if (!s) return -1;
  s->has_gauss = has_gauss ? 1 : 0;
  s->gauss = gauss;
  return 0;
}

extern "C" int ghm_sampler_get_gauss(const ghm_sampler* s, int* has_gauss, double* gauss) {
  if (!s || !has_gauss || !gauss) return -1;
  *has_gauss = s->has_gauss;
  *gauss = s->gauss;
  return 0;
}

extern "C" int ghm_sampler_randn(ghm_sampler* s, double* out, int64_t n) {
  if (!s || (!out && n)) return -1;
  for (int64_t i = 0; i < n; ++i) out[i] = legacy_gauss(s);
  return 0;
}

// ConditionalDenoiseSampler.get_batch (guide=False) draws, in the reference's
// stream order: choice(V, B) shared roots (:863), the text tree (:865), the image
// tree (:866), then np.random.randn(T, B) * sigma + leaves (:869) — drawn
// leaf-major ([T][B] C order) and written transposed as z[b][t] (the .T at :882).
// z == NULL: the trees only (NextWordPredictSampler.get_batch, :902-907).
extern "C" int ghm_sampler_next_cdm(ghm_sampler* s, int B, double sigma, uint8_t* t_leaves,
                                    uint8_t* i_leaves, uint8_t* root, double* z) {
  if (!s || B < 1 || !t_leaves || !i_leaves) return -1;
  const int V = s->V, T = s->tree[1].T;  // z lives on the image leaves
  std::vector<uint8_t> r(B);
  for (int b = 0; b < B; ++b) r[b] = static_cast<uint8_t>(s->mt.bounded(V - 1));
  std::vector<int> sel(B);
  for (int b = 0; b < B; ++b) sel[b] = b;
  draw_trees(s, B, r.data(), r.data(), sel.data(), B, t_leaves, i_leaves);
  for (int t = 0; z && t < T; ++t) {
    for (int b = 0; b < B; ++b) {
      const double g = legacy_gauss(s);
      z[static_cast<size_t>(b) * T + t] = g * sigma + static_cast<double>(i_leaves[static_cast<size_t>(b) * T + t]);
    }
  }
  if (root) std::memcpy(root, r.data(), B);
  return 0;
}
