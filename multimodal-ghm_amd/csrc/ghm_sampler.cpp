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
#include <cstring>
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

  void generate() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    int kk = 0;
    uint32_t y;
    for (; kk < kN - kM; ++kk) {
      y = (key[kk] & 0x80000000u) | (key[kk + 1] & 0x7fffffffu);
      key[kk] = key[kk + kM] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < kN - 1; ++kk) {
      y = (key[kk] & 0x80000000u) | (key[kk + 1] & 0x7fffffffu);
      key[kk] = key[kk + (kM - kN)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (key[kN - 1] & 0x80000000u) | (key[0] & 0x7fffffffu);
    key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ mag01[y & 1u];
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

struct ghm_sampler {
  int n_layer, n_child, V, K, T;
  // cdf[tree][layer][child][row][col], cumulative sums in the reference's order
  std::vector<double> cdf;
  MT19937 mt;
  int has_gauss = 0;  // numpy legacy Gaussian cache (RandomState state[3], state[4])
  double gauss = 0.0;
  std::vector<uint8_t> plane_a, plane_b;  // [n_nodes][rows] value planes
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

static void build_cdf(const double* trans, int n_layer, int n_child, int V, double* out) {
  const int nm = n_layer * n_child;
  for (int m = 0; m < nm; ++m) {
    for (int r = 0; r < V; ++r) {
      double acc = 0.0;  // np.cumsum: sequential float64 adds
      for (int c = 0; c < V; ++c) {
        acc += trans[(static_cast<size_t>(m) * V + r) * V + c];
        out[(static_cast<size_t>(m) * V + r) * V + c] = acc;
      }
    }
  }
}

extern "C" ghm_sampler* ghm_sampler_create(const double* t_trans, const double* i_trans, int n_layer,
                                           int n_child, int V, int K) {
  if (!t_trans || !i_trans || n_layer < 1 || n_child < 1 || V < 1 || V > 255 || K < 2) return nullptr;
  long T = 1;
  for (int l = 0; l < n_layer; ++l) T *= n_child;
  if (T > (1 << 20)) return nullptr;
  ghm_sampler* s = new ghm_sampler();
  s->n_layer = n_layer; s->n_child = n_child; s->V = V; s->K = K; s->T = static_cast<int>(T);
  const size_t per = static_cast<size_t>(n_layer) * n_child * V * V;
  s->cdf.resize(2 * per);
  build_cdf(t_trans, n_layer, n_child, V, s->cdf.data());
  build_cdf(i_trans, n_layer, n_child, V, s->cdf.data() + per);
  s->mt.seed(0);
  return s;
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

// One tree: roots [rows] -> leaves [rows][T] (uint8, row-major).
static void sample_tree(ghm_sampler* s, const double* cdf, const uint8_t* root, int rows,
                        uint8_t* leaves) {
  const int V = s->V, C = s->n_child;
  std::vector<uint8_t>& cur = s->plane_a;
  std::vector<uint8_t>& nxt = s->plane_b;
  cur.assign(root, root + rows);
  int n_par = 1;
  for (int layer = 0; layer < s->n_layer; ++layer) {
    nxt.resize(static_cast<size_t>(n_par) * C * rows);
    for (int p = 0; p < n_par; ++p) {
      const uint8_t* pv = cur.data() + static_cast<size_t>(p) * rows;
      for (int c = 0; c < C; ++c) {
        const double* m = cdf + static_cast<size_t>(layer * C + c) * V * V;
        uint8_t* out = nxt.data() + (static_cast<size_t>(p) * C + c) * rows;
        for (int b = 0; b < rows; ++b) {
          const double u = s->mt.next_double();
          const double* row = m + static_cast<size_t>(pv[b]) * V;
          int v = 0;  // (u < cdf).argmax(): first True, 0 when none is True
          for (int k = 0; k < V; ++k) {
            if (u < row[k]) { v = k; break; }
          }
          out[b] = static_cast<uint8_t>(v);
        }
      }
    }
    std::swap(cur, nxt);
    n_par *= C;
  }
  // cur: [T][rows] -> leaves [rows][T]
  const int T = s->T;
  for (int t = 0; t < T; ++t) {
    const uint8_t* src = cur.data() + static_cast<size_t>(t) * rows;
    for (int b = 0; b < rows; ++b) leaves[static_cast<size_t>(b) * T + t] = src[b];
  }
}

extern "C" int ghm_sampler_next(ghm_sampler* s, int B, uint8_t* t_leaves, uint8_t* i_leaves,
                                uint8_t* t_root, uint8_t* i_root) {
  if (!s || B < 1 || !t_leaves || !i_leaves) return -1;
  const int K = s->K, V = s->V;
  const int rows = B * (K + 1);
  std::vector<uint8_t> tr(rows), ir(rows);
  for (int r = 0; r < rows; ++r) tr[r] = static_cast<uint8_t>(s->mt.bounded(V - 1));
  for (int r = 0; r < 2 * B; ++r) ir[r] = tr[r];
  for (int r = 2 * B; r < rows; ++r) ir[r] = static_cast<uint8_t>(s->mt.bounded(V - 1));
  const size_t per = static_cast<size_t>(s->n_layer) * s->n_child * V * V;
  sample_tree(s, s->cdf.data(), tr.data(), rows, t_leaves);
  sample_tree(s, s->cdf.data() + per, ir.data(), rows, i_leaves);
  if (t_root) std::memcpy(t_root, tr.data(), rows);
  if (i_root) std::memcpy(i_root, ir.data(), rows);
  return 0;
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
  const int V = s->V, T = s->T;
  std::vector<uint8_t> r(B);
  for (int b = 0; b < B; ++b) r[b] = static_cast<uint8_t>(s->mt.bounded(V - 1));
  const size_t per = static_cast<size_t>(s->n_layer) * s->n_child * V * V;
  sample_tree(s, s->cdf.data(), r.data(), B, t_leaves);
  sample_tree(s, s->cdf.data() + per, r.data(), B, i_leaves);
  for (int t = 0; z && t < T; ++t) {
    for (int b = 0; b < B; ++b) {
      const double g = legacy_gauss(s);
      z[static_cast<size_t>(b) * T + t] = g * sigma + static_cast<double>(i_leaves[static_cast<size_t>(b) * T + t]);
    }
  }
  if (root) std::memcpy(root, r.data(), B);
  return 0;
}
