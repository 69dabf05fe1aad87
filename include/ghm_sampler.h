/* ghm_sampler.h — native host GHM sampler (C ABI), libghm_host.so.
 *
 * Replaces the per-step host producer of the reference CLIP loop:
 *   ClipSampler.get_batch          src/ghmclip/data/data_random_GHM.py:753-784
 *   GHMTree.gen_values (root given) src/ghmclip/data/data_random_GHM.py:145-165
 * and reproduces numpy's legacy RandomState stream bit-exactly (MT19937,
 * random_sample = (a>>5, b>>6) 53-bit doubles, randint via masked rejection), so
 * a batch drawn here equals the reference's draw from the same numpy state.
 *
 * Ownership: the handle owns only host memory; output buffers are caller-owned.
 * Errors: int return, 0 = success, negative GHM_E* on bad arguments.
 * Threading: one handle per calling thread (each handle owns a small worker pool
 * for the tree expansion); no global state.  Fork: a handle used in a child
 * process (fork after ghm_sampler_create) expands serially on the calling
 * thread — same draws, no deadlock on the parent's absent workers.
 */
#ifndef GHM_SAMPLER_H
#define GHM_SAMPLER_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ghm_sampler ghm_sampler;

/* t_trans / i_trans: [n_layer][n_child][V][V] float64 row-stochastic matrices
 * (the distinct per-(layer, child-slot) templates of a translation-invariant
 * GenTransition, data_random_GHM.py:43-89).  K = number of CLIP blocks minus one
 * (batch rows = B*(K+1)).  Returns NULL on bad arguments. */
ghm_sampler* ghm_sampler_create(const double* t_trans, const double* i_trans, int n_layer,
                                int n_child, int V, int K);
/* General form: one [V][V] matrix per edge of each tree, in the reference's
 * order transition[layer][parent * n_child + child] (layer 0 first; n_child +
 * n_child^2 + ... + n_child^n_layer edges), so non-translation-invariant
 * GenTransition trees (data_random_GHM.py:80-85) and text / image trees of
 * different shapes (ClipSampler n_layers / n_childs, :645-658) draw
 * bit-exactly.  Leaves: text rows [n_child_t^n_layer_t], image rows
 * [n_child_i^n_layer_i]. */
ghm_sampler* ghm_sampler_create_edges(const double* t_edges, int t_layer, int t_child, const double* i_edges,
                                      int i_layer, int i_child, int V, int K);
void ghm_sampler_destroy(ghm_sampler* s);
/* the source hash of this library's build (as ghm_build_id in ghm_hip.h) */
const char* ghm_sampler_build_id(void);

/* Seed like numpy.random.seed(int) (init_genrand). */
int ghm_sampler_seed(ghm_sampler* s, uint32_t seed);
/* Import / export the numpy legacy MT19937 state: key[624] and pos (0..624). */
int ghm_sampler_set_state(ghm_sampler* s, const uint32_t* key, int pos);
int ghm_sampler_get_state(const ghm_sampler* s, uint32_t* key, int* pos);

/* One ClipSampler.get_batch(batch_size=B, guide=False):
 *   t_leaves, i_leaves : [B*(K+1)][n_child**n_layer] uint8, row = sequence
 *   t_root, i_root     : [B*(K+1)] uint8 (may be NULL)
 * Stream order: choice(V, B(K+1)) text roots, choice(V, B(K-1)) image roots
 * (image rows [0,2B) reuse the text roots), text tree, image tree. */
int ghm_sampler_next(ghm_sampler* s, int B, uint8_t* t_leaves, uint8_t* i_leaves,
                     uint8_t* t_root, uint8_t* i_root);

/* The same draw (the stream advances by the WHOLE batch, as get_batch(B) does),
 * returning only the data-parallel shard: rows [k*B + lo, k*B + lo + n) of every
 * block k = 0..K, i.e. outputs are [(K+1)*n][T] (and [(K+1)*n] roots).  The
 * serial part is the MT19937 stream; the inverse-CDF expansion runs only for the
 * shard's rows, on $GHM_SAMPLER_THREADS (default 4) threads.  Replaces
 * get_batch + the per-rank row slice of the data-parallel CLI. */
int ghm_sampler_next_shard(ghm_sampler* s, int B, int lo, int n, uint8_t* t_leaves, uint8_t* i_leaves,
                           uint8_t* t_root, uint8_t* i_root);

/* One ConditionalDenoiseSampler.get_batch(batch_size=B) draw
 * (data_random_GHM.py:854-869; replaces the per-node Python loop and np.random.randn):
 *   t_leaves, i_leaves : [B][n_child**n_layer] uint8 (trees sharing one root per row)
 *   root               : [B] uint8 (may be NULL)
 *   z                  : [B][n_child**n_layer] float64 noisy image observations
 *                        randn * sigma + leaf (the reference's image_tree_noise, transposed)
 * Stream order: choice(V, B), text tree, image tree, randn(T, B) leaf-major.
 * z == NULL draws the two trees only: NextWordPredictSampler.get_batch (:902-907). */
int ghm_sampler_next_cdm(ghm_sampler* s, int B, double sigma, uint8_t* t_leaves, uint8_t* i_leaves,
                         uint8_t* root, double* z);
/* numpy legacy Gaussian cache (RandomState.get_state()[3:5]): import / export. */
int ghm_sampler_set_gauss(ghm_sampler* s, int has_gauss, double gauss);
int ghm_sampler_get_gauss(const ghm_sampler* s, int* has_gauss, double* gauss);
/* n draws of numpy.random.randn() (legacy polar method, cached second deviate). */
int ghm_sampler_randn(ghm_sampler* s, double* out, int64_t n);

/* Raw stream access for tests: n doubles of numpy.random.random_sample(). */
int ghm_sampler_random_sample(ghm_sampler* s, double* out, int64_t n);
/* n draws of numpy.random.choice(V) (legacy masked rejection). */
int ghm_sampler_choice(ghm_sampler* s, int V, int64_t n, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif
