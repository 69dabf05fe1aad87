/* ghm_hip.h — C ABI of libghm_hip.so, the MI355X (gfx950) kernels of the GHM
 * CLIP training step.  Each entry point launches HIP work asynchronously on the
 * caller's stream and returns 0, a hipError_t value (>0) or a negative GHM_E*
 * code; ghm_last_error_string() gives detail.  No entry point allocates, frees
 * or synchronises, so every call is graph-capturable.  All device buffers are
 * caller-owned (PyTorch's caching allocator in the Python host).
 *
 * Layouts (one encoder): M = n_seq * T tokens; activations row-major [M][D]
 * fp32 with D = 128; weights exactly as nn.Linear stores them ([out][in]).
 * Every function replaces part of the reference's PyTorch-eager hot path; the
 * reference file:line is given with each (paths under src/ghmclip/).
 */
#ifndef GHM_HIP_H
#define GHM_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GHM_OK 0
#define GHM_EINVAL (-22)   /* bad pointer / shape / unsupported configuration */

const char* ghm_last_error_string(void);
/* 1 when the library was built for gfx950 and a device is visible, else 0. */
int ghm_device_ok(void);
/* 16 hex digits: the hash of the sources this library was built from
 * (every file of multimodal-ghm_amd/csrc, the headers in include, the Makefile;
 * ghmclip/_buildid.py).
 * smoke() and bench.py require it to equal the hash of the tree they run in. */
const char* ghm_build_id(void);
/* Cross-stream ordering (the two-tower step's fork / join / cross waits,
 * replacing torch Stream.wait_stream in train_CLIP's step, which has no
 * reference counterpart: the reference runs the towers one after the other).
 * ghm_event_create(mode): 1 an event recorded with a device-scope release
 * (hipEventReleaseToDevice), 2 with hipEventDisableSystemFence, 0 a default one
 * (all without timing).  ghm_event_record / ghm_stream_wait:
 * hipEventRecord / hipStreamWaitEvent (streams: hipStream_t or NULL). */
void* ghm_event_create(int mode);
int ghm_event_destroy(void* ev);
int ghm_event_record(void* ev, void* stream);
int ghm_stream_wait(void* stream, void* ev);

/* ---- forward ---------------------------------------------------------- */

/* H0 = tok_w[tokens] + pos_w[t]  —  models/model.py:764-765 (EncoderTransformer.forward)
 * tokens: uint8 [n_seq][T]; tok_w [V][D]; pos_w [T][D]; H0 [M][D]. */
int ghm_embed_fwd(const uint8_t* tokens, const float* tok_w, const float* pos_w, float* H0,
                  int64_t n_seq, int T, int V, int D, void* stream);

/* qkv[:, 0:128|128:256|256:384] = LN1(H) Wq^T | Wk^T | Wv^T; stats[m] = (mean, rstd)
 * —  models/model.py:772-775 (ln1 + _queries/_keys/_values). */
int ghm_ln_qkv_fwd(const float* H, const float* ln_w, const float* ln_b, const float* Wq,
                   const float* Wk, const float* Wv, float* qkv, float* stats, int64_t M, int D,
                   float eps, void* stream);

/* H_mid = H + softmax(Q K^T / scale_div) V, single head over all D dims (no W_O);
 * the probabilities are saved for backward dense and padded, P[n_seq][96][96]
 * (P[n][q][key]; keys >= T hold 0, rows q >= T are unused)  —  model.py:778-782. */
int ghm_attn_fwd(const float* qkv, const float* H, float* H_mid, float* P, int64_t n_seq, int T,
                 int D, float scale_div, void* stream);

/* H_out = H_mid + W2 GELU(W1 LN2(H_mid) + b1) + b2, U = W1 LN2(H_mid) + b1; saves
 * G = GELU(U) and Dg = GELU'(U) [M][F] for backward (both null: saves nothing, for
 * a backward that recomputes U); stats = LN2 (mean, rstd)
 * —  models/model.py:741-747,784-788. */
int ghm_ln_mlp_fwd(const float* H_mid, const float* ln_w, const float* ln_b, const float* W1,
                   const float* b1, const float* W2, const float* b2, float* H_out, float* G,
                   float* Dg, float* stats, int64_t M, int D, int F, float eps, void* stream);

/* emb[n][c] = b_out + sum_t w_out[t] (b_ro[c] + H[n,t,:] . W_ro[c,:])
 * —  models/model.py:802-805 (_read_out, transpose, _out). */
int ghm_readout_fwd(const float* H, const float* W_ro, const float* b_ro, const float* w_out,
                    const float* b_out, float* emb, int64_t n_seq, int T, int D, int C,
                    void* stream);

/* K-way symmetric CLIP loss (GuidedClipLoss, guide=False) and its gradient
 * d(loss)/d(emb) for both towers; loss_out[0] = loss_out[1] = loss.  If hist is
 * non-NULL, hist[*step] = loss (step read on device, for graph replay).
 * dt_emb = di_emb = NULL: the loss value only (ghm_readout_bwd_clip computes the
 * gradient rows)
 * —  models/model.py:877-907; train_CLIP.py:153-161. */
int ghm_clip_loss(const float* t_emb, const float* i_emb, float* dt_emb, float* di_emb,
                  float* loss_out, float* hist, const int32_t* step, int B, int K, int C,
                  void* stream);

/* ---- backward (autograd of train_CLIP.py:158) ------------------------- */

/* dH_L and per-sequence partial parameter grads of the readout; reduce the
 * partials with ghm_reduce_partials over n_seq  —  backward of model.py:802-805. */
int ghm_readout_bwd(const float* H, const float* W_ro, const float* b_ro, const float* w_out,
                    const float* d_emb, float* dH, float* part_wro, float* part_bro,
                    float* part_wout, float* part_bout, int64_t n_seq, int T, int D, int C,
                    void* stream);

/* ghm_readout_bwd of one CLIP tower (0 text, 1 image) with the K-way loss
 * gradient of each row recomputed from both towers' embeddings (t_emb, i_emb;
 * n_seq = (K + 1) B rows) instead of read: d_emb is written, equal to
 * ghm_clip_loss's; the towers' backwards then need no loss kernel between the
 * forward and the backward  —  backward of model.py:877-907 and :802-805. */
int ghm_readout_bwd_clip(const float* H, const float* W_ro, const float* b_ro, const float* w_out,
                         const float* t_emb, const float* i_emb, int tower, int B, int K, float* d_emb,
                         float* dH, float* part_wro, float* part_bro, float* part_wout, float* part_bout,
                         int64_t n_seq, int T, int D, int C, void* stream);

/* Token- and position-embedding gradient PARTIALS of one encoder in one pass over
 * dH0 [n_seq][T][D] (D = 128, V = 10): part = [S T][V][D] token sums (rows of
 * dH0 by token id, per (split, position)), then [S][T][D] position sums (over
 * the split's sequences), S = ghm_embed_bwd_splits(), ghm_embed_bwd_part_elems(T, V)
 * floats.  Reduce them with ghm_reduce_batch: tok_grad = the sum over S T of the
 * first region, pos_grad = the sum over S of the second.  Deterministic  —
 * backward of models/model.py:764-765 (token_embeddings(x) + position_embeddings). */
int ghm_embed_bwd_splits(void);
int64_t ghm_embed_bwd_part_elems(int T, int V);
int ghm_embed_bwd_part(const float* dH0, const uint8_t* tokens, int64_t n_seq, int T, int V, int D, float* part,
                       void* stream);

/* MLP + LN2 backward for one layer (Dg = GELU'(U) from ghm_ln_mlp_fwd, passed as U):
 * writes dU [M][F] and dH_mid = dH_out + dLN2;
 * part_ln [n_blocks][2][D] = partial (dgamma, dbeta) of LN2 where
 * n_blocks = ghm_token_blocks(M)  —  backward of model.py:784-788. */
int ghm_mlp_bwd(const float* dH_out, const float* H_mid, const float* stats, const float* ln_w,
                const float* W1, const float* W2, const float* U, float* dU, float* dH_mid,
                float* part_ln, int64_t M, int D, int F, void* stream);

/* Attention backward: dqkv[:, q|k|v] from dH_mid, qkv and P (layout of
 * ghm_attn_fwd); dS: caller scratch [n_seq][96][96]  —  backward of model.py:778-782. */
int ghm_attn_bwd(const float* qkv, const float* P, const float* dH_mid, float* dS, float* dqkv,
                 int64_t n_seq, int T, int D, float scale_div, void* stream);
/* ghm_attn_fwd / ghm_attn_bwd with the attention activation of the reference's
 * get_activation (models/model.py:121-130, applied at :781): act 0 softmax
 * (identical to the plain entry points), 1 relu, 2 gelu (erf form) of the
 * scaled scores, keys past T contributing 0.  P holds act(s); for gelu the
 * forward also writes GELU'(s) to Pd (P's layout, required) and the backward
 * reads it.  dS: caller scratch as in ghm_attn_bwd. */
int ghm_attn_fwd_act(const float* qkv, const float* H, float* H_mid, float* P, float* Pd, int64_t n_seq, int T,
                     int D, float scale_div, int act, void* stream);
int ghm_attn_bwd_act(const float* qkv, const float* P, const float* Pd, const float* dH_mid, float* dS, float* dqkv,
                     int64_t n_seq, int T, int D, float scale_div, int act, void* stream);

/* QKV + LN1 backward: dH = dH_mid + dLN1(dqkv W); part_ln as in ghm_mlp_bwd
 * —  backward of model.py:772-775. */
int ghm_qkv_bwd(const float* dqkv, const float* H, const float* stats, const float* ln_w,
                const float* Wq, const float* Wk, const float* Wv, const float* dH_mid, float* dH,
                float* part_ln, int64_t M, int D, void* stream);

/* Split-K weight gradient C[a][b] = sum_m A[m][a] * op(B)[m][b] over token
 * chunks of tok_per_split tokens: part [n_split][A_cols][B_cols];
 * bias_part [n_split][A_cols] = sum_m A[m][a] (may be NULL).
 * b_mode: 0 plain, 1 GELU(B), 2 LayerNorm(B; stats, ln_w, ln_b).
 * A_cols and B_cols must be multiples of 128; tok_per_split a positive multiple of 32.
 * Used for dW1/db1, dW2/db2, dWq|k|v (nn.Linear weight/bias grads). */
int ghm_wgrad(const float* A, int lda, int A_cols, const float* B, int ldb, int B_cols,
              int b_mode, const float* stats, const float* ln_w, const float* ln_b, float* part,
              float* bias_part, int64_t M, int tok_per_split, void* stream);

/* (The embedding gradients of model.py:764-765 are ghm_wcolsum by token id and
 * ghm_colsum over the sequences, declared with the VLM GEMM entry points.) */

/* out[i] = sum_{s<n_split} part[s*n + i] in fixed order (deterministic).  The
 * n outputs are written to up to 4 destination segments: segment k takes
 * outputs [off[k], off[k+1]) into dst[k] (off[0] = 0, off[n_seg] = n). */
int ghm_reduce_partials(const float* part, int n_split, int64_t n, int n_seg,
                        float* const* dst, const int64_t* off, void* stream);

/* Up to 32 independent partial reductions in one launch (same semantics). */
typedef struct ghm_reduce_job {
  const float* part;
  int32_t n_split;
  int32_t n_seg;
  int64_t n;
  float* dst[4];
  int64_t off[5];
} ghm_reduce_job;
int ghm_reduce_batch(const ghm_reduce_job* jobs, int n_jobs, void* stream);

/* ---- clip_grad_norm_ + AdamW (train_CLIP.py:163-167, optimizer.py:41-85) ---- */

/* hyper[0] = ||g||_2, hyper[1] = min(1, max_norm/(||g|| + 1e-6)), then
 * hyper[2..3] = sched[2*s .. 2*s+1] (lr_t, lr*weight_decay) for s = *step,
 * and *step += 1.  work: >= 1024 floats of scratch. */
int ghm_clip_prepare(const float* grad, int64_t n, float max_norm, const float* sched,
                     int n_sched, int32_t* step, float* hyper, float* work, void* stream);

/* In place over flat fp32 buffers (reference op order, IEEE rounding, no FMA
 * contraction): g *= hyper[1]; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
 * p -= lr_t m / (sqrt(v) + eps); p -= (lr wd) p. */
int ghm_adamw(float* param, const float* grad, float* m, float* v, int64_t n, const float* hyper,
              float b1, float one_minus_b1, float b2, float one_minus_b2, float eps,
              void* stream);

/* ---- split-bf16 ("x3") path ------------------------------------------------
 * Same semantics and buffers as the f32 entry points above; every product is
 * evaluated as hi*hi + hi*lo + lo*hi with the operands split into bf16
 * hi = bf16(x), lo = bf16(x - hi) and f32 accumulation (v_mfma_f32_32x32x16_bf16):
 * ~2^-16 relative error per product instead of exact-f32 MFMA, at 5.3x the
 * matrix-core rate.  Weights come from a per-layer "pack" of pre-split bf16
 * planes written by ghm_split_weights (GHM_SPLIT_PACK_ELEMS bf16 per layer,
 * 16-byte aligned); re-split after every parameter update. */
#define GHM_SPLIT_PACK_ELEMS 983040
#define GHM_SPLIT_MAX_JOBS 16
typedef struct ghm_split_job {
  const float* Wq;  /* [128][128] each, nn.Linear layout [out][in] */
  const float* Wk;
  const float* Wv;
  const float* W1;  /* [512][128] */
  const float* W2;  /* [128][512] */
  void* pack;       /* GHM_SPLIT_PACK_ELEMS bf16 */
} ghm_split_job;
/* Split one layer's Q/K/V/MLP weights per job into its pack (up to 16 jobs). */
int ghm_split_weights(const ghm_split_job* jobs, int n_jobs, void* stream);
/* As ghm_ln_qkv_fwd (model.py:772-775). */
int ghm_ln_qkv_fwd_x3(const float* H, const float* ln_w, const float* ln_b, const void* pack, float* qkv,
                      float* stats, int64_t M, int D, float eps, void* stream);
/* ghm_ln_qkv_fwd_x3 that also writes the split LN1 rows it multiplies as bf16
 * (hi, lo) planes xs [2][M][128] (the B operand of ghm_wgrad_x3p for dWq|k|v;
 * round 6)  —  model.py:772-775. */
int ghm_ln_qkv_fwd_x3s(const float* H, const float* ln_w, const float* ln_b, const void* pack, float* qkv,
                       float* stats, void* xs, int64_t M, int D, float eps, void* stream);
/* LN2 + MLP + residual forward of one layer (as ghm_ln_mlp_fwd, model.py:741-747,
 * 784-788) on split-bf16 products, 16 tokens per wave (v_mfma_f32_16x16x32_bf16);
 * b1 [512], b2 [128] stay f32.  Only H_out and the LN2 stats leave the chip: the
 * backward, ghm_mlp_bwd_rc_x3, recomputes U. */
int ghm_ln_mlp_fwd_x3b(const float* H_mid, const float* ln_w, const float* ln_b, const void* pack,
                       const float* b1, const float* b2, float* H_out, float* stats, int64_t M, int D, int F,
                       float eps, void* stream);
/* ghm_ln_mlp_fwd_x3b that also writes the split LN2 rows as bf16 (hi, lo) planes
 * xs [2][M][128] (the B operand of ghm_wgrad_x3p for dW1; round 6). */
int ghm_ln_mlp_fwd_x3bs(const float* H_mid, const float* ln_w, const float* ln_b, const void* pack,
                        const float* b1, const float* b2, float* H_out, float* stats, void* xs, int64_t M, int D,
                        int F, float eps, void* stream);
/* Third split planes ("lo2": x = hi + lo + lo2) of each job's weights into job.pack,
 * a pack3 of GHM_SPLIT3_PACK_ELEMS bf16: W1 as the pack's W1_N image, W2 as its
 * W2_P32 image, [Wq; Wk; Wv] as its QKV_N image (round 6). */
#define GHM_SPLIT3_PACK_ELEMS 180224
int ghm_split3_weights(const ghm_split_job* jobs, int n_jobs, void* stream);
/* ghm_ln_qkv_fwd_x3 on three-way split operands (six bf16 MFMAs per product); pack3
 * from ghm_split3_weights (precision "f32fwd", $GHM_F32FWD qkv6; round 6). */
int ghm_ln_qkv_fwd_x6(const float* H, const float* ln_w, const float* ln_b, const void* pack, const void* pack3,
                      float* qkv, float* stats, int64_t M, int D, float eps, void* stream);
/* ghm_ln_mlp_fwd_x3b with every product on three-way split operands (six bf16
 * MFMAs, ~2^-24 relative: the exact-f32 level) and the exact GELU; pack3 from
 * ghm_split3_weights (precision "f32fwd", $GHM_F32FWD mlp6; round 6).  G / Dg
 * (both or neither): also saves GELU(U) and GELU'(U) [M][F] as ghm_ln_mlp_fwd does,
 * for the exact-f32 backward (precision "f32x6"). */
int ghm_ln_mlp_fwd_x6(const float* H_mid, const float* ln_w, const float* ln_b, const void* pack,
                      const void* pack3, const float* b1, const float* b2, float* H_out, float* stats, float* G,
                      float* Dg, int64_t M, int D, int F, float eps, void* stream);
/* MLP + LN2 backward with the up-projection recomputed from H_mid and the LN2
 * stats of the forward (which then saves no [M][F] tensor): writes G = GELU(U)
 * and dU = (dH_out W2) * GELU'(U) [M][F] (inputs of the dW2 / dW1 reductions),
 * dH_mid = dH_out + dLN2 (must not alias dH_out) and part_ln as ghm_mlp_bwd
 * (n_blocks = ghm_mlp_bwd_rc_x3_blocks(M))  —  backward of model.py:741-747,784-788.
 * split_out 0: G and dU f32 [M][F]; 1: pre-split bf16 planes for
 * ghm_wgrad_ring_x3's format 2 (hi [M][F] at the pointer, lo [M][F] right after
 * it: the same bytes), the columns of every 32-group in perm32 order (k-slot
 * 8g + i holds unit 4g + i for i < 4, 16 + 4g + i - 4 else). */
int ghm_mlp_bwd_rc_x3(const float* dH_out, const float* H_mid, const float* stats, const float* ln_w,
                      const float* ln_b, const void* pack, const float* b1, void* G, void* dU, float* dH_mid,
                      float* part_ln, int64_t M, int D, int F, int split_out, void* stream);
/* The same launch with per-workgroup clock stamps for bench.py's in-graph
 * kernel timing: stamps[2 b], stamps[2 b + 1] = s_memrealtime (100 MHz) at
 * workgroup b's start and end, 2 x ghm_mlp_bwd_rc_x3_blocks(M) uint64.  twin
 * (1 or 2) picks one of two identical kernel instantiations, so a profiler
 * trace separates two measurements. */
int ghm_mlp_bwd_rc_x3_stamped(const float* dH_out, const float* H_mid, const float* stats, const float* ln_w,
                              const float* ln_b, const void* pack, const float* b1, void* G, void* dU,
                              float* dH_mid, float* part_ln, int64_t M, int D, int F, int split_out,
                              uint64_t* stamps, int twin, void* stream);
/* As ghm_qkv_bwd (backward of model.py:772-775), with the LN1 statistics
 * recomputed from H exactly as the forward computed them (eps = the LayerNorm
 * eps); stats (the forward's [M][2] buffer) is accepted and not read
 * (DESIGN.md §4 "Determinism"). */
int ghm_qkv_bwd_x3(const float* dqkv, const float* H, const float* stats, const float* ln_w, const void* pack,
                   const float* dH_mid, float* dH, float* part_ln, int64_t M, int D, float eps, void* stream);
/* Diagnostic twin of ghm_qkv_bwd_x3 (tools/race_probe.py, DESIGN.md §4
 * "Determinism"): the LN1 statistics read from the forward's stats buffer,
 * mode 1 plain vector load (the round-2 load), 2 agent scope through a buffer
 * descriptor (sc0 sc1), 3 agent-scope global load (sc1), 4 recomputed with
 * the plain load issued beside: dbg[m] = (loaded mean, loaded rstd, recomputed
 * mean, recomputed rstd) [M][4], 5 as 1 with dbg[m] = (used mean, used rstd,
 * 0, 0).  Not on the training path. */
int ghm_qkv_bwd_x3_probe(const float* dqkv, const float* H, const float* stats, const float* ln_w, const void* pack,
                         const float* dH_mid, float* dH, float* part_ln, float* dbg, int64_t M, int D, float eps,
                         int mode, void* stream);

/* As ghm_attn_fwd / ghm_attn_bwd (model.py:778-782 and its backward); P and dS
 * are stored fp32 in the same dense padded layout. */
int ghm_attn_fwd_x3(const float* qkv, const float* H, float* H_mid, float* P, int64_t n_seq, int T, int D,
                    float scale_div, void* stream);
int ghm_attn_bwd_x3(const float* qkv, const float* P, const float* dH_mid, float* dS, float* dqkv, int64_t n_seq,
                    int T, int D, float scale_div, void* stream);
/* The same attention with the activation of the reference's get_activation
 * (models/model.py:121-130, applied at :781; train_CLIP --clip_activation):
 * act 0 softmax (identical to ghm_attn_fwd_x3 / ghm_attn_bwd_x3), 1 relu, 2
 * gelu (erf form) of the scaled scores, keys past T contributing 0.  P holds
 * act(s); for gelu the forward also writes GELU'(s) to Pd (same layout,
 * required) and the backward reads it.  The backward is the fused one-kernel
 * form (no dS buffer). */
int ghm_attn_fwd_x3_act(const float* qkv, const float* H, float* H_mid, float* P, float* Pd, int64_t n_seq, int T,
                        int D, float scale_div, int act, void* stream);
int ghm_attn_bwd_x3_act(const float* qkv, const float* P, const float* Pd, const float* dH_mid, float* dqkv,
                        int64_t n_seq, int T, int D, float scale_div, int act, void* stream);
/* As ghm_wgrad (b_mode 0 plain or 2 layernorm). */
int ghm_wgrad_x3(const float* A, int lda, int A_cols, const float* B, int ldb, int B_cols, int b_mode,
                 const float* stats, const float* ln_w, const float* ln_b, float* part, float* bias_part, int64_t M,
                 int tok_per_split, void* stream);
/* ghm_wgrad_x3 with B pre-split: Bp = the bf16 hi plane [M][ldb] of LN(x) written
 * by ghm_ln_qkv_fwd_x3s / ghm_ln_mlp_fwd_x3bs, the lo plane bplane elements on (no
 * LayerNorm transform, statistics or split in the kernel; round 6)  —  the
 * nn.Linear weight / bias gradients of model.py:772-775, 784-788. */
int ghm_wgrad_x3p(const float* A, int lda, int A_cols, const void* Bp, int ldb, int B_cols, int64_t bplane,
                  float* part, float* bias_part, int64_t M, int tok_per_split, void* stream);
/* Split-K weight (and bias) gradient partials of the encoder projections on an
 * LDS-DMA ring with producer / consumer waves (csrc/ghm_wgrad.hip):
 *   part[z][a][b] = sum_{m in split z} A[m][a] op(B)[m][b], bias_part[z][a] = sum A[m][a]
 * (bias_part may be NULL), z over ceil(M / tok_per_split) splits, A_cols and
 * B_cols multiples of 128.  Operand formats: 0 f32 rows of ld elements; 1 (B
 * only) f32 through LayerNorm with stats [M][2] (mean, rstd), ln_w, ln_b;
 * 2 pre-split bf16 planes of ghm_mlp_bwd_rc_x3(split_out = 1): hi [M][ld] at
 * the pointer, lo `plane` elements on, perm32 column order (the output rows /
 * columns are in natural order).  One operand must be format 0 or 1.  The
 * weight gradients of model.py:773-775 (dWq|k|v = dqkv^T LN1(H)) and :787-788
 * (dW2 = dY^T G, db2; dW1 = dU^T LN2(H_mid), db1) under autograd (train_CLIP.py:158). */
int ghm_wgrad_ring_x3(const void* A, int lda, int A_cols, int a_fmt, int64_t a_plane, const void* B, int ldb,
                      int B_cols, int b_fmt, int64_t b_plane, const float* stats, const float* ln_w,
                      const float* ln_b, float* part, float* bias_part, int64_t M, int tok_per_split,
                      void* stream);

/* ---- guided CLIP (clip_guide=True) ------------------------------------------
 * Exact BP_CLS messages of each sequence's GHM tree (data_random_GHM.py:185-208,
 * guided_info :526-549) from its leaves: trans = [L][C][V][V] f64 templates
 * (parent value, child value) of a translation-invariant tree (per_edge 0), or
 * (per_edge 1) every edge's matrix, layer by layer: [sum_l C^(l+1)][V][V], layer
 * l's edges in child order (parent * C + slot; GenTransition(translation_invariance=
 * False), data_random_GHM.py:43-89); msgs = [n_seq][n_total][V] f32 with
 * n_total = (C^L - 1)/(C - 1), levels in guided-target order (depth L-1 first,
 * root last), log-domain, max-shifted per node. */
int ghm_bp_cls(const double* trans, const uint8_t* tokens, float* msgs, int64_t n_seq, int L, int C, int V,
               int per_edge, void* stream);
/* part[n] = sum_{t,c<V} (H[n,t,c] - msgs[n][node_level(t)][c])^2 for guided target
 * `level` (model.py:790-800, 909-924); H is a [n_seq*T][128] residual stream. */
int ghm_guide_fwd(const float* H, const float* msgs, float* part, int64_t n_seq, int L, int C, int V, int level,
                  void* stream);
/* dH[n,t,c] += scale * (H[n,t,c] - msgs[...][c]) for c < V (scale = 2*penalty/n_seq). */
int ghm_guide_bwd(const float* H, const float* msgs, float* dH, int64_t n_seq, int L, int C, int V, int level,
                  float scale, void* stream);
/* loss_io[1] = loss_io[0] + penalty * mean_n sum_k part[k][n]; loss_io[2] = that mean / penalty;
 * phist[*step] = loss_io[1] if phist.  part: [n_parts][n_seq]. */
int ghm_guide_total(const float* part, int n_parts, int64_t n_seq, float penalty, float* loss_io, float* phist,
                    const int32_t* step, void* stream);

/* Module-API helpers (dense guided targets): out[r] = sum_e (a - b)^2 over rows of
 * row_len; out = scale[0]*alpha*(a - b); dst[m][c] += src[m][c] for c < V (dst [M][128]). */
int ghm_sqdiff_rows(const float* a, const float* b, float* out, int64_t rows, int64_t row_len, void* stream);
int ghm_scaled_diff(const float* a, const float* b, const float* scale, float alpha, float* out, int64_t n,
                    void* stream);
int ghm_add_cols(float* dst, const float* src, int64_t M, int V, void* stream);

/* Guided joint CDM (train_CDNS.py --guide=True; model.py:502-527, 1023-1040):
 * one guided block = V columns [col, col+V) of the tokens [tok0, tok0+ntok) of a
 * residual stream H [n_seq][T][128], against a BP message that each tree node
 * repeats over `ext` consecutive tokens (data_random_GHM.py:551-592):
 *   target(n,t,c) = msgs[n*msg_stride + moff + (t/ext)*V + c]
 * fwd: part[n] = sum (H - target)^2;  bwd: dH += scale * (H - target). */
int ghm_guide_blk_fwd(const float* H, int T, int tok0, int ntok, int col, const float* msgs, int64_t msg_stride,
                      int64_t moff, int ext, int V, float* part, int64_t n_seq, void* stream);
int ghm_guide_blk_bwd(const float* H, int T, int tok0, int ntok, int col, const float* msgs, int64_t msg_stride,
                      int64_t moff, int ext, int V, float* dH, float scale, int64_t n_seq, void* stream);
/* The same for a list of nb <= 32 blocks in one launch (block k: residual stream
 * H[k], messages msgs[k], desc[6k..6k+5] = {T, tok0, ntok, col, ext, V},
 * desc64[2k..2k+1] = {msg_stride, moff}); blocks apply in list order.
 * fwd: part[k*n_seq + n];  bwd: every block adds into the one dH. */
int ghm_guide_blks_fwd(const float* const* H, const float* const* msgs, const int32_t* desc, const int64_t* desc64,
                       int nb, float* part, int64_t n_seq, void* stream);
int ghm_guide_blks_bwd(const float* const* H, const float* const* msgs, const int32_t* desc, const int64_t* desc64,
                       int nb, float* dH, float scale, int64_t n_seq, void* stream);
/* The same for a residual stream of row pitch D (block columns col + V <= D): the
 * guided joint VLM (train_NWP.py --guide=True, model.py:303-331, loss :1122-1149,
 * D = 256, dense per-position targets: ext = 1). */
int ghm_guide_blks_fwd_d(const float* const* H, const float* const* msgs, const int32_t* desc,
                         const int64_t* desc64, int nb, int D, float* part, int64_t n_seq, void* stream);
int ghm_guide_blks_bwd_d(const float* const* H, const float* const* msgs, const int32_t* desc,
                         const int64_t* desc64, int nb, int D, float* dH, float scale, int64_t n_seq, void* stream);
/* Largest nb the block-list launches take (32). */
int ghm_guide_max_blocks(void);

/* ---- sequential conditional denoising (CDM, train_sequential_DNS.py) ---------
 * ConditionalDenoiseEncoderTransformer (models/model.py:337-532, sequential=True)
 * runs the encoder layer kernels above at T = T_img + n_cond tokens; only the
 * embedding, the readout, the loss and the BP posterior differ. */
/* H0 = token embedding + position embedding (model.py:404-423, :437): image token
 * t < T_img gets -((d - z[n,t])^2)/2 in features d < V, conditioning token
 * j = t - T_img gets cond[n, j, d] (row stride cond_ld) in d < V; all else 0.
 * z: f32 [n_seq][T_img]; cond: f32 [n_seq][T - T_img][cond_ld]; pos_w [T][128]. */
int ghm_cdm_embed_fwd(const float* z, const float* cond, int cond_ld, const float* pos_w, float* H0,
                      int64_t n_seq, int T, int T_img, int V, int D, void* stream);
/* Joint CDM (train_CDNS.py: sequential=False, model.py:408-423): text token
 * t >= T_img gets the row t_emb[tok[n, t - T_img]] ([V][128]); image tokens as
 * above.  tok uint8 [n_seq][T - T_img]; T <= 192. */
int ghm_cdm_embed_joint_fwd(const float* z, const uint8_t* tok, const float* t_emb, const float* pos_w, float* H0,
                            int64_t n_seq, int T, int T_img, int V, int D, void* stream);
/* Exact BP, f64, one workgroup per sample: the text tree's BP_CLS root message
 * (data_random_GHM.py:185-208) conditions BP_DNS of the image tree (:467-523,
 * external message :875-877).  trans: [L][C][V][V] templates, or per-edge tables
 * as ghm_bp_cls (per_edge bit 0: the text tree, bit 1: the image tree); t_tokens uint8
 * [n_seq][C_t^L_t]; z f64 [n_seq][C_i^L_i] noisy observations.  Writes the
 * posterior means post (f32, the "Compare" target, train_sequential_DNS.py:145)
 * and z32 = (float)z, the model input (torch.tensor(noise, float32), :882). */
int ghm_bp_dns(const double* t_trans, const double* i_trans, const uint8_t* t_tokens, const double* z,
               double sigma, float* post, float* z32, int64_t n_seq, int L_t, int C_t, int L_i, int C_i, int V,
               int per_edge, void* stream);
/* As ghm_bp_dns, and also the image tree's messages for the guided CDM
 * (data_random_GHM.py:551-592): msgs f32 [n_seq][3][n_nodes][V], planes hd, qd,
 * bu; n_nodes = non-root nodes + 1; depth d (1..L_i) nodes breadth-first from
 * offset sum_{e<d} C_i^e - 1, the root last (its qd plane is unused; its hd
 * plane holds bu, as the reference's in-place `+=` aliases them, :501-504). */
int ghm_bp_dns_msgs(const double* t_trans, const double* i_trans, const uint8_t* t_tokens, const double* z,
                    double sigma, float* post, float* z32, float* msgs, int64_t n_seq, int L_t, int C_t, int L_i,
                    int C_i, int V, int per_edge, void* stream);
/* pred[n, t] = H[n, t, :] . w_ro + b_ro for t < T_img (_read_out Linear(128, 1),
 * model.py:527-531).  H [n_seq][T][128]. */
int ghm_cdm_readout_fwd(const float* H, const float* w_ro, const float* b_ro, float* pred, int64_t n_seq, int T,
                        int T_img, int D, void* stream);
/* loss = mean_n sum_t (pred - target)^2 (ConditionalGuidedLsLoss guide=False and
 * LsLoss, model.py:997-998, :1152-1160); compare = the same against post (may be
 * NULL); dpred = 2 (pred - target) / n_seq (may be NULL).  loss_out[0..1] <- loss,
 * compare; hist / chist [*step] likewise when non-NULL.  Deterministic. */
int ghm_ls_loss(const float* pred, const uint8_t* target, const float* post, float* dpred, float* loss_out,
                float* hist, float* chist, const int32_t* step, int64_t n_seq, int T_img, void* stream);
/* Readout backward: dH[n, t, :] = dpred[n, t] w_ro (t < T_img; 0 for the
 * conditioning tokens), per-sequence partials part_w [n_seq][128] and part_b
 * [n_seq] of d_read_out.weight / .bias (reduce with ghm_reduce_batch). */
int ghm_cdm_readout_bwd(const float* H, const float* w_ro, const float* dpred, float* dH, float* part_w,
                        float* part_b, int64_t n_seq, int T, int T_img, int D, void* stream);

/* ---- sequential VLM (next-word prediction, train_sequential_NWP.py) ----------
 * AutoRegressiveTransformer (models/model.py:132-335, sequential=True,
 * auto_regressive=True) at width D (256 in exp_vlm_*.sh): its plain projections
 * (QKV, MLP, readout) are library GEMMs in the host code; these are the operators
 * between them.  Layouts row-major [rows][D] fp32, M = n_seq * T. */
/* H0 = token embedding + positions (model.py:274-293, :305): prefix token t < P gets
 * feat[n, t, 0:V] zero-padded to D, text token t >= P gets tok_w[xt[n, t - P]].
 * onehot (may be NULL) [M][V] = the text tokens' one-hot rows (0 on prefix rows). */
int ghm_vlm_embed_fwd(const uint8_t* xt, const float* feat, const float* tok_w, const float* pos_w, float* H0,
                      float* onehot, int64_t n_seq, int T, int P, int V, int D, void* stream);
/* Joint VLM (train_NWP.py, sequential=False, model.py:221-232): prefix (image) token
 * t < P gets i_w[it[n, t]] (it uint8 [n_seq][P]), text token t >= P gets
 * tok_w[xt[n, t - P]]; onehot_t / onehot_i (may be NULL) [M][V] one-hot rows of the
 * text / image tokens (0 on the other kind). */
int ghm_vlm_embed_joint_fwd(const uint8_t* xt, const uint8_t* it, const float* i_w, const float* tok_w,
                            const float* pos_w, float* H0, float* onehot_t, float* onehot_i, int64_t n_seq, int T,
                            int P, int V, int D, void* stream);
/* Row LayerNorm Y = LN(X) (nn.LayerNorm(D), biased variance), stats [M] (mean, rstd);
 * D in {128, 256, 512}. */
int ghm_ln_rows_fwd(const float* X, const float* w, const float* b, float* Y, float* stats, int64_t M, int D,
                    float eps, void* stream);
/* dX = dres + LayerNorm backward of dY (dres may alias dX); part [n_blocks][2][D]
 * per-block (dgamma, dbeta) partials, n_blocks = ghm_ln_rows_blocks(M). */
int64_t ghm_ln_rows_blocks(int64_t M);
int ghm_ln_rows_bwd(const float* dY, const float* X, const float* stats, const float* w, const float* dres,
                    float* dX, float* part, int64_t M, int D, void* stream);
/* H_mid = H + A V + (A / D) V with A = softmax((Q K^T + mask) / scale_div), the
 * prefix-causal mask of generate_mask (model.py:24-33) and the reference's double
 * attention residual (:338-341); P [n_seq][96][96] saved for backward.  q, k, v
 * [M][D] (T <= 96, D % 64 == 0). */
int ghm_vlm_attn_fwd(const float* q, const float* k, const float* v, const float* H, float* H_mid, float* P,
                     int64_t n_seq, int T, int D, int n_prefix, float scale_div, void* stream);
/* Backward of ghm_vlm_attn_fwd: dq, dk, dv [M][D] from dH_mid (the residual term
 * dH += dH_mid is the caller's). */
int ghm_vlm_attn_bwd(const float* q, const float* k, const float* v, const float* P, const float* dH_mid, float* dq,
                     float* dk, float* dv, int64_t n_seq, int T, int D, float scale_div, void* stream);
/* G = GELU(U), Dg = GELU'(U) (nn.GELU, approximate='none'); out = a * b; out = a + b. */
int ghm_gelu_fwd(const float* U, float* G, float* Dg, int64_t n, void* stream);
int ghm_mul(const float* a, const float* b, float* out, int64_t n, void* stream);
int ghm_add(const float* a, const float* b, float* out, int64_t n, void* stream);
/* Next-token cross entropy over the text rows t >= n_prefix of logits [n_seq][T][V]
 * (ConditionalGuidedCELoss guide=False, model.py:1087-1098) and the batchmean KL of
 * post [n_seq][T - n_prefix][V] against softmax(logits) (KLdiv, :1067-1078; post may
 * be NULL); dlogits (may be NULL) = (softmax - onehot) / rows on text rows, 0 on
 * prefix rows.  loss_out[0..1] <- loss, compare; loss_out[2..] holds per-workgroup
 * partials: the buffer has ghm_ce_kl_out_elems(n_seq, T, n_prefix) floats.
 * hist / chist [*step] when non-NULL. */
int64_t ghm_ce_kl_out_elems(int64_t n_seq, int T, int n_prefix);
int ghm_ce_kl(const float* logits, const uint8_t* targets, const float* post, float* dlogits, float* loss_out,
              float* hist, float* chist, const int32_t* step, int64_t n_seq, int T, int n_prefix, int V,
              void* stream);

/* Split-bf16 MFMA form of ghm_vlm_attn_fwd / _bwd (csrc/ghm_vlm_x3.hip) on the fused
 * projection layout: q, k, v are columns [0, D), [D, 2D), [2D, 3D) of qkv [M][3D];
 * the backward writes dq, dk, dv into dqkv [M][3D] the same way, with dS
 * [n_seq][96][96] scratch.  D in {128, 256}, T <= 96. */
int ghm_vlm_attn_fwd_x3(const float* qkv, const float* H, float* H_mid, float* P, int64_t n_seq, int T, int D,
                        int n_prefix, float scale_div, void* stream);
int ghm_vlm_attn_bwd_x3(const float* qkv, const float* P, const float* dH_mid, float* dS, float* dqkv, int64_t n_seq,
                        int T, int D, float scale_div, void* stream);

/* General form of the two above: prefix-causal mask with n_prefix (n_prefix = T: no
 * mask), H_mid = (H + o) + o * dbl (dbl = 1/D: the VLM's double residual; 0: the
 * plain residual of the CLIP / CDM encoders, model.py:391-394, 474-478).  D in
 * {128, 256}, T <= 192 (P, dS [n_seq][192][192] when T > 96, else [n_seq][96][96]).
 * The joint CDM (train_CDNS.py, T = 162) and joint VLM (train_NWP.py, T = 161) run on it. */
int ghm_attn_ext_fwd_x3(const float* qkv, const float* H, float* H_mid, float* P, int64_t n_seq, int T, int D,
                        int n_prefix, float scale_div, float dbl, void* stream);
int ghm_attn_ext_bwd_x3(const float* qkv, const float* P, const float* dH_mid, float* dS, float* dqkv, int64_t n_seq,
                        int T, int D, int n_prefix, float scale_div, float dbl, void* stream);
/* The same with the attention activation of model.py:121-130 (get_activation,
 * applied at :485 for the CDM): act 1 relu, 2 gelu of the scaled score,
 * elementwise (no row normalisation; masked entries 0); gelu writes GELU'(score)
 * to Pd (same shape as P) for the backward, which takes dS = act'(score) dA /
 * scale_div.  D == 128 (the joint CDM at T = 162 under train_CDNS.py --activation) or
 * 256 (the VLM, AutoRegressiveTransformer(activation="relu"), model.py:163, 287). */
int ghm_attn_ext_fwd_x3_act(const float* qkv, const float* H, float* H_mid, float* P, float* Pd, int64_t n_seq,
                            int T, int D, int n_prefix, float scale_div, float dbl, int act, void* stream);
int ghm_attn_ext_bwd_x3_act(const float* qkv, const float* P, const float* Pd, const float* dH_mid, float* dS,
                            float* dqkv, int64_t n_seq, int T, int D, int n_prefix, float scale_div, float dbl,
                            int act, void* stream);

/* ---- split-bf16 (x3) GEMM for the VLM projections (csrc/ghm_gemm.hip) -------
 * Replaces the nn.Linear products of AutoRegressiveTransformer (models/model.py:
 * 203-216 _queries/_keys/_values/_mlps, applied at :330-347) and their autograd
 * backward.  C[m][n] = sum_k A(m,k) B(k,n), fp32 in/out, split-bf16 MFMA inside:
 *   ta = 0: A(m,k) = A[m*lda + k];  ta = 1: A(m,k) = A[k*lda + m]
 *   tb = 1: B(k,n) = Bq[n*ldb + k]; tb = 0: B(k,n) = Bq[k*ldb + n]
 * B may be three tensors B0, B1, B2 stacked along its storage rows (n for tb = 1,
 * k for tb = 0), b_chunk rows each (0: B0 only).  N % 128 == 0.
 * epi: 0 C = acc; 1 (u = acc + bias[n]) C = GELU(u), C2 = GELU'(u); 2 C = acc +
 * bias[n] + R[m][n]; 3 C = acc * R[m][n]; 4 split-k partials C[z][M][N] (nsplit
 * slabs of ghm_gemm_slab_elems floats in total), summed by ghm_gemm_reduce; with
 * ta = 1 and C2 set, also C2[z][m] = the split's sum over k of A(m, k) (nsplit x M
 * floats: the Linear bias gradient as a by-product of its weight gradient). */
int64_t ghm_gemm_slab_elems(int64_t M, int64_t N, int nsplit);
int ghm_gemm_x3(int ta, int tb, int epi, const float* A, int64_t lda, const float* B0, const float* B1,
                const float* B2, int64_t ldb, int64_t b_chunk, float* C, int64_t ldc, float* C2, const float* bias,
                const float* R, int64_t ldr, int64_t M, int64_t N, int64_t K, int nsplit, void* stream);
/* The same product with exact f32 MFMA (v_mfma_f32_32x32x2f32, no split) and the
 * erf GELU in epilogue 1: the VLM's precision "f32" mode (replaces the torch.mm /
 * addmm library calls of rounds 1-3).  Arguments and limits as ghm_gemm_x3. */
int ghm_gemm_f32(int ta, int tb, int epi, const float* A, int64_t lda, const float* B0, const float* B1,
                 const float* B2, int64_t ldb, int64_t b_chunk, float* C, int64_t ldc, float* C2, const float* bias,
                 const float* R, int64_t ldr, int64_t M, int64_t N, int64_t K, int nsplit, void* stream);
/* ghm_gemm_x3 with ta = 0 and B pre-split (round 5; the VLM's weight products,
 * nn.Linear in model.py:132-335): C = A(m,k) B(k,n) with B(k,n) = Bp[n][k], Bp
 * the bf16 hi image [N][K] (pitch ldbp) and the lo image bplane elements on, as
 * ghm_split_pack writes them; the K loop copies B's tiles without splitting
 * them.  Epilogues as ghm_gemm_x3 (C2: GELU' only); N % 128 == 0, K % 32 == 0,
 * ldbp and bplane % 8 == 0. */
int ghm_gemm_x3p(int epi, const float* A, int64_t lda, const void* Bp, int64_t ldbp, int64_t bplane, float* C,
                 int64_t ldc, float* C2, const float* bias, const float* R, int64_t ldr, int64_t M, int64_t N,
                 int64_t K, int nsplit, void* stream);
/* Split f32 matrices into bf16 (hi, lo) images for ghm_gemm_x3p: jobs is a
 * DEVICE array of n_jobs x 8 int64 (src pointer, src pitch, rows, cols, dst
 * pointer (bf16 hi), dst pitch, lo-plane offset in elements, transpose 0 / 1:
 * dst[c][r] = split(src[r][c])); max_tiles >= the largest job's count of 64 x 64
 * tiles.  Once per step, after the optimizer. */
int ghm_split_pack(const int64_t* jobs, int n_jobs, int max_tiles, void* stream);
/* D[m][n] = sum_z slab[z][m][n] (z in order: deterministic); rows stacked into
 * D0, D1, D2 by chunk (0: D0 only). */
int ghm_gemm_reduce(const float* slab, int nsplit, int64_t M, int64_t N, float* D0, float* D1, float* D2,
                    int64_t chunk, void* stream);
/* ghm_gemm_reduce plus, in the same launch, bdst[m] = sum_z bslab[z][m] (the row
 * sums of a ta = 1 slab GEMM; M % 4 == 0).  bslab = bdst = NULL: ghm_gemm_reduce.
 * Replaces the bias-gradient column sums of the MLP Linears (model.py:344-347). */
int ghm_gemm_reduce_bias(const float* slab, int nsplit, int64_t M, int64_t N, float* D0, float* D1, float* D2,
                         int64_t chunk, const float* bslab, float* bdst, void* stream);
/* out[n] = sum_m X[m][n] (deterministic two-stage), X [M][N] fp32, N % 4 == 0 and
 * N/4 dividing 256 or >= 256; part scratch of ghm_colsum_part_elems(M, N) floats.
 * The bias gradients of the Linear layers and the position-embedding gradient
 * (autograd's sum over batch rows, model.py:291-293, :330-347). */
int64_t ghm_colsum_part_elems(int64_t M, int64_t N);
int ghm_colsum(const float* X, int64_t M, int64_t N, float* out, float* part, void* stream);
/* Weighted column sums: out[c][n] = sum_m w(m, c) X[xrow(m)][n] and (if wsum)
 * wsum[c] = sum_m w(m, c) (dense W only), c < C <= 64, N/4 dividing 256.  w(m, c) = W[m][c]
 * (dense [M][C]; the readout weight and bias gradients from dlogits) or
 * [tok[m] == c] when W is NULL (token ids [M]; the t_embedding / i_embedding
 * gradients, autograd's embedding backward of model.py:238-241 and :444); xrow(m) = (m / rps) * seq_rows + off + m % rps.  Deterministic two
 * stages; part scratch of ghm_wcolsum_part_elems(M, N, C) floats. */
int64_t ghm_wcolsum_part_elems(int64_t M, int64_t N, int C);
int ghm_wcolsum(const float* W, const uint8_t* tok, int C, const float* X, int64_t rps, int64_t seq_rows, int64_t off,
                int64_t M, int64_t N, float* out, float* wsum, float* part, void* stream);
/* The readout Linear for C <= 64 classes, D in {128, 256} (model.py:332 _read_out):
 * Y[m][c] = b[c] + sum_d X[m][d] W[c][d]; its data gradient
 * dX[m][d] = sum_c dZ[m][c] W[c][d]. */
int ghm_rows_linear(const float* X, const float* W, const float* b, float* Y, int64_t M, int D, int C, void* stream);
int ghm_rows_linear_t(const float* dZ, const float* W, float* dX, int64_t M, int D, int C, void* stream);

/* ---- generic-width CLIP encoder ends (csrc/ghm_genc.hip, models/gemm_encoder.py:
 * n_embd != 128, e.g. the reference CLI default clip_{t,i}model_deb = 64,
 * utils/config.py:58-59; its layers run on ghm_gemm_x3, ghm_ln_rows_* and
 * ghm_attn_ext_*_x3 at D = n_embd) ------------------------------------------ */

/* H0[n, t, :] = tok_w[tokens[n, t]] + pos_w[t], D floats per row
 * —  models/model.py:762-765 (token_embeddings(x) + position_embeddings). */
int ghm_tok_embed_fwd(const uint8_t* tokens, const float* tok_w, const float* pos_w, float* H0, int64_t n_seq, int T,
                      int V, int D, void* stream);

/* emb[n][c] = b_out + sum_t w_out[t] Z[n][t][c], Z = H_L W_ro^T + b_ro (ghm_rows_linear)
 * —  models/model.py:802-805 (_read_out, transpose, _out). */
int ghm_tok_readout_fwd(const float* Z, const float* w_out, const float* b_out, float* emb, int64_t n_seq, int T,
                        int C, void* stream);

/* Backward of the token-axis Linear(n_token -> 1): dZ[n][t][c] = w_out[t] d_emb[n][c],
 * d_wout[t] = sum_{n,c} d_emb[n][c] Z[n][t][c], d_bout[0] = sum d_emb (fixed-order
 * sums; one launch)  —  backward of models/model.py:804-805. */
int ghm_tok_readout_bwd(const float* Z, const float* d_emb, const float* w_out, float* dZ, float* d_wout,
                        float* d_bout, int64_t n_seq, int T, int C, void* stream);

/* ---- zero-shot classification (figures/eval-zsc-risk.py:107-118) --------
 * logits[q][r][c] = log( mean_{k < n_list[q]} exp(<i_emb[r], t_emb[proto_idx[c][k]]>) )
 * for every image row r < n_rows and class c < n_class: the reference's
 * torch.log(exp(i_embeddings @ t_embeddings.T)[:, index].mean(dim=1)) for the
 * first n_list[q] text samples of class c, without forming the N x N matrix.
 * i_emb [n_rows][D], t_emb [*][D] fp32 (D <= 16); proto_idx int32
 * [n_class][n_proto] (rows of t_emb); n_list int32 [n_j] (n_j <= 8, each in
 * 1..n_proto); logits fp32 [n_j][n_rows][n_class].  Exact f32 MFMA products. */
int ghm_zsc_logits(const float* i_emb, int64_t n_rows, const float* t_emb, int D, const int32_t* proto_idx,
                   int n_class, int n_proto, const int32_t* n_list, int n_j, float* logits, void* stream);

/* ---- helpers ----------------------------------------------------------- */
/* number of 128-token blocks the token-parallel kernels use for M tokens */
int64_t ghm_token_blocks(int64_t M);
/* number of LN-partial rows (token workgroups) ghm_mlp_bwd_rc_x3 writes for M tokens */
int64_t ghm_mlp_bwd_rc_x3_blocks(int64_t M);

#ifdef __cplusplus
}
#endif
#endif
