"""ORACLE — CPU restatement of the reference's zero-shot-classification
evaluation (figures/eval-zsc-risk.py:62-121, zsc_loss).

TEST INFRASTRUCTURE ONLY: only tests/ may import it, as the checker of
ghmclip.evaluation.zsc and the ghm_zsc_logits kernel.  Nothing in
multimodal-ghm_amd/ imports it.

Parity pinning: tests/golden/zsc_small.npz holds the reference's own draw
(DoubleSampler.get_zeroshot_batch), both towers' embeddings and the losses the
reference's zsc_loss returned for them (tests/golden/make_golden_zsc.py imports
the reference); tests/test_zsc_host.py checks this restatement against them.

Reference file:line it follows:
  prototypes   figures/eval-zsc-risk.py:86-91 (first num_samples text samples per class)
  embeddings   :96-105  total // 200 minibatches of 200: the last total % 200 rows stay 0
  similarity   :107   exp_similarity = exp(i_embeddings @ t_embeddings.T)     (f32)
  logits       :109-116  log(exp_similarity[:, index].mean(dim=1)) per class
  risk         :118-119  cross_entropy(model_predict, t_leaves[:, 0])
  Bayes        :73-82    i_pp projected through every text transition's slot-0
                         matrix, log, cross entropy against the first text leaf
"""
import numpy as np


def reference_rows(emb, minibatch=200):
    """The embeddings zsc_loss actually uses (:98-105): it fills
    total // minibatch minibatches of 200 rows, so the last total % 200 rows keep
    their torch.zeros initial value (e.g. 100 of 300, 100 of 7500)."""
    out = np.array(emb, np.float32, copy=True)
    out[(len(out) // minibatch) * minibatch:] = 0.0
    return out


def prototype_index(first, n_class, n_max):
    """[n_class][n_max] int32: the first n_max sample indices whose first text
    leaf is c (torch.where(t_leaves[:, 0] == c)[0][:n], :88-90)."""
    out = np.empty((n_class, n_max), np.int32)
    for c in range(n_class):
        idx = np.nonzero(np.asarray(first) == c)[0]
        if len(idx) < n_max:
            raise ValueError(f"class {c} only has {len(idx)} text samples")
        out[c] = idx[:n_max]
    return out


def zsc_logits(i_emb, t_emb, proto_idx, n_list):
    """[len(n_list)][N][n_class] float32: log of the mean of exp(<i_r, t_k>) over
    each class's first n prototypes, evaluated in float32 as the reference does."""
    i_emb = np.asarray(i_emb, np.float32)
    t_emb = np.asarray(t_emb, np.float32)
    S = np.exp(i_emb @ t_emb.T)  # [N, N] float32
    n_class = proto_idx.shape[0]
    out = np.empty((len(n_list), len(i_emb), n_class), np.float32)
    for q, n in enumerate(n_list):
        for c in range(n_class):
            out[q, :, c] = np.log(S[:, proto_idx[c, :n]].mean(axis=1, dtype=np.float32))
    return out


def cross_entropy(logits, labels):
    """mean over rows of logsumexp(logits) - logits[label] (float64 accumulation)."""
    x = np.asarray(logits, np.float64)
    m = x.max(axis=1, keepdims=True)
    lse = (m[:, 0] + np.log(np.exp(x - m).sum(axis=1)))
    return float((lse - x[np.arange(len(x)), np.asarray(labels)]).mean())


def zsc_risks(i_emb, t_emb, first, n_list, n_class=10):
    """The model losses zsc_loss reports for one encoder pair, one per n (from
    the full embeddings; the reference's zero tail applied here)."""
    idx = prototype_index(first, n_class, max(n_list))
    lg = zsc_logits(reference_rows(i_emb), reference_rows(t_emb), idx, n_list)
    return [cross_entropy(lg[q], first) for q in range(len(n_list))]


def bayes_risk(i_pp, t_transition, first):
    """:73-82: the image root posterior pushed through the text tree's slot-0
    transition of every layer, as logits of the first text leaf."""
    p = np.asarray(i_pp, np.float64)
    for layer in t_transition:
        p = p @ np.asarray(layer[0], np.float64)
    return cross_entropy(np.log(p.astype(np.float32)), first)
