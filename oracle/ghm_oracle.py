"""ORACLE — CPU restatement of the reference CLIP training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (multimodal-ghm_amd/)
imports this file.  Only tests/, __graft_entry__.smoke() and bench.py's
``cpu_baseline`` leg may import it, and only as the checker / the timed CPU
baseline, never as the thing measured or shipped.

Parity pinning: this restatement is checked against golden fixtures produced by
importing the real reference (tests/golden/make_golden.py, committed with its
outputs): the sampler bit-exactly (sampler_*.npz), one/two full training steps
of a tiny and a d=128 config (clip_tiny.npz, clip_d128.npz), the 200-step loss
curve of the default config (clip_default_curve.npz) and the 20 published
Bayes CLIP risks (bayes.json, from figures/data/ghm-data/clip-risk.json:90-110).

Everything cites the reference file:line it follows (paths relative to the
reference root, src/ghmclip/...).
  sampler      data/data_random_GHM.py:43-96 (GenTransition, _softmax_row),
               :145-165 (GHMTree.gen_values), :753-784 (ClipSampler.get_batch)
  Bayes        data/data_random_GHM.py:185-221 (BP_CLS), :786-817 (get_Bayes)
  encoder      models/model.py:690-808 (EncoderTransformer)
  loss         models/model.py:867-926 (GuidedClipLoss, guide=False)
  optimizer    models/optimizer.py:34-85 (AdamW, get_lr_cosine_schedule)
  loop         training/train_CLIP.py:62-201
"""
import math
import random
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------
# seeding — models/model.py:12-22
# ----------------------------------------------------------------------------
def seed_everything(seed):
    random.seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


# ----------------------------------------------------------------------------
# sampler — data/data_random_GHM.py
# ----------------------------------------------------------------------------
def _softmax_row(x):
    """data_random_GHM.py:91-96"""
    e = np.exp(x - np.max(x, axis=1, keepdims=True))
    return e / e.sum(axis=1, keepdims=True)


def gen_transition(n_layer, n_child, V, p_flip, flip_scale=1.0):
    """Translation-invariant GenTransition (data_random_GHM.py:43-89).

    Returns an array [n_layer, n_child, V, V]: the distinct per-(layer, child-slot)
    matrices.  The reference repeats each layer's n_child templates n_child**layer
    times (:71-76), so transition[layer][id*n_child + c] == out[layer, c].
    RNG consumption order (permutation, then one normal(V,V) per child) is kept.
    """
    out = np.zeros((n_layer, n_child, V, V))
    for layer in range(n_layer):
        skel = np.identity(V)[np.random.permutation(V), :]
        for c in range(n_child):
            out[layer, c] = (1 - p_flip) * skel + p_flip * _softmax_row(
                np.random.normal(0, flip_scale, [V, V]))
    return out


def gen_leaves(trans, root):
    """GHMTree.gen_values with a given root (data_random_GHM.py:145-165).

    The reference draws ``np.random.rand(B, 1)`` per (parent node, child slot) in
    breadth-first order; drawing one rand(n_parent, n_child, B) block per layer
    consumes the identical stream in the identical order.  ``(u < cdf).argmax``
    reproduces the inverse CDF including the all-False -> 0 case.
    Returns leaves [B, n_child**n_layer] (int64), position = BFS leaf index.
    """
    n_layer, n_child = trans.shape[0], trans.shape[1]
    B = root.shape[0]
    vals = root[None, :].astype(np.int64)  # [n_nodes, B]
    for layer in range(n_layer):
        n_par = vals.shape[0]
        u = np.random.rand(n_par, n_child, B)
        cdf = trans[layer].cumsum(axis=2)  # [n_child, V, V]
        child = np.empty((n_par, n_child, B), dtype=np.int64)
        for c in range(n_child):
            rows = cdf[c][vals]  # [n_par, B, V]
            child[:, c, :] = (u[:, c, :, None] < rows).argmax(axis=2)
        vals = child.reshape(n_par * n_child, B)
    return vals.T.copy()


class ClipSamplerOracle:
    """ClipSampler (data_random_GHM.py:746-784) for translation-invariant trees."""

    def __init__(self, n_layers, n_childs, p_flips, K=4, flip_scale=1, variable_type=10,
                 seedtree=42):
        self.K, self.V = K, variable_type
        self.n_layers, self.n_childs = n_layers, n_childs
        np.random.seed(seedtree)  # DoubleSampler.__init__ :654
        self.t_trans = gen_transition(n_layers[0], n_childs[0], variable_type, p_flips[0], flip_scale)
        self.i_trans = gen_transition(n_layers[1], n_childs[1], variable_type, p_flips[1], flip_scale)

    def get_batch(self, batch_size=128):
        """:753-784 (guide=False).  Returns (t_leaves, t_root, i_leaves, i_root) numpy."""
        B, K = batch_size, self.K
        t_root = np.random.choice(self.V, size=B * (K + 1))
        i_root = np.random.choice(self.V, size=B * (K - 1))
        i_root = np.append(t_root[:2 * B], i_root)
        t_leaves = gen_leaves(self.t_trans, t_root)
        i_leaves = gen_leaves(self.i_trans, i_root)
        return t_leaves, t_root, i_leaves, i_root


def bp_cls_posterior(trans, leaves, p_y):
    """Vectorised BP_CLS (data_random_GHM.py:185-221): p(root | leaves), [B, V].

    Same message arithmetic (log-domain, per-node max shift); nodes of a layer are
    processed together since translation invariance makes their matrices equal per
    child slot.
    """
    n_layer, n_child, V, _ = trans.shape
    B = leaves.shape[0]
    lv = leaves.T  # [n_leaves, B]
    n_par = lv.shape[0] // n_child
    # leaves -> depth L-1 nodes: sum_c log T_c[:, x_child]  (:191-197)
    msg = np.zeros((n_par, V, B))
    for c in range(n_child):
        msg += np.log(trans[-1, c][:, lv[c::n_child]].transpose(1, 0, 2))
    msg -= msg.max(axis=1, keepdims=True)
    for layer in range(n_layer - 2, -1, -1):  # :201-208
        n_par = msg.shape[0] // n_child
        new = np.zeros((n_par, V, B))
        for c in range(n_child):
            ch = msg[c::n_child]  # [n_par, V, B]
            new += np.log(np.einsum("ij,njb->nib", trans[layer, c], np.exp(ch)))
        new -= new.max(axis=1, keepdims=True)
        msg = new
    h0 = msg[0] + np.log(p_y).reshape(-1, 1)  # :213
    h0 -= h0.max(axis=0)
    pp = np.exp(h0) / np.exp(h0).sum(axis=0)
    return pp.T


def bp_cls_messages(trans, leaves):
    """Per-level BP_CLS messages (data_random_GHM.py:185-208) as GHMTree.guided_info
    returns them (:526-549), compactly: one entry per tree node instead of one per
    descendant leaf.  Returns [msg_depth_{L-1}, ..., msg_root], each float64
    [B, n_nodes, V] (n_nodes = 27, 9, 3, 1 for L=4, C=3), node order BFS."""
    n_layer, n_child, V, _ = trans.shape
    lv = leaves.T  # [n_leaves, B]
    n_par = lv.shape[0] // n_child
    msg = np.zeros((n_par, V, lv.shape[1]))
    for c in range(n_child):
        msg += np.log(trans[-1, c][:, lv[c::n_child]].transpose(1, 0, 2))
    msg -= msg.max(axis=1, keepdims=True)
    out = [msg]
    for layer in range(n_layer - 2, -1, -1):
        n_par = msg.shape[0] // n_child
        new = np.zeros((n_par, V, msg.shape[2]))
        for c in range(n_child):
            new += np.log(np.einsum("ij,njb->nib", trans[layer, c], np.exp(msg[c::n_child])))
        new -= new.max(axis=1, keepdims=True)
        msg = new
        out.append(msg)
    return [m.transpose(2, 0, 1) for m in out]


def expand_messages(msgs, n_leaves):
    """[B, n_nodes, V] per level -> the reference's guided targets [B, n_leaves, V]
    (float32, torch.tensor(..., dtype=torch.float) in guided_info)."""
    return [torch.from_numpy(np.repeat(m, n_leaves // m.shape[1], axis=1).astype(np.float32)) for m in msgs]


def clip_bayes(sampler, n_eval=10000):
    """ClipSampler.get_Bayes (data_random_GHM.py:786-817) without the dense kron."""
    t_l, _, i_l, _ = sampler.get_batch(n_eval)
    p_y = np.ones(sampler.V) / sampler.V
    tp = bp_cls_posterior(sampler.t_trans, t_l, p_y).T  # [V, 5n]
    ip = bp_cls_posterior(sampler.i_trans, i_l, p_y).T
    K, V, n = sampler.K, sampler.V, n_eval

    def fold(x):  # S_indep.dot(kron(ones(K-1,1), eye(n)))  (:801)
        return x.reshape(K - 1, n).sum(axis=0)

    S_match = np.sum(tp[:, :n] * ip[:, :n], 0) * V
    S_indep = fold(np.sum(tp[:, 2 * n:] * np.tile(ip[:, :n], (1, K - 1)), 0)) * V
    S = -np.log(S_match / (S_indep + S_match))
    S_match = np.sum(tp[:, n:2 * n] * ip[:, n:2 * n], 0) * V
    S_indep = fold(np.sum(ip[:, 2 * n:] * np.tile(tp[:, n:2 * n], (1, K - 1)), 0)) * V
    S = S - np.log(S_match / (S_indep + S_match))
    return float(np.mean(S)), float(np.std(S) / np.sqrt(n))


# ----------------------------------------------------------------------------
# encoder — models/model.py:690-808 (normalize_attn=True; attention activation
# softmax | relu | gelu as get_activation, models/model.py:121-130)
# ----------------------------------------------------------------------------
class OracleEncoder(nn.Module):
    """Same module construction order as the reference so torch.manual_seed gives
    identical initial weights and identical state_dict keys (model.py:725-758)."""

    def __init__(self, n_token, num_class, n_embd=128, n_layer=12, n_mlp_multiplier=4,
                 normalize_attn=True, guide=False, n_guided_layer=4, activation="softmax"):
        super().__init__()
        self.n_embd, self.normalize_attn = n_embd, normalize_attn
        if activation not in ("softmax", "relu", "gelu"):
            raise NotImplementedError(activation)  # :129-130
        self.activation = activation
        self.vocab_size = num_class
        # guided layer flags, model.py:716-718,751-755
        gap = max(1, n_layer // n_guided_layer)
        self.guided_layer_flag, cnt = [False] * n_layer, 0
        for i in range(n_layer):
            if guide and cnt < n_guided_layer and (i + 1) % gap == 0:
                self.guided_layer_flag[i] = True
                cnt += 1
        self.token_embeddings = nn.Embedding(num_class, n_embd)
        self.position_embeddings = nn.Embedding(n_token, n_embd)
        self._queries, self._keys, self._values = nn.ModuleList(), nn.ModuleList(), nn.ModuleList()
        self._mlps, self._lns_1, self._lns_2 = nn.ModuleList(), nn.ModuleList(), nn.ModuleList()
        h = n_embd * n_mlp_multiplier
        for _ in range(n_layer):
            self._queries.append(nn.Linear(n_embd, n_embd, bias=False))
            self._keys.append(nn.Linear(n_embd, n_embd, bias=False))
            self._values.append(nn.Linear(n_embd, n_embd, bias=False))
            self._lns_1.append(nn.LayerNorm([n_embd]))
            self._mlps.append(nn.Sequential(nn.Linear(n_embd, h), nn.GELU(), nn.Linear(h, n_embd)))
            self._lns_2.append(nn.LayerNorm([n_embd]))
        self._read_out = nn.Linear(n_embd, num_class)
        self._out = nn.Linear(n_token, 1)

    def forward(self, x):
        B, T = x.shape
        pos = torch.arange(T, device=x.device).expand(B, T)
        H = self.token_embeddings(x) + self.position_embeddings(pos)  # :765
        guided = []
        # test hooks: `scores` (a list) records each layer's scaled scores; `relu_masks`
        # (per layer, [B, T, T]) replaces relu's own mask with given ones, so that a
        # float64 gradient can be taken with the masks a kernel used (tests/test_gpu_width.py)
        for l, (q, k, v, mlp, ln1, ln2, flag) in enumerate(zip(self._queries, self._keys, self._values,
                                                               self._mlps, self._lns_1, self._lns_2,
                                                               self.guided_layer_flag)):
            H1 = ln1(H)  # :772
            S = torch.matmul(q(H1), k(H1).transpose(-2, -1))  # :778
            if self.normalize_attn:
                S = S / np.sqrt(self.n_embd)  # :779-780
            if getattr(self, "scores", None) is not None:
                self.scores.append(S.detach())
            if self.activation == "softmax":  # :781 through get_activation (:121-130)
                A = F.softmax(S, dim=-1)
            elif self.activation == "relu":
                masks = getattr(self, "relu_masks", None)
                A = F.relu(S) if masks is None else S * masks[l].to(S.dtype)
            else:
                A = F.gelu(S)
            H = H + torch.einsum("bij,bjd->bid", A, v(H1))  # :782
            H = H + mlp(ln2(H))  # :784-788
            if flag:  # :790-800 — the slice index never advances (_layer_count stays 0)
                guided.append(H[:, :, 0:self.vocab_size])
        P = self._read_out(H).transpose(1, 2)  # :802-804
        return self._out(P)[:, :, 0], guided  # :805-808


def clip_loss(t, i, K, B):
    """GuidedClipLoss.forward, guide=False (model.py:877-907).  The block fold
    ``S_indep @ kron(ones(K-1,1), eye(B))`` is a sum over the K-1 negative blocks."""
    def fold(x):
        return x.reshape(K - 1, B).sum(dim=0)

    tm, im, ti = t[:B], i[:B], t[2 * B:]
    Sm = torch.exp((tm * im).sum(1))
    Si = fold(torch.exp((ti * torch.cat([im] * (K - 1), 0)).sum(1)))
    l1 = -torch.log(Sm / (Sm + Si))
    tm, im, ii = t[B:2 * B], i[B:2 * B], i[2 * B:]
    Sm = torch.exp((tm * im).sum(1))
    Si = fold(torch.exp((ii * torch.cat([tm] * (K - 1), 0)).sum(1)))
    l2 = -torch.log(Sm / (Sm + Si))
    return (l1 + l2).mean()


def guide_penalty(t_guided, i_guided, t_targets, i_targets, penalty):
    """GuidedClipLoss guide branch (model.py:909-924): per-sample sum over guided
    layers of penalty * ||H_l[:, :, :V] - target_l||_F^2 for both towers; returns
    (the mean over samples, which is added to the loss, and mean / penalty)."""
    loss3 = 0
    for g, t in zip(t_guided, t_targets):
        loss3 = loss3 + penalty * torch.pow(torch.linalg.norm(g - t, dim=(1, 2), ord="fro"), 2)
    for g, t in zip(i_guided, i_targets):
        loss3 = loss3 + penalty * torch.pow(torch.linalg.norm(g - t, dim=(1, 2), ord="fro"), 2)
    m = loss3.mean()
    return m, m.item() / penalty


# ----------------------------------------------------------------------------
# optimizer — models/optimizer.py:34-85
# ----------------------------------------------------------------------------
class OracleAdamW:
    """AdamW with bias correction folded into lr and decay applied AFTER the
    Adam update to the already-updated weights (optimizer.py:46-75)."""

    def __init__(self, params, weight_decay=0.001, betas=(0.9, 0.999), eps=1e-8):
        self.params = list(params)
        self.wd, (self.b1, self.b2), self.eps = weight_decay, betas, eps
        self.state = {id(p): {"t": 0, "m": torch.zeros_like(p), "v": torch.zeros_like(p)}
                      for p in self.params}
        self.lr = None

    def set_lr(self, lr):
        self.lr = lr

    @torch.no_grad()
    def step(self):
        for p in self.params:
            if p.grad is None:
                continue
            st = self.state[id(p)]
            t = st["t"] + 1
            g = p.grad
            m = self.b1 * st["m"] + (1 - self.b1) * g
            v = self.b2 * st["v"] + (1 - self.b2) * g ** 2
            lr_t = self.lr * (1 - self.b2 ** t) ** 0.5 / (1 - self.b1 ** t)
            p.data -= lr_t * m / (v ** 0.5 + self.eps)
            p.data -= self.lr * self.wd * p.data
            st["t"], st["m"], st["v"] = t, m, v


def lr_cosine(t, lr_max, lr_min, warmup_iters, total_iters):
    """optimizer.py:78-85"""
    if t < warmup_iters:
        return lr_max * t / warmup_iters
    elif t < total_iters:
        return lr_min + 0.5 * (lr_max - lr_min) * (
            1 + np.cos((t - warmup_iters) / (total_iters - warmup_iters) * 3.141592653589793))
    return lr_min


# ----------------------------------------------------------------------------
# training loop — training/train_CLIP.py:62-201 (raw=True, guide=False)
# ----------------------------------------------------------------------------
def build_encoders(T=81, L=5, d=128, V=10, guide=False, activation="softmax"):
    return (OracleEncoder(T, V, d, L, guide=guide, activation=activation),
            OracleEncoder(T, V, d, L, guide=guide, activation=activation))


class OracleTrainer:
    def __init__(self, p=0.2, B=128, L=5, d=128, K=4, lr_max=3e-4, lr_min=3e-7, warmup=0,
                 total_iters=3000, max_norm=1.0, seed=224, seedtree=42, n_layer_tree=4,
                 n_child=3, guide=False, penalty=1e-3, activation="softmax"):
        self.sampler = ClipSamplerOracle([n_layer_tree] * 2, [n_child] * 2, [p, p], K=K,
                                         seedtree=seedtree)
        seed_everything(seed)  # :83
        T = n_child ** n_layer_tree
        self.tm, self.im = build_encoders(T, L, d, guide=guide, activation=activation)
        self.guide, self.penalty = guide, penalty
        self.last_penalty = 0.0
        self.params = list(self.tm.parameters()) + list(self.im.parameters())
        self.opt = OracleAdamW(self.params)
        self.B, self.K = B, K
        self.sched = (lr_max, lr_min, warmup, total_iters)
        self.max_norm = max_norm
        self.it = 0

    def step(self, batch=None):
        for p in self.params:
            p.grad = None
        if batch is None:
            batch = self.sampler.get_batch(self.B)
        t_l, _, i_l, _ = batch
        t, tg = self.tm(torch.as_tensor(t_l, dtype=torch.long))
        i, ig = self.im(torch.as_tensor(i_l, dtype=torch.long))
        loss = clip_loss(t, i, self.K, self.B)
        self.last_loss_nop = float(loss.item())
        if self.guide:  # train_CLIP.py:145-158 with clip_guide=True
            T = t_l.shape[1]
            tt = expand_messages(bp_cls_messages(self.sampler.t_trans, t_l), T)
            it = expand_messages(bp_cls_messages(self.sampler.i_trans, i_l), T)
            pen, self.last_penalty = guide_penalty(tg, ig, tt, it, self.penalty)
            loss = loss + pen
        loss.backward()
        norm = torch.nn.utils.clip_grad_norm_(self.params, self.max_norm, norm_type=2)
        lr = lr_cosine(self.it, *self.sched)
        self.opt.set_lr(lr)
        self.opt.step()
        self.it += 1
        return float(loss.item()), float(norm.item())
