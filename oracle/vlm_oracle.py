"""ORACLE — CPU restatement of the reference's sequential vision-language (VLM,
next-word prediction) training path (BASELINE config 5:
scripts/experiments/exp_vlm_standardTF.sh).

TEST INFRASTRUCTURE ONLY, like ghm_oracle.py: only tests/, __graft_entry__.smoke()
and bench.py's ``cpu_baseline`` leg may import it.  Nothing in multimodal-ghm_amd/
imports it.

Parity pinning: checked against fixtures produced by importing the real reference
(tests/golden/make_golden_vlm.py): sampler draws, BP_NWP_autoregressive posteriors
and the Bayes risk (vlm_sampler.npz), two training steps (vlm_tiny.npz) and the
first steps of the default config (vlm_curve.npz).

Reference file:line it follows (relative to src/ghmclip/):
  sampler    data/data_random_GHM.py:896-929 (NextWordPredictSampler.get_batch),
             :931-942 (get_Bayes)
  BP         data/data_random_GHM.py:185-215 (BP_CLS root message), :336-466
             (BP_NWP_autoregressive, guide_info=False)
  mask       models/model.py:24-33 (generate_mask)
  model      models/model.py:132-335 (AutoRegressiveTransformer, sequential=True,
             auto_regressive=True)
  losses     models/model.py:1080-1149 (ConditionalGuidedCELoss, guide=False),
             :1067-1078 (KLdiv)
  loop       training/train_sequential_NWP.py:65-185
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .ghm_oracle import OracleAdamW, OracleEncoder, bp_cls_messages, gen_leaves, gen_transition, lr_cosine


def bp_nwp_autoregressive(trans, leaves, ext):
    """BP_NWP_autoregressive(guide_info=False) (data_random_GHM.py:336-466),
    vectorised over the batch.  trans [L][C][V][V] translation-invariant
    templates (node k of a level uses slot k % C); leaves [B, n_leaves]; ext: the
    image tree's BP_CLS root message [V, B].  Returns p(leaf p+1 | leaves <= p,
    image) as [B, n_leaves - 1, V].

    State follows the reference's mutable tree: qd[level][k] of a node is
    overwritten whenever the node is an ancestor of the current leaf, so a
    completed earlier sibling keeps its last (complete) message."""
    n_layer, C, V, _ = trans.shape
    B, n_leaves = leaves.shape
    lv = leaves.T  # [n_leaves, B]
    qd = {d: np.zeros((C ** d, V, B)) for d in range(1, n_layer + 1)}
    hd = {d: np.zeros((C ** d, V, B)) for d in range(1, n_layer)}
    out = np.zeros((B, n_leaves - 1, V))

    def lmv(mat, msg):  # log(mat @ exp(msg)) column-wise
        return np.log(mat @ np.exp(msg))

    for p in range(n_leaves - 1):
        q = np.log(trans[-1, p % C][:, lv[p]])  # :370-371
        qd[n_layer][p] = q - q.max(0)
        idn = p
        goal = [p + 1]  # goal-path node index per level, leaf level first
        share = [False]
        for layer in range(n_layer - 1, 0, -1):  # downward process :381-406
            par = idn // C
            h = 0
            for c in range(C):
                if c + par * C <= idn:
                    h = h + qd[layer + 1][par * C + c]
            h = h - h.max(0)
            hd[layer][par] = h
            qq = lmv(trans[layer - 1, par % C], h)
            qd[layer][par] = qq - qq.max(0)
            goal.append(goal[-1] // C)
            idn = par
            share.append(idn == goal[-1])
        h = 0  # root :410-417
        for c in range(C):
            if c <= idn:
                h = h + qd[1][c]
        h = h - h.max(0)
        bu = h + ext  # :420-424 (bu aliases hd in the reference; same values)
        bu = bu - bu.max(0)
        for layer in range(1, n_layer + 1):  # upward process :435-452
            k = goal[-layer]
            mat = trans[layer - 1, k % C].T
            if share[-layer]:
                b = hd[layer][k] + lmv(mat, bu - qd[layer][k])
            else:
                b = lmv(mat, bu)
            bu = b - b.max(0)
        w = np.exp(bu)
        out[:, p, :] = (w / w.sum(0)).T
    return out


class NwpSamplerOracle:
    """NextWordPredictSampler (data_random_GHM.py:896-942), translation-invariant trees."""

    def __init__(self, n_layers, n_childs, p_flips, flip_scale=1, variable_type=10, seedtree=42):
        self.V = variable_type
        np.random.seed(seedtree)  # DoubleSampler.__init__ :654
        self.t_trans = gen_transition(n_layers[0], n_childs[0], variable_type, p_flips[0], flip_scale)
        self.i_trans = gen_transition(n_layers[1], n_childs[1], variable_type, p_flips[1], flip_scale)

    def get_batch(self, batch_size=128):
        """:902-929.  Returns (text inputs [B, T-1], text targets [B, T-1],
        posterior [B, T-1, V], image leaves [B, T_i], image root [B])."""
        B = batch_size
        root = np.random.choice(self.V, size=B)
        t_leaves = gen_leaves(self.t_trans, root)
        i_leaves = gen_leaves(self.i_trans, root)
        ext = bp_cls_messages(self.i_trans, i_leaves)[-1][:, 0, :].T  # image root hd_message [V, B]
        post = bp_nwp_autoregressive(self.t_trans, t_leaves, ext)
        return t_leaves[:, :-1], t_leaves[:, 1:], post, i_leaves, root

    def get_Bayes(self, n_eval=30000):
        """:931-942 — mean and standard error of -log p(target) under the posterior
        (float32 like the reference's predict_pp tensor and its torch reductions)."""
        _, target, post, _, _ = self.get_batch(n_eval)
        pred = torch.from_numpy(post.astype(np.float32)).reshape(-1, self.V)
        tc = torch.from_numpy(target.reshape(-1))
        loss = -torch.log(pred[torch.arange(len(tc)), tc])
        return float(torch.mean(loss)), float(torch.std(loss) / np.sqrt(n_eval))


def vlm_mask(n_token, n_i_token):
    """generate_mask (model.py:24-33): the image prefix attends only within itself,
    text tokens attend to the image prefix and causally to text."""
    n_t = n_token - n_i_token
    mask = torch.zeros(n_token, n_token)
    mask[:n_i_token, n_i_token:] = float("-inf")
    mask[n_i_token:, n_i_token:] = torch.triu(torch.ones(n_t, n_t) * float("-inf"), diagonal=1)
    return mask


class OracleVlm(nn.Module):
    """AutoRegressiveTransformer, sequential=True, auto_regressive=True, guide=False
    (model.py:132-335).  Construction order as the reference: position embedding,
    the (then empty) ModuleLists, t_embedding, i_embedding, per layer q, k, v, ln1,
    mlp, ln2, then _read_out Linear(d -> V) and the unused _out."""

    def __init__(self, n_token, n_i_token=1, num_class=10, n_embd=256, n_layer=9, n_mlp_hidden=1024, sequential=True,
                 activation="softmax", layernorm=True):
        super().__init__()
        self.layernorm = layernorm  # model.py:269-277, 294-301: False = Q / K / V and the MLP on H itself
        self.V, self.n_i_token, self.n_embd, self.n_token = num_class, n_i_token, n_embd, n_token
        self.sequential = sequential
        self.activation = activation  # get_activation (model.py:121-130): softmax / relu
        self.position_embeddings = nn.Embedding(n_token, n_embd)
        self._queries, self._keys, self._values = nn.ModuleList(), nn.ModuleList(), nn.ModuleList()
        self._mlps, self._lns_1, self._lns_2 = nn.ModuleList(), nn.ModuleList(), nn.ModuleList()
        self.t_embedding = nn.Embedding(num_class, n_embd)
        self.i_embedding = nn.Embedding(num_class, n_embd)
        for _ in range(n_layer):
            self._queries.append(nn.Linear(n_embd, n_embd, bias=False))
            self._keys.append(nn.Linear(n_embd, n_embd, bias=False))
            self._values.append(nn.Linear(n_embd, n_embd, bias=False))
            self._lns_1.append(nn.LayerNorm([n_embd]))
            self._mlps.append(nn.Sequential(nn.Linear(n_embd, n_mlp_hidden), nn.GELU(),
                                            nn.Linear(n_mlp_hidden, n_embd)))
            self._lns_2.append(nn.LayerNorm([n_embd]))
        self._read_out = nn.Linear(n_embd, num_class)
        self._out = nn.Linear(n_token, 1)

    def forward(self, xt, zi):
        """xt: text tokens [B, T1] (long); zi: the frozen CLIP image feature
        [B, 1, V] (sequential) or the image leaves [B, n_i_token] (long; joint,
        sequential=False).  Returns next-token logits [B, T1, V] (model.py:301-335)."""
        B, T1 = xt.shape
        T = T1 + zi.shape[1]
        mask = vlm_mask(self.n_token, self.n_i_token)
        emb = torch.zeros(B, T, self.n_embd)
        if self.sequential:
            x2 = torch.cat([zi, torch.zeros(B, zi.shape[1], self.n_embd - self.V)], dim=2)  # :281-286
            emb[:, 0, :] = x2[:, 0, :]
        else:
            emb[:, :self.n_i_token, :] = self.i_embedding(zi)  # :287-289
        emb[:, self.n_i_token:, :] = self.t_embedding(xt)  # :292
        H = emb + self.position_embeddings(torch.arange(T).expand(B, T))  # :305
        for q, k, v, mlp, ln1, ln2 in zip(self._queries, self._keys, self._values, self._mlps, self._lns_1,
                                          self._lns_2):
            H1 = ln1(H) if self.layernorm else H
            S = torch.matmul(q(H1), k(H1).transpose(-2, -1))  # :329
            S = S + mask  # :333
            S = S / np.sqrt(self.n_embd)  # :335-336
            A = F.softmax(S, dim=-1) if self.activation == "softmax" else F.relu(S)  # :287
            Vv = v(H1)
            H = H + torch.einsum("bij,bjd->bid", A, Vv)  # :338
            A = A / H.shape[2]  # :339-340
            H = H + torch.einsum("bij,bjd->bid", A, Vv)  # :341
            H = H + mlp(ln2(H) if self.layernorm else H)  # :344-347
        return self._read_out(H)[:, self.n_i_token:, :]  # :397-401


def ce_loss(logits, targets):
    """ConditionalGuidedCELoss(guide=False) (model.py:1087-1098): per-token CE,
    mean over the sequence, mean over samples."""
    loss = F.cross_entropy(logits.reshape(-1, logits.size(-1)), targets.reshape(-1), reduction="none")
    return loss.reshape(-1, targets.shape[1]).mean(dim=1).mean()


def kl_compare(logits, post):
    """KLdiv (model.py:1067-1078): batchmean KL(post || softmax(logits)) over rows."""
    inputs = F.log_softmax(logits.reshape(-1, logits.size(-1)), dim=1)
    return F.kl_div(inputs, post.reshape(-1, post.size(-1)), reduction="batchmean")


class OracleVlmTrainer:
    """train_sequential_NWP.py:65-185 (raw=True: no get_Bayes draw; guide=False),
    the frozen CLIP image encoder at seeded weights (torch.manual_seed(clip_seed)
    just before its construction; the script loads a trained CLIP checkpoint)."""

    def __init__(self, p=0.2, B=128, L=9, d=256, lr_max=1e-3, lr_min=1e-6, warmup=0, total_iters=30000,
                 max_norm=1.0, seed=224, seedtree=42, clip_seed=7, n_layer_tree=4, n_child=3, activation="softmax",
                 layernorm=True):
        self.sampler = NwpSamplerOracle([n_layer_tree] * 2, [n_child] * 2, [p, p], seedtree=seedtree)
        T = n_child ** n_layer_tree
        torch.manual_seed(clip_seed)
        self.clip = OracleEncoder(T, 10, 128, 5)
        torch.manual_seed(seed)  # seed_everything(seed) before the model (:120)
        np.random.seed(seed)
        self.model = OracleVlm(T, 1, 10, d, L, 4 * d, activation=activation, layernorm=layernorm)
        self.params = list(self.model.parameters())
        self.opt = OracleAdamW(self.params)
        self.B = B
        self.sched = (lr_max, lr_min, warmup, total_iters)
        self.max_norm = max_norm
        self.it = 0

    def step(self, batch=None):
        """Returns (ploss, loss, compare)."""
        for p in self.params:
            p.grad = None
        if batch is None:
            batch = self.sampler.get_batch(self.B)
        xt, yt, post, il = batch[:4]
        with torch.no_grad():
            feat = self.clip(torch.as_tensor(il, dtype=torch.long))[0].unsqueeze(1)
        self.last_feat = feat
        logits = self.model(torch.as_tensor(xt, dtype=torch.long), feat)
        self.last_logits = logits.detach()
        loss = ce_loss(logits, torch.as_tensor(yt, dtype=torch.long))
        loss.backward()
        with torch.no_grad():
            cmp = kl_compare(logits, torch.as_tensor(post, dtype=torch.float32))
        with_grad = [p for p in self.params if p.grad is not None]
        torch.nn.utils.clip_grad_norm_(with_grad, self.max_norm, norm_type=2)
        self.opt.set_lr(lr_cosine(self.it, *self.sched))
        self.opt.step()
        self.it += 1
        return float(loss.item()), float(loss.item()), float(cmp.item())


class OracleVlmJointTrainer:
    """train_NWP.py:60-160 (raw=True, guide=False): the joint model (sequential=False,
    T = 161: 81 image leaves through i_embedding as the prefix, 80 text tokens), no
    CLIP.  RNG order: sampler (seedtree) -> [get_Bayes, unseeded, skipped] ->
    seed_everything(seed) -> model -> loop."""

    def __init__(self, p=0.2, B=128, L=9, d=256, lr_max=1e-3, lr_min=1e-6, warmup=0, total_iters=30000,
                 max_norm=1.0, seed=224, seedtree=42, n_layer_tree=4, n_child=3):
        self.sampler = NwpSamplerOracle([n_layer_tree] * 2, [n_child] * 2, [p, p], seedtree=seedtree)
        T = n_child ** n_layer_tree
        torch.manual_seed(seed)  # seed_everything(seed) (:72)
        np.random.seed(seed)
        self.model = OracleVlm(2 * T - 1, T, 10, d, L, 4 * d, sequential=False)
        self.params = list(self.model.parameters())
        self.opt = OracleAdamW(self.params)
        self.B = B
        self.sched = (lr_max, lr_min, warmup, total_iters)
        self.max_norm = max_norm
        self.it = 0

    def step(self, batch=None):
        """Returns (ploss, loss, compare)."""
        for p in self.params:
            p.grad = None
        if batch is None:
            batch = self.sampler.get_batch(self.B)
        xt, yt, post, il = batch[:4]
        logits = self.model(torch.as_tensor(xt, dtype=torch.long), torch.as_tensor(np.asarray(il), dtype=torch.long))
        self.last_logits = logits.detach()
        loss = ce_loss(logits, torch.as_tensor(yt, dtype=torch.long))
        loss.backward()
        with torch.no_grad():
            cmp = kl_compare(logits, torch.as_tensor(post, dtype=torch.float32))
        with_grad = [p for p in self.params if p.grad is not None]
        torch.nn.utils.clip_grad_norm_(with_grad, self.max_norm, norm_type=2)
        self.opt.set_lr(lr_cosine(self.it, *self.sched))
        self.opt.step()
        self.it += 1
        return float(loss.item()), float(loss.item()), float(cmp.item())
