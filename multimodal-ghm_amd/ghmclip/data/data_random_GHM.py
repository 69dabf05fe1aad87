"""GHM sampler API of the reference (src/ghmclip/data/data_random_GHM.py).

Per-step draws run in the native host sampler (libghm_host.so, C++), which
reproduces numpy's legacy MT19937 stream bit-exactly.  ``ClipSampler.get_batch``
takes numpy's global RandomState, advances it exactly as the reference's
per-node Python loop would, and writes it back — so interleaving with other
numpy RNG users (seed_everything, get_Bayes) gives the reference's draws.

Transition matrices are generated once at start-up with numpy, in the
reference's RNG order (GenTransition, :43-89).  get_Bayes runs a vectorised
BP_CLS (:185-221) on the host once per run.
"""
import ctypes

import numpy as np
import torch

from .. import _native

__all__ = ["GenTransition", "PPCLIPLoss", "DoubleSampler", "ClipSampler", "bp_cls_posterior", "guided_targets",
           "vlm_guide_planes",
           "NativeClipSampler", "ConditionalDenoiseSampler", "bp_dns_posterior", "bp_cls_root_message",
           "NextWordPredictSampler", "bp_nwp_posterior"]


def _softmax_row(x):
    """data_random_GHM.py:91-96"""
    e_x = np.exp(x - np.max(x, axis=1, keepdims=True))
    return e_x / e_x.sum(axis=1, keepdims=True)


def GenTransition(n_layer, n_child, variable_type, p_flip=0.3, flip_scale=1.0,
                  translation_invariance=True, verbose=False):
    """data_random_GHM.py:43-89: list over layers of n_child**(layer+1) matrices."""
    transition = [[] for _ in range(n_layer)]
    skeleton = []
    if translation_invariance:
        for layer in range(n_layer):
            skel = np.identity(variable_type)[np.random.permutation(variable_type), :]
            templ = [(1 - p_flip) * skel + p_flip * _softmax_row(
                np.random.normal(0, flip_scale, [variable_type, variable_type])) for _ in range(n_child)]
            for _ in range(n_child ** layer):
                transition[layer].extend(templ)
            skeleton.append(skel)
    else:
        for layer in range(n_layer):
            for _ in range(n_child ** layer):
                transition[layer].extend([(1 - p_flip) * np.identity(variable_type)[np.random.permutation(variable_type), :]
                                          + p_flip * _softmax_row(np.random.normal(0, flip_scale, [variable_type, variable_type]))
                                          for _ in range(n_child)])
    return (transition, skeleton) if verbose else transition


def _templates(transition, n_child):
    """Distinct per-(layer, child slot) matrices [n_layer, n_child, V, V] of a
    translation-invariant tree (what the device BP kernels take), or None when
    the tree is not translation invariant (GenTransition(translation_invariance=
    False): a matrix per edge)."""
    out = np.stack([np.stack(layer[:n_child]) for layer in transition])
    for l, layer in enumerate(transition):
        for k, mat in enumerate(layer):
            if not np.array_equal(mat, out[l, k % n_child]):
                return None
    return np.ascontiguousarray(out)


class DeviceTree:
    """A GHM tree's transition matrices as the device BP kernels take them
    (ghm_bp_cls / ghm_bp_dns, include/ghm_hip.h): the per-(layer, child slot)
    templates [L][C][V][V] of a translation-invariant tree (per_edge 0), or every
    edge's own matrix layer by layer, [sum_l C^(l+1)][V][V] with layer l's edges in
    child order (per_edge 1: GenTransition(translation_invariance=False),
    data_random_GHM.py:43-89)."""

    def __init__(self, trans, L, C, V, per_edge):
        self.trans = np.ascontiguousarray(trans, dtype=np.float64)
        self.L, self.C, self.V, self.per_edge = int(L), int(C), int(V), int(per_edge)

    @classmethod
    def of(cls, x):
        """A DeviceTree from itself, a template array [L][C][V][V], or a list of
        per-layer edge tables ([C^(l+1)][V][V] each)."""
        if isinstance(x, DeviceTree):
            return x
        if isinstance(x, np.ndarray) and x.ndim == 4:
            return cls(x, x.shape[0], x.shape[1], x.shape[2], 0)
        layers = [np.asarray(t, dtype=np.float64) for t in x]
        return cls(np.concatenate(layers, axis=0), len(layers), layers[0].shape[0], layers[0].shape[-1], 1)


def _edge_tables(transition):
    """Per-layer edge matrices [n_child^(l+1), V, V] (layer l, edge parent*C +
    child: the reference's transition[l] list as an array)."""
    return [np.ascontiguousarray(np.stack(layer), dtype=np.float64) for layer in transition]


def _tables(tr):
    """BP input as per-layer edge tables: a template array [L, C, V, V] is
    expanded (node n of layer l uses template n % C), a list of per-layer edge
    tables passes through, a DeviceTree is split back into either."""
    if isinstance(tr, DeviceTree):
        if not tr.per_edge:
            return _tables(tr.trans)
        cuts = np.cumsum([tr.C ** (l + 1) for l in range(tr.L)])[:-1]
        return np.split(tr.trans, cuts)
    if isinstance(tr, np.ndarray) and tr.ndim == 4:
        L, C = tr.shape[0], tr.shape[1]
        return [np.tile(tr[l], (C ** l, 1, 1)) for l in range(L)]
    return [np.asarray(t, dtype=np.float64) for t in tr]


class NativeClipSampler:
    """Thin owner of a libghm_host sampler handle.  Built from per-edge
    transition tables of each tree (any shapes, translation invariant or not),
    or from two equal-shape template arrays [L, C, V, V]."""

    def __init__(self, t_tr, i_tr, V, K):
        t_tab, i_tab = _tables(t_tr), _tables(i_tr)
        self.t_shape = (len(t_tab), t_tab[0].shape[0])
        self.i_shape = (len(i_tab), i_tab[0].shape[0])
        if self.t_shape == self.i_shape:
            self.n_layer, self.n_child = self.t_shape
        self.V, self.K = V, K
        self.T_t = self.t_shape[1] ** self.t_shape[0]
        self.T_i = self.i_shape[1] ** self.i_shape[0]
        self.T = self.T_t if self.T_t == self.T_i else None  # one T only for equal trees
        self._t = np.ascontiguousarray(np.concatenate(t_tab))  # [n_edges][V][V], kept alive
        self._i = np.ascontiguousarray(np.concatenate(i_tab))
        lib = _native.host_lib()
        self._lib = lib
        self._h = lib.ghm_sampler_create_edges(self._t.ctypes.data, self.t_shape[0], self.t_shape[1],
                                               self._i.ctypes.data, self.i_shape[0], self.i_shape[1], V, K)
        if not self._h:
            raise RuntimeError("ghm_sampler_create_edges failed")

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.ghm_sampler_destroy(self._h)
            self._h = None

    def seed(self, seed):
        self._lib.ghm_sampler_seed(self._h, int(seed) & 0xFFFFFFFF)

    def set_state(self, key, pos):
        key = np.ascontiguousarray(key, dtype=np.uint32)
        assert key.shape == (624,)
        _native_check(self._lib.ghm_sampler_set_state(self._h, key.ctypes.data, int(pos)))

    def get_state(self):
        key = np.zeros(624, dtype=np.uint32)
        pos = ctypes.c_int(0)
        _native_check(self._lib.ghm_sampler_get_state(self._h, key.ctypes.data, ctypes.byref(pos)))
        return key, pos.value

    def next_into(self, B, t_leaves, i_leaves, t_root=None, i_root=None):
        """Fill caller-owned uint8 numpy/pinned buffers [B(K+1), T]."""
        rc = self._lib.ghm_sampler_next(self._h, B, _addr(t_leaves), _addr(i_leaves),
                                        _addr(t_root) if t_root is not None else None,
                                        _addr(i_root) if i_root is not None else None)
        _native_check(rc)

    def next_shard_into(self, B, lo, n, t_leaves, i_leaves, t_root=None, i_root=None):
        """The same draw, keeping only rows [k*B + lo, k*B + lo + n) of every block
        k (the data-parallel shard): buffers [(K+1)*n, T]."""
        rc = self._lib.ghm_sampler_next_shard(self._h, B, lo, n, _addr(t_leaves), _addr(i_leaves),
                                              _addr(t_root) if t_root is not None else None,
                                              _addr(i_root) if i_root is not None else None)
        _native_check(rc)

    # numpy global-state bridge -------------------------------------------------
    def next_cdm_into(self, B, sigma, t_leaves, i_leaves, z, root=None):
        """ConditionalDenoiseSampler draw into caller-owned buffers: uint8 [B, T]
        leaves, float64 [B, T] noisy observations z, optional uint8 [B] roots."""
        rc = self._lib.ghm_sampler_next_cdm(self._h, B, float(sigma), _addr(t_leaves), _addr(i_leaves),
                                            _addr(root) if root is not None else None,
                                            _addr(z) if z is not None else None)
        _native_check(rc)

    def set_gauss(self, has_gauss, gauss):
        _native_check(self._lib.ghm_sampler_set_gauss(self._h, int(has_gauss), float(gauss)))

    def get_gauss(self):
        h, g = ctypes.c_int(0), ctypes.c_double(0.0)
        _native_check(self._lib.ghm_sampler_get_gauss(self._h, ctypes.byref(h), ctypes.byref(g)))
        return h.value, g.value

    def pull_numpy_state(self):
        st = np.random.get_state()
        if st[0] != "MT19937":
            raise RuntimeError("unexpected numpy RNG")
        self.set_state(st[1], st[2])
        self.set_gauss(st[3], st[4])

    def push_numpy_state(self):
        key, pos = self.get_state()
        has_gauss, cached = self.get_gauss()
        np.random.set_state(("MT19937", key, pos, has_gauss, cached))


def _addr(a):
    if isinstance(a, torch.Tensor):
        return a.data_ptr()
    return a.ctypes.data


def _native_check(rc):
    if rc != 0:
        raise RuntimeError(f"native sampler call failed ({rc})")


def _bp_levels(templ, leaves):
    """BP_CLS messages (data_random_GHM.py:185-208), vectorised over the nodes of a
    layer with each node's own edge matrices (translation-invariant templates
    are expanded, _tables).  Returns the per-level messages [n_nodes, V, B],
    depth L-1 first, root last."""
    tab = _tables(templ)
    n_layer = len(tab)
    C = tab[0].shape[0]
    lv = np.asarray(leaves).astype(np.int64).T
    n_par = lv.shape[0] // C
    msg = np.zeros((n_par, tab[-1].shape[1], lv.shape[1]))
    for c in range(C):  # leaf edge par*C + c: column leaf value of its matrix
        msg += np.log(np.take_along_axis(tab[-1][c::C], lv[c::C][:, None, :], axis=2))
    msg -= msg.max(axis=1, keepdims=True)
    levels = [msg]
    for layer in range(n_layer - 2, -1, -1):
        n_par = msg.shape[0] // C
        new = np.zeros((n_par, msg.shape[1], msg.shape[2]))
        for c in range(C):
            new += np.log(np.einsum("nij,njb->nib", tab[layer][c::C], np.exp(msg[c::C])))
        new -= new.max(axis=1, keepdims=True)
        msg = new
        levels.append(msg)
    return levels


def guided_targets(templ, leaves, device="cpu"):
    """GHMTree.guided_info for classification (data_random_GHM.py:526-539): one
    float32 [B, T, V] tensor per tree level (depth L-1 first, root last), every
    leaf position carrying its ancestor's BP message.  On a HIP device the
    messages come from the ghm_bp_cls kernel (the path ClipTrainer uses);
    otherwise from the host BP above."""
    leaves = np.asarray(leaves)
    B, T = leaves.shape
    dev = torch.device(device)
    if dev.type == "cuda":
        dt = DeviceTree.of(templ)
        L, C, V = dt.L, dt.C, dt.V
        n_total = (C ** L - 1) // (C - 1)
        tok = torch.from_numpy(np.ascontiguousarray(leaves, dtype=np.uint8)).to(dev)
        tr = torch.from_numpy(dt.trans).to(dev)
        msgs = torch.empty(B, n_total, V, dtype=torch.float32, device=dev)
        _native.call("ghm_bp_cls", tr.data_ptr(), tok.data_ptr(), msgs.data_ptr(), B, L, C, V, dt.per_edge,
                     torch.cuda.current_stream().cuda_stream)
        out, off, nodes = [], 0, T // C
        for _ in range(L):
            out.append(msgs[:, off:off + nodes].repeat_interleave(T // nodes, dim=1))
            off += nodes
            nodes //= C
        return out
    out = []
    for m in _bp_levels(templ, leaves):
        ext = T // m.shape[0]
        out.append(torch.from_numpy(np.repeat(m.transpose(2, 0, 1), ext, axis=1).astype(np.float32)).to(dev))
    return out


def bp_cls_posterior(templ, leaves, p_y):
    """BP_CLS (data_random_GHM.py:185-221): p(root | leaves) [B, V].
    templ [n_layer, n_child, V, V]; leaves [B, T]."""
    msg = _bp_levels(templ, leaves)[-1]
    h0 = msg[0] + np.log(p_y).reshape(-1, 1)
    h0 -= h0.max(axis=0)
    return (np.exp(h0) / np.exp(h0).sum(axis=0)).T


def PPCLIPLoss(t_pp, i_pp, n_eval, K=4, variable_type=10):
    """data_random_GHM.py:13-41 (posterior form of the CLIP loss), without the
    dense kron: the K-1 negative blocks are folded by a reshape-sum."""
    def fold(x):
        return x.reshape(K - 1, n_eval).sum(axis=0)

    S_match = np.sum(t_pp[:, :n_eval] * i_pp[:, :n_eval], 0) * variable_type
    S_indep = fold(np.sum(t_pp[:, 2 * n_eval:] * np.tile(i_pp[:, :n_eval], (1, K - 1)), 0)) * variable_type
    S = -np.log(S_match / (S_indep + S_match))
    S_match = np.sum(t_pp[:, n_eval:2 * n_eval] * i_pp[:, n_eval:2 * n_eval], 0) * variable_type
    S_indep = fold(np.sum(i_pp[:, 2 * n_eval:] * np.tile(t_pp[:, n_eval:2 * n_eval], (1, K - 1)), 0)) * variable_type
    S = S - np.log(S_match / (S_indep + S_match))
    return np.mean(S), np.std(S) / np.sqrt(n_eval)


class DoubleSampler:
    """data_random_GHM.py:641-658: seeds numpy with seedtree and builds both
    modalities' transitions."""

    def __init__(self, n_layers, n_childs, p_ys, p_flips, flip_scale=1, variable_type=10,
                 translation_invariance=True, seedtree=42):
        self.n_layers = n_layers
        self.n_childs = n_childs
        self.p_ys = p_ys
        self.p_flips = p_flips
        self.flip_scale = flip_scale
        self.variable_type = variable_type
        self.seedtree = seedtree
        np.random.seed(seedtree)
        self.t_transition = GenTransition(n_layers[0], n_childs[0], variable_type, p_flips[0], flip_scale,
                                          translation_invariance=translation_invariance)
        self.i_transition = GenTransition(n_layers[1], n_childs[1], variable_type, p_flips[1], flip_scale,
                                          translation_invariance=translation_invariance)
        self.translation_invariance = translation_invariance
        # per-layer edge tables (host BP, the native sampler) and, for translation-
        # invariant trees, the per-child-slot templates the device BP kernels take
        self.t_tables, self.i_tables = _edge_tables(self.t_transition), _edge_tables(self.i_transition)
        self.t_templ = _templates(self.t_transition, n_childs[0])
        self.i_templ = _templates(self.i_transition, n_childs[1])
        self._zs = None

    def _p_y(self, tree):
        """The root prior of the text (0) or image (1) tree, as the reference builds
        each GHMTree with p_ys[0] / p_ys[1] (data_random_GHM.py:665-666, 762-764,
        860-861, 908-909) and BP_CLS combines it with the root message (:213)."""
        return np.asarray(self.p_ys[tree], np.float64)

    def _native_sampler(self, K):
        return NativeClipSampler(self.t_tables, self.i_tables, self.variable_type, K)

    def device_templates(self, what="this path"):
        """(text, image) transitions for the device BP kernels: the per-child-slot
        templates of a translation-invariant tree, else a DeviceTree of its
        per-edge tables (`what` names the caller; kept for the signature)."""
        t = self.t_templ if self.t_templ is not None else DeviceTree.of(self.t_tables)
        i = self.i_templ if self.i_templ is not None else DeviceTree.of(self.i_tables)
        return t, i

    def get_zeroshot_batch(self, batch_size=128, return_tree=False):
        """:670-683: text and image trees sharing one root per sample (the draw of
        figures/eval-zsc-risk.py:66).  Returns text leaves, image leaves (int64
        [B, T]), their BP_CLS root posteriors (float64 [B, V]) and the roots (int64
        [B]); the trees come from the native sampler on numpy's global stream
        (root choice, then the text tree, then the image tree, as GHMTree draws
        them)."""
        if return_tree:
            raise NotImplementedError("return_tree: the trees are drawn natively, no GHMTree objects exist")
        if getattr(self, "_zs", None) is None:
            self._zs = self._native_sampler(2)
        nat = self._zs
        t_templ, i_templ = self.t_tables, self.i_tables
        B = batch_size
        tl = np.empty((B, nat.T_t), np.uint8)
        il = np.empty((B, nat.T_i), np.uint8)
        root = np.empty(B, np.uint8)
        nat.pull_numpy_state()
        nat.next_cdm_into(B, 0.0, tl, il, None, root)
        nat.push_numpy_state()
        t_pp = bp_cls_posterior(t_templ, tl, np.asarray(self.p_ys[0], np.float64))
        i_pp = bp_cls_posterior(i_templ, il, np.asarray(self.p_ys[1], np.float64))
        return tl.astype(np.int64), il.astype(np.int64), t_pp, i_pp, root.astype(np.int64)


class ClipSampler(DoubleSampler):
    """data_random_GHM.py:746-817 with the per-step draw in native code."""

    def __init__(self, n_layers, n_childs, p_ys, p_flips, K=4, flip_scale=1, variable_type=10,
                 translation_invariance=True, seedtree=42):
        super().__init__(n_layers, n_childs, p_ys, p_flips, flip_scale, variable_type,
                         translation_invariance, seedtree)
        self.K = K
        self.native = self._native_sampler(K)
        self.T, self.T_t, self.T_i = self.native.T, self.native.T_t, self.native.T_i

    def draw_numpy(self, batch_size):
        """One reference-identical draw from numpy's global state (uint8 arrays;
        text rows T_t wide, image rows T_i wide)."""
        rows = batch_size * (self.K + 1)
        tl = np.empty((rows, self.T_t), np.uint8)
        il = np.empty((rows, self.T_i), np.uint8)
        tr = np.empty(rows, np.uint8)
        ir = np.empty(rows, np.uint8)
        self.native.pull_numpy_state()
        self.native.next_into(batch_size, tl, il, tr, ir)
        self.native.push_numpy_state()
        return tl, tr, il, ir

    def get_batch(self, device="cpu", batch_size=128, guide=False):
        """:753-784.  Returns [text_leaves, text_root, guided_info, t_pp],
        [image ...] with leaves as int64 [B(K+1), T] on ``device``; with guide=True
        guided_info is the list of per-level BP guide targets (float32 [B(K+1),
        T, V] on ``device``) and t_pp the BP_CLS posteriors [B(K+1), V] (numpy),
        else both are None."""
        tl, tr, il, ir = self.draw_numpy(batch_size)
        to = lambda a: torch.from_numpy(a.astype(np.int64)).to(device)  # noqa: E731
        tg = ig = tp = ip = None
        if guide:
            tg = guided_targets(self.t_templ if self.t_templ is not None else self.t_tables, tl, device)
            ig = guided_targets(self.i_templ if self.i_templ is not None else self.i_tables, il, device)
            tp = bp_cls_posterior(self.t_tables, tl, self._p_y(0))
            ip = bp_cls_posterior(self.i_tables, il, self._p_y(1))
        return [to(tl), to(tr), tg, tp], [to(il), to(ir), ig, ip]

    def get_Bayes(self, n_eval=10000):
        """:786-817 — exact Bayes CLIP loss from BP posteriors (host, once per run)."""
        tl, _, il, _ = self.draw_numpy(n_eval)
        tp = bp_cls_posterior(self.t_tables, tl, self._p_y(0)).T
        ip = bp_cls_posterior(self.i_tables, il, self._p_y(1)).T
        return PPCLIPLoss(tp, ip, n_eval, self.K, self.variable_type)


def bp_cls_root_message(templ, leaves):
    """The max-shifted BP_CLS root message [V, B] (data_random_GHM.py:201-208) — the
    text tree's evidence the conditional denoiser's image BP receives (:875-877)."""
    return _bp_levels(templ, leaves)[-1][0]


def bp_dns_posterior(templ, z, sigma, ext):
    """BP_DNS (data_random_GHM.py:467-523) on the host, vectorised over the nodes of a
    layer (translation invariance: node n uses its child-slot matrix n % C).
    z: noisy leaf observations [n_leaves, B] float64; ext: external root message
    [V, B].  Returns the posterior means [n_leaves, B]."""
    return bp_dns_levels(templ, z, sigma, ext)[-1]


def bp_dns_levels(templ, z, sigma, ext):
    """bp_dns_posterior's messages as well: (hd, qd, bu, root_bu, post) with hd / qd /
    bu dicts depth 1..L -> [n_nodes, V, B] (the per-node hd_message, qd_message and
    bu_message of data_random_GHM.py:481-512), the root's bu [V, B] (its hd aliases
    it, :501-504) and the posterior means [n_leaves, B]."""
    tab = _tables(templ)
    n_layer, C, V = len(tab), tab[0].shape[0], tab[0].shape[1]
    vt = np.linspace(0, V - 1, V).reshape(1, V, 1)

    def up(msg, mats, transpose=False):  # node n of the layer: its edge matrix mats[n]
        eq = "nji,njb->nib" if transpose else "nij,njb->nib"
        return np.log(np.einsum(eq, mats, np.exp(msg)))

    def children_sum(q):  # sum(child.qd for child in children), children in slot order
        acc = q[0::C].copy()
        for c in range(1, C):
            acc += q[c::C]
        return acc

    hd = {n_layer: -0.5 * (np.asarray(z, dtype=np.float64)[:, None, :] - vt) ** 2 / (sigma ** 2)}
    qd = {n_layer: up(hd[n_layer], tab[-1])}
    for layer in range(n_layer - 1, 0, -1):  # leaves -> root (:489-495)
        h = children_sum(qd[layer + 1])
        h -= h.max(axis=1, keepdims=True)
        hd[layer], qd[layer] = h, up(h, tab[layer - 1])
    bu = children_sum(qd[1])  # root (:499-504)
    bu -= bu.max(axis=1, keepdims=True)
    bu = bu + np.asarray(ext)[None]
    root_bu, bus = bu[0], {}
    for layer in range(1, n_layer + 1):  # root -> leaves (:507-512)
        b = hd[layer] + up(np.repeat(bu, C, axis=0) - qd[layer], tab[layer - 1], transpose=True)
        bu = b - b.max(axis=1, keepdims=True)
        bus[layer] = bu
    w = np.exp(bu)
    return hd, qd, bus, root_bu, ((vt * w).sum(axis=1) / w.sum(axis=1))


class ConditionalDenoiseSampler(DoubleSampler):
    """data_random_GHM.py:846-894 with the per-step draw (trees + Gaussian noise) in
    native code.  The BP posteriors of get_batch run vectorised on the host; the
    CDM trainer computes them on the device instead (ghm_bp_dns)."""

    def __init__(self, n_layers, n_childs, p_ys, p_flips, sigma=1, flip_scale=1, variable_type=10,
                 translation_invariance=True, seedtree=42):
        super().__init__(n_layers, n_childs, p_ys, p_flips, flip_scale, variable_type,
                         translation_invariance, seedtree)
        self.sigma = sigma
        self.native = self._native_sampler(2)
        self.T = self.native.T  # None for trees of different leaf counts
        self.T_t, self.T_i = self.native.T_t, self.native.T_i

    def draw_numpy(self, batch_size):
        """One reference-identical draw from numpy's global state: (text leaves uint8
        [B, T_t], roots uint8 [B], z float64 [B, T_i], image leaves uint8 [B, T_i])
        (the noise lives on the image leaves, :862)."""
        B = batch_size
        tl = np.empty((B, self.T_t), np.uint8)
        il = np.empty((B, self.T_i), np.uint8)
        root = np.empty(B, np.uint8)
        z = np.empty((B, self.T_i), np.float64)
        self.native.pull_numpy_state()
        self.native.next_cdm_into(B, self.sigma, tl, il, z, root)
        self.native.push_numpy_state()
        return tl, root, z, il

    def posterior(self, tl, z):
        """(text BP_CLS posteriors [V, B], image BP_DNS posterior means [B, T])."""
        t_pp = bp_cls_posterior(self.t_tables, tl, self._p_y(0)).T
        ext = bp_cls_root_message(self.t_tables, tl)
        return t_pp, bp_dns_posterior(self.i_tables, np.asarray(z).T, self.sigma, ext).T

    def get_batch(self, batch_size=128, device="cpu", guide=False):
        """:854-884.  Returns (text_leaves int64 [B, T_t], text_root int64 [B],
        text guided_info, t_pp [V, B]), (z float32 [B, T_i], image_leaves int64
        [B, T_i], image guided_info, posterior means float64 [B, T_i]).  guide=True:
        the host BP's guided_info lists (:526-592) -- the text tree's BP_CLS
        message of every leaf's ancestor, depth L_t-1 first ([B, T_t, V] each), and
        the image tree's BP_DNS messages: (hd, qd) of depths L_i .. 1, the root's
        (hd, bu), then (hd, qd, bu) of depths 1 .. L_i ([B, T_i, 2V] / [B, T_i, 3V],
        float32); guide=False: None (the fused CdmTrainer step computes its targets
        on the device, ghm_bp_dns_msgs / ghm_bp_cls)."""
        tl, root, z, il = self.draw_numpy(batch_size)
        t_levels = _bp_levels(self.t_tables, tl)
        t_pp = bp_cls_posterior(self.t_tables, tl, self._p_y(0)).T
        hd, qd, bu, root_bu, post = bp_dns_levels(self.i_tables, np.asarray(z).T, self.sigma, t_levels[-1][0])
        post = post.T
        t_info = i_info = None
        if guide:
            T_t, T_i = tl.shape[1], il.shape[1]
            t_info = [torch.from_numpy(np.repeat(m.transpose(2, 0, 1), T_t // m.shape[0], axis=1)
                                       .astype(np.float32)).to(device) for m in t_levels]

            def rep(*ms):  # [n_nodes, V, B] each -> [B, T_i, k V]
                cat = np.concatenate(ms, axis=1)
                return torch.from_numpy(np.repeat(cat.transpose(2, 0, 1), T_i // cat.shape[0], axis=1)
                                        .astype(np.float32)).to(device)

            L = len(hd)
            i_info = [rep(hd[d], qd[d]) for d in range(L, 0, -1)]
            i_info.append(rep(root_bu[None], root_bu[None]))
            i_info += [rep(hd[d], qd[d], bu[d]) for d in range(1, L + 1)]
        to = lambda a: torch.from_numpy(a.astype(np.int64)).to(device)  # noqa: E731
        return ((to(tl), to(root), t_info, t_pp),
                (torch.from_numpy(z.astype(np.float32)).to(device), to(il), i_info, post))

    def get_Bayes(self, n_eval=30000):
        """:886-894 — mean and standard error of the Bayes (posterior-mean) squared error."""
        tl, _, z, il = self.draw_numpy(n_eval)
        _, post = self.posterior(tl, z)
        loss = np.sum(np.power(post - il.astype(np.int64), 2), 1)
        return np.mean(loss), np.std(loss) / np.sqrt(n_eval)


def bp_nwp_posterior(templ, leaves, ext, guide=False):
    """BP_NWP_autoregressive (data_random_GHM.py:336-466) on the host, vectorised
    over the batch: p(leaf p+1 | leaves <= p, image evidence ext) for every
    position p, [B, n_leaves - 1, V] float32 (the reference's predict_pp tensor
    dtype).  templ [L][C][V][V]; leaves [B, n_leaves]; ext [V, B].
    A node's qd message is rewritten whenever it is an ancestor of the current
    leaf, so completed earlier siblings keep their last (complete) message, as in
    the reference's mutable tree.
    guide=True (guide_info=True) also returns the 2L + 1 guide targets of every
    position, float32: [0] the leaf's qd [B, n-1, V] (:372-373); [1..L-1] the
    (hd, qd) of its ancestors at depth L-1 .. 1 [B, n-1, 2V] (:392-394); [L] the
    root's (hd, bu) — one array in the reference (bu_message = hd_message, then
    += in place, :414-421), so both halves hold the final bu; [L+1 .. 2L] the bu
    of the target leaf's path from depth 1 down to the leaf [B, n-1, V] (:449-451)."""
    tab = _tables(templ)
    n_layer, C, V = len(tab), tab[0].shape[0], tab[0].shape[1]
    lv = np.asarray(leaves).astype(np.int64).T
    n_leaves, B = lv.shape
    qd = [None] + [np.zeros((C ** d, V, B)) for d in range(1, n_layer + 1)]
    hd = [None] + [np.zeros((C ** d, V, B)) for d in range(1, n_layer)]
    out = np.zeros((B, n_leaves - 1, V), dtype=np.float32)
    if guide:
        gl = ([np.zeros((B, n_leaves - 1, V), np.float32)] +
              [np.zeros((B, n_leaves - 1, 2 * V), np.float32) for _ in range(n_layer)] +
              [np.zeros((B, n_leaves - 1, V), np.float32) for _ in range(n_layer)])
    for p in range(n_leaves - 1):
        q = np.log(tab[-1][p][:, lv[p]])  # leaf message :370-371 (leaf p's edge)
        qd[n_layer][p] = q - q.max(0)
        if guide:
            gl[0][:, p, :] = qd[n_layer][p].T
        idn, goal, share = p, [p + 1], [False]
        for layer in range(n_layer - 1, 0, -1):  # prefix evidence up to the root :381-406
            par = idn // C
            h = qd[layer + 1][par * C].copy()
            for c in range(1, C):
                if c + par * C <= idn:
                    h += qd[layer + 1][par * C + c]
            h -= h.max(0)
            hd[layer][par] = h
            qq = np.log(tab[layer - 1][par] @ np.exp(h))
            qd[layer][par] = qq - qq.max(0)
            if guide:
                gl[n_layer - layer][:, p, :V] = h.T
                gl[n_layer - layer][:, p, V:] = qd[layer][par].T
            goal.append(goal[-1] // C)
            idn = par
            share.append(idn == goal[-1])
        bu = qd[1][0].copy()  # root :410-426
        for c in range(1, C):
            if c <= idn:
                bu += qd[1][c]
        bu -= bu.max(0)
        bu = bu + ext
        bu -= bu.max(0)
        if guide:
            gl[n_layer][:, p, :V] = bu.T
            gl[n_layer][:, p, V:] = bu.T
        for layer in range(1, n_layer + 1):  # down the target's path :435-452
            k = goal[-layer]
            mat = tab[layer - 1][k].T
            if share[-layer]:
                b = hd[layer][k] + np.log(mat @ np.exp(bu - qd[layer][k]))
            else:
                b = np.log(mat @ np.exp(bu))
            bu = b - b.max(0)
            if guide:
                gl[n_layer + layer][:, p, :] = bu.T
        w = np.exp(bu)
        out[:, p, :] = (w / w.sum(0)).T
    return (out, gl) if guide else out


def vlm_guide_planes(text_targets, image_targets, V, out=None):
    """Pack the guided-VLM targets into the per-sample block planes the fused
    trainer's penalty kernels read (VLM_GUIDE_BLOCKS order): the 13 text blocks
    [n_text][V] (leaf q; (hd, qd) of depths L-1 .. 1 and of the root, split in
    two; the path bu), then the L image blocks [n_image][V].  Returns float32
    [B, 13 * n_text * V + L * n_image * V]."""
    planes = []
    for t in text_targets:
        if t.shape[2] == V:
            planes.append(t)
        else:
            planes += [t[:, :, :V], t[:, :, V:]]
    planes += [np.asarray(x) for x in image_targets]
    B = planes[0].shape[0]
    flat = [np.ascontiguousarray(p, dtype=np.float32).reshape(B, -1) for p in planes]
    if out is None:
        return np.concatenate(flat, axis=1)
    off = 0
    for p in flat:
        out[:, off:off + p.shape[1]] = p
        off += p.shape[1]
    return out


class NextWordPredictSampler(DoubleSampler):
    """data_random_GHM.py:896-942 with the trees drawn in native code and the BP
    posteriors (BP_CLS of the image tree, BP_NWP_autoregressive of the text tree)
    vectorised on the host."""

    def __init__(self, n_layers, n_childs, p_ys, p_flips, flip_scale=1, variable_type=10,
                 translation_invariance=True, seedtree=42):
        super().__init__(n_layers, n_childs, p_ys, p_flips, flip_scale, variable_type,
                         translation_invariance, seedtree)
        self.native = self._native_sampler(2)
        self.T, self.T_t, self.T_i = self.native.T, self.native.T_t, self.native.T_i

    def draw_numpy(self, batch_size):
        """One reference-identical draw of the paired trees from numpy's global
        state: (text leaves uint8 [B, T_t], image leaves uint8 [B, T_i], roots [B])."""
        B = batch_size
        tl = np.empty((B, self.T_t), np.uint8)
        il = np.empty((B, self.T_i), np.uint8)
        root = np.empty(B, np.uint8)
        self.native.pull_numpy_state()
        self.native.next_cdm_into(B, 0.0, tl, il, None, root)
        self.native.push_numpy_state()
        return tl, il, root

    def posterior(self, tl, il, guide=False):
        """(next-word posteriors [B, T-1, V] float32, image BP_CLS posteriors [B, V]);
        guide=True: (posteriors, image posteriors, text guide targets (the 2L + 1
        arrays of bp_nwp_posterior), image guide targets (GHMTree.guided_info of the
        image tree: L float32 [B, T, V]))."""
        ext = bp_cls_root_message(self.i_tables, il)
        i_pp = bp_cls_posterior(self.i_tables, il, self._p_y(1))
        if not guide:
            return bp_nwp_posterior(self.t_tables, tl, ext), i_pp
        post, tg = bp_nwp_posterior(self.t_tables, tl, ext, guide=True)
        ig = [m.numpy() for m in guided_targets(self.i_tables, il)]
        return post, i_pp, tg, ig

    def get_batch(self, batch_size=128, device="cpu", guide=False):
        """:902-929.  Returns (text inputs int64 [B, T-1], targets [B, T-1], text
        guide targets, posteriors float32 [B, T-1, V] (torch, on device)), (image
        leaves int64 [B, T], roots [B], image guide targets, image posteriors
        [B, V]); the guide targets (guide=True, else None) are lists of float32
        torch tensors in the reference's order (BP_NWP_autoregressive guide_info,
        GHMTree.guided_info)."""
        tl, il, root = self.draw_numpy(batch_size)
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.int64)).to(device)  # noqa: E731
        if guide:
            post, i_pp, tg, ig = self.posterior(tl, il, guide=True)
            tg = [torch.from_numpy(x).to(device) for x in tg]
            ig = [torch.from_numpy(x).to(device) for x in ig]
        else:
            (post, i_pp), tg, ig = self.posterior(tl, il), None, None
        return ((to(tl[:, :-1]), to(tl[:, 1:]), tg, torch.from_numpy(post).to(device)),
                (to(il), to(root), ig, i_pp))

    def get_Bayes(self, n_eval=30000):
        """:931-942 — mean and standard error of -log p(next leaf) under the exact
        posterior (float32, as the reference's torch reductions)."""
        tl, il, _ = self.draw_numpy(n_eval)
        post, _ = self.posterior(tl, il)
        pred = torch.from_numpy(post).reshape(-1, self.variable_type)
        tc = torch.from_numpy(tl[:, 1:].astype(np.int64).reshape(-1))
        loss = -torch.log(pred[torch.arange(len(tc)), tc])
        return torch.mean(loss), torch.std(loss) / np.sqrt(n_eval)
