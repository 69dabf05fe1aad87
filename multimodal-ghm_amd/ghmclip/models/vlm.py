"""Sequential VLM (next-word prediction, BASELINE config 5) on the HIP path.

Reference: models/model.py:132-335 (AutoRegressiveTransformer, sequential=True,
auto_regressive=True), :24-33 (generate_mask), :1080-1149 (ConditionalGuidedCELoss),
:1067-1078 (KLdiv); trained by training/train_sequential_NWP.py with a frozen CLIP
image encoder supplying the one prefix token.

``VlmPlan`` runs one model at one batch shape with no autograd, in one of two
matrix-product modes:
  "x3" (default): Q/K/V and the MLP's two Linear layers, forward, data gradient and
       weight gradient, on the hand-written split-bf16 MFMA GEMM (csrc/ghm_gemm.hip;
       GELU / GELU', bias + residual and the GELU' product fused into its epilogues,
       Q/K/V fused into one [M][3D] product), attention on the split-bf16 MFMA
       kernels of csrc/ghm_vlm_x3.hip;
  "f32": the same GEMM template with exact f32 products (ghm_gemm_f32:
       v_mfma_f32_32x32x2f32 on f32 LDS images, erf GELU in the epilogue; Q, K
       and V as three products into separate buffers) and the fp32 attention
       kernels of csrc/ghm_vlm.hip.
Both use the hand-written embedding, row LayerNorm forward/backward, readout
(ghm_rows_linear), bias / embedding gradient sums (ghm_colsum / ghm_wcolsum) and
cross-entropy + KL kernels; no library GEMM runs in either mode.  All buffers are
allocated once; a step is a fixed launch sequence (graph-capturable).

HBM layout (M = n_seq * T tokens, D = n_embd, F = 4 D, fp32 row-major):
  H [L+1][M][D], Hmid / X1 (LN1 out) / X2 (LN2 out) / q / k / v [L][M][D],
  G, Dg (GELU(U), GELU'(U)) [L][M][F], P [L][n_seq][96][96], st1 / st2 [L][M][2];
  backward scratch dH [2][M][D], dX, dq, dk, dv [M][D], dG [M][F].  (x3 keeps
  q | k | v as one [L][M][3D] buffer and dq | dk | dv as [M][3D].)
"""
import ctypes
import math
import os

import torch
import torch.nn as nn

from .. import _native
from .hip_encoder import PRECISIONS, default_precision, require_hip

__all__ = ["AutoRegressiveTransformer", "ConditionalGuidedCELoss", "KLdiv", "VlmPlan", "vlm_param_names", "vlm_untrained",
           "vlm_guide_blocks", "vlm_guide_plane_elems",
           "VLM_UNTRAINED", "VLM_JOINT_UNTRAINED"]

# never given a gradient by the reference in sequential mode (the image prefix is a
# frozen CLIP feature, _out is unused): AdamW and clip_grad_norm_ skip them
VLM_UNTRAINED = ("i_embedding.weight", "_out.weight", "_out.bias")
# joint model (sequential=False, train_NWP.py): the image leaves go through i_embedding
VLM_JOINT_UNTRAINED = ("_out.weight", "_out.bias")


def vlm_untrained(model):
    """Parameters the reference never gives a gradient (AdamW and clip_grad_norm_
    skip them): VLM_UNTRAINED / VLM_JOINT_UNTRAINED, and with layernorm=False the
    unused LayerNorms (model.py:269-277, 294-301)."""
    names = VLM_UNTRAINED if model.sequential else VLM_JOINT_UNTRAINED
    if not getattr(model, "layernorm", True):
        names = names + tuple(f"_lns_{k}.{l}.{w}" for k in (1, 2) for l in range(model.n_layer)
                              for w in ("weight", "bias"))
    return names


def vlm_param_names(n_layer):
    """state_dict keys of AutoRegressiveTransformer in registration order
    (model.py:177-218: the ModuleLists are registered before t_/i_embedding)."""
    names = ["position_embeddings.weight"]
    names += [f"_queries.{l}.weight" for l in range(n_layer)]
    names += [f"_keys.{l}.weight" for l in range(n_layer)]
    names += [f"_values.{l}.weight" for l in range(n_layer)]
    for l in range(n_layer):
        names += [f"_mlps.{l}.0.weight", f"_mlps.{l}.0.bias", f"_mlps.{l}.2.weight", f"_mlps.{l}.2.bias"]
    for l in range(n_layer):
        names += [f"_lns_1.{l}.weight", f"_lns_1.{l}.bias"]
    for l in range(n_layer):
        names += [f"_lns_2.{l}.weight", f"_lns_2.{l}.bias"]
    names += ["t_embedding.weight", "i_embedding.weight", "_read_out.weight", "_read_out.bias", "_out.weight",
              "_out.bias"]
    return names


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _gemm(ta, tb, epi, A, lda, Bs, ldb, b_chunk, C, ldc, M, N, K, C2=None, bias=None, R=None, ldr=0, nsplit=1,
          s=None, f32=False):
    """ghm_gemm_x3 / ghm_gemm_f32 (include/ghm_hip.h): C = A(m,k) B(k,n) with the epilogue epi."""
    Bs = list(Bs) + [None] * (3 - len(Bs))
    pp = lambda t: None if t is None else _ptr(t)  # noqa: E731
    _native.call("ghm_gemm_f32" if f32 else "ghm_gemm_x3", ta, tb, epi, _ptr(A), lda, pp(Bs[0]), pp(Bs[1]), pp(Bs[2]), ldb, b_chunk, _ptr(C),
                 ldc, pp(C2), pp(bias), pp(R), ldr, M, N, K, nsplit, _stream() if s is None else s)


EPI_STORE, EPI_GELU, EPI_RESID, EPI_MUL, EPI_SLAB = range(5)


class VlmPlan:
    def __init__(self, n_layer, n_token, n_seq, n_prefix=1, num_class=10, n_embd=256, eps=1e-5,
                 normalize_attn=True, device="cuda", precision=None, joint=False, activation="softmax",
                 layernorm=True):
        if n_embd not in (128, 256, 512):
            raise ValueError(f"the HIP VLM kernels take n_embd in (128, 256, 512) (got {n_embd})")
        self.L, self.T, self.N, self.P, self.V, self.D = n_layer, n_token, n_seq, n_prefix, num_class, n_embd
        self.F = 4 * n_embd
        self.M = M = n_seq * n_token
        self.eps = float(eps)
        self.scale_div = float(math.sqrt(n_embd)) if normalize_attn else 1.0  # model.py:335-336
        self.device = torch.device(device)
        self.precision = default_precision() if precision is None else precision
        if self.precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}")
        if self.precision == "x3" and n_embd not in (128, 256):
            raise ValueError(f"the split-bf16 VLM kernels take n_embd in (128, 256) (got {n_embd})")
        # attention activation (model.py:121-130): softmax, or relu on the split-bf16
        # kernels (gelu of the -inf-masked scores is NaN in the reference: refused)
        if activation not in ("softmax", "relu") or (activation == "relu" and self.precision != "x3"):
            raise NotImplementedError(f"HIP VLM attention: softmax, or relu with precision x3 (got {activation}, "
                                      f"{self.precision})")
        self.act = 1 if activation == "relu" else 0
        if n_token > 192 or (n_token > 96 and self.precision != "x3"):
            raise ValueError(f"the HIP attention kernels take sequences of <= 96 tokens, <= 192 with the split-bf16 "
                             f"(x3) kernels (got {n_token}, precision {self.precision})")
        # joint model (sequential=False): image prefix tokens through i_embedding;
        # sequences past 96 tokens (161) run on ghm_attn_ext_*_x3 with P / dS padded to 192
        self.joint = joint
        self.long_attn = n_token > 96
        pad = 192 if self.long_attn else 96
        L, D, F, N = n_layer, n_embd, self.F, n_seq
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)  # noqa: E731
        self.H = e(L + 1, M, D)
        self.Hmid = e(L, M, D)
        # layernorm=False (model.py:269-277, 294-301): Q / K / V read H and the MLP
        # reads Hmid directly; their backward adds dX into the residual gradient
        self.layernorm = bool(layernorm)
        if self.layernorm:
            self.X1, self.X2 = e(L, M, D), e(L, M, D)
        else:
            self.X1, self.X2 = self.H[:L], self.Hmid
        self.G, self.Dg = e(L, M, F), e(L, M, F)
        self.Pm = torch.zeros(L, N, pad, pad, dtype=torch.float32, device=self.device)
        self.st1, self.st2 = e(L, M, 2), e(L, M, 2)
        self.logits, self.dlogits = e(M, num_class), e(M, num_class)
        self.dH = e(2, M, D)
        self.dX = e(M, D)
        self.dG = e(M, F)
        self.f32 = self.precision != "x3"
        if self.f32:  # separate q / k / v (the fp32 attention kernels' layout)
            self.q, self.k, self.v = e(L, M, D), e(L, M, D), e(L, M, D)
            self.dq, self.dk, self.dv = e(M, D), e(M, D), e(M, D)
            self.zero_b = torch.zeros(D, dtype=torch.float32, device=self.device)
        else:
            # fused projections: q | k | v columns of one [M][3D] buffer
            self.qkv = e(L, M, 3 * D)
            self.dqkv = e(M, 3 * D)
            self.dS = torch.zeros(N, pad, pad, dtype=torch.float32, device=self.device)
        # split-k weight-gradient slabs, column-sum partials
        self.nsplit = max(1, min(int(os.environ.get("GHM_VLM_NSPLIT", "16")), M // 256))
        self.slab = e(self.nsplit * max(D * F, 3 * D * D))
        self.bslab = e(self.nsplit * F)  # MLP bias-gradient row-sum partials
        # data gradients dX = dY W over K = 4D / 3D: k split in dsplit slabs (the
        # N = D products have only 2 x M / 64 output tiles: ~1.3 workgroups per CU)
        self.dsplit = max(1, int(os.environ.get("GHM_VLM_DSPLIT", "1")))
        self.dslab = e(self.dsplit * M * D) if self.dsplit > 1 else None
        # x3 (default; GHM_VLM_PACK=0 turns it off): the weights' (hi, lo) bf16
        # images for ghm_gemm_x3p, split once per forward by ghm_split_pack, instead
        # of the GEMMs splitting them per tile
        self.pack_on = not self.f32 and os.environ.get("GHM_VLM_PACK", "1") == "1"
        if self.pack_on:
            self._img_sizes = {"qkv": 3 * D * D, "qkvT": 3 * D * D, "w1": F * D, "w1T": F * D, "w2": F * D,
                               "w2T": F * D}
            per = 2 * sum(self._img_sizes.values())
            self.wpack = torch.empty(L * per, dtype=torch.bfloat16, device=self.device)
            self._img_off, o = {}, 0
            for l in range(L):
                for k, n in self._img_sizes.items():
                    self._img_off[(l, k)] = o
                    o += 2 * n
            # the job table lives in one device buffer for the plan's lifetime: a
            # captured ghm_split_pack node keeps its address, so a table rewritten
            # for moved weights is refreshed in place (never reallocated), and only
            # outside a capture (_split_weights)
            self._pack_key = None
            self.pack_jobs = torch.zeros(L * 10, 8, dtype=torch.int64, device=self.device)
            self._pack_tiles = 1
        lib = _native.hip_lib()
        self.colpart = e(max(lib.ghm_colsum_part_elems(M, F), lib.ghm_colsum_part_elems(M, D),
                             lib.ghm_colsum_part_elems(N, n_token * D),
                             lib.ghm_wcolsum_part_elems(M, D, num_class)))
        self.nblk = int(_native.hip_lib().ghm_ln_rows_blocks(M))
        self.part_ln = e(self.nblk, 2, D)
        self.xt = torch.empty(N, n_token - n_prefix, dtype=torch.uint8, device=self.device)
        if joint:
            self.itok = torch.empty(N, n_prefix, dtype=torch.uint8, device=self.device)
        self._gen = 0

    # ------------------------------------------------------------------
    def forward(self, p, xt, feat):
        """p: name -> fp32 device tensor; xt uint8 [N, T - P] text tokens; feat
        f32 [N, P, V] prefix features (unused by the joint model: self.itok holds
        the image leaves).  Returns self.logits [M, V] (all rows)."""
        return self._forward_hip(p, xt, feat)

    def backward(self, p, g, dlogits=None, layer_grad=None):
        """Writes d(loss)/d(param) into g[name] for every trained parameter (not
        VLM_UNTRAINED) from dlogits [M, V] (defaults to self.dlogits).  Returns
        dL/dH_0 [M, D] (its prefix rows give the gradient of the features).
        layer_grad: optional {layer l: fn(dH, stream)} adding a loss term's gradient
        w.r.t. H[l+1] (the guided layers, model.py:303-331) before layer l's
        backward."""
        return self._backward_hip(p, g, dlogits, layer_grad)

    # ------------------------------------------------------------------
    # every projection on the hand-written GEMM (ghm_gemm_x3, or ghm_gemm_f32 in the
    # f32 mode; GELU, bias, residual and GELU' products fused into its epilogues),
    # attention on ghm_attn_ext_*_x3 (x3) or ghm_vlm_attn_* (f32)
    def _gemm(self, *a, **k):
        _gemm(*a, f32=self.f32, **k)

    def _img(self, l, k):
        """(hi pointer, pitch, lo-plane offset) of layer l's pre-split image k: B(k,n)
        of a weight product is img[n][k] (qkv / w1 / w2: the forward's W; qkvT /
        w1T / w2T: the data gradients' W^T)."""
        D, F = self.D, self.F
        pitch = {"qkv": D, "qkvT": 3 * D, "w1": D, "w1T": F, "w2": F, "w2T": D}[k]
        return self.wpack.data_ptr() + 2 * self._img_off[(l, k)], pitch, self._img_sizes[k]

    def _gemmp(self, epi, A, lda, img, C, ldc, M, N, K, C2=None, bias=None, R=None, ldr=0, nsplit=1, s=None):
        """ghm_gemm_x3p: C = A B with B pre-split (self._img)."""
        pp = lambda t: None if t is None else _ptr(t)  # noqa: E731
        bp, ldbp, plane = img
        _native.call("ghm_gemm_x3p", epi, _ptr(A), lda, ctypes.c_void_p(bp), ldbp, plane, _ptr(C), ldc, pp(C2),
                     pp(bias), pp(R), ldr, M, N, K, nsplit, _stream() if s is None else s)

    def _split_weights(self, p, s):
        """Write every layer's six weight images (ghm_split_pack, one launch); the
        job table is rebuilt only when a weight's storage moved."""
        D, F = self.D, self.F
        names = [(f"_queries.{l}.weight", f"_keys.{l}.weight", f"_values.{l}.weight", f"_mlps.{l}.0.weight",
                  f"_mlps.{l}.2.weight") for l in range(self.L)]
        key = tuple(p[n].data_ptr() for ns in names for n in ns)
        if key != self._pack_key:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("VlmPlan: the weights moved during a graph capture; run one eager forward with "
                                   "the same parameter tensors before capturing")
            jobs = []
            for l, (nq, nk, nv, n1, n2) in enumerate(names):
                qkv, _, pq = self._img(l, "qkv")
                qkvT, _, pqT = self._img(l, "qkvT")
                for i, n in enumerate((nq, nk, nv)):
                    jobs.append((p[n].data_ptr(), D, D, D, qkv + 2 * i * D * D, D, pq, 0))  # rows iD.. of [3D][D]
                    jobs.append((p[n].data_ptr(), D, D, D, qkvT + 2 * i * D, 3 * D, pqT, 1))  # columns iD.. of [D][3D]
                for n, (rows, cols), k, kt in ((n1, (F, D), "w1", "w1T"), (n2, (D, F), "w2", "w2T")):
                    b, _, pl = self._img(l, k)
                    bt, _, plt = self._img(l, kt)
                    jobs.append((p[n].data_ptr(), cols, rows, cols, b, cols, pl, 0))
                    jobs.append((p[n].data_ptr(), cols, rows, cols, bt, rows, plt, 1))
            assert len(jobs) == self.pack_jobs.shape[0]
            self.pack_jobs.copy_(torch.tensor(jobs, dtype=torch.int64))
            self._pack_tiles = max(-(-r // 64) * -(-c // 64) for (_, _, r, c, _, _, _, _) in jobs)
            self._pack_key = key
        _native.call("ghm_split_pack", _ptr(self.pack_jobs), len(self.pack_jobs), self._pack_tiles, s)

    def _forward_hip(self, p, xt, feat):
        s = _stream()
        c = _native.call
        M, D, F, T, N = self.M, self.D, self.F, self.T, self.N
        if self.joint:  # feat unused: self.itok holds the image leaves
            c("ghm_vlm_embed_joint_fwd", _ptr(xt), _ptr(self.itok), _ptr(p["i_embedding.weight"]),
              _ptr(p["t_embedding.weight"]), _ptr(p["position_embeddings.weight"]), _ptr(self.H[0]),
              None, None, N, T, self.P, self.V, D, s)
        else:
            c("ghm_vlm_embed_fwd", _ptr(xt), _ptr(feat), _ptr(p["t_embedding.weight"]),
              _ptr(p["position_embeddings.weight"]), _ptr(self.H[0]), None, N, T, self.P, self.V, D, s)
        if self.pack_on:
            self._split_weights(p, s)
        for l in range(self.L):
            if self.layernorm:
                c("ghm_ln_rows_fwd", _ptr(self.H[l]), _ptr(p[f"_lns_1.{l}.weight"]), _ptr(p[f"_lns_1.{l}.bias"]),
                  _ptr(self.X1[l]), _ptr(self.st1[l]), M, D, self.eps, s)
            wqkv = (p[f"_queries.{l}.weight"], p[f"_keys.{l}.weight"], p[f"_values.{l}.weight"])
            if self.f32:
                for w, out in zip(wqkv, (self.q[l], self.k[l], self.v[l])):
                    self._gemm(0, 1, EPI_STORE, self.X1[l], D, (w,), D, 0, out, D, M, D, D, s=s)
                c("ghm_vlm_attn_fwd", _ptr(self.q[l]), _ptr(self.k[l]), _ptr(self.v[l]), _ptr(self.H[l]),
                  _ptr(self.Hmid[l]), _ptr(self.Pm[l]), N, T, D, self.P, self.scale_div, s)
            else:
                if self.pack_on:
                    self._gemmp(EPI_STORE, self.X1[l], D, self._img(l, "qkv"), self.qkv[l], 3 * D, M, 3 * D, D, s=s)
                else:
                    self._gemm(0, 1, EPI_STORE, self.X1[l], D, wqkv, D, D, self.qkv[l], 3 * D, M, 3 * D, D, s=s)
                if self.act:  # relu(score) (model.py:287), masked entries 0
                    c("ghm_attn_ext_fwd_x3_act", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]),
                      _ptr(self.Pm[l]), None, N, T, D, self.P, self.scale_div, 1.0 / D, self.act, s)
                else:
                    c("ghm_attn_ext_fwd_x3", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]),
                      _ptr(self.Pm[l]), N, T, D, self.P, self.scale_div, 1.0 / D, s)
            if self.layernorm:
                c("ghm_ln_rows_fwd", _ptr(self.Hmid[l]), _ptr(p[f"_lns_2.{l}.weight"]),
                  _ptr(p[f"_lns_2.{l}.bias"]), _ptr(self.X2[l]), _ptr(self.st2[l]), M, D, self.eps, s)
            if self.pack_on:
                self._gemmp(EPI_GELU, self.X2[l], D, self._img(l, "w1"), self.G[l], F, M, F, D, C2=self.Dg[l],
                            bias=p[f"_mlps.{l}.0.bias"], s=s)
                self._gemmp(EPI_RESID, self.G[l], F, self._img(l, "w2"), self.H[l + 1], D, M, D, F,
                            bias=p[f"_mlps.{l}.2.bias"], R=self.Hmid[l], ldr=D, s=s)  # :344-347
            else:
                self._gemm(0, 1, EPI_GELU, self.X2[l], D, (p[f"_mlps.{l}.0.weight"],), D, 0, self.G[l], F, M, F, D,
                           C2=self.Dg[l], bias=p[f"_mlps.{l}.0.bias"], s=s)
                self._gemm(0, 1, EPI_RESID, self.G[l], F, (p[f"_mlps.{l}.2.weight"],), F, 0, self.H[l + 1], D, M, D,
                           F, bias=p[f"_mlps.{l}.2.bias"], R=self.Hmid[l], ldr=D, s=s)  # :344-347
        c("ghm_rows_linear", _ptr(self.H[self.L]), _ptr(p["_read_out.weight"]), _ptr(p["_read_out.bias"]),
          _ptr(self.logits), M, D, self.V, s)  # model.py:332
        self._xt_fwd = xt
        self._gen += 1
        return self.logits

    def _wgrad(self, A, lda, m, B, ldb, n, dst, chunk, s, bias=None):
        """dst (rows stacked by chunk) = A^T B over the M tokens: split-k slabs + fixed-order reduce.
        bias: also its gradient, the column sums of A over the tokens, from the same
        staged tiles (C2 row-sum partials) and the same reduce launch."""
        bs = None if bias is None else self.bslab
        self._gemm(1, 0, EPI_SLAB, A, lda, (B,), ldb, 0, self.slab, n, m, n, self.M, C2=bs, nsplit=self.nsplit, s=s)
        d = list(dst) + [None] * (3 - len(dst))
        pp = lambda t: None if t is None else _ptr(t)  # noqa: E731
        _native.call("ghm_gemm_reduce_bias", _ptr(self.slab), self.nsplit, m, n, pp(d[0]), pp(d[1]), pp(d[2]), chunk,
                     pp(bs), pp(bias), s)

    def _dgrad(self, A, lda, Bs, b_chunk, K, s, img=None):
        """self.dX [M][D] = A [M][K] @ B (B [K][D] rows stacked by b_chunk, or the
        pre-split image img of B^T), split-k over dsplit slabs + the fixed-order
        reduce when dsplit > 1."""
        M, D = self.M, self.D
        ns = self.dsplit
        if ns > 1 and (ns - 1) * ((-(-K // ns) + 31) // 32 * 32) < K:
            if img is not None:
                self._gemmp(EPI_SLAB, A, lda, img, self.dslab, D, M, D, K, nsplit=ns, s=s)
            else:
                self._gemm(0, 0, EPI_SLAB, A, lda, Bs, D, b_chunk, self.dslab, D, M, D, K, nsplit=ns, s=s)
            _native.call("ghm_gemm_reduce", _ptr(self.dslab), ns, M, D, _ptr(self.dX), None, None, 0, s)
        elif img is not None:
            self._gemmp(EPI_STORE, A, lda, img, self.dX, D, M, D, K, s=s)
        else:
            self._gemm(0, 0, EPI_STORE, A, lda, Bs, D, b_chunk, self.dX, D, M, D, K, s=s)

    def _backward_hip(self, p, g, dlogits=None, layer_grad=None):
        s = _stream()
        c = _native.call
        M, D, F = self.M, self.D, self.F
        dz = self.dlogits if dlogits is None else dlogits
        cur, nxt = self.dH[0], self.dH[1]
        c("ghm_rows_linear_t", _ptr(dz), _ptr(p["_read_out.weight"]), _ptr(cur), M, D, self.V, s)
        c("ghm_wcolsum", _ptr(dz), None, self.V, _ptr(self.H[self.L]), M, M, 0, M, D, _ptr(g["_read_out.weight"]),
          _ptr(g["_read_out.bias"]), _ptr(self.colpart), s)
        for l in reversed(range(self.L)):
            if layer_grad and l in layer_grad:
                layer_grad[l](cur, s)
            w1, w2 = p[f"_mlps.{l}.0.weight"], p[f"_mlps.{l}.2.weight"]
            self._wgrad(cur, D, D, self.G[l], F, F, (g[f"_mlps.{l}.2.weight"],), 0, s, bias=g[f"_mlps.{l}.2.bias"])
            if self.pack_on:  # dU
                self._gemmp(EPI_MUL, cur, D, self._img(l, "w2T"), self.dG, F, M, F, D, R=self.Dg[l], ldr=F, s=s)
            else:
                self._gemm(0, 0, EPI_MUL, cur, D, (w2,), F, 0, self.dG, F, M, F, D, R=self.Dg[l], ldr=F, s=s)
            self._wgrad(self.dG, F, F, self.X2[l], D, D, (g[f"_mlps.{l}.0.weight"],), 0, s, bias=g[f"_mlps.{l}.0.bias"])
            self._dgrad(self.dG, F, (w1,), 0, F, s, img=self._img(l, "w1T") if self.pack_on else None)
            if self.layernorm:
                c("ghm_ln_rows_bwd", _ptr(self.dX), _ptr(self.Hmid[l]), _ptr(self.st2[l]),
                  _ptr(p[f"_lns_2.{l}.weight"]), _ptr(cur), _ptr(nxt), _ptr(self.part_ln), M, D, s)
                self._reduce_ln(g, 2, l, s)
            else:
                c("ghm_add", _ptr(cur), _ptr(self.dX), _ptr(nxt), M * D, s)
            # attention (nxt = dHmid) -> dq | dk | dv
            wqkv = (p[f"_queries.{l}.weight"], p[f"_keys.{l}.weight"], p[f"_values.{l}.weight"])
            gqkv = (g[f"_queries.{l}.weight"], g[f"_keys.{l}.weight"], g[f"_values.{l}.weight"])
            if self.f32:
                c("ghm_vlm_attn_bwd", _ptr(self.q[l]), _ptr(self.k[l]), _ptr(self.v[l]), _ptr(self.Pm[l]), _ptr(nxt),
                  _ptr(self.dq), _ptr(self.dk), _ptr(self.dv), self.N, self.T, D, self.scale_div, s)
                dqkv = (self.dq, self.dk, self.dv)
                for d, gw in zip(dqkv, gqkv):
                    self._wgrad(d, D, D, self.X1[l], D, D, (gw,), 0, s)
                # dX = dq Wq, then (dk Wk + 0) + dX and (dv Wv + 0) + dX in place
                self._gemm(0, 0, EPI_STORE, self.dq, D, (wqkv[0],), D, 0, self.dX, D, M, D, D, s=s)
                for d, w in zip(dqkv[1:], wqkv[1:]):
                    self._gemm(0, 0, EPI_RESID, d, D, (w,), D, 0, self.dX, D, M, D, D, bias=self.zero_b, R=self.dX,
                               ldr=D, s=s)
            else:
                if self.act:  # dS = [P > 0] dA / scale_div
                    c("ghm_attn_ext_bwd_x3_act", _ptr(self.qkv[l]), _ptr(self.Pm[l]), None, _ptr(nxt),
                      _ptr(self.dS), _ptr(self.dqkv), self.N, self.T, D, self.P, self.scale_div, 1.0 / D, self.act, s)
                else:
                    c("ghm_attn_ext_bwd_x3", _ptr(self.qkv[l]), _ptr(self.Pm[l]), _ptr(nxt), _ptr(self.dS),
                      _ptr(self.dqkv), self.N, self.T, D, self.P, self.scale_div, 1.0 / D, s)
                self._wgrad(self.dqkv, 3 * D, 3 * D, self.X1[l], D, D, gqkv, D, s)
                self._dgrad(self.dqkv, 3 * D, wqkv, D, 3 * D, s, img=self._img(l, "qkvT") if self.pack_on else None)
            if self.layernorm:
                c("ghm_ln_rows_bwd", _ptr(self.dX), _ptr(self.H[l]), _ptr(self.st1[l]),
                  _ptr(p[f"_lns_1.{l}.weight"]), _ptr(nxt), _ptr(cur), _ptr(self.part_ln), M, D, s)
                self._reduce_ln(g, 1, l, s)
            else:
                c("ghm_add", _ptr(nxt), _ptr(self.dX), _ptr(cur), M * D, s)
        self._colsum(cur, self.N, self.T * D, g["position_embeddings.weight"], s)  # sum over sequences
        # token-embedding gradients: rows of dH0 summed per token value (text rows
        # t >= P; the joint model's prefix rows through i_embedding)
        T, P, N = self.T, self.P, self.N
        c("ghm_wcolsum", None, _ptr(self._xt_fwd), self.V, _ptr(cur), T - P, T, P, N * (T - P), D,
          _ptr(g["t_embedding.weight"]), None, _ptr(self.colpart), s)
        if self.joint:
            c("ghm_wcolsum", None, _ptr(self.itok), self.V, _ptr(cur), P, T, 0, N * P, D,
              _ptr(g["i_embedding.weight"]), None, _ptr(self.colpart), s)
        return cur

    def _colsum(self, X, rows, cols, out, s):
        _native.call("ghm_colsum", _ptr(X), rows, cols, _ptr(out), _ptr(self.colpart), s)

    def _reduce_ln(self, g, which, l, s):
        j = _native.ReduceJob()
        j.part = self.part_ln.data_ptr()
        j.n_split = self.nblk
        j.n_seg = 2
        j.n = 2 * self.D
        j.dst[0] = g[f"_lns_{which}.{l}.weight"].data_ptr()
        j.dst[1] = g[f"_lns_{which}.{l}.bias"].data_ptr()
        j.off[0], j.off[1], j.off[2] = 0, self.D, 2 * self.D
        _native.call("ghm_reduce_batch", (_native.ReduceJob * 1)(j), 1, s)


def vlm_guide_blocks(model, n_text, V):
    """The guided outputs of AutoRegressiveTransformer.forward (model.py:303-331) as
    column blocks of H[l+1] and their targets in vlm_guide_planes' per-sample
    layout: {layer: [(tok0, ntok, col, plane_offset, group)]} in the reference's
    loss-term order, group in ("loss2", "loss4", "loss5", "loss3") = the
    ConditionalGuidedCELoss penalty terms (model.py:1122-1144: text downward incl.
    the leaf, text root, text upward, image).  Text block k (k-th text-guided
    layer): k = 0 the leaf q at columns index_q; 0 < k <= n_t the (h, q) pair at
    (index_h, index_q); k > n_t the u at index_u; image blocks at index_i."""
    n_t, P = model.n_t_guided_layer, model.n_i_token
    n_tplanes = 3 * n_t + 1
    tplane = lambda k: n_text * V * k  # noqa: E731
    iplane = lambda j: n_text * V * n_tplanes + P * V * j  # noqa: E731
    index_q, index_h, index_u, index_i = 0, (n_t + 1) * V, (2 * n_t + 1) * V, 0
    counter, img = 0, 0
    blocks = {}
    for l in range(model.n_layer):
        blks = []
        if model.t_guided_layer_flag[l]:
            if counter == 0:
                blks.append((P, n_text, index_q, tplane(0), "loss2"))
                index_q += V
            elif counter < n_t + 1:
                grp = "loss2" if counter < n_t else "loss4"
                blks.append((P, n_text, index_h, tplane(2 * counter - 1), grp))
                blks.append((P, n_text, index_q, tplane(2 * counter), grp))
                index_h += V
                index_q += V
            else:
                blks.append((P, n_text, index_u, tplane(2 * n_t + counter - n_t), "loss5"))
                index_u += V
            counter += 1
        if model.i_guided_layer_flag[l]:
            blks.append((0, P, index_i, iplane(img), "loss3"))
            index_i += V
            img += 1
        if blks:
            blocks[l] = blks
    return blocks


def _guided_slices(model, n_text):
    """The reference's guided outputs in return order: text outputs (one per
    text-guided layer; the (h, q) pair concatenated) then image outputs, each as
    (layer, [(tok0, ntok, col)], kind)."""
    blocks = vlm_guide_blocks(model, n_text, model.vocab_size)
    text, image = [], []
    for l in sorted(blocks):
        tb = [(t0, nt, c) for (t0, nt, c, _, g) in blocks[l] if g != "loss3"]
        ib = [(t0, nt, c) for (t0, nt, c, _, g) in blocks[l] if g == "loss3"]
        if tb:
            text.append((l, tb, "t"))
        if ib:
            image.append((l, ib, "i"))
    return text + image


def vlm_guide_plane_elems(model, n_text, V):
    """Floats per sample of the guide target planes (vlm_guide_planes): the text
    blocks, then (joint model) one [n_i_token][V] plane per image-guided layer.  The
    sequential model's image guides all target the frozen CLIP feature
    (train_sequential_NWP.py:165), which the fused trainer reads from the CLIP
    encoder's output in place: no image planes."""
    n = n_text * V * (3 * model.n_t_guided_layer + 1)
    if not model.sequential:
        n += model.n_i_token * V * sum(model.i_guided_layer_flag)
    return n


class _VlmFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, module, xt, zi, *params):
        N, T1 = xt.shape
        plan = module._plan(N, T1 + zi.shape[1], zi.shape[1], xt.device)
        pd = dict(zip(module._names, params))
        plan.xt.copy_(xt.to(torch.uint8))
        if plan.joint:  # zi: image leaves (token ids)
            plan.itok.copy_(zi.to(torch.uint8))
            logits = plan.forward(pd, plan.xt, None)
        else:
            feat = zi.contiguous().float()
            logits = plan.forward(pd, plan.xt, feat)
        ctx.module, ctx.plan, ctx.gen = module, plan, plan._gen
        ctx.save_for_backward(*params)
        out = logits.view(N, T1 + zi.shape[1], -1)[:, zi.shape[1]:, :].clone()
        if not module.guide:
            return out
        # guided outputs (model.py:303-331): copies of the column blocks of H[l+1]
        ctx.gslices = _guided_slices(module, T1)
        Hv = plan.H.view(plan.L + 1, N, plan.T, plan.D)
        guided = [torch.cat([Hv[l + 1, :, t0:t0 + nt, c:c + module.vocab_size] for (t0, nt, c) in blks], dim=2)
                  for (l, blks, _) in ctx.gslices]
        return (out, *guided)

    @staticmethod
    def backward(ctx, dlog, *dguided):
        plan = ctx.plan
        layer_grad = None
        if ctx.module.guide:  # add each guided output's gradient into dH[l+1] before layer l's backward
            V = ctx.module.vocab_size
            hooks = {}
            for (l, blks, _), gd in zip(ctx.gslices, dguided):
                if gd is None:
                    continue

                def fn(dH, s, blks=blks, gd=gd):
                    dv = dH.view(plan.N, plan.T, plan.D)
                    for j, (t0, nt, c) in enumerate(blks):
                        dv[:, t0:t0 + nt, c:c + V] += gd[:, :, j * V:(j + 1) * V]
                hooks.setdefault(l, []).append(fn)
            layer_grad = {l: (lambda dH, s, fs=fs: [f(dH, s) for f in fs]) for l, fs in hooks.items()}
        if plan._gen != ctx.gen:
            raise RuntimeError("AutoRegressiveTransformer: another forward of this module overwrote the "
                               "activations saved for backward")
        params = ctx.saved_tensors
        names = ctx.module._names
        untrained = vlm_untrained(ctx.module)
        grads = {n: torch.empty_like(p) for n, p in zip(names, params) if n not in untrained}
        dz = torch.zeros(plan.N, plan.T, plan.V, dtype=torch.float32, device=dlog.device)
        dz[:, plan.P:, :] = dlog
        dH0 = plan.backward(dict(zip(names, params)), grads, dlogits=dz.view(plan.M, plan.V), layer_grad=layer_grad)
        d_zi = None
        if ctx.needs_input_grad[2] and not plan.joint:
            d_zi = dH0.view(plan.N, plan.T, plan.D)[:, :plan.P, :plan.V].clone()
        return (None, None, d_zi, *[grads.get(n) for n in names])


class AutoRegressiveTransformer(nn.Module):
    """Reference: models/model.py:132-335.  Same constructor, parameter creation order
    (so torch.manual_seed gives identical weights) and state_dict keys.  The HIP path
    covers the configurations the VLM experiments train: sequential
    (exp_vlm_{standard,shallow}TF.sh: a frozen-CLIP image feature prefix token, T = 81)
    and joint (exp_vlm_jointtrain.sh: the 81 image leaves through i_embedding as the
    prefix, T = 161, split-bf16 only); prefix-causal mask, softmax attention (relu on
    the split-bf16 kernels), LayerNorm, MLP; guide=True for both (train_NWP.py /
    train_sequential_NWP.py --guide=True); n_embd in (128, 256, 512) (joint: 128, 256)."""

    def __init__(self, n_token=9, n_i_token=4, num_class=10, n_embd=128, n_layer=12, n_guided_layers=(3, 3),
                 n_head=4, n_mlp_hidden=512, activation="softmax", mlp=True, normalize_attn=True,
                 auto_regressive=False, sequential=False, layernorm=True, guide=False):
        super().__init__()
        self.name = f"EncoderTF_embd={n_embd}_layer={n_layer}_head={n_head}"
        self.vocab_size = num_class
        self.context_length = n_token
        self.n_token = n_token
        self.n_i_token = n_i_token
        self.n_embd = n_embd
        self.n_head = n_head
        self.n_layer = n_layer
        self.n_mlp_hidden = n_mlp_hidden
        self.sequential = sequential
        self.activation = activation
        self.mlp = mlp
        self.normalize_attn = normalize_attn
        self.layernorm = layernorm
        self.auto_regressive = auto_regressive
        self.guide = guide
        self.n_t_guided_layer = n_guided_layers[0]
        self.n_i_guided_layer = n_guided_layers[1]
        self.guided_layer_gap = n_layer // (n_guided_layers[0] * 2 + 1)
        if activation not in ("softmax", "relu") or not mlp:
            raise NotImplementedError("HIP VLM: softmax or relu attention, mlp=True")
        if not auto_regressive or (sequential and n_i_token != 1):
            raise NotImplementedError("HIP VLM: auto_regressive=True; sequential=True takes one prefix token "
                                      "(train_sequential_NWP.py), sequential=False the image leaves "
                                      "(train_NWP.py)")
        if n_mlp_hidden != 4 * n_embd:
            raise NotImplementedError("HIP VLM: n_mlp_hidden = 4 * n_embd")
        # construction (RNG) order of the reference, model.py:177-218
        self.position_embeddings = nn.Embedding(self.context_length, self.n_embd)
        self._queries = nn.ModuleList()
        self._keys = nn.ModuleList()
        self._values = nn.ModuleList()
        self._mlps = nn.ModuleList()
        self._lns_1 = nn.ModuleList()
        self._lns_2 = nn.ModuleList()
        self.t_guided_layer_flag = [False] * n_layer
        self.i_guided_layer_flag = [False] * n_layer
        self.t_embedding = nn.Embedding(self.vocab_size, self.n_embd)
        self.i_embedding = nn.Embedding(self.vocab_size, self.n_embd)
        counter = 0
        for i in range(n_layer):
            self._queries.append(nn.Linear(n_embd, n_embd, bias=False))
            self._keys.append(nn.Linear(n_embd, n_embd, bias=False))
            self._values.append(nn.Linear(n_embd, n_embd, bias=False))
            self._lns_1.append(nn.LayerNorm([self.n_embd]))
            self._mlps.append(nn.Sequential(nn.Linear(n_embd, n_mlp_hidden), nn.GELU(),
                                            nn.Linear(n_mlp_hidden, n_embd)))
            self._lns_2.append(nn.LayerNorm([self.n_embd]))
            # guided-layer flags (model.py:207-216); n_layer < 2 n_t + 1 divides by
            # zero in the reference too
            if guide and counter < self.n_t_guided_layer * 2 + 1 and (i + 1) % self.guided_layer_gap == 0:
                self.t_guided_layer_flag[i] = True
                if counter < self.n_i_guided_layer:
                    self.i_guided_layer_flag[i] = True
                if counter == self.n_t_guided_layer - 1 and self.n_i_guided_layer < self.n_t_guided_layer:
                    self.i_guided_layer_flag[i] = True
                counter += 1
        self._read_out = nn.Linear(n_embd, self.vocab_size)
        self._out = nn.Linear(n_token, 1)
        self._names = vlm_param_names(n_layer)
        self._plans = {}
        # matrix-product mode of the HIP plan ("x3" / "f32"; None: $GHM_PRECISION or "x3")
        self.precision = None

    def _plan(self, n_seq, T, P, device):
        key = (n_seq, T, P, str(device), self.precision)
        if key not in self._plans:
            self._plans.clear()
            self._plans[key] = VlmPlan(self.n_layer, T, n_seq, n_prefix=P, num_class=self.vocab_size,
                                       n_embd=self.n_embd, normalize_attn=self.normalize_attn, device=device,
                                       precision=self.precision, joint=not self.sequential,
                                       activation=self.activation, layernorm=self.layernorm)
        return self._plans[key]

    def forward(self, xt, zi):
        """xt: text tokens [B, T1] (long); zi: the frozen CLIP image feature [B, 1,
        num_class] (sequential) or the image leaves [B, n_i_token] (long; joint,
        sequential=False).  Returns (next-token logits [B, T1, num_class], [[], []])."""
        require_hip(xt)
        B, T1 = xt.shape
        if self.sequential:
            if zi.dim() != 3 or zi.shape[0] != B or zi.shape[1] != self.n_i_token or zi.shape[2] != self.vocab_size:
                raise ValueError(f"expected zi of shape [{B}, {self.n_i_token}, {self.vocab_size}], "
                                 f"got {tuple(zi.shape)}")
        elif zi.dim() != 2 or zi.shape[0] != B or zi.shape[1] != self.n_i_token:
            raise ValueError(f"expected image leaves of shape [{B}, {self.n_i_token}], got {tuple(zi.shape)}")
        if T1 + self.n_i_token != self.n_token:
            raise ValueError(f"expected {self.n_token - self.n_i_token} text tokens, got {T1}")
        for t in ((xt,) if self.sequential else (xt, zi)):
            if t.numel() and (int(t.min()) < 0 or int(t.max()) >= self.vocab_size):
                raise IndexError("token id out of range")
        sd = dict(self.named_parameters())
        params = [sd[n] for n in self._names]
        for prm in params:
            if prm.dtype != torch.float32 or not prm.is_contiguous():
                raise RuntimeError("HIP VLM parameters must be contiguous fp32")
        res = _VlmFn.apply(self, xt, zi, *params)
        if not self.guide:
            return res, [[], []]
        n_t = sum(self.t_guided_layer_flag)
        return res[0], [list(res[1:1 + n_t]), list(res[1 + n_t:])]


class ConditionalGuidedCELoss(nn.Module):
    """models/model.py:1080-1149: per-sample mean cross entropy; with guide the
    penalty * squared Frobenius norms of the guided outputs against their BP
    targets, grouped as the reference logs them (text downward incl. the leaf,
    text root, text upward, image).  Returns (loss, loss2, loss4, loss5, loss3).
    The fused VlmTrainer evaluates the same terms on the device."""

    def __init__(self, penalty=1e-4, guide=False):
        super().__init__()
        self.penalty = penalty
        self.guide = guide

    def forward(self, inputs, targets, verbose=False):
        logits = inputs[0].reshape(-1, inputs[0].size(-1))
        loss = nn.functional.cross_entropy(logits, targets[0].reshape(-1), reduction="none")
        loss = loss.reshape(-1, targets[0].shape[1]).mean(dim=1)
        if not self.guide:
            return loss.mean(), 0, 0, 0, 0
        sq = lambda a, b: self.penalty * ((a - b) ** 2).sum(dim=(1, 2))  # noqa: E731
        gin, gtg = inputs[1][0], targets[1][0]
        half = len(gin) // 2
        loss2 = sum(sq(gin[i], gtg[i]) for i in range(half))
        loss5 = sum(sq(gin[i + half + 1], gtg[i + half + 1]) for i in range(half))
        loss4 = sq(gin[half], gtg[half])
        loss3 = sum(sq(a, b) for a, b in zip(inputs[1][1], targets[1][1]))
        total = loss + loss2 + loss3 + loss4 + loss5
        return (total.mean(), loss2.mean().item(), loss4.mean().item(), loss5.mean().item(),
                loss3.mean().item())


class KLdiv(nn.Module):
    """models/model.py:1067-1078: batchmean KL of the target distributions against
    softmax(inputs)."""

    def forward(self, inputs, targets):
        inputs = nn.functional.log_softmax(inputs.reshape(-1, inputs.size(-1)), dim=1)
        return nn.functional.kl_div(inputs, targets.reshape(-1, targets.size(-1)), reduction="batchmean")
