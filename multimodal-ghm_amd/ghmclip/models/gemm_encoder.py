"""EncoderTransformer at widths other than 128 (reference: models/model.py:690-808).

The fused token-parallel kernels of hip_encoder.EncoderPlan are built for
n_embd = 128 (the width every shipped experiment script passes).  The reference
CLI's own default is clip_{t,i}model_deb = 64 (utils/config.py:58-59), and
EncoderTransformer takes any n_embd (model.py:693).  ``GemmEncoderPlan`` runs
those widths (64 and 256) on the same building blocks as the VLM (models/vlm.py):

  LN1 / LN2          ghm_ln_rows_fwd / _bwd (one wave per row, D = 64 / 256)
  Q | K | V          one split-bf16 GEMM (ghm_gemm_x3, the three weights stacked
                     as B; 64-column tiles when D = 64)
  attention          ghm_attn_ext_{fwd,bwd}_x3 (softmax; relu / gelu by _act):
                     unmasked (n_prefix = T), plain residual (dbl = 0),
                     scores / sqrt(n_embd) (model.py:779-781)
  MLP                GEMM with the GELU / GELU' epilogue, GEMM with bias + residual
  weight gradients   split-k slab GEMMs + the fixed-order slab reduce (bias
                     gradients from the same staged tiles)
  embedding          ghm_tok_embed_fwd; gradients ghm_wcolsum by token id and
                     ghm_colsum over the sequences
  readout            ghm_rows_linear (Z = H W_ro^T + b_ro) + ghm_tok_readout_fwd
                     (the token-axis Linear(n_token -> 1)); backward
                     ghm_tok_readout_bwd, ghm_rows_linear_t, ghm_wcolsum
Split-bf16 (x3) only: the exact-f32 GEMM variant has no 64-column tiles.

HBM layout (M = n_seq * T tokens, D = n_embd, F = 4 D, fp32 row-major):
  H [L+1][M][D], Hmid / X1 / X2 [L][M][D], qkv [L][M][3D], G / Dg [L][M][F],
  P (and Pd for gelu) [L][n_seq][pad][pad] (pad = 96, or 192 past 96 tokens),
  st1 / st2 [L][M][2], Z [M][C]; backward scratch dH [2][M][D], dX [M][D],
  dG [M][F], dqkv [M][3D], dS [n_seq][pad][pad], dZ [M][C], split-k slabs.
No PyTorch math runs here: torch allocates and provides the stream.
"""
import ctypes
import math

import torch

from .. import _native
from .hip_encoder import ENCODER_PRECISIONS, EncoderPlan, default_precision
from .vlm import EPI_GELU, EPI_MUL, EPI_RESID, EPI_SLAB, EPI_STORE, _gemm

GEMM_WIDTHS = (64, 256)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def make_encoder_plan(n_layer, n_token, n_seq, n_embd=128, **kw):
    """The plan for one EncoderTransformer: the fused kernels at n_embd = 128,
    the GEMM path otherwise."""
    if n_embd == 128:
        return EncoderPlan(n_layer, n_token, n_seq, n_embd=n_embd, **kw)
    kw.pop("defer_reduce", None)
    kw.pop("ln_presplit", None)
    kw.pop("wgrad_target_blocks", None)
    kw.pop("wgrad_min_tokens", None)
    return GemmEncoderPlan(n_layer, n_token, n_seq, n_embd=n_embd, **kw)


class GemmEncoderPlan:
    def __init__(self, n_layer, n_token, n_seq, num_class=10, vocab=10, n_embd=64, eps=1e-5, normalize_attn=True,
                 device="cuda", precision=None, activation="softmax"):
        if n_embd not in GEMM_WIDTHS:
            raise ValueError(f"the HIP encoder takes n_embd = 128 (fused kernels) or one of {GEMM_WIDTHS} "
                             f"(GEMM path), got {n_embd}")
        self.precision = default_precision(allowed=ENCODER_PRECISIONS) if precision is None else precision
        if self.precision not in ENCODER_PRECISIONS:
            raise ValueError(f"precision must be one of {ENCODER_PRECISIONS}")
        if self.precision != "x3":
            raise NotImplementedError(f"n_embd = {n_embd}: the encoder's GEMM path is split-bf16 (precision x3) only")
        if n_token > 192:
            raise ValueError(f"the HIP attention kernels take sequences of <= 192 tokens (got {n_token})")
        if vocab > 256 or num_class > 64:
            raise ValueError("vocabulary <= 256 and num_class <= 64")
        acts = {"softmax": 0, "relu": 1, "gelu": 2}
        if activation not in acts:
            raise NotImplementedError(f"attention activation {activation!r}")
        self.act = acts[activation]
        self.L, self.T, self.N, self.C, self.V = n_layer, n_token, n_seq, num_class, vocab
        self.D, self.F = n_embd, 4 * n_embd
        self.M = M = n_seq * n_token
        self.eps = float(eps)
        self.scale_div = float(math.sqrt(n_embd)) if normalize_attn else 1.0  # model.py:779-780
        self.device = dev = torch.device(device)
        L, D, F, N, T = n_layer, self.D, self.F, n_seq, n_token
        pad = 192 if T > 96 else 96
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.H, self.Hmid = e(L + 1, M, D), e(L, M, D)
        self.X1, self.X2 = e(L, M, D), e(L, M, D)
        self.qkv = e(L, M, 3 * D)
        self.G, self.Dg = e(L, M, F), e(L, M, F)
        self.P = torch.zeros(L, N, pad, pad, dtype=torch.float32, device=dev)
        self.Pd = torch.zeros(L, N, pad, pad, dtype=torch.float32, device=dev) if self.act == 2 else None
        self.st1, self.st2 = e(L, M, 2), e(L, M, 2)
        self.Z = e(M, num_class)
        self.emb, self.d_emb, self.d_other = e(N, num_class), e(N, num_class), e(N, num_class)
        self.loss_scr = e(2)
        self.tokens = self.token_buf = torch.empty(N, T, dtype=torch.uint8, device=dev)
        self.dH, self.dX, self.dG, self.dqkv = e(2, M, D), e(M, D), e(M, F), e(M, 3 * D)
        self.dS = torch.zeros(N, pad, pad, dtype=torch.float32, device=dev)
        self.dZ = e(M, num_class)
        # split-k weight gradients: ~256 workgroups per product (the tiles are few:
        # 64 x 64 / 64 x 128 output tiles of 64 x 256 matrices), slabs of >= 256 tokens
        self.nsplit = {}
        for key, (m, n) in {"w2": (D, F), "w1": (F, D), "qkv": (3 * D, D)}.items():
            tiles = -(-m // 64) * -(-n // (128 if n % 128 == 0 else 64))
            self.nsplit[key] = max(1, min(256, 256 // tiles, M // 256))
        self.slab = e(max(self.nsplit[k] * mn for k, mn in
                          (("w2", D * F), ("w1", F * D), ("qkv", 3 * D * D))))
        self.bslab = e(max(self.nsplit["w2"] * D, self.nsplit["w1"] * F))
        lib = _native.hip_lib()
        self.colpart = e(max(lib.ghm_colsum_part_elems(N, T * D), lib.ghm_wcolsum_part_elems(M, D, num_class),
                             lib.ghm_wcolsum_part_elems(M, D, vocab)))
        self.nblk = int(lib.ghm_ln_rows_blocks(M))
        self.part_ln = e(self.nblk, 2, D)
        self.pending = []  # nothing deferred: every gradient is final when written
        self._written = set()
        self._gen = 0

    # -- interface shared with EncoderPlan (ClipTrainer, the modules) --------------
    def split_weights(self, p, s=None):
        """(EncoderPlan's weight pre-split; the GEMM path splits per tile.)"""

    def probs_dense(self, l):
        return self.P[l, :, :self.T, :self.T]

    def flush_pending(self):
        """(Nothing is deferred on the GEMM path.)"""

    def queued_grad_ptrs(self):
        """Addresses of the parameter gradients the running backward has made
        final so far (ClipTrainer's data-parallel bucket check)."""
        return set(self._written)

    def forward(self, p, tokens=None, split=True):
        for _ in self.forward_iter(p, tokens, split):
            pass
        return self.emb

    def backward(self, p, g, d_emb=None, tokens=None, layer_grad=None):
        for _ in self.backward_iter(p, g, d_emb, tokens, layer_grad):
            pass

    # ------------------------------------------------------------------------------
    def forward_iter(self, p, tokens=None, split=True):
        """forward() as a generator yielding after the embedding, each layer and the
        readout (launches on the stream current when each is issued)."""
        tok = self.tokens if tokens is None else tokens
        c = _native.call
        M, D, F, T, N, L = self.M, self.D, self.F, self.T, self.N, self.L
        c("ghm_tok_embed_fwd", _ptr(tok), _ptr(p["token_embeddings.weight"]), _ptr(p["position_embeddings.weight"]),
          _ptr(self.H[0]), N, T, self.V, D, _stream())
        yield
        for l in range(L):
            s = _stream()
            c("ghm_ln_rows_fwd", _ptr(self.H[l]), _ptr(p[f"_lns_1.{l}.weight"]), _ptr(p[f"_lns_1.{l}.bias"]),
              _ptr(self.X1[l]), _ptr(self.st1[l]), M, D, self.eps, s)
            wqkv = (p[f"_queries.{l}.weight"], p[f"_keys.{l}.weight"], p[f"_values.{l}.weight"])
            _gemm(0, 1, EPI_STORE, self.X1[l], D, wqkv, D, D, self.qkv[l], 3 * D, M, 3 * D, D, s=s)
            if self.act:
                c("ghm_attn_ext_fwd_x3_act", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]), _ptr(self.P[l]),
                  None if self.Pd is None else _ptr(self.Pd[l]), N, T, D, T, self.scale_div, 0.0, self.act, s)
            else:
                c("ghm_attn_ext_fwd_x3", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]), _ptr(self.P[l]),
                  N, T, D, T, self.scale_div, 0.0, s)
            c("ghm_ln_rows_fwd", _ptr(self.Hmid[l]), _ptr(p[f"_lns_2.{l}.weight"]), _ptr(p[f"_lns_2.{l}.bias"]),
              _ptr(self.X2[l]), _ptr(self.st2[l]), M, D, self.eps, s)
            _gemm(0, 1, EPI_GELU, self.X2[l], D, (p[f"_mlps.{l}.0.weight"],), D, 0, self.G[l], F, M, F, D,
                  C2=self.Dg[l], bias=p[f"_mlps.{l}.0.bias"], s=s)
            _gemm(0, 1, EPI_RESID, self.G[l], F, (p[f"_mlps.{l}.2.weight"],), F, 0, self.H[l + 1], D, M, D, F,
                  bias=p[f"_mlps.{l}.2.bias"], R=self.Hmid[l], ldr=D, s=s)
            yield
        s = _stream()
        c("ghm_rows_linear", _ptr(self.H[L]), _ptr(p["_read_out.weight"]), _ptr(p["_read_out.bias"]), _ptr(self.Z),
          M, D, self.C, s)
        c("ghm_tok_readout_fwd", _ptr(self.Z), _ptr(p["_out.weight"]), _ptr(p["_out.bias"]), _ptr(self.emb), N, T,
          self.C, s)
        self._gen += 1

    def _wgrad(self, key, A, lda, m, B, ldb, n, dst, chunk, s, bias=None):
        """dst (rows stacked by chunk) = A^T B over the M tokens: split-k slabs + the
        fixed-order reduce; bias: also its gradient (the column sums of A)."""
        ns = self.nsplit[key]
        bs = None if bias is None else self.bslab
        _gemm(1, 0, EPI_SLAB, A, lda, (B,), ldb, 0, self.slab, n, m, n, self.M, C2=bs, nsplit=ns, s=s)
        d = list(dst) + [None] * (3 - len(dst))
        pp = lambda t: None if t is None else _ptr(t)  # noqa: E731
        _native.call("ghm_gemm_reduce_bias", _ptr(self.slab), ns, m, n, pp(d[0]), pp(d[1]), pp(d[2]), chunk, pp(bs),
                     pp(bias), s)
        self._written.update(t.data_ptr() for t in dst)
        if bias is not None:
            self._written.add(bias.data_ptr())

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
        self._written.update((j.dst[0], j.dst[1]))

    def backward_iter(self, p, g, d_emb=None, tokens=None, layer_grad=None, clip=None):
        """backward() as a generator yielding after the readout and after each layer.
        d_emb: d(loss)/d(emb) [n_seq, C] (defaults to self.d_emb); clip = (t_emb,
        i_emb, tower, B, K): ClipTrainer's K-way CLIP loss gradient of this tower's
        rows, recomputed here from both towers' embeddings (ghm_clip_loss)."""
        tok = self.tokens if tokens is None else tokens
        c = _native.call
        M, D, F, T, N, L, C = self.M, self.D, self.F, self.T, self.N, self.L, self.C
        self._written = set()
        s = _stream()
        de = self.d_emb if d_emb is None else d_emb
        if clip is not None:
            te, ie, tower, B, K = clip
            dt, di = (self.d_emb, self.d_other) if tower == 0 else (self.d_other, self.d_emb)
            c("ghm_clip_loss", _ptr(te), _ptr(ie), _ptr(dt), _ptr(di), _ptr(self.loss_scr), None, None, B, K, C, s)
            de = self.d_emb
        c("ghm_tok_readout_bwd", _ptr(self.Z), _ptr(de), _ptr(p["_out.weight"]), _ptr(self.dZ), _ptr(g["_out.weight"]),
          _ptr(g["_out.bias"]), N, T, C, s)
        cur, nxt = self.dH[0], self.dH[1]
        c("ghm_rows_linear_t", _ptr(self.dZ), _ptr(p["_read_out.weight"]), _ptr(cur), M, D, C, s)
        c("ghm_wcolsum", _ptr(self.dZ), None, C, _ptr(self.H[L]), M, M, 0, M, D, _ptr(g["_read_out.weight"]),
          _ptr(g["_read_out.bias"]), _ptr(self.colpart), s)
        self._written.update(g[k].data_ptr() for k in ("_out.weight", "_out.bias", "_read_out.weight",
                                                       "_read_out.bias"))
        yield
        for l in reversed(range(L)):
            s = _stream()
            if layer_grad and l in layer_grad:
                layer_grad[l](cur, s)
            w1, w2 = p[f"_mlps.{l}.0.weight"], p[f"_mlps.{l}.2.weight"]
            # MLP (model.py:784-788): dW2 = dY^T G, dU = (dY W2) GELU'(U), dW1 = dU^T LN2(Hmid), dX2 = dU W1
            self._wgrad("w2", cur, D, D, self.G[l], F, F, (g[f"_mlps.{l}.2.weight"],), 0, s,
                        bias=g[f"_mlps.{l}.2.bias"])
            _gemm(0, 0, EPI_MUL, cur, D, (w2,), F, 0, self.dG, F, M, F, D, R=self.Dg[l], ldr=F, s=s)
            self._wgrad("w1", self.dG, F, F, self.X2[l], D, D, (g[f"_mlps.{l}.0.weight"],), 0, s,
                        bias=g[f"_mlps.{l}.0.bias"])
            _gemm(0, 0, EPI_STORE, self.dG, F, (w1,), D, 0, self.dX, D, M, D, F, s=s)
            c("ghm_ln_rows_bwd", _ptr(self.dX), _ptr(self.Hmid[l]), _ptr(self.st2[l]), _ptr(p[f"_lns_2.{l}.weight"]),
              _ptr(cur), _ptr(nxt), _ptr(self.part_ln), M, D, s)
            self._reduce_ln(g, 2, l, s)
            # attention (model.py:772-783): nxt = dHmid -> dq | dk | dv
            if self.act:
                c("ghm_attn_ext_bwd_x3_act", _ptr(self.qkv[l]), _ptr(self.P[l]),
                  None if self.Pd is None else _ptr(self.Pd[l]), _ptr(nxt), _ptr(self.dS), _ptr(self.dqkv), N, T, D,
                  T, self.scale_div, 0.0, self.act, s)
            else:
                c("ghm_attn_ext_bwd_x3", _ptr(self.qkv[l]), _ptr(self.P[l]), _ptr(nxt), _ptr(self.dS),
                  _ptr(self.dqkv), N, T, D, T, self.scale_div, 0.0, s)
            wqkv = (p[f"_queries.{l}.weight"], p[f"_keys.{l}.weight"], p[f"_values.{l}.weight"])
            gqkv = (g[f"_queries.{l}.weight"], g[f"_keys.{l}.weight"], g[f"_values.{l}.weight"])
            self._wgrad("qkv", self.dqkv, 3 * D, 3 * D, self.X1[l], D, D, gqkv, D, s)
            _gemm(0, 0, EPI_STORE, self.dqkv, 3 * D, wqkv, D, D, self.dX, D, M, D, 3 * D, s=s)
            c("ghm_ln_rows_bwd", _ptr(self.dX), _ptr(self.H[l]), _ptr(self.st1[l]), _ptr(p[f"_lns_1.{l}.weight"]),
              _ptr(nxt), _ptr(cur), _ptr(self.part_ln), M, D, s)
            self._reduce_ln(g, 1, l, s)
            yield
        s = _stream()
        # embeddings (model.py:764-765): dH0 rows summed per token id; positions over the sequences
        c("ghm_wcolsum", None, _ptr(tok), self.V, _ptr(cur), T, T, 0, M, D, _ptr(g["token_embeddings.weight"]),
          None, _ptr(self.colpart), s)
        c("ghm_colsum", _ptr(cur), N, T * D, _ptr(g["position_embeddings.weight"]), _ptr(self.colpart), s)
        self._written.update(g[k].data_ptr() for k in ("token_embeddings.weight", "position_embeddings.weight"))
