"""HIP execution plan of one EncoderTransformer (reference: models/model.py:690-808).

An ``EncoderPlan`` owns the device workspaces of one encoder at one batch shape
and issues the native kernels (include/ghm_hip.h) on the current stream.  No
PyTorch math runs here: torch only allocates memory and provides the stream.

HBM layout (one encoder, M = n_seq * T tokens, fp32):
  H    [L+1, M, 128]   residual stream entering each layer (+ final output)
  Hmid [L,   M, 128]   residual after attention
  qkv  [L,   M, 384]   Q | K | V
  P    [L, n_seq, 96, 96] attention probabilities, dense and padded (backward input);
       [L, n_seq, 192, 192] for sequences past 96 tokens (x3 only)
  G/Dg [L,   M, 512]   GELU(U) and GELU'(U) of the MLP pre-activation U (f32 mode only:
       the x3 forward saves nothing of the MLP; its backward recomputes U and writes
       G [M, 512] as per-layer scratch for dW2)
  st1/st2 [L, M, 2]    LayerNorm (mean, rstd)
  pack [L, 983040] bf16 (precision "x3" only): per-layer pre-split weight planes
Backward scratch (reused across layers): dH ping-pong [2, M, 128], dqkv
[M, 384], dU [M, 512], and split-K / per-block partial buffers.
"""
import ctypes
import math
import os

import torch

from .. import _native

D_MODEL = 128
D_HIDDEN = 512


def param_names(n_layer):
    """state_dict keys of the reference EncoderTransformer, registration order
    (model.py:725-758)."""
    names = ["token_embeddings.weight", "position_embeddings.weight"]
    names += [f"_queries.{l}.weight" for l in range(n_layer)]
    names += [f"_keys.{l}.weight" for l in range(n_layer)]
    names += [f"_values.{l}.weight" for l in range(n_layer)]
    for l in range(n_layer):
        names += [f"_mlps.{l}.0.weight", f"_mlps.{l}.0.bias", f"_mlps.{l}.2.weight", f"_mlps.{l}.2.bias"]
    for l in range(n_layer):
        names += [f"_lns_1.{l}.weight", f"_lns_1.{l}.bias"]
    for l in range(n_layer):
        names += [f"_lns_2.{l}.weight", f"_lns_2.{l}.bias"]
    names += ["_read_out.weight", "_read_out.bias", "_out.weight", "_out.bias"]
    return names


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def perm32(q):
    """k-slot q of a 32-group of the MLP backward's split G / dU planes holds unit
    perm32(q) (csrc/ghm_x3.hip perm32)."""
    base, r = q & ~31, q & 31
    return base + (4 * ((r >> 3) & 3) + (r & 3) if (r & 7) < 4 else 16 + 4 * ((r >> 3) & 3) + (r & 3))


def inv_perm32_index(device):
    """index tensor idx with natural[:, u] = permuted[:, idx[u]] over 512 units."""
    inv = [0] * D_HIDDEN
    for q in range(D_HIDDEN):
        inv[perm32(q)] = q
    return torch.tensor(inv, dtype=torch.long, device=device)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


PRECISIONS = ("f32", "x3")
# the encoder plans (n_embd = 128) also take "f32fwd" (the forward at f32 accuracy,
# the backward split-bf16) and "f32x6" (the forward's LN + QKV / LN + MLP on the
# three-way split kernels, the backward exact f32)
ENCODER_PRECISIONS = PRECISIONS + ("f32fwd", "f32x6")


def default_precision(fallback="x3", allowed=PRECISIONS):
    """GHM_PRECISION env var: "x3" (split-bf16 MFMA, fp32-accurate to ~1e-5
    relative per product; the CLIP and VLM default: the reference code's whole
    3001-step CLIP run within 1.4e-6) or "f32" (exact-f32 MFMA for the
    projections and the MLP; the joint CDM default, whose lr-1e-2 guided run
    amplifies x3 rounding past the reference's own thread-count spread,
    DESIGN.md §2)."""
    p = os.environ.get("GHM_PRECISION", fallback)
    if p not in allowed:
        raise ValueError(f"GHM_PRECISION must be one of {allowed} (got {p!r})")
    return p


def forward_stages(precision, env=None):
    """The forward stages an encoder plan keeps at f32 accuracy, as a frozenset of
    qkv / attn / mlp (the exact-f32 kernels) and qkv6 / mlp6 (three-way split
    operands, six bf16 MFMAs per product: 2e-6 from float64 where the f32 kernel is
    at 1e-6 and x3 at 1e-5); the stages not named run split-bf16 x3.  "x3": none;
    "f32": all three exact; "f32x6": qkv6, attn, mlp6 (with the exact-f32
    backward); "f32fwd" (split-bf16 backward): $GHM_F32FWD (env: a mapping standing
    in for os.environ), default qkv6,mlp6.  The guided 3001-step CLIP run needs
    both projections' stages at f32 accuracy (worst ratio to its bound: qkv,mlp
    0.377, all three 0.359; mlp alone 4.96, attn + mlp 4.44, qkv + attn 4.22,
    profiles/r6_f32mix_curves.txt); qkv6,mlp6 0.499 at 4.72 ms per guided step
    against 5.44-5.68 for qkv,mlp (profiles/r6_x6_curves.txt, r6_x6_ab.txt)."""
    if precision == "x3":
        return frozenset()
    if precision == "f32":
        return frozenset({"qkv", "attn", "mlp"})
    if precision == "f32x6":
        return frozenset({"qkv6", "attn", "mlp6"})
    if precision != "f32fwd":
        raise ValueError(f"precision must be one of {ENCODER_PRECISIONS}")
    env = os.environ if env is None else env
    parts = {q for q in env.get("GHM_F32FWD", "qkv6,mlp6").split(",") if q}
    if not parts <= {"qkv", "qkv6", "attn", "mlp", "mlp6"} or {"mlp", "mlp6"} <= parts or {"qkv", "qkv6"} <= parts:
        raise ValueError(f"GHM_F32FWD: comma list of qkv or qkv6 / attn / mlp or mlp6 (got {sorted(parts)})")
    return frozenset(parts)


def require_hip(t):
    if not (isinstance(t, torch.Tensor) and t.is_cuda and torch.version.hip):
        raise RuntimeError("ghmclip (MI355X build) runs on a HIP device only; "
                           "move the model and inputs to 'cuda' on a ROCm build of PyTorch")


class EncoderPlan:
    def __init__(self, n_layer, n_token, n_seq, num_class=10, vocab=10, n_embd=128, eps=1e-5,
                 normalize_attn=True, device="cuda", wgrad_target_blocks=256, precision=None,
                 wgrad_min_tokens=None, defer_reduce=False, activation="softmax", ln_presplit=None):
        """ln_presplit (x3; $GHM_LN_PRESPLIT=1, default off): the LN1 / LN2 forwards
        also write the split rows they multiply as bf16 (hi, lo) planes, which the
        dWq|k|v / dW1 weight gradients then read directly (ghm_wgrad_x3p) instead of
        re-normalising and splitting H / Hmid per tile.  Faster alone (dW1 44.1 ->
        39.4, dWq|k|v 35.8 -> 31.5 us) and slower in the step (4.10 -> 4.20 ms: the
        planes add 530 MB of writes per step, profiles/r6_lnps2_ab.txt).
        defer_reduce: every layer keeps its own parameter-gradient partial
        buffers and backward() reduces all of them at its end in batched launches
        of up to 32 jobs (2 launches per encoder instead of one per layer), as a
        fully parallel, bandwidth-bound pass instead of L short latency-bound ones."""
        if n_embd != D_MODEL:
            raise ValueError(f"the HIP encoder is built for n_embd=128 (got {n_embd})")
        if num_class != 10 or vocab > 16:
            raise ValueError("the HIP readout is built for num_class == 10 and a vocabulary <= 16")
        self.precision = default_precision(allowed=ENCODER_PRECISIONS) if precision is None else precision
        if self.precision not in ENCODER_PRECISIONS:
            raise ValueError(f"precision must be one of {ENCODER_PRECISIONS}")
        self.fwd_x3 = self.precision == "x3"
        self.bwd_x3 = self.precision in ("x3", "f32fwd")
        self.fwd_f32 = forward_stages(self.precision)
        # mlp6 / qkv6: the LN2 + MLP / LN1 + QKV forward on three-way split operands
        # (ghm_ln_mlp_fwd_x6 / ghm_ln_qkv_fwd_x6: near the exact-f32 level, on the bf16
        # pipe), the weights' third planes in pack3
        self.mlp6 = "mlp6" in self.fwd_f32
        self.qkv6 = "qkv6" in self.fwd_f32
        if n_token > 192:
            raise ValueError(f"the HIP attention kernels take sequences of <= 192 tokens (got {n_token})")
        # sequences past 96 tokens (the joint CDM's 162) run on ghm_attn_ext_*_x3 with
        # P / dS padded to 192; precision "f32" there takes the exact-f32 attention of
        # _attn_fwd_f32 / _attn_bwd_f32 (fp32 library products: a validation mode that
        # separates the split-bf16 rounding from the curve's chaos)
        self.long_attn = n_token > 96
        pad = 192 if self.long_attn else 96
        # attention activation (model.py:121-130): softmax, or elementwise relu / gelu
        # on every attention kernel: the one-sequence ones up to 96 tokens
        # (ghm_attn_{fwd,bwd}_act exact f32, ghm_attn_{fwd,bwd}_x3_act split-bf16), the
        # multi-workgroup ones past 96 (ghm_attn_ext_{fwd,bwd}_x3_act, which every
        # precision's long attention uses)
        acts = {"softmax": 0, "relu": 1, "gelu": 2}
        if activation not in acts:
            raise NotImplementedError(f"attention activation {activation!r}")
        self.act = acts[activation]
        self.L, self.T, self.N, self.C, self.V = n_layer, n_token, n_seq, num_class, vocab
        self.M = M = n_seq * n_token
        self.eps = float(eps)
        # reference: attn / np.sqrt(n_embd) (model.py:779-780) — a true division
        self.scale_div = float(math.sqrt(n_embd)) if normalize_attn else 1.0
        self.device = torch.device(device)
        L, T, N, f32 = n_layer, n_token, n_seq, torch.float32
        dev = self.device
        e = lambda *s: torch.empty(*s, dtype=f32, device=dev)  # noqa: E731
        self.H = e(L + 1, M, D_MODEL)
        self.Hmid = e(L, M, D_MODEL)
        self.qkv = e(L, M, 3 * D_MODEL)
        self.P = torch.zeros(L, N, pad, pad, dtype=f32, device=dev)
        # gelu attention: GELU'(scores) saved beside P for the backward
        self.Pd = torch.zeros(L, N, pad, pad, dtype=f32, device=dev) if self.act == 2 else None
        # x3: the MLP forward saves nothing and its backward recomputes U
        self.mlp_rc = self.bwd_x3
        # past 96 tokens the f32 plan runs the attention core on the split-bf16
        # ghm_attn_ext kernels (the joint CDM's curves stay inside the reference's
        # own thread-count spread with them: DESIGN.md §2); GHM_LONG_ATTN=f32
        # selects the exact-f32 torch validation path instead
        self.attn_f32 = (self.long_attn and self.precision == "f32"
                         and os.environ.get("GHM_LONG_ATTN", "x3") == "f32")
        if self.attn_f32 and self.act:
            raise NotImplementedError("GHM_LONG_ATTN=f32 (the exact torch validation attention) is softmax only")
        # x3 weight gradients on the LDS-DMA ring kernel (ghm_wgrad_ring_x3, producer /
        # consumer waves) instead of ghm_wgrad_x3: $GHM_WGRAD_RING bit mask, 1 | 2 = dW2
        # and dW1 (the MLP backward then writes G / dU as pre-split planes), 4 = dWq|k|v.
        # Default 0: isolated the ring is faster (33.3 / 39.9 / 32.7 vs 42.3 / 45.3 /
        # 35.8 us) but the two-tower step slower (4.19-4.21 vs 4.05-4.09 ms, r5_ring4:
        # its 130-150 KB of LDS hold a whole CU)
        ring = int(os.environ.get("GHM_WGRAD_RING", "0")) if self.bwd_x3 else 0
        self.wgrad_ring = bool(ring & 3)      # dW2 / dW1 on the ring, G / dU pre-split
        self.wgrad_ring_qkv = bool(ring & 4)  # dWq|k|v on the ring
        if self.mlp_rc:  # backward scratch (k_mlp_bwd_rc_x3 -> dW2): f32 [M][512], or the
            # bf16 hi / lo planes [2][M][512] of the ring path in the same bytes
            # (f32fwd: the f32 forward saves no G / GELU' either)
            self.G, self.Dg = e(M, D_HIDDEN), None
        else:
            self.G, self.Dg = e(L, M, D_HIDDEN), e(L, M, D_HIDDEN)
        self.st1 = e(L, M, 2)
        self.st2 = e(L, M, 2)
        self.emb = e(N, num_class)
        self.tokens = self.token_buf = torch.empty(N, T, dtype=torch.uint8, device=dev)
        # backward scratch
        self.dH = e(2, M, D_MODEL)
        self.dqkv = e(M, 3 * D_MODEL)
        self.dU = e(M, D_HIDDEN)
        self.dS = torch.zeros(N, pad, pad, dtype=f32, device=dev)
        self.nblk = int(_native.hip_lib().ghm_token_blocks(M))
        self.nblk_rc = int(_native.hip_lib().ghm_mlp_bwd_rc_x3_blocks(M))
        # split-K plans (A_cols x B_cols output tiles of 128x128): ~wgrad_target_blocks
        # workgroups of at least wgrad_min_tokens tokens per split (measured on the
        # CDM's 10.5 K tokens: 32 -> 3.01 ms/step, 256 -> 3.09, 512 -> 3.50: the
        # extra parallelism outweighs the larger partial reduction)
        wgrad_target_blocks = int(os.environ.get("GHM_WGRAD_BLOCKS", wgrad_target_blocks))
        if wgrad_min_tokens is None:
            wgrad_min_tokens = int(os.environ.get("GHM_WGRAD_MIN_TOKENS", "32"))
        self.wg = {}
        for key, (ac, bc) in {"w2": (D_MODEL, D_HIDDEN), "w1": (D_HIDDEN, D_MODEL),
                              "qkv": (3 * D_MODEL, D_MODEL)}.items():
            tiles = (ac // 128) * (bc // 128)
            nsplit = max(1, min(int(round(wgrad_target_blocks / tiles)), M // max(32, wgrad_min_tokens)))
            tps = -(-M // nsplit)
            tps = -(-tps // 32) * 32  # multiple of the 32-token k-step
            nsplit = -(-M // tps)
            self.wg[key] = (tps, nsplit)
        # one partial buffer per pending reduction job of a layer: flushed once per
        # layer, or (defer_reduce) one set per layer, flushed at the end of backward()
        self.defer_reduce = bool(defer_reduce)
        nl = L if self.defer_reduce else 1
        self.lpart = {"w2": e(nl, self.wg["w2"][1] * D_MODEL * D_HIDDEN),
                      "w1": e(nl, self.wg["w1"][1] * D_HIDDEN * D_MODEL),
                      "wq": e(nl, self.wg["qkv"][1] * 3 * D_MODEL * D_MODEL),
                      "b2": e(nl, self.wg["w2"][1] * D_MODEL),
                      "b1": e(nl, self.wg["w1"][1] * D_HIDDEN),
                      "ln": e(nl, self.nblk * 2 * D_MODEL),
                      "ln2": e(nl, max(self.nblk, self.nblk_rc) * 2 * D_MODEL)}
        self.part_w2, self.part_w1, self.part_wq = self.lpart["w2"][0], self.lpart["w1"][0], self.lpart["wq"][0]
        self.part_b2, self.part_b1 = self.lpart["b2"][0], self.lpart["b1"][0]
        self.part_ln = self.lpart["ln"][0].view(self.nblk, 2, D_MODEL)
        self.part_ln2 = self.lpart["ln2"][0].view(max(self.nblk, self.nblk_rc), 2, D_MODEL)
        self.part_w = self.part_w2  # (kbench / legacy name)
        self.part_b = self.part_b1
        self.part_ro = e(N * num_class * D_MODEL)
        self.part_bro = e(N * num_class)
        self.part_wout = e(N * T)
        self.part_bout = e(N)
        lib = _native.hip_lib()
        # embedding backward scratch: token sums by id (ghm_wcolsum), then the
        # position gradient's sum over sequences (ghm_colsum), one after the other
        self.part_emb = e(max(lib.ghm_wcolsum_part_elems(M, D_MODEL, vocab),
                              lib.ghm_colsum_part_elems(N, T * D_MODEL),
                              lib.ghm_embed_bwd_part_elems(T, vocab)))
        self.d_emb = e(N, num_class)
        self.pack = None
        if self.bwd_x3:
            npk = int(_native.GHM_SPLIT_PACK_ELEMS)
            self.pack = torch.empty(L, npk, dtype=torch.bfloat16, device=dev)
        self.pack3 = (torch.empty(L, int(_native.GHM_SPLIT3_PACK_ELEMS), dtype=torch.bfloat16, device=dev)
                      if self.mlp6 or self.qkv6 else None)
        if self.pack is None and self.pack3 is not None:  # the x6 kernels read the hi / lo planes too
            self.pack = torch.empty(L, int(_native.GHM_SPLIT_PACK_ELEMS), dtype=torch.bfloat16, device=dev)
        # pre-split LN outputs: xs[l][0] = LN1(H_l), xs[l][1] = LN2(Hmid_l), each the hi
        # plane [M][128] then the lo plane (bf16: the bytes of one f32 plane)
        if ln_presplit is None:
            ln_presplit = os.environ.get("GHM_LN_PRESPLIT", "0") == "1"
        self.ln_presplit = bool(ln_presplit) and self.precision == "x3"
        # G for dW2 as natural-order bf16 planes from the MLP backward (split_out 2,
        # ghm_wgrad_x3p): $GHM_G_PRESPLIT=1 (x3, not with the ring weight gradients)
        self.g_presplit = (self.ln_presplit and not self.wgrad_ring
                           and os.environ.get("GHM_G_PRESPLIT", "0") == "1")
        self.xs = (torch.empty(L, 2, 2, M, D_MODEL, dtype=torch.bfloat16, device=dev) if self.ln_presplit
                   else None)
        self._gen = 0

    def mlp_scratch_f32(self, name="G"):
        """The MLP backward's G or dU scratch as f32 [M][512] in natural column
        order (inspection / tests): the ring path stores them as bf16 hi / lo
        planes with the columns of each 32-group in perm32 order."""
        t = getattr(self, name)
        if name == "G" and getattr(self, "g_presplit", False):  # natural-order (hi, lo) planes
            planes = t.view(torch.bfloat16).view(2, self.M, D_HIDDEN).float()
            return planes[0] + planes[1]
        if not self.wgrad_ring:
            return t
        planes = t.view(torch.bfloat16).view(2, self.M, D_HIDDEN).float()
        v = planes[0] + planes[1]
        return v[:, inv_perm32_index(v.device)]

    def probs_dense(self, l):
        """Layer l's attention probabilities [n_seq, T, T] (inspection helper)."""
        return self.P[l, :, :self.T, :self.T]

    # ------------------------------------------------------------------
    def forward(self, p, tokens=None, split=True):
        """p: dict name -> fp32 device tensor (state_dict keys).  tokens: uint8
        [n_seq, T] on the device (defaults to self.tokens).  Returns self.emb.
        split=False reuses the weight packs of the previous forward (frozen weights)."""
        for _ in self.forward_iter(p, tokens, split):
            pass
        return self.emb

    def forward_iter(self, p, tokens=None, split=True):
        """forward() as a generator that yields after the embedding, after each
        layer and after the readout; every launch goes to the stream current at
        the time it is issued (so a caller can interleave two encoders' launch
        sequences on two streams, ClipTrainer)."""
        tok = self.tokens if tokens is None else tokens
        c = _native.call
        T, N, L = self.T, self.N, self.L
        s = _stream()
        if self.pack is not None and split:
            self.split_weights(p, s)
        c("ghm_embed_fwd", _ptr(tok), _ptr(p["token_embeddings.weight"]),
          _ptr(p["position_embeddings.weight"]), _ptr(self.H[0]), N, T, self.V, D_MODEL, s)
        yield
        for l in range(L):
            self._layer_fwd(p, l, _stream())
            yield
        c("ghm_readout_fwd", _ptr(self.H[L]), _ptr(p["_read_out.weight"]), _ptr(p["_read_out.bias"]),
          _ptr(p["_out.weight"]), _ptr(p["_out.bias"]), _ptr(self.emb), N, T, D_MODEL, self.C, _stream())
        self._gen += 1

    def layers_fwd(self, p, s):
        """The n_layer encoder layers (model.py:769-800) from H[0] to H[L]:
        LN1+QKV, attention+residual, LN2+MLP+residual per layer."""
        for l in range(self.L):
            self._layer_fwd(p, l, s)

    def _layer_fwd(self, p, l, s):
        c = _native.call
        M = self.M
        pk = _ptr(self.pack[l]) if self.pack is not None else None
        if self.qkv6:
            c("ghm_ln_qkv_fwd_x6", _ptr(self.H[l]), _ptr(p[f"_lns_1.{l}.weight"]), _ptr(p[f"_lns_1.{l}.bias"]), pk,
              _ptr(self.pack3[l]), _ptr(self.qkv[l]), _ptr(self.st1[l]), M, D_MODEL, self.eps, s)
        elif "qkv" in self.fwd_f32:
            c("ghm_ln_qkv_fwd", _ptr(self.H[l]), _ptr(p[f"_lns_1.{l}.weight"]), _ptr(p[f"_lns_1.{l}.bias"]),
              _ptr(p[f"_queries.{l}.weight"]), _ptr(p[f"_keys.{l}.weight"]), _ptr(p[f"_values.{l}.weight"]),
              _ptr(self.qkv[l]), _ptr(self.st1[l]), M, D_MODEL, self.eps, s)
        elif self.ln_presplit:
            c("ghm_ln_qkv_fwd_x3s", _ptr(self.H[l]), _ptr(p[f"_lns_1.{l}.weight"]),
              _ptr(p[f"_lns_1.{l}.bias"]), pk, _ptr(self.qkv[l]), _ptr(self.st1[l]), _ptr(self.xs[l, 0]), M,
              D_MODEL, self.eps, s)
        else:
            c("ghm_ln_qkv_fwd_x3", _ptr(self.H[l]), _ptr(p[f"_lns_1.{l}.weight"]),
              _ptr(p[f"_lns_1.{l}.bias"]), pk, _ptr(self.qkv[l]), _ptr(self.st1[l]), M, D_MODEL, self.eps, s)
        self._attn_fwd(l, s)
        if self.mlp6:
            c("ghm_ln_mlp_fwd_x6", _ptr(self.Hmid[l]), _ptr(p[f"_lns_2.{l}.weight"]), _ptr(p[f"_lns_2.{l}.bias"]), pk,
              _ptr(self.pack3[l]), _ptr(p[f"_mlps.{l}.0.bias"]), _ptr(p[f"_mlps.{l}.2.bias"]), _ptr(self.H[l + 1]),
              _ptr(self.st2[l]), None if self.mlp_rc else _ptr(self.G[l]), None if self.mlp_rc else _ptr(self.Dg[l]),
              M, D_MODEL, D_HIDDEN, self.eps, s)
            return
        if "mlp" in self.fwd_f32:
            c("ghm_ln_mlp_fwd", _ptr(self.Hmid[l]), _ptr(p[f"_lns_2.{l}.weight"]), _ptr(p[f"_lns_2.{l}.bias"]),
              _ptr(p[f"_mlps.{l}.0.weight"]), _ptr(p[f"_mlps.{l}.0.bias"]), _ptr(p[f"_mlps.{l}.2.weight"]),
              _ptr(p[f"_mlps.{l}.2.bias"]), _ptr(self.H[l + 1]), None if self.mlp_rc else _ptr(self.G[l]),
              None if self.mlp_rc else _ptr(self.Dg[l]), _ptr(self.st2[l]), M, D_MODEL, D_HIDDEN, self.eps, s)
            return
        mlp_args = (_ptr(self.Hmid[l]), _ptr(p[f"_lns_2.{l}.weight"]), _ptr(p[f"_lns_2.{l}.bias"]), pk,
                    _ptr(p[f"_mlps.{l}.0.bias"]), _ptr(p[f"_mlps.{l}.2.bias"]), _ptr(self.H[l + 1]),
                    _ptr(self.st2[l]))
        if self.ln_presplit:
            c("ghm_ln_mlp_fwd_x3bs", *mlp_args, _ptr(self.xs[l, 1]), M, D_MODEL, D_HIDDEN, self.eps, s)
        else:
            c("ghm_ln_mlp_fwd_x3b", *mlp_args, M, D_MODEL, D_HIDDEN, self.eps, s)

    def _attn_fwd(self, l, s):
        """Layer l's attention + residual (model.py:776-783): Hmid[l] = H[l] + A V
        from qkv[l], P (and Pd) saved for the backward."""
        c = _native.call
        N, T = self.N, self.T
        if self.attn_f32:
            self._attn_fwd_f32(l)
        elif self.long_attn:  # unmasked (n_prefix = T), plain residual (dbl = 0)
            self._attn_ext_fwd(l, s)
        elif "attn" not in self.fwd_f32:
            if self.act:
                c("ghm_attn_fwd_x3_act", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]), _ptr(self.P[l]),
                  None if self.Pd is None else _ptr(self.Pd[l]), N, T, D_MODEL, self.scale_div, self.act, s)
            else:
                c("ghm_attn_fwd_x3", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]), _ptr(self.P[l]),
                  N, T, D_MODEL, self.scale_div, s)
        elif self.act:
            c("ghm_attn_fwd_act", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]), _ptr(self.P[l]),
              None if self.Pd is None else _ptr(self.Pd[l]), N, T, D_MODEL, self.scale_div, self.act, s)
        else:
            c("ghm_attn_fwd", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]), _ptr(self.P[l]),
              N, T, D_MODEL, self.scale_div, s)

    def _attn_bwd(self, l, cur, s):
        """Backward of _attn_fwd: dqkv from cur = dL/dHmid[l] (the residual term
        stays the caller's)."""
        c = _native.call
        N, T = self.N, self.T
        x3 = self.bwd_x3
        if self.attn_f32:
            self._attn_bwd_f32(l, cur)
        elif self.long_attn:
            self._attn_ext_bwd(l, cur, s)
        elif self.act and x3:
            c("ghm_attn_bwd_x3_act", _ptr(self.qkv[l]), _ptr(self.P[l]),
              None if self.Pd is None else _ptr(self.Pd[l]), _ptr(cur), _ptr(self.dqkv), N, T, D_MODEL,
              self.scale_div, self.act, s)
        elif self.act:
            c("ghm_attn_bwd_act", _ptr(self.qkv[l]), _ptr(self.P[l]),
              None if self.Pd is None else _ptr(self.Pd[l]), _ptr(cur), _ptr(self.dS), _ptr(self.dqkv), N, T,
              D_MODEL, self.scale_div, self.act, s)
        else:
            c("ghm_attn_bwd_x3" if x3 else "ghm_attn_bwd", _ptr(self.qkv[l]), _ptr(self.P[l]), _ptr(cur),
              _ptr(self.dS), _ptr(self.dqkv), N, T, D_MODEL, self.scale_div, s)

    def _attn_ext_fwd(self, l, s):
        """Attention past 96 tokens on the multi-workgroup split-bf16 kernels:
        unmasked (n_prefix = T), plain residual (dbl = 0); relu / gelu via the _act
        variants."""
        N, T = self.N, self.T
        if self.act:
            _native.call("ghm_attn_ext_fwd_x3_act", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]),
                         _ptr(self.P[l]), None if self.Pd is None else _ptr(self.Pd[l]), N, T, D_MODEL, T,
                         self.scale_div, 0.0, self.act, s)
        else:
            _native.call("ghm_attn_ext_fwd_x3", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]),
                         _ptr(self.P[l]), N, T, D_MODEL, T, self.scale_div, 0.0, s)

    def _attn_ext_bwd(self, l, cur, s):
        N, T = self.N, self.T
        if self.act:
            _native.call("ghm_attn_ext_bwd_x3_act", _ptr(self.qkv[l]), _ptr(self.P[l]),
                         None if self.Pd is None else _ptr(self.Pd[l]), _ptr(cur), _ptr(self.dS), _ptr(self.dqkv),
                         N, T, D_MODEL, T, self.scale_div, 0.0, self.act, s)
        else:
            _native.call("ghm_attn_ext_bwd_x3", _ptr(self.qkv[l]), _ptr(self.P[l]), _ptr(cur), _ptr(self.dS),
                         _ptr(self.dqkv), N, T, D_MODEL, T, self.scale_div, 0.0, s)

    def _attn_fwd_f32(self, l):
        """Exact-f32 single-head attention past 96 tokens (model.py:489-497 of the
        joint CDM: softmax(QK^T / sqrt(d)) V, plain residual), on the current stream:
        Hmid = H + P V, P saved (dense, padded) for the backward."""
        N, T = self.N, self.T
        q = self.qkv[l].view(N, T, 3 * D_MODEL)
        Q, K, V = q[..., :D_MODEL], q[..., D_MODEL:2 * D_MODEL], q[..., 2 * D_MODEL:]
        A = torch.softmax(torch.bmm(Q, K.transpose(1, 2)) / self.scale_div, dim=-1)
        self.P[l, :, :T, :T] = A
        torch.baddbmm(self.H[l].view(N, T, D_MODEL), A, V, out=self.Hmid[l].view(N, T, D_MODEL))

    def _attn_bwd_f32(self, l, dHmid):
        """Backward of _attn_fwd_f32 into dqkv = [dQ | dK | dV] (the residual's
        gradient stays in dHmid, as ghm_attn_bwd)."""
        N, T = self.N, self.T
        q = self.qkv[l].view(N, T, 3 * D_MODEL)
        Q, K, V = q[..., :D_MODEL], q[..., D_MODEL:2 * D_MODEL], q[..., 2 * D_MODEL:]
        A = self.P[l, :, :T, :T]
        dO = dHmid.view(N, T, D_MODEL)
        dq = self.dqkv.view(N, T, 3 * D_MODEL)
        dA = torch.bmm(dO, V.transpose(1, 2))
        dS = A * (dA - (dA * A).sum(-1, keepdim=True)) / self.scale_div
        dq[..., :D_MODEL] = torch.bmm(dS, K)
        dq[..., D_MODEL:2 * D_MODEL] = torch.bmm(dS.transpose(1, 2), Q)
        dq[..., 2 * D_MODEL:] = torch.bmm(A.transpose(1, 2), dO)

    def split_weights(self, p, s=None):
        """Write every layer's pre-split bf16 weight pack (precision "x3")."""
        s = _stream() if s is None else s
        jobs = []
        for l in range(self.L):
            j = _native.SplitJob()
            j.Wq = p[f"_queries.{l}.weight"].data_ptr()
            j.Wk = p[f"_keys.{l}.weight"].data_ptr()
            j.Wv = p[f"_values.{l}.weight"].data_ptr()
            j.W1 = p[f"_mlps.{l}.0.weight"].data_ptr()
            j.W2 = p[f"_mlps.{l}.2.weight"].data_ptr()
            j.pack = self.pack[l].data_ptr()
            jobs.append(j)
        for a in range(0, len(jobs), 16):
            chunk = jobs[a:a + 16]
            _native.call("ghm_split_weights", (_native.SplitJob * len(chunk))(*chunk), len(chunk), s)
        if self.pack3 is not None:  # the weights' third planes for the x6 kernels
            for j, l in zip(jobs, range(self.L)):
                j.pack = self.pack3[l].data_ptr()
            for a in range(0, len(jobs), 16):
                chunk = jobs[a:a + 16]
                _native.call("ghm_split3_weights", (_native.SplitJob * len(chunk))(*chunk), len(chunk), s)

    # ------------------------------------------------------------------
    @staticmethod
    def _job(part, n_split, dsts):
        j = _native.ReduceJob()
        j.part = part.data_ptr()
        j.n_split = n_split
        j.n_seg = len(dsts)
        offs = [0]
        for t in dsts:
            offs.append(offs[-1] + t.numel())
        j.n = offs[-1]
        for k, t in enumerate(dsts):
            j.dst[k] = t.data_ptr()
        for k in range(5):
            j.off[k] = offs[min(k, len(dsts))]
        return j

    def _lp(self, key, l):
        """Layer l's partial buffer `key` (the shared one unless defer_reduce)."""
        return self.lpart[key][l if self.defer_reduce else 0]

    def _flush(self, jobs, s):
        for a in range(0, len(jobs), 32):
            chunk = jobs[a:a + 32]
            arr = (_native.ReduceJob * len(chunk))(*chunk)
            _native.call("ghm_reduce_batch", arr, len(chunk), s)
        jobs.clear()

    def _reduce(self, part, n_split, n, dsts, s):
        j = self._job(part, n_split, dsts)
        assert j.n == n
        self._flush([j], s)

    def backward(self, p, g, d_emb=None, tokens=None, layer_grad=None):
        """Accumulate nothing: writes d(loss)/d(param) into g[name] (fp32 device
        tensors, same keys as p).  d_emb: [n_seq, C] (defaults to self.d_emb).
        layer_grad: optional {layer l: fn(dH, stream)} — adds a loss term's gradient
        w.r.t. the residual stream H[l+1] leaving layer l (guided layers,
        model.py:790-800) before that layer's backward runs.
        Parameter-gradient partials are reduced by one batched launch per layer."""
        for _ in self.backward_iter(p, g, d_emb, tokens, layer_grad):
            pass

    def backward_iter(self, p, g, d_emb=None, tokens=None, layer_grad=None, clip=None):
        """backward() as a generator yielding after the readout backward and after
        each layer (launches on the stream current when each is issued).
        clip = (t_emb, i_emb, tower, B, K): the CLIP trainer's readout backward,
        which recomputes this tower's rows of d(loss)/d(emb) from both towers'
        embeddings (ghm_readout_bwd_clip) instead of reading d_emb."""
        tok = self.tokens if tokens is None else tokens
        de = self.d_emb if d_emb is None else d_emb
        c = _native.call
        J = self._job
        T, N, L, C = self.T, self.N, self.L, self.C
        cur = self.dH[0]
        jobs = []
        self.pending = jobs  # flush_pending() reduces what is queued so far (data-parallel buckets)
        ro = (_ptr(self.H[L]), _ptr(p["_read_out.weight"]), _ptr(p["_read_out.bias"]), _ptr(p["_out.weight"]))
        parts = (_ptr(cur), _ptr(self.part_ro), _ptr(self.part_bro), _ptr(self.part_wout), _ptr(self.part_bout))
        if clip is None:
            c("ghm_readout_bwd", *ro, _ptr(de), *parts, N, T, D_MODEL, C, _stream())
        else:
            te, ie, tower, B, K = clip
            c("ghm_readout_bwd_clip", *ro, _ptr(te), _ptr(ie), tower, B, K, _ptr(de), *parts, N, T, D_MODEL, C,
              _stream())
        jobs += [J(self.part_ro, N, [g["_read_out.weight"]]), J(self.part_bro, N, [g["_read_out.bias"]]),
                 J(self.part_wout, N, [g["_out.weight"]]), J(self.part_bout, N, [g["_out.bias"]])]
        yield
        cur, nxt = self.dH[0], self.dH[1]
        for l in reversed(range(self.L)):
            cur, nxt = self._layer_bwd(p, g, l, cur, nxt, jobs, _stream(), layer_grad)
            yield
        s = _stream()
        # embeddings (model.py:765 via autograd): dH0 rows summed by token id,
        # and over the sequences for the positions
        if self.V == 10:  # one pass over dH0 for both; their partials join the final reduction
            c("ghm_embed_bwd_part", _ptr(cur), _ptr(tok), N, T, self.V, D_MODEL, _ptr(self.part_emb), s)
            S = int(_native.hip_lib().ghm_embed_bwd_splits())
            ntok = S * T * self.V * D_MODEL
            jobs += [J(self.part_emb, S * T, [g["token_embeddings.weight"]]),
                     J(self.part_emb[ntok:], S, [g["position_embeddings.weight"]])]
            self._flush(jobs, s)
        else:
            self._flush(jobs, s)
            c("ghm_wcolsum", None, _ptr(tok), self.V, _ptr(cur), self.M, self.M, 0, self.M, D_MODEL,
              _ptr(g["token_embeddings.weight"]), None, _ptr(self.part_emb), s)
            c("ghm_colsum", _ptr(cur), N, T * D_MODEL, _ptr(g["position_embeddings.weight"]), _ptr(self.part_emb), s)

    def flush_pending(self):
        """Reduce the parameter-gradient partials queued by the running
        backward_iter so far (on the current stream): those gradients are final
        from here on."""
        self._flush(self.pending, _stream())

    def queued_grad_ptrs(self):
        """Addresses of the parameter gradients whose partials the running
        backward_iter has queued so far (final once flush_pending() has run)."""
        return {j.dst[i] for j in self.pending for i in range(j.n_seg)}

    def layers_bwd(self, p, g, jobs, s, layer_grad=None):
        """Backward of the n_layer encoder layers from dH[0] (= dL/dH_L, written by
        the caller's readout backward) down to dL/dH_0, which is returned (one of
        the dH ping-pong buffers).  Parameter-gradient partials are reduced by one
        batched launch per layer (pending jobs in `jobs` are flushed with them)."""
        cur, nxt = self.dH[0], self.dH[1]
        for l in reversed(range(self.L)):
            cur, nxt = self._layer_bwd(p, g, l, cur, nxt, jobs, s, layer_grad)
        return cur

    def _layer_bwd(self, p, g, l, cur, nxt, jobs, s, layer_grad=None):
        """One layer's backward: cur = dL/dH_{l+1} in, returns (dL/dH_l, the free
        ping-pong buffer)."""
        c = _native.call
        J = self._job
        M = self.M
        x3 = self.bwd_x3
        wgrad = "ghm_wgrad_x3" if x3 else "ghm_wgrad"
        P_ln, P_ln2 = self._lp("ln", l), self._lp("ln2", l)
        P_w2, P_w1, P_wq = self._lp("w2", l), self._lp("w1", l), self._lp("wq", l)
        P_b2, P_b1 = self._lp("b2", l), self._lp("b1", l)
        if True:
            if layer_grad and l in layer_grad:
                layer_grad[l](cur, s)
            # MLP + LN2: cur = dH_{l+1} -> nxt = dHmid_l
            if x3:  # recomputes U; writes G (scratch) and dU
                args = (_ptr(cur), _ptr(self.Hmid[l]), _ptr(self.st2[l]), _ptr(p[f"_lns_2.{l}.weight"]),
                        _ptr(p[f"_lns_2.{l}.bias"]), _ptr(self.pack[l]), _ptr(p[f"_mlps.{l}.0.bias"]),
                        _ptr(self.G), _ptr(self.dU), _ptr(nxt), _ptr(P_ln2), M, D_MODEL, D_HIDDEN,
                        2 if self.g_presplit else int(self.wgrad_ring))
                if getattr(self, "stamps", None) is not None:  # bench.py's in-graph timing
                    c("ghm_mlp_bwd_rc_x3_stamped", *args, _ptr(self.stamps[l]), self.stamp_twin, s)
                else:
                    c("ghm_mlp_bwd_rc_x3", *args, s)
            else:
                c("ghm_mlp_bwd", _ptr(cur), _ptr(self.Hmid[l]), _ptr(self.st2[l]), _ptr(p[f"_lns_2.{l}.weight"]),
                  _ptr(p[f"_mlps.{l}.0.weight"]), _ptr(p[f"_mlps.{l}.2.weight"]), _ptr(self.Dg[l]), _ptr(self.dU),
                  _ptr(nxt), _ptr(P_ln2), M, D_MODEL, D_HIDDEN, s)
            nb2 = self.nblk_rc if (x3 and self.mlp_rc) else self.nblk
            jobs.append(J(P_ln2, nb2, [g[f"_lns_2.{l}.weight"], g[f"_lns_2.{l}.bias"]]))
            tps, ns = self.wg["w2"]  # dW2[o][hid] = sum dY[m][o] G[m][hid]; db2 = sum dY
            if self.g_presplit:  # dY f32 x G as the MLP backward split it (natural order)
                c("ghm_wgrad_x3p", _ptr(cur), D_MODEL, D_MODEL, _ptr(self.G), D_HIDDEN, D_HIDDEN, M * D_HIDDEN,
                  _ptr(P_w2), _ptr(P_b2), M, tps, s)
            elif self.wgrad_ring:  # dY f32 (format 0) x G pre-split (format 2)
                c("ghm_wgrad_ring_x3", _ptr(cur), D_MODEL, D_MODEL, 0, 0, _ptr(self.G), D_HIDDEN, D_HIDDEN, 2,
                  M * D_HIDDEN, None, None, None, _ptr(P_w2), _ptr(P_b2), M, tps, s)
            else:
                c(wgrad, _ptr(cur), D_MODEL, D_MODEL, _ptr(self.G if self.mlp_rc else self.G[l]), D_HIDDEN,
                  D_HIDDEN, 0, None, None, None, _ptr(P_w2), _ptr(P_b2), M, tps, s)
            jobs += [J(P_w2, ns, [g[f"_mlps.{l}.2.weight"]]), J(P_b2, ns, [g[f"_mlps.{l}.2.bias"]])]
            tps, ns = self.wg["w1"]  # dW1[hid][in] = sum dU[m][hid] LN2(Hmid)[m][in]; db1 = sum dU
            if self.wgrad_ring:  # dU pre-split (format 2) x LN2(Hmid) (format 1)
                c("ghm_wgrad_ring_x3", _ptr(self.dU), D_HIDDEN, D_HIDDEN, 2, M * D_HIDDEN, _ptr(self.Hmid[l]),
                  D_MODEL, D_MODEL, 1, 0, _ptr(self.st2[l]), _ptr(p[f"_lns_2.{l}.weight"]),
                  _ptr(p[f"_lns_2.{l}.bias"]), _ptr(P_w1), _ptr(P_b1), M, tps, s)
            elif x3 and self.ln_presplit:  # dU (f32) x LN2(Hmid) as the forward split it
                c("ghm_wgrad_x3p", _ptr(self.dU), D_HIDDEN, D_HIDDEN, _ptr(self.xs[l, 1]), D_MODEL, D_MODEL,
                  M * D_MODEL, _ptr(P_w1), _ptr(P_b1), M, tps, s)
            else:
                c(wgrad, _ptr(self.dU), D_HIDDEN, D_HIDDEN, _ptr(self.Hmid[l]), D_MODEL, D_MODEL, 2,
                  _ptr(self.st2[l]), _ptr(p[f"_lns_2.{l}.weight"]), _ptr(p[f"_lns_2.{l}.bias"]),
                  _ptr(P_w1), _ptr(P_b1), M, tps, s)
            jobs += [J(P_w1, ns, [g[f"_mlps.{l}.0.weight"]]), J(P_b1, ns, [g[f"_mlps.{l}.0.bias"]])]
            cur, nxt = nxt, cur  # cur = dHmid_l
            self._attn_bwd(l, cur, s)
            tps, ns = self.wg["qkv"]  # dWq|k|v[o][in] = sum dqkv[m][o] LN1(H)[m][in]
            if self.wgrad_ring_qkv:  # dqkv f32 (format 0) x LN1(H) (format 1)
                c("ghm_wgrad_ring_x3", _ptr(self.dqkv), 3 * D_MODEL, 3 * D_MODEL, 0, 0, _ptr(self.H[l]), D_MODEL,
                  D_MODEL, 1, 0, _ptr(self.st1[l]), _ptr(p[f"_lns_1.{l}.weight"]), _ptr(p[f"_lns_1.{l}.bias"]),
                  _ptr(P_wq), None, M, tps, s)
            elif x3 and self.ln_presplit:  # dqkv (f32) x LN1(H) as the forward split it
                c("ghm_wgrad_x3p", _ptr(self.dqkv), 3 * D_MODEL, 3 * D_MODEL, _ptr(self.xs[l, 0]), D_MODEL, D_MODEL,
                  M * D_MODEL, _ptr(P_wq), None, M, tps, s)
            else:
                c(wgrad, _ptr(self.dqkv), 3 * D_MODEL, 3 * D_MODEL, _ptr(self.H[l]), D_MODEL, D_MODEL, 2,
                  _ptr(self.st1[l]), _ptr(p[f"_lns_1.{l}.weight"]), _ptr(p[f"_lns_1.{l}.bias"]),
                  _ptr(P_wq), None, M, tps, s)
            jobs.append(J(P_wq, ns, [g[f"_queries.{l}.weight"], g[f"_keys.{l}.weight"],
                                             g[f"_values.{l}.weight"]]))
            if x3:
                c("ghm_qkv_bwd_x3", _ptr(self.dqkv), _ptr(self.H[l]), _ptr(self.st1[l]), _ptr(p[f"_lns_1.{l}.weight"]),
                  _ptr(self.pack[l]), _ptr(cur), _ptr(nxt), _ptr(P_ln), M, D_MODEL, self.eps, s)
            else:
                c("ghm_qkv_bwd", _ptr(self.dqkv), _ptr(self.H[l]), _ptr(self.st1[l]), _ptr(p[f"_lns_1.{l}.weight"]),
                  _ptr(p[f"_queries.{l}.weight"]), _ptr(p[f"_keys.{l}.weight"]), _ptr(p[f"_values.{l}.weight"]),
                  _ptr(cur), _ptr(nxt), _ptr(P_ln), M, D_MODEL, s)
            jobs.append(J(P_ln, self.nblk, [g[f"_lns_1.{l}.weight"], g[f"_lns_1.{l}.bias"]]))
            if not self.defer_reduce:
                self._flush(jobs, s)  # every partial buffer is reused by the next layer
            cur, nxt = nxt, cur  # cur = dH_l
        return cur, nxt
