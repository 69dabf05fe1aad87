"""Sequential conditional denoiser (CDM, BASELINE config 4) on the HIP path.

Reference: models/model.py:337-532 (ConditionalDenoiseEncoderTransformer),
:989-1041 (ConditionalGuidedLsLoss), :1152-1160 (LsLoss); trained by
training/train_sequential_DNS.py with a frozen CLIP text encoder supplying the
one conditioning token.

The denoiser is the CLIP encoder's layer stack at T = 81 image + 1 conditioning
token, so ``CdmPlan`` reuses EncoderPlan's layer kernels and adds the CDM
embedding (continuous leaf features), the Linear(d -> 1) readout and the
position-embedding gradient (csrc/ghm_cdm.hip).
"""
import ctypes
import os

import torch
import torch.nn as nn

from .. import _native
from .hip_encoder import D_HIDDEN, D_MODEL, ENCODER_PRECISIONS, EncoderPlan, default_precision, require_hip
from .vlm import EPI_GELU, EPI_MUL, EPI_RESID, EPI_SLAB, EPI_STORE, _gemm

__all__ = ["ConditionalDenoiseEncoderTransformer", "ConditionalGuidedLsLoss", "LsLoss", "CdmPlan",
           "cdm_param_names", "cdm_untrained", "CDM_UNTRAINED", "CDM_JOINT_UNTRAINED", "NoLnLayers"]

# parameters the reference never gives a gradient in sequential mode (the
# conditioning token bypasses t_embedding, _out is unused by forward): AdamW and
# clip_grad_norm_ skip them (optimizer.py:55-56)
CDM_UNTRAINED = ("t_embedding.weight", "_out.weight", "_out.bias")
# joint model (sequential=False, train_CDNS.py): the text leaves go through t_embedding
CDM_JOINT_UNTRAINED = ("_out.weight", "_out.bias")


def cdm_untrained(model):
    """Parameters the reference never gives a gradient (AdamW and clip_grad_norm_
    skip them): CDM_UNTRAINED / CDM_JOINT_UNTRAINED, and with layernorm=False the
    unused LayerNorms (model.py:470-477, 488-498)."""
    names = CDM_UNTRAINED if model.sequential else CDM_JOINT_UNTRAINED
    if not getattr(model, "layernorm", True):
        names = names + tuple(f"_lns_{k}.{l}.{w}" for k in (1, 2) for l in range(model.n_layer)
                              for w in ("weight", "bias"))
    return names


def cdm_precision(precision, joint, guide, layernorm):
    """The CDM's matrix-product mode: an explicit `precision` (or $GHM_PRECISION)
    wins; else the joint model with LayerNorm runs the LN + QKV / LN + MLP forwards
    on the f32-accurate three-way split kernels and, unguided, the rest split-bf16
    ("f32fwd": its reference curve at f32's distance, 4.66 -> 3.22 ms per step) or,
    guided (lr 1e-2, whose curve needs an f32 backward), the backward exact f32
    ("f32x6": 4.91 -> 4.37 ms, its curve inside the f32 bound); everything else
    CdmPlan's default."""
    if precision is None and joint and layernorm and "GHM_PRECISION" not in os.environ:
        return "f32x6" if guide else "f32fwd"
    return precision


class NoLnLayers:
    """The CDM layer stack with layernorm=False (model.py:470-477: Q / K / V read
    H; :488-498: H = H + mlp(H) after the attention residual).  The LayerNorm is
    fused into EncoderPlan's token-parallel kernels, so this stack runs the
    projections on the tiled GEMM instead (ghm_gemm_x3, or ghm_gemm_f32 in the f32
    mode: GELU / GELU', bias + residual and the GELU' product in its epilogues,
    split-k weight gradients with the bias sums) around the plan's own attention
    kernels (EncoderPlan._attn_fwd / _attn_bwd, every activation and length);
    the residual gradients add with ghm_add.  HBM: G, GELU'(U) [L][M][512] saved by
    the forward, dU [M][512], dX [M][128] and the split-k slabs."""

    def __init__(self, plan):
        self.plan = plan
        L, M = plan.L, plan.M
        dev = plan.device
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.f32 = plan.precision != "x3"
        self.G, self.Dg = e(L, M, D_HIDDEN), e(L, M, D_HIDDEN)
        self.dG, self.dX = e(M, D_HIDDEN), e(M, D_MODEL)
        self.nsplit = max(1, min(16, M // 256))
        self.slab = e(self.nsplit * max(D_MODEL * D_HIDDEN, 3 * D_MODEL * D_MODEL))
        self.bslab = e(self.nsplit * D_HIDDEN)

    def _gemm(self, *a, **k):
        _gemm(*a, f32=self.f32, **k)

    def _wgrad(self, A, lda, m, B, ldb, n, dst, chunk, s, bias=None):
        """dst (rows stacked by chunk) = A^T B over the M tokens (+ the bias gradient,
        the column sums of A, from the same launch), as VlmPlan._wgrad."""
        bs = None if bias is None else self.bslab
        self._gemm(1, 0, EPI_SLAB, A, lda, (B,), ldb, 0, self.slab, n, m, n, self.plan.M, C2=bs, nsplit=self.nsplit,
                   s=s)
        d = list(dst) + [None] * (3 - len(dst))
        pp = lambda t: None if t is None else _ptr(t)  # noqa: E731
        _native.call("ghm_gemm_reduce_bias", _ptr(self.slab), self.nsplit, m, n, pp(d[0]), pp(d[1]), pp(d[2]), chunk,
                     pp(bs), pp(bias), s)

    def fwd(self, p, l, s):
        pl, D, F, M = self.plan, D_MODEL, D_HIDDEN, self.plan.M
        wqkv = (p[f"_queries.{l}.weight"], p[f"_keys.{l}.weight"], p[f"_values.{l}.weight"])
        self._gemm(0, 1, EPI_STORE, pl.H[l], D, wqkv, D, D, pl.qkv[l], 3 * D, M, 3 * D, D, s=s)
        pl._attn_fwd(l, s)
        self._gemm(0, 1, EPI_GELU, pl.Hmid[l], D, (p[f"_mlps.{l}.0.weight"],), D, 0, self.G[l], F, M, F, D,
                   C2=self.Dg[l], bias=p[f"_mlps.{l}.0.bias"], s=s)
        self._gemm(0, 1, EPI_RESID, self.G[l], F, (p[f"_mlps.{l}.2.weight"],), F, 0, pl.H[l + 1], D, M, D, F,
                   bias=p[f"_mlps.{l}.2.bias"], R=pl.Hmid[l], ldr=D, s=s)

    def bwd(self, p, g, l, cur, nxt, s, layer_grad=None):
        """cur = dL/dH[l+1] in; returns (dL/dH[l], the free ping-pong buffer)."""
        pl, D, F, M = self.plan, D_MODEL, D_HIDDEN, self.plan.M
        if layer_grad and l in layer_grad:
            layer_grad[l](cur, s)
        w1, w2 = p[f"_mlps.{l}.0.weight"], p[f"_mlps.{l}.2.weight"]
        self._wgrad(cur, D, D, self.G[l], F, F, (g[f"_mlps.{l}.2.weight"],), 0, s, bias=g[f"_mlps.{l}.2.bias"])
        self._gemm(0, 0, EPI_MUL, cur, D, (w2,), F, 0, self.dG, F, M, F, D, R=self.Dg[l], ldr=F, s=s)  # dU
        self._wgrad(self.dG, F, F, pl.Hmid[l], D, D, (g[f"_mlps.{l}.0.weight"],), 0, s, bias=g[f"_mlps.{l}.0.bias"])
        self._gemm(0, 0, EPI_STORE, self.dG, F, (w1,), D, 0, self.dX, D, M, D, F, s=s)
        _native.call("ghm_add", _ptr(cur), _ptr(self.dX), _ptr(nxt), M * D, s)  # nxt = dL/dHmid[l]
        pl._attn_bwd(l, nxt, s)
        wqkv = (p[f"_queries.{l}.weight"], p[f"_keys.{l}.weight"], p[f"_values.{l}.weight"])
        gqkv = (g[f"_queries.{l}.weight"], g[f"_keys.{l}.weight"], g[f"_values.{l}.weight"])
        self._wgrad(pl.dqkv, 3 * D, 3 * D, pl.H[l], D, D, gqkv, D, s)
        self._gemm(0, 0, EPI_STORE, pl.dqkv, 3 * D, wqkv, D, D, self.dX, D, M, D, 3 * D, s=s)
        _native.call("ghm_add", _ptr(nxt), _ptr(self.dX), _ptr(cur), M * D, s)  # cur = dL/dH[l]
        return cur, nxt


def cdm_param_names(n_layer):
    """state_dict keys of ConditionalDenoiseEncoderTransformer in registration order
    (model.py:382-402: the ModuleLists are registered before t_embedding)."""
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
    names += ["t_embedding.weight", "_read_out.weight", "_read_out.bias", "_out.weight", "_out.bias"]
    return names


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class CdmPlan(EncoderPlan):
    """Device workspaces of one ConditionalDenoiseEncoderTransformer at one batch
    shape: the EncoderPlan layer buffers at T = n_token plus the readout/loss ones.
    HBM layout: H [L+1][N*T][128] etc. as EncoderPlan; pred, dpred [N][T_img];
    readout partials part_rw [N][128], part_rb [N] (distinct from EncoderPlan's
    split-K buffers part_w1 / part_b1)."""

    def __init__(self, n_layer, n_token, n_i_token, n_seq, num_class=10, n_embd=128, eps=1e-5,
                 normalize_attn=True, device="cuda", precision=None, joint=False, activation="softmax",
                 layernorm=True):
        if precision is None:
            # exact f32 by default where split-bf16 leaves the parity bound: the joint
            # model (T = 162), and relu / gelu attention without
            # LayerNorm (un-normalised scores on un-normalised activations: an MLP
            # weight gradient 6.2e-4 off at x3 against the 5e-4 bound)
            f32_default = joint or (activation != "softmax" and not layernorm)
            precision = default_precision("f32" if f32_default else "x3", allowed=ENCODER_PRECISIONS)
        # attention activation (model.py:485 through get_activation, :121-130): relu / gelu
        # on the split-bf16 attention kernels (EncoderPlan: one-sequence up to 96 tokens,
        # the multi-workgroup ghm_attn_ext_*_act past 96, the joint model's 162)
        if precision in ("f32fwd", "f32x6") and not layernorm:
            raise NotImplementedError(f"precision {precision}: the LayerNorm-fused forward kernels (layernorm=True)")
        super().__init__(n_layer, n_token, n_seq, num_class=num_class, vocab=num_class, n_embd=n_embd, eps=eps,
                         normalize_attn=normalize_attn, device=device, precision=precision, activation=activation)
        if not 1 <= n_i_token <= n_token:
            raise ValueError("n_i_token must be in [1, n_token]")
        self.Ti = n_i_token
        self.joint = joint
        if joint:  # text leaves as tokens through t_embedding (sequential=False)
            self.tok = torch.empty(n_seq, n_token - n_i_token, dtype=torch.uint8, device=self.device)
            lib = _native.hip_lib()
            self.wpart = torch.empty(lib.ghm_wcolsum_part_elems(n_seq * (n_token - n_i_token), D_MODEL, num_class),
                                     dtype=torch.float32, device=self.device)
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)  # noqa: E731
        # layernorm=False: the layer stack on the GEMM path (NoLnLayers)
        self.layernorm = bool(layernorm)
        self.noln = None if self.layernorm else NoLnLayers(self)
        self.pred = e(n_seq, n_i_token)
        self.dpred = e(n_seq, n_i_token)
        self.part_rw = e(n_seq, D_MODEL)
        self.part_rb = e(n_seq)

    def forward(self, p, z, cond, cond_ld, split=True):
        """z: f32 [N, T_img] noisy observations; cond: f32 [N, T - T_img, cond_ld]
        conditioning features (first V used).  Returns self.pred [N, T_img]."""
        s = _stream()
        if self.pack is not None and split and self.layernorm:
            self.split_weights(p, s)
        if self.joint:  # cond unused: self.tok holds the text leaves
            _native.call("ghm_cdm_embed_joint_fwd", _ptr(z), _ptr(self.tok), _ptr(p["t_embedding.weight"]),
                         _ptr(p["position_embeddings.weight"]), _ptr(self.H[0]), self.N, self.T, self.Ti, self.C,
                         D_MODEL, s)
        else:
            _native.call("ghm_cdm_embed_fwd", _ptr(z), _ptr(cond) if cond is not None else None, cond_ld,
                         _ptr(p["position_embeddings.weight"]), _ptr(self.H[0]), self.N, self.T, self.Ti, self.C,
                         D_MODEL, s)
        self.layers_fwd(p, s)
        _native.call("ghm_cdm_readout_fwd", _ptr(self.H[self.L]), _ptr(p["_read_out.weight"]),
                     _ptr(p["_read_out.bias"]), _ptr(self.pred), self.N, self.T, self.Ti, D_MODEL, s)
        self._gen += 1
        return self.pred

    def layers_fwd(self, p, s):
        if self.layernorm:
            return super().layers_fwd(p, s)
        for l in range(self.L):
            self.noln.fwd(p, l, s)

    def layers_bwd(self, p, g, jobs, s, layer_grad=None):
        if self.layernorm:
            return super().layers_bwd(p, g, jobs, s, layer_grad)
        cur, nxt = self.dH[0], self.dH[1]
        for l in reversed(range(self.L)):
            cur, nxt = self.noln.bwd(p, g, l, cur, nxt, s, layer_grad)
        return cur

    def backward(self, p, g, dpred=None, layer_grad=None):
        """Writes d(loss)/d(param) into g[name] for every trained parameter (not
        CDM_UNTRAINED); dpred [N, T_img] defaults to self.dpred.  Returns dL/dH_0
        [N*T, 128] (its conditioning rows give the gradient of cond)."""
        s = _stream()
        J = self._job
        dp = self.dpred if dpred is None else dpred
        cur = self.dH[0]
        _native.call("ghm_cdm_readout_bwd", _ptr(self.H[self.L]), _ptr(p["_read_out.weight"]), _ptr(dp), _ptr(cur),
                     _ptr(self.part_rw), _ptr(self.part_rb), self.N, self.T, self.Ti, D_MODEL, s)
        jobs = [J(self.part_rw, self.N, [g["_read_out.weight"]]), J(self.part_rb, self.N, [g["_read_out.bias"]])]
        cur = self.layers_bwd(p, g, jobs, s, layer_grad)
        jobs.append(J(cur, self.N, [g["position_embeddings.weight"]]))
        self._flush(jobs, s)
        if self.joint:  # d t_embedding[v] = sum of the text rows of dH_0 holding token v
            Tt = self.T - self.Ti
            _native.call("ghm_wcolsum", None, _ptr(self.tok), self.V, _ptr(cur), Tt, self.T, self.Ti, self.N * Tt,
                         D_MODEL, _ptr(g["t_embedding.weight"]), None, _ptr(self.wpart), s)
        return cur


class _CdmFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, module, xt, zi, *params):
        N, T2 = zi.shape
        T1 = xt.shape[1]
        plan = module._plan(N, T1 + T2, T2, zi.device)
        pd = dict(zip(module._names, params))
        z = zi.contiguous().float()
        if plan.joint:
            plan.tok.copy_(xt.to(torch.uint8))
            pred = plan.forward(pd, z, None, 0).clone()
        else:
            cond = xt.contiguous().float()
            pred = plan.forward(pd, z, cond, cond.shape[2]).clone()
        ctx.module, ctx.plan, ctx.gen = module, plan, plan._gen
        ctx.T1 = T1
        ctx.save_for_backward(*params)
        return pred

    @staticmethod
    def backward(ctx, dpred):
        plan = ctx.plan
        if plan._gen != ctx.gen:
            raise RuntimeError("ConditionalDenoiseEncoderTransformer: another forward of this module "
                               "overwrote the activations saved for backward")
        params = ctx.saved_tensors
        names = ctx.module._names
        untrained = cdm_untrained(ctx.module)
        trained = [n not in untrained for n in names]
        grads = {n: torch.empty_like(p) for n, p, t in zip(names, params, trained) if t}
        dH0 = plan.backward(dict(zip(names, params)), grads, dpred=dpred.contiguous().float())
        d_xt = None
        if ctx.needs_input_grad[1] and not plan.joint:
            V = ctx.module.vocab_size
            d_xt = torch.zeros(plan.N, ctx.T1, ctx.module.vocab_size, dtype=torch.float32, device=dH0.device)
            d_xt.copy_(dH0.view(plan.N, plan.T, D_MODEL)[:, plan.Ti:, :V])
        return (None, d_xt, None, *[grads.get(n) for n in names])


class ConditionalDenoiseEncoderTransformer(nn.Module):
    """Reference: models/model.py:337-532.  Same constructor, parameter creation
    order (so torch.manual_seed gives identical weights) and state_dict keys.
    The HIP path covers the configurations the CDM experiments train: sequential
    (exp_cdm_{standard,shallow}TF.sh: a frozen-CLIP feature token, T = 82; guided:
    eg_sdns.sh) and joint (exp_cdm_jointtrain.sh / exp_cdm_guidedTF.sh: the 81 text
    leaves through t_embedding, T = 162, on the split-bf16 attention for sequences
    past 96 tokens); softmax attention, LayerNorm, MLP, no causal mask, n_embd 128.
    guide=True: the guided penalties run inside the fused CdmTrainer step."""

    def __init__(self, n_token, n_i_token, num_class, n_embd=128, n_layer=12, n_guided_layers=(3, 3), n_head=4,
                 n_mlp_hidden=512, activation="softmax", mlp=True, normalize_attn=True, auto_regressive=False,
                 sequential=False, layernorm=True, maxnorm=False, guide=False, sigma=1):
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
        self.maxnorm = maxnorm
        self.auto_regressive = auto_regressive
        self.guide = guide
        self.n_t_guided_layer = n_guided_layers[0]
        self.n_i_guided_layer = n_guided_layers[1]
        self.guided_layer_gap = n_layer // (n_guided_layers[1] * 2 + 1)
        self.sigma = sigma
        if activation not in ("softmax", "relu", "gelu") or not mlp or maxnorm or auto_regressive:
            raise NotImplementedError("HIP CDM: softmax / relu / gelu attention, mlp=True, maxnorm=False, "
                                      "auto_regressive=False")
        if guide and self.guided_layer_gap == 0:
            raise ValueError("guide=True needs n_layer >= 2 * n_guided_layers[1] + 1 (model.py:372)")
        if n_mlp_hidden != 4 * n_embd:
            raise NotImplementedError("HIP CDM: n_mlp_hidden = 4 * n_embd")
        # construction (RNG) order of the reference, model.py:382-402
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
        counter = 0
        for i in range(n_layer):  # guided-layer flags of model.py:392-416
            if guide and counter < 2 * self.n_i_guided_layer + 1 and (i + 1) % self.guided_layer_gap == 0:
                self.i_guided_layer_flag[i] = True
                if counter < self.n_t_guided_layer or (counter == self.n_i_guided_layer - 1
                                                       and self.n_t_guided_layer < self.n_i_guided_layer):
                    self.t_guided_layer_flag[i] = True
                counter += 1
        for _ in range(n_layer):
            self._queries.append(nn.Linear(n_embd, n_embd, bias=False))
            self._keys.append(nn.Linear(n_embd, n_embd, bias=False))
            self._values.append(nn.Linear(n_embd, n_embd, bias=False))
            self._lns_1.append(nn.LayerNorm([self.n_embd]))
            self._mlps.append(nn.Sequential(nn.Linear(n_embd, n_mlp_hidden), nn.GELU(),
                                            nn.Linear(n_mlp_hidden, n_embd)))
            self._lns_2.append(nn.LayerNorm([self.n_embd]))
        self._read_out = nn.Linear(n_embd, 1)
        self._out = nn.Linear(n_token, 1)
        self._names = cdm_param_names(n_layer)
        self._plans = {}
        self.precision = None  # None -> $GHM_PRECISION or "x3" (hip_encoder.py)

    def _plan(self, n_seq, T, T_img, device):
        key = (n_seq, T, T_img, str(device), self.precision)
        if key not in self._plans:
            self._plans.clear()
            self._plans[key] = CdmPlan(self.n_layer, T, T_img, n_seq, num_class=self.vocab_size,
                                       n_embd=self.n_embd, normalize_attn=self.normalize_attn, device=device,
                                       precision=cdm_precision(self.precision, not self.sequential,
                                                               getattr(self, "guide", False), self.layernorm),
                                       joint=not self.sequential, activation=self.activation,
                                       layernorm=self.layernorm)
        return self._plans[key]

    def forward(self, xt, zi):
        """sequential: xt = conditioning features [B, T1, num_class] (the frozen CLIP
        text embedding, unsqueezed); joint (sequential=False): xt = text leaves
        [B, T1] (token ids).  zi: noisy image observations [B, T2] (float).
        Returns (denoised predictions [B, T2], guided layers [[], []])."""
        require_hip(zi)
        B, T2 = zi.shape
        if not self.sequential:
            if xt.dim() != 2 or xt.shape[0] != B:
                raise ValueError(f"expected text leaves of shape [{B}, T1], got {tuple(xt.shape)}")
            if xt.numel() and (int(xt.min()) < 0 or int(xt.max()) >= self.vocab_size):
                raise IndexError("token id out of range")
        elif xt.dim() != 3 or xt.shape[0] != B or xt.shape[2] != self.vocab_size:
            raise ValueError(f"expected xt of shape [{B}, T1, {self.vocab_size}], got {tuple(xt.shape)}")
        if T2 != self.n_i_token or xt.shape[1] + T2 != self.n_token:
            raise ValueError(f"expected {self.n_i_token} image + {self.n_token - self.n_i_token} conditioning tokens")
        sd = dict(self.named_parameters())
        params = [sd[n] for n in self._names]
        for prm in params:
            if prm.dtype != torch.float32 or not prm.is_contiguous():
                raise RuntimeError("HIP CDM parameters must be contiguous fp32")
        pred = _CdmFn.apply(self, xt, zi, *params)
        return pred, [[], []]


def cdm_guide_blocks(model, t_tree, i_tree, V):
    """The guided outputs of the CDM (model.py:458-527) as blocks of the residual
    stream, each paired with the target that the trainer lines up against it, in
    ConditionalGuidedLsLoss order (:1023-1040).  t_tree / i_tree = (L, C).  Returns
    {layer l: [block, ...]}, block = (src, tok0, ntok, col, moff, ext) with src
    "i" (image messages [n][3][n_nodes][V] of ghm_bp_dns_msgs: planes hd, qd, bu;
    data_random_GHM.py:551-592), "t" (joint model: text BP_CLS messages
    [n][n_total][V] of ghm_bp_cls, depth Lt-1 first) or "c" (sequential model,
    train_sequential_DNS.py:145: the frozen CLIP text embedding [n][V] that is also
    the conditioning token, for every text-guided layer)."""
    Lt, Ct = t_tree
    Li, Ci = i_tree
    Ti, Tt = Ci ** Li, Ct ** Lt
    n_nodes = sum(Ci ** d for d in range(1, Li + 1)) + 1

    def node0(depth):  # first node of a depth in the ghm_bp_dns_msgs order
        return n_nodes - 1 if depth == 0 else sum(Ci ** e for e in range(1, depth))

    def img(plane, depth, col, ext):
        return ("i", 0, Ti, col, (plane * n_nodes + node0(depth)) * V, ext)

    nt = model.n_t_guided_layer
    blocks = {}
    ig = [l for l, f in enumerate(model.i_guided_layer_flag) if f]
    tg = [l for l, f in enumerate(model.t_guided_layer_flag) if f]
    if len(ig) != 2 * Li + 1 or (not model.sequential and len(tg) > Lt):
        raise ValueError("guided layers do not match the trees (n_guided_layers vs tree depths)")
    for k, l in enumerate(ig):
        if k <= Li:  # downward h / q (root: hd / bu), :505-511
            depth, ext = Li - k, Ci ** k
            b = [img(0, depth, k * V, ext), img(1 if depth else 2, depth, (nt + k) * V, ext)]
        else:  # upward h / q / u, :512-518
            j = k - Li - 1
            depth = j + 1
            ext = Ci ** (Li - depth)
            b = [img(0, depth, (2 * Li + 1 - k) * V, ext), img(1, depth, (nt + 2 * Li + 1 - k) * V, ext),
                 img(2, depth, (2 * nt + j) * V, ext)]
        blocks.setdefault(l, []).extend(b)
    if model.sequential:  # text id blocks (:522-527) of the one conditioning token vs the CLIP feature
        for k, l in enumerate(tg):
            blocks.setdefault(l, []).append(("c", Ti, model.n_token - Ti, k * V, 0, 1))
        return blocks
    off = 0
    nodes = Tt // Ct
    for k, l in enumerate(tg):  # text id blocks, :522-527 against BP_CLS depth Lt-1-k
        blocks.setdefault(l, []).append(("t", Ti, Tt, k * V, off * V, Ct ** (k + 1)))
        off += nodes
        nodes //= Ct
    return blocks


class LsLoss(nn.Module):
    """models/model.py:1152-1160: mean over samples of the summed squared error."""

    def forward(self, inputs, targets):
        return torch.sum(torch.pow(inputs - targets, 2), dim=1).mean()


class ConditionalGuidedLsLoss(nn.Module):
    """models/model.py:989-1041: returns (loss, 0, 0, 0, 0); the guide=True branch is
    computed by CdmTrainer (fused, on the device)."""

    def __init__(self, penalty=1e-4, guide=False):
        super().__init__()
        self.penalty = penalty
        self.guide = guide

    def forward(self, inputs, targets, verbose=False):
        if self.guide:
            raise NotImplementedError("guided CDM penalties run inside the fused CdmTrainer step "
                                      "(training/cdm_trainer.py, train_CDNS.py --guide=True), not on module outputs")
        loss = torch.sum(torch.pow(inputs[0] - targets[0], 2), dim=1)
        return loss.mean(), 0, 0, 0, 0
