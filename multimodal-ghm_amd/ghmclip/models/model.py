"""Drop-in module API of the reference (src/ghmclip/models/model.py) on the HIP path.

Same class names, constructor signatures, parameter registration order and
state_dict keys as the reference, so ``torch.manual_seed`` yields identical
initial weights and reference checkpoints load unchanged.  The compute runs in
the native kernels (models/hip_encoder.py -> libghm_hip.so); there is no CPU
path: calling a module on CPU tensors raises.
"""
import os
import random

import numpy as np
import torch
import torch.nn as nn

from .. import _native
from .gemm_encoder import make_encoder_plan
from .hip_encoder import param_names, require_hip

__all__ = ["seed_everything", "get_activation", "EncoderTransformer", "GuidedClipLoss", "ClipLoss"]


def seed_everything(seed: int):
    """models/model.py:12-22 — same RNG calls in the same order."""
    random.seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = True


def get_activation(activation="softmax"):
    """models/model.py:121-130: the attention activation by name ("softmax",
    "relu", "gelu"; anything else raises NotImplementedError, as the reference).
    Returned as the name: the HIP attention kernels apply it (relu / gelu on the
    split-bf16 kernels, sequences of <= 96 tokens)."""
    if activation in ("softmax", "relu", "gelu"):
        return activation
    raise NotImplementedError


class _EncoderFn(torch.autograd.Function):
    """Outputs: the embedding [N, C] and, for a guided encoder, H_{l+1}[:, :, 0:V]
    of every flagged layer l (model.py:790-800) as [N, T, V] tensors."""

    @staticmethod
    def forward(ctx, module, tokens, *params):
        plan = module._plan(tokens.shape[0], tokens.shape[1], tokens.device)
        pd = dict(zip(module._names, params))
        emb = plan.forward(pd, tokens).clone()
        ctx.module, ctx.plan, ctx.gen = module, plan, plan._gen
        ctx.save_for_backward(tokens, *params)
        N, T, V = tokens.shape[0], tokens.shape[1], module.vocab_size
        guided = [plan.H[l + 1].view(N, T, -1)[:, :, :V].contiguous() for l in module._guided_layers()]
        return (emb, *guided)

    @staticmethod
    def backward(ctx, d_emb, *d_guided):
        plan = ctx.plan
        if plan._gen != ctx.gen:
            raise RuntimeError("EncoderTransformer: another forward of this module overwrote the "
                               "activations saved for backward")
        tokens, *params = ctx.saved_tensors
        names = ctx.module._names
        grads = {n: torch.empty_like(p) for n, p in zip(names, params)}
        hooks = {}
        V = ctx.module.vocab_size
        for l, dg in zip(ctx.module._guided_layers(), d_guided):
            if dg is None:
                continue
            dg = dg.contiguous().float()
            if ctx.module.n_embd == 128:
                def fn(dH, s, dg=dg):
                    _native.call("ghm_add_cols", dH.data_ptr(), dg.data_ptr(), plan.M, V, s)
            else:  # the GEMM path's residual stream has row pitch n_embd
                def fn(dH, s, dg=dg):
                    dH.view(-1, ctx.module.n_embd)[:, :V] += dg.view(-1, V)
            hooks[l] = fn
        plan.backward(dict(zip(names, params)), grads, d_emb=d_emb.contiguous().float(), tokens=tokens,
                      layer_grad=hooks)
        return (None, None, *[grads[n] for n in names])


class EncoderTransformer(nn.Module):
    """Reference: models/model.py:690-808.  Single-head full-width attention
    (n_head is stored but unused, as in the reference), no attention output
    projection, LayerNorm always applied, token-axis Linear(n_token -> 1) readout."""

    def __init__(self, n_token, num_class, n_embd=128, n_layer=12, n_guided_layer=3, n_head=4,
                 n_mlp_multiplier=4, activation="softmax", mlp=True, normalize_attn=True,
                 layernorm=True, maxnorm=False, guide=False, guide_contract=False):
        super().__init__()
        self.name = f"EncoderTF_embd={n_embd}_layer={n_layer}_head={n_head}"
        self.vocab_size = num_class
        self.context_length = n_token
        self.n_token = n_token
        self.n_embd = n_embd
        self.n_head = n_head
        self.n_layer = n_layer
        self.n_mlp_hidden = n_embd * n_mlp_multiplier
        self.activation = get_activation(activation)
        self.mlp = mlp
        self.normalize_attn = normalize_attn
        self.layernorm = layernorm
        self.maxnorm = maxnorm
        self.guide = guide
        self.n_guided_layer = n_guided_layer
        self.guided_layer_gap = n_layer // n_guided_layer
        self.guide_contract = guide_contract
        if not mlp or maxnorm or n_mlp_multiplier != 4:
            raise NotImplementedError("HIP encoder: mlp=True, maxnorm=False, n_mlp_multiplier=4 only")
        # identical construction (and so RNG) order to the reference, model.py:725-758
        self.token_embeddings = nn.Embedding(self.vocab_size, self.n_embd)
        self.position_embeddings = nn.Embedding(self.context_length, self.n_embd)
        self._queries = nn.ModuleList()
        self._keys = nn.ModuleList()
        self._values = nn.ModuleList()
        self._mlps = nn.ModuleList()
        self._lns_1 = nn.ModuleList()
        self._lns_2 = nn.ModuleList()
        self.guided_layer_flag = [False] * n_layer
        _layer_count = 0
        for i in range(n_layer):
            self._queries.append(nn.Linear(n_embd, n_embd, bias=False))
            self._keys.append(nn.Linear(n_embd, n_embd, bias=False))
            self._values.append(nn.Linear(n_embd, n_embd, bias=False))
            self._lns_1.append(nn.LayerNorm([self.n_embd]))
            self._mlps.append(nn.Sequential(nn.Linear(n_embd, self.n_mlp_hidden), nn.GELU(),
                                            nn.Linear(self.n_mlp_hidden, n_embd)))
            self._lns_2.append(nn.LayerNorm([self.n_embd]))
            if guide and _layer_count < self.n_guided_layer and (i + 1) % self.guided_layer_gap == 0:
                self.guided_layer_flag[i] = True
                _layer_count += 1
        self._read_out = nn.Linear(n_embd, num_class)
        self._out = nn.Linear(n_token, 1)
        self._names = param_names(n_layer)
        self._plans = {}
        # matrix-product mode of the HIP kernels: None -> $GHM_PRECISION or "x3";
        # "f32" exact-f32 MFMA, "x3" split-bf16 MFMA (hip_encoder.py)
        self.precision = None

    def _plan(self, n_seq, T, device):
        key = (n_seq, T, str(device), self.precision, self.activation)
        if key not in self._plans:
            self._plans.clear()  # keep one workspace set alive per module
            self._plans[key] = make_encoder_plan(self.n_layer, T, n_seq, num_class=self.vocab_size,
                                                 vocab=self.vocab_size, n_embd=self.n_embd,
                                                 normalize_attn=self.normalize_attn, device=device,
                                                 precision=self.precision, activation=self.activation)
        return self._plans[key]

    def _guided_layers(self):
        """Indices of the guided layers (model.py:751-755 flags)."""
        return [l for l, f in enumerate(self.guided_layer_flag) if f] if self.guide else []

    def forward(self, x):
        """x: LongTensor [B, n_token] on the HIP device -> (prediction [B, num_class],
        guided layers: [H_{l+1}[:, :, 0:num_class] for each flagged layer l])."""
        require_hip(x)
        B, T = x.shape
        if T != self.n_token:
            raise ValueError(f"expected {self.n_token} tokens, got {T}")
        if x.numel() and (int(x.min()) < 0 or int(x.max()) >= self.vocab_size):
            raise IndexError("token id out of range")
        tokens = x.to(torch.uint8).contiguous()
        sd = dict(self.named_parameters())
        params = [sd[n] for n in self._names]
        for prm in params:
            if prm.dtype != torch.float32 or not prm.is_contiguous():
                raise RuntimeError("HIP encoder parameters must be contiguous fp32")
        out = _EncoderFn.apply(self, tokens, *params)
        return out[0], list(out[1:])


class _ClipLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, i, K, B):
        require_hip(t)
        t = t.contiguous().float()
        i = i.contiguous().float()
        if t.shape != i.shape or t.shape[0] != B * (K + 1):
            raise ValueError(f"expected embeddings of shape [{B * (K + 1)}, C], got {tuple(t.shape)}")
        dt, di = torch.empty_like(t), torch.empty_like(i)
        out = torch.empty(2, dtype=torch.float32, device=t.device)
        s = torch.cuda.current_stream().cuda_stream
        _native.call("ghm_clip_loss", t.data_ptr(), i.data_ptr(), dt.data_ptr(), di.data_ptr(),
                     out.data_ptr(), None, None, B, K, t.shape[1], s)
        ctx.save_for_backward(dt, di)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        dt, di = ctx.saved_tensors
        return dt * g, di * g, None, None


class _GuidePenaltyFn(torch.autograd.Function):
    """mean_n sum_k penalty * ||g_k[n] - t_k[n]||_F^2 (model.py:913-924) with the
    squared differences and their gradient in libghm_hip (ghm_sqdiff_rows,
    ghm_scaled_diff)."""

    @staticmethod
    def forward(ctx, penalty, n, *gt):
        g = [x.contiguous().float() for x in gt[:n]]
        t = [x.to(g[0].device).contiguous().float() for x in gt[n:]]
        N = g[0].shape[0]
        s = torch.cuda.current_stream().cuda_stream
        rows = torch.empty(n, N, dtype=torch.float32, device=g[0].device)
        for k in range(n):
            if g[k].shape != t[k].shape:
                raise ValueError(f"guided layer {k}: {tuple(g[k].shape)} vs target {tuple(t[k].shape)}")
            _native.call("ghm_sqdiff_rows", g[k].data_ptr(), t[k].data_ptr(), rows[k].data_ptr(), N,
                         g[k].numel() // N, s)
        ctx.save_for_backward(*g, *t)
        ctx.penalty, ctx.n = penalty, n
        return (rows.sum(0) * penalty).mean()

    @staticmethod
    def backward(ctx, up):
        saved = ctx.saved_tensors
        n = ctx.n
        g, t = saved[:n], saved[n:]
        up = up.contiguous().float()
        s = torch.cuda.current_stream().cuda_stream
        out = []
        for k in range(n):
            d = torch.empty_like(g[k])
            _native.call("ghm_scaled_diff", g[k].data_ptr(), t[k].data_ptr(), up.data_ptr(),
                         2.0 * ctx.penalty / g[k].shape[0], d.data_ptr(), d.numel(), s)
            out.append(d)
        return (None, None, *out, *[None] * n)


class GuidedClipLoss(nn.Module):
    """Reference: models/model.py:867-926.  Returns (loss, guided_penalty)."""

    def __init__(self, K, batch_size, penalty=1e-4, guide=False):
        super().__init__()
        self.K = K
        self.batch_size = batch_size
        self.penalty = penalty
        self.guide = guide

    def forward(self, tmodel_outputs, imodel_outputs, targets):
        loss = _ClipLossFn.apply(tmodel_outputs[0], imodel_outputs[0], self.K, self.batch_size)
        if not self.guide:
            return loss, 0
        # :909-924 — per-sample sum of penalty * ||guided - target||_F^2 over both
        # towers' guided layers, averaged over samples
        g = list(tmodel_outputs[1]) + list(imodel_outputs[1])
        t = list(targets[0]) + list(targets[1])
        if len(g) != len(t):
            raise ValueError(f"{len(g)} guided layers but {len(t)} targets")
        loss3 = _GuidePenaltyFn.apply(self.penalty, len(g), *g, *t)
        return loss + loss3, loss3.item() / self.penalty


class ClipLoss(nn.Module):
    """Reference: models/model.py:829-865 (same objective without the guide term)."""

    def __init__(self, K, batch_size):
        super().__init__()
        self.K, self.batch_size = K, batch_size

    def forward(self, tmodel_output, imodel_output):
        return _ClipLossFn.apply(tmodel_output, imodel_output, self.K, self.batch_size)
