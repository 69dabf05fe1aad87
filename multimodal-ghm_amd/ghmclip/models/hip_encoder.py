"""HIP execution plan of one EncoderTransformer (reference: models/model.py:690-808).

An ``EncoderPlan`` owns the device workspaces of one encoder at one batch shape
and issues the native kernels (include/ghm_hip.h) on the current stream.  No
PyTorch math runs here: torch only allocates memory and provides the stream.

HBM layout (one encoder, M = n_seq * T tokens, fp32):
  H    [L+1, M, 128]   residual stream entering each layer (+ final output)
  Hmid [L,   M, 128]   residual after attention
  qkv  [L,   M, 384]   Q | K | V
  P    [L, n_seq, nkt, nkt, 16, 64] attention probabilities in the attention
                       kernel's register-native layout (nkt = ceil(T/32)), backward input
  U    [L,   M, 512]   MLP pre-activation (backward input)
  st1/st2 [L, M, 2]    LayerNorm (mean, rstd)
Backward scratch (reused across layers): dH ping-pong [2, M, 128], dqkv
[M, 384], dU [M, 512], and split-K / per-block partial buffers.
"""
import ctypes
import math

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


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def require_hip(t):
    if not (isinstance(t, torch.Tensor) and t.is_cuda and torch.version.hip):
        raise RuntimeError("ghmclip (MI355X build) runs on a HIP device only; "
                           "move the model and inputs to 'cuda' on a ROCm build of PyTorch")


class EncoderPlan:
    def __init__(self, n_layer, n_token, n_seq, num_class=10, vocab=10, n_embd=128, eps=1e-5,
                 normalize_attn=True, device="cuda", wgrad_target_blocks=1024):
        if n_embd != D_MODEL:
            raise ValueError(f"the HIP encoder is built for n_embd=128 (got {n_embd})")
        if n_token > 96:
            raise ValueError(f"the HIP attention kernels take sequences of <= 96 tokens (got {n_token})")
        if num_class > 16 or vocab > 16:
            raise ValueError("num_class / vocabulary must be <= 16")
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
        self.nkt = -(-T // 32)
        self.P = e(L, N, self.nkt, self.nkt, 16, 64)
        self.U = e(L, M, D_HIDDEN)
        self.st1 = e(L, M, 2)
        self.st2 = e(L, M, 2)
        self.emb = e(N, num_class)
        self.tokens = torch.empty(N, T, dtype=torch.uint8, device=dev)
        # backward scratch
        self.dH = e(2, M, D_MODEL)
        self.dqkv = e(M, 3 * D_MODEL)
        self.dU = e(M, D_HIDDEN)
        self.nblk = int(_native.hip_lib().ghm_token_blocks(M))
        self.part_ln = e(self.nblk, 2, D_MODEL)
        # split-K plans (A_cols x B_cols output tiles of 128x128)
        self.wg = {}
        for key, (ac, bc) in {"w2": (D_MODEL, D_HIDDEN), "w1": (D_HIDDEN, D_MODEL),
                              "qkv": (3 * D_MODEL, D_MODEL)}.items():
            tiles = (ac // 128) * (bc // 128)
            nsplit = max(1, min(int(round(wgrad_target_blocks / tiles)), (M + 1) // 2))
            tps = -(-M // nsplit)
            tps = -(-tps // 32) * 32  # multiple of the 32-token k-step
            nsplit = -(-M // tps)
            self.wg[key] = (tps, nsplit)
        max_part = max(ns * 128 * 512 if k != "qkv" else ns * 384 * 128 for k, (t, ns) in self.wg.items())
        self.part_w = e(max_part)
        self.part_b = e(max(ns * 512 for (_, ns) in self.wg.values()))
        self.part_ro = e(N * num_class * D_MODEL)
        self.part_bro = e(N * num_class)
        self.part_wout = e(N * T)
        self.part_bout = e(N)
        self.part_tok = e(N * vocab * D_MODEL)
        self.d_emb = e(N, num_class)
        self._gen = 0

    def probs_dense(self, l):
        """Layer l's attention probabilities as a dense [n_seq, T, T] tensor
        (test / inspection helper; un-permutes the native layout)."""
        nkt, T = self.nkt, self.T
        lane = torch.arange(64, device=self.device)
        r = torch.arange(16, device=self.device)
        w = torch.arange(nkt, device=self.device)
        kt = torch.arange(nkt, device=self.device)
        q = (32 * w[:, None, None, None] + (lane & 31)[None, None, None, :]).expand(nkt, nkt, 16, 64)
        key = (32 * kt[None, :, None, None] + 8 * (r >> 2)[None, None, :, None] + 4 * (lane >> 5)[None, None, None, :]
               + (r & 3)[None, None, :, None]).expand(nkt, nkt, 16, 64)
        dense = torch.zeros(self.N, 32 * nkt, 32 * nkt, device=self.device)
        dense[:, q.reshape(-1), key.reshape(-1)] = self.P[l].reshape(self.N, -1)
        return dense[:, :T, :T]

    # ------------------------------------------------------------------
    def forward(self, p, tokens=None):
        """p: dict name -> fp32 device tensor (state_dict keys).  tokens: uint8
        [n_seq, T] on the device (defaults to self.tokens).  Returns self.emb."""
        tok = self.tokens if tokens is None else tokens
        s = _stream()
        c = _native.call
        M, T, N, L = self.M, self.T, self.N, self.L
        c("ghm_embed_fwd", _ptr(tok), _ptr(p["token_embeddings.weight"]),
          _ptr(p["position_embeddings.weight"]), _ptr(self.H[0]), N, T, self.V, D_MODEL, s)
        for l in range(L):
            c("ghm_ln_qkv_fwd", _ptr(self.H[l]), _ptr(p[f"_lns_1.{l}.weight"]), _ptr(p[f"_lns_1.{l}.bias"]),
              _ptr(p[f"_queries.{l}.weight"]), _ptr(p[f"_keys.{l}.weight"]), _ptr(p[f"_values.{l}.weight"]),
              _ptr(self.qkv[l]), _ptr(self.st1[l]), M, D_MODEL, self.eps, s)
            c("ghm_attn_fwd", _ptr(self.qkv[l]), _ptr(self.H[l]), _ptr(self.Hmid[l]), _ptr(self.P[l]),
              N, T, D_MODEL, self.scale_div, s)
            c("ghm_ln_mlp_fwd", _ptr(self.Hmid[l]), _ptr(p[f"_lns_2.{l}.weight"]), _ptr(p[f"_lns_2.{l}.bias"]),
              _ptr(p[f"_mlps.{l}.0.weight"]), _ptr(p[f"_mlps.{l}.0.bias"]), _ptr(p[f"_mlps.{l}.2.weight"]),
              _ptr(p[f"_mlps.{l}.2.bias"]), _ptr(self.H[l + 1]), _ptr(self.U[l]), _ptr(self.st2[l]),
              M, D_MODEL, D_HIDDEN, self.eps, s)
        c("ghm_readout_fwd", _ptr(self.H[L]), _ptr(p["_read_out.weight"]), _ptr(p["_read_out.bias"]),
          _ptr(p["_out.weight"]), _ptr(p["_out.bias"]), _ptr(self.emb), N, T, D_MODEL, self.C, s)
        self._gen += 1
        return self.emb

    # ------------------------------------------------------------------
    def _reduce(self, part, n_split, n, dsts, s):
        n_seg = len(dsts)
        arr = (ctypes.c_void_p * 4)(*[t.data_ptr() for t in dsts], *([0] * (4 - n_seg)))
        offs = [0]
        for t in dsts:
            offs.append(offs[-1] + t.numel())
        assert offs[-1] == n, (offs, n)
        off = (ctypes.c_int64 * 5)(*offs, *([n] * (5 - len(offs))))
        _native.call("ghm_reduce_partials", _ptr(part), n_split, n, n_seg, arr, off, s)

    def backward(self, p, g, d_emb=None, tokens=None):
        """Accumulate nothing: writes d(loss)/d(param) into g[name] (fp32 device
        tensors, same keys as p).  d_emb: [n_seq, C] (defaults to self.d_emb)."""
        tok = self.tokens if tokens is None else tokens
        de = self.d_emb if d_emb is None else d_emb
        s = _stream()
        c = _native.call
        M, T, N, L, C = self.M, self.T, self.N, self.L, self.C
        cur, nxt = self.dH[0], self.dH[1]
        c("ghm_readout_bwd", _ptr(self.H[L]), _ptr(p["_read_out.weight"]), _ptr(p["_read_out.bias"]),
          _ptr(p["_out.weight"]), _ptr(de), _ptr(cur), _ptr(self.part_ro), _ptr(self.part_bro),
          _ptr(self.part_wout), _ptr(self.part_bout), N, T, D_MODEL, C, s)
        self._reduce(self.part_ro, N, C * D_MODEL, [g["_read_out.weight"]], s)
        self._reduce(self.part_bro, N, C, [g["_read_out.bias"]], s)
        self._reduce(self.part_wout, N, T, [g["_out.weight"]], s)
        self._reduce(self.part_bout, N, 1, [g["_out.bias"]], s)
        for l in reversed(range(L)):
            # MLP + LN2: cur = dH_{l+1} -> nxt = dHmid_l
            c("ghm_mlp_bwd", _ptr(cur), _ptr(self.Hmid[l]), _ptr(self.st2[l]), _ptr(p[f"_lns_2.{l}.weight"]),
              _ptr(p[f"_mlps.{l}.0.weight"]), _ptr(p[f"_mlps.{l}.2.weight"]), _ptr(self.U[l]), _ptr(self.dU),
              _ptr(nxt), _ptr(self.part_ln), M, D_MODEL, D_HIDDEN, s)
            self._reduce(self.part_ln, self.nblk, 2 * D_MODEL,
                         [g[f"_lns_2.{l}.weight"], g[f"_lns_2.{l}.bias"]], s)
            tps, ns = self.wg["w2"]  # dW2[o][hid] = sum dY[m][o] GELU(U)[m][hid]; db2 = sum dY
            c("ghm_wgrad", _ptr(cur), D_MODEL, D_MODEL, _ptr(self.U[l]), D_HIDDEN, D_HIDDEN, 1,
              None, None, None, _ptr(self.part_w), _ptr(self.part_b), M, tps, s)
            self._reduce(self.part_w, ns, D_MODEL * D_HIDDEN, [g[f"_mlps.{l}.2.weight"]], s)
            self._reduce(self.part_b, ns, D_MODEL, [g[f"_mlps.{l}.2.bias"]], s)
            tps, ns = self.wg["w1"]  # dW1[hid][in] = sum dU[m][hid] LN2(Hmid)[m][in]; db1 = sum dU
            c("ghm_wgrad", _ptr(self.dU), D_HIDDEN, D_HIDDEN, _ptr(self.Hmid[l]), D_MODEL, D_MODEL, 2,
              _ptr(self.st2[l]), _ptr(p[f"_lns_2.{l}.weight"]), _ptr(p[f"_lns_2.{l}.bias"]),
              _ptr(self.part_w), _ptr(self.part_b), M, tps, s)
            self._reduce(self.part_w, ns, D_HIDDEN * D_MODEL, [g[f"_mlps.{l}.0.weight"]], s)
            self._reduce(self.part_b, ns, D_HIDDEN, [g[f"_mlps.{l}.0.bias"]], s)
            cur, nxt = nxt, cur  # cur = dHmid_l
            c("ghm_attn_bwd", _ptr(self.qkv[l]), _ptr(self.P[l]), _ptr(cur), _ptr(self.dqkv), N, T, D_MODEL,
              self.scale_div, s)
            tps, ns = self.wg["qkv"]  # dWq|k|v[o][in] = sum dqkv[m][o] LN1(H)[m][in]
            c("ghm_wgrad", _ptr(self.dqkv), 3 * D_MODEL, 3 * D_MODEL, _ptr(self.H[l]), D_MODEL, D_MODEL, 2,
              _ptr(self.st1[l]), _ptr(p[f"_lns_1.{l}.weight"]), _ptr(p[f"_lns_1.{l}.bias"]),
              _ptr(self.part_w), None, M, tps, s)
            self._reduce(self.part_w, ns, 3 * D_MODEL * D_MODEL,
                         [g[f"_queries.{l}.weight"], g[f"_keys.{l}.weight"], g[f"_values.{l}.weight"]], s)
            c("ghm_qkv_bwd", _ptr(self.dqkv), _ptr(self.H[l]), _ptr(self.st1[l]), _ptr(p[f"_lns_1.{l}.weight"]),
              _ptr(p[f"_queries.{l}.weight"]), _ptr(p[f"_keys.{l}.weight"]), _ptr(p[f"_values.{l}.weight"]),
              _ptr(cur), _ptr(nxt), _ptr(self.part_ln), M, D_MODEL, s)
            self._reduce(self.part_ln, self.nblk, 2 * D_MODEL,
                         [g[f"_lns_1.{l}.weight"], g[f"_lns_1.{l}.bias"]], s)
            cur, nxt = nxt, cur  # cur = dH_l
        c("ghm_embed_bwd", _ptr(cur), _ptr(tok), _ptr(self.part_tok), N, T, self.V, D_MODEL, s)
        self._reduce(self.part_tok, N, self.V * D_MODEL, [g["token_embeddings.weight"]], s)
        self._reduce(cur, N, T * D_MODEL, [g["position_embeddings.weight"]], s)
