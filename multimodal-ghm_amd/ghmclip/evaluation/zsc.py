"""Zero-shot classification risk on the device (figures/eval-zsc-risk.py:62-121).

``zsc_loss(sampler, model_dicts, num_samples_list, device)`` keeps the
reference function's signature and result dict: it draws N = 30 x max(n)
shared-root text/image pairs (DoubleSampler.get_zeroshot_batch), embeds both
modalities with each encoder pair (the HIP encoder forward), and scores every
image against every class's first n text samples through the all-pairs
contraction exp(i_emb @ t_emb.T) — here the ``ghm_zsc_logits`` kernel, which
reads only the 10 x n_max prototype columns the risk uses instead of forming
the N x N matrix.  The reference embeds only total // 200 full minibatches of
200 rows (:98-105); the rows past them keep zero embeddings there, and here.

Data parallel (optional, when a process group is up): every rank draws the
same N pairs (same numpy stream) and embeds a contiguous 1/world of the rows of
both modalities; the text embeddings are all-gathered so every rank holds all
prototypes; each rank scores its own image rows; the cross-entropy sums are
all-reduced (SUM) and divided by N.  The result equals the single-process one.
"""
from collections import defaultdict

import numpy as np
import torch
import torch.nn.functional as F

from .. import _native
from ..models.hip_encoder import _ptr, _stream, require_hip

EMBED_CHUNK = 2048  # sequences per encoder forward (any size gives the same rows)
REF_MINIBATCH = 200  # eval-zsc-risk.py:98: only total // 200 full minibatches are embedded


def shard_rows(n, rank, world):
    """Contiguous [lo, hi) of n rows for `rank`, ceil(n / world) rows per rank."""
    per = -(-n // world)
    return min(n, rank * per), min(n, (rank + 1) * per), per


def gather_rows(local, n, per, group=None):
    """All-gather equal-size row shards (zero-padded to `per` rows) and return
    the first n rows of the concatenation, in rank order."""
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    dev = local.device if dist.get_backend(group) == "nccl" else torch.device("cpu")  # gloo gathers host tensors
    pad = torch.zeros(per, *local.shape[1:], dtype=local.dtype, device=dev)
    pad[:len(local)] = local
    out = torch.empty(ws * per, *local.shape[1:], dtype=local.dtype, device=dev)
    dist.all_gather_into_tensor(out, pad, group=group)
    return out[:n].to(local.device)


def _embed(model, leaves, n_valid, device, D=10):
    """Embeddings of `leaves`; rows at or past n_valid stay zero (the
    reference's torch.zeros buffer past its last full minibatch, :96-105)."""
    out = torch.zeros(len(leaves), D, dtype=torch.float32, device=device)
    with torch.no_grad():
        for a in range(0, min(n_valid, len(leaves)), EMBED_CHUNK):
            b = min(a + EMBED_CHUNK, n_valid)
            tok = torch.from_numpy(np.ascontiguousarray(leaves[a:b])).to(device)
            out[a:b] = model(tok)[0].float()
    return out


def zsc_logits(i_emb, t_emb, proto_idx, n_list):
    """[len(n_list), rows, n_class] device logits (ghm_zsc_logits).
    Every support size must lie in 1..n_proto (the kernel divides the first n
    prototypes' sum by n) and at most 8 sizes are scored per launch; the
    prototype indices must address rows of t_emb."""
    require_hip(i_emb)
    n_rows, D = i_emb.shape
    n_class, n_proto = proto_idx.shape
    n_list = [int(n) for n in n_list]
    if not 1 <= len(n_list) <= 8:
        raise ValueError(f"zsc_logits scores 1..8 support sizes per call, got {len(n_list)}")
    if any(n < 1 or n > n_proto for n in n_list):
        raise ValueError(f"support sizes {n_list} must lie in 1..{n_proto} (prototypes per class)")
    if t_emb.shape[1] != D or D > 16:
        raise ValueError(f"embedding widths {D} / {t_emb.shape[1]} must match and be <= 16")
    if proto_idx.numel() and (int(proto_idx.min()) < 0 or int(proto_idx.max()) >= t_emb.shape[0]):
        raise ValueError("prototype indices must address rows of t_emb")
    out = torch.empty(len(n_list), n_rows, n_class, dtype=torch.float32, device=i_emb.device)
    nl = torch.tensor(n_list, dtype=torch.int32, device=i_emb.device)
    ie, te = i_emb.contiguous(), t_emb.contiguous()
    pi = proto_idx.to(torch.int32).contiguous()
    _native.call("ghm_zsc_logits", _ptr(ie), n_rows, _ptr(te), D, _ptr(pi), n_class, n_proto, _ptr(nl), len(n_list),
                 _ptr(out), _stream())
    return out


def zsc_loss(sampler, model_dicts, num_samples_list, device="cuda", process_group=None):
    """figures/eval-zsc-risk.py:62-121 on the device.  Returns the same dict:
    {"num_samples_list": [...], "Bayes": [loss], name: [loss per n]}."""
    import torch.distributed as dist
    dev = torch.device(device)
    n_list = [int(n) for n in np.asarray(num_samples_list).reshape(-1)]
    total = max(n_list) * 30
    t_leaves, i_leaves, t_pp, i_pp, root = sampler.get_zeroshot_batch(batch_size=total)
    V = sampler.variable_type
    ip = np.asarray(i_pp, np.float64)
    for layer_pps in sampler.t_transition:  # :73-76
        ip = ip @ layer_pps[0]
    first = torch.from_numpy(np.asarray(t_leaves[:, 0], np.int64)).to(dev)
    res = defaultdict(list)
    res["num_samples_list"] = list(n_list)
    res["Bayes"].append(F.cross_entropy(torch.log(torch.tensor(ip, dtype=torch.float, device=dev)), first).item())
    protos = []
    for c in range(V):  # :86-91
        idx = np.nonzero(t_leaves[:, 0] == c)[0]
        if len(idx) < max(n_list):
            raise AssertionError(f"Class {c} only has {len(idx)} text samples")
        protos.append(idx[:max(n_list)])
    proto_idx = torch.from_numpy(np.stack(protos).astype(np.int32)).to(dev)
    on = dist.is_available() and dist.is_initialized() and dist.get_world_size(process_group) > 1
    ws = dist.get_world_size(process_group) if on else 1
    rank = dist.get_rank(process_group) if on else 0
    lo, hi, per = shard_rows(total, rank, ws)
    for name, (t_model, i_model) in model_dicts.items():
        t_model.eval()
        i_model.eval()
        n_valid = max(0, (total // REF_MINIBATCH) * REF_MINIBATCH - lo)
        i_emb = _embed(i_model, i_leaves[lo:hi], n_valid, dev, V)
        t_emb = _embed(t_model, t_leaves[lo:hi], n_valid, dev, V)
        if on:
            t_emb = gather_rows(t_emb, total, per, process_group)
        sums = torch.zeros(len(n_list), dtype=torch.float64, device=dev)
        if hi > lo:
            lg = zsc_logits(i_emb, t_emb, proto_idx, n_list)
            for q in range(len(n_list)):
                sums[q] = F.cross_entropy(lg[q], first[lo:hi], reduction="sum").double()
        if on:
            s = sums if dist.get_backend(process_group) == "nccl" else sums.cpu()
            dist.all_reduce(s, op=dist.ReduceOp.SUM, group=process_group)
            sums = s.to(dev)
        for q in range(len(n_list)):
            res[name].append(float(sums[q].item() / total))
    return res
