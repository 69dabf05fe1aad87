"""Determinism check: run the default CLIP step N times (eager; graph captured
after step 3 when N > 3) and print digests of the loss history, the forward
buffers of both plans and every gradient, so two runs can be compared bit for
bit to find the first tensor that differs.

    python tools/det_check.py [steps]
"""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multimodal-ghm_amd"))
import bench  # noqa: E402


def digest(t):
    return hashlib.sha1(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:10]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sampler, tr = bench.build(0, 128, 5, 0.2, 3000, "x3")
    ring = bench.make_ring(sampler, 128, 4)
    for k in range(steps):
        tr.set_tokens(ring[k % 4, 0], ring[k % 4, 1])
        tr.step()
        if k == 2 and steps > 3:
            tr.capture()
    torch.cuda.synchronize()
    h = np.asarray(tr.loss_history()[:steps])
    print("loss", digest(torch.as_tensor(h)), "params", digest(tr.pflat), f"last {h[-1]:.9f}")
    for i, plan in enumerate(tr.plans):
        for name in ("H", "Hmid", "qkv", "P", "st1", "st2", "emb", "d_emb"):
            t = getattr(plan, name, None)
            if t is not None:
                if t.dim() >= 2 and name in ("H", "Hmid", "qkv", "P", "st1", "st2"):
                    print(f"tower{i} {name}", " ".join(digest(t[l]) for l in range(t.shape[0])))
                else:
                    print(f"tower{i} {name}", digest(t))
    for i, (_, gd, _, _) in enumerate(tr.views):
        for name, g in gd.items():
            print(f"grad{i} {name}", digest(g))




def layer_snapshots(steps=1):
    """Snapshots of tower 0's backward scratch at the start of each layer's
    backward (hook on the residual-stream gradient): dH_{l+1}, and the scratch
    the previous (deeper) layer left (its qkv_bwd LN partials, dqkv, G, dU)."""
    sampler, tr = bench.build(0, 128, 5, 0.2, 3000, "x3")
    ring = bench.make_ring(sampler, 128, 4)
    plan = tr.plans[0]
    snaps = []

    def hooks(tower):
        if tower != 0:
            return None
        def mk(l):
            def fn(dH, s):
                snaps.append((l, {"dH_in": dH.clone(), "part_ln": plan.part_ln.clone(), "dqkv": plan.dqkv.clone(),
                                  "G": plan.G.clone(), "dU": plan.dU.clone(), "part_ln2": plan.part_ln2.clone()}))
            return fn
        return {l: mk(l) for l in range(plan.L)}
    tr._guide_hooks = hooks
    for k in range(steps):
        tr.set_tokens(ring[k % 4, 0], ring[k % 4, 1])
        tr.step()
    torch.cuda.synchronize()
    for l, d in snaps:
        print(f"layer {l}: " + " ".join(f"{k}={digest(v)}" for k, v in d.items()))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "layers":
        layer_snapshots(int(sys.argv[1]))
    else:
        main()
