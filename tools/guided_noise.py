"""Diagnostic (not product code): which op group's rounding does the guided CLIP
run (exp_clip_guidedTF.sh) amplify?  Runs the guided trainer for N steps,
eagerly, and after one kernel group's launches multiplies that group's output by
(1 + eps*u), u ~ U(-1, 1) per element (eps = 2^-23: one ulp-level rounding
difference per element per launch), then writes every run's loss history to
gpurun_out/guided_noise.npz for comparison against the reference's CPU runs.

Usage: python tools/guided_noise.py STEPS PRECISION GROUP[,GROUP...]
GROUP: none, qkv_f, attn_f, P, mlp_f, readout, dloss, readout_b, mlp_b, dU, attn_b,
qkv_b, guide_b, targets, grads, params."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "multimodal-ghm_amd"))
from ghmclip import _native  # noqa: E402
from test_gpu_parity import _guided_trainer  # noqa: E402

# kernel -> [(argument index of an output, group)] (f32 and x3 entry points)
OUTS = {
    "ghm_ln_qkv_fwd": [(6, "qkv_f")], "ghm_ln_qkv_fwd_x3": [(4, "qkv_f")],
    "ghm_attn_fwd": [(2, "attn_f"), (3, "P")], "ghm_attn_fwd_x3": [(2, "attn_f"), (3, "P")],
    "ghm_ln_mlp_fwd": [(7, "mlp_f")], "ghm_ln_mlp_fwd_x3b": [(6, "mlp_f")],
    "ghm_readout_fwd": [(5, "readout")],
    "ghm_clip_loss": [(2, "dloss"), (3, "dloss")],
    "ghm_readout_bwd": [(5, "readout_b")],
    "ghm_mlp_bwd": [(8, "mlp_b"), (7, "dU")], "ghm_mlp_bwd_rc_x3": [(9, "mlp_b"), (8, "dU")],
    "ghm_attn_bwd": [(4, "attn_b")], "ghm_attn_bwd_x3": [(4, "attn_b")],
    "ghm_qkv_bwd": [(8, "qkv_b")], "ghm_qkv_bwd_x3": [(6, "qkv_b")],
    "ghm_guide_bwd": [(2, "guide_b")],
    "ghm_bp_cls": [(2, "targets")],
    "ghm_adamw": [(0, "params")],
}
PRE = {"ghm_clip_prepare": [(0, "grads")]}  # perturbed before the launch


def run(steps, precision, groups, eps=2.0 ** -23, seed=1):
    sampler, tr = _guided_trainer(5, 128, precision)
    reg = {}
    for pl in tr.plans:
        for t in list(pl.H) + list(pl.Hmid) + list(pl.qkv) + list(pl.P) + [pl.dH[0], pl.dH[1], pl.dqkv,
                                                                            pl.dU, pl.emb, pl.d_emb]:
            reg[t.data_ptr()] = t
        reg[pl.G.data_ptr()] = pl.G
    for t in [tr.gflat, tr.pflat] + list(tr.gmsgs):
        reg[t.data_ptr()] = t
    gen = torch.Generator(device="cuda").manual_seed(seed)
    real = _native.call

    def noise(name, args, table):
        for idx, grp in table.get(name, ()):
            if grp in groups:
                a = args[idx]
                ptr = a.value if isinstance(a, ctypes.c_void_p) else int(a)
                t = reg[ptr]
                u = torch.rand(t.shape, device=t.device, generator=gen) * 2 - 1
                t.mul_(1 + eps * u)

    def call(name, *args):
        noise(name, args, PRE)
        real(name, *args)
        noise(name, args, OUTS)
    _native.call = call
    try:
        for _ in range(steps):
            tl, _, il, _ = sampler.draw_numpy(128)
            tr.set_tokens(torch.from_numpy(tl), torch.from_numpy(il))
            tr.step()
        torch.cuda.synchronize()
    finally:
        _native.call = real
    return tr.loss_history()


def main():
    steps, precision = int(sys.argv[1]), sys.argv[2]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = os.path.join(ROOT, "gpurun_out", f"guided_noise_{precision}.npz")
    res = dict(np.load(out)) if os.path.exists(out) else {}
    for g in sys.argv[3].split(","):
        t0 = time.time()
        h = run(steps, precision, set(g.split("+")))
        res[g] = h
        np.savez(out, **res)
        print(f"{precision} {g}: {steps} steps in {time.time() - t0:.1f}s, final {h[-1]:.6f}", flush=True)


if __name__ == "__main__":
    main()
