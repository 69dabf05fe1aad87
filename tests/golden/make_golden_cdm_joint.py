"""Golden fixtures of the JOINT conditional-denoising path (train_CDNS.py,
scripts/experiments/exp_cdm_jointtrain.sh: ConditionalDenoiseEncoderTransformer
with sequential=False, the 81 text leaves through t_embedding, T = 162), generated
by importing the real reference.

Run ONLY in the build container, where the read-only reference is mounted:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_cdm_joint.py [--curve-steps 30]

Each fixture mirrors training/train_CDNS.py:60-150 (raw=True) in its RNG order:
ConditionalDenoiseSampler(seedtree=42) -> get_Bayes (unseeded; it does not affect
what follows) -> seed_everything(seed) -> the model -> loop.

Fixtures
--------
cdm_joint_tiny.npz   L=1, d=128, B=4, 2 steps: the batch (text leaves, z, image
                     leaves, posterior means), predictions, losses, per-tensor
                     grad / param checksums (sum, sum of squares, first 64 values).
cdm_joint_curve.npz  default joint config (p=0.2, L=9, d=128, B=128, lr 1e-3 ->
                     1e-6 over 30000 iters): ploss / loss / compare of the first N steps.
cdm_guided_tiny.npz  guided joint model (exp_cdm_guidedTF.sh: guide=True, penalty
                     0.1, lr 1e-2 -> 1e-5), L=9, B=4, 2 steps: batches, the
                     sampler's guided targets, predictions, losses, grad checksums.
cdm_guided_curve.npz the guided default config (B=128): first N ploss / loss / compare.
cdm_joint_curve_t2.npz, cdm_guided_curve_t2.npz  (--spread) the same two curves with
                     2 CPU threads instead of 8: the reference's own reduction-order
                     spread, which bounds the curve tolerance where it exceeds 1e-4.
"""
import argparse
import os
import sys
import time

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REF, "src"))

import torch  # noqa: E402
from ghmclip.models.model import (ConditionalDenoiseEncoderTransformer, ConditionalGuidedLsLoss, LsLoss,  # noqa: E402
                                  seed_everything)
from ghmclip.models.optimizer import AdamW, get_lr_cosine_schedule  # noqa: E402
from ghmclip.data.data_random_GHM import ConditionalDenoiseSampler  # noqa: E402

sys.path.insert(0, HERE)
from make_golden_cdm import checksums  # noqa: E402

P_Y = np.ones(10) / 10


class Loop:
    """train_CDNS.py:60-150 (raw=True, guide=False)."""

    def __init__(self, p, L, B, seed=224, total_iters=30000, lr_max=1e-3, lr_min=1e-6, penalty=0.1, max_norm=1.0,
                 guide=False):
        self.s = ConditionalDenoiseSampler([4, 4], [3, 3], [P_Y, P_Y], [p, p], sigma=1, flip_scale=1,
                                           variable_type=10, translation_invariance=True, seedtree=42)
        seed_everything(seed)  # :74
        self.model = ConditionalDenoiseEncoderTransformer(n_token=162, n_i_token=81, num_class=10, n_embd=128,
                                                          n_layer=L, n_guided_layers=[4, 4], n_head=4,
                                                          n_mlp_hidden=512, activation="softmax", mlp=True,
                                                          normalize_attn=True, layernorm=True, maxnorm=False,
                                                          sequential=False, guide=guide)  # :75-89
        self.loss = ConditionalGuidedLsLoss(penalty=penalty, guide=guide)
        self.guide = guide
        self.loss_nop = LsLoss()
        self.opt = AdamW(params=self.model.parameters(), lr=None)
        self.B, self.it = B, 0
        self.sched = (lr_max, lr_min, 0, total_iters)
        self.max_norm = max_norm

    def step(self):
        self.opt.zero_grad()
        rt, ri = self.s.get_batch(device="cpu", batch_size=self.B, guide=self.guide)
        guided = [rt[2], ri[2]]
        post = torch.tensor(ri[3], dtype=torch.float32)
        out = self.model(rt[0], ri[0])
        outputs = self.loss(out, [ri[1], guided])
        outputs[0].backward()
        nop = self.loss_nop(out[0], ri[1])
        cmp = self.loss_nop(out[0], post)
        grads = [(n, p.grad) for n, p in self.model.named_parameters() if p.grad is not None]
        torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.max_norm, norm_type=2)
        lr = get_lr_cosine_schedule(self.it, *self.sched)
        self.opt.set_lr(lr)
        self.opt.step()
        self.it += 1
        return dict(ploss=outputs[0].item(), loss=nop.item(), compare=cmp.item(), pred=out[0].detach(),
                    grads=[(n, g.clone()) for n, g in grads], batch=(rt, ri))


def tiny_fixture(L=1, B=4, nsteps=2, p=0.2):
    lp = Loop(p, L, B)
    init = checksums(lp.model.named_parameters())
    rec = {}
    for k in range(nsteps):
        r = lp.step()
        rec[f"ploss{k}"] = r["ploss"]
        rec[f"loss{k}"] = r["loss"]
        rec[f"compare{k}"] = r["compare"]
        rec[f"pred{k}"] = r["pred"].numpy()
        rt, ri = r["batch"]
        rec[f"t_leaves{k}"] = rt[0].numpy().astype(np.uint8)
        rec[f"z{k}"] = ri[0].numpy()
        rec[f"i_leaves{k}"] = ri[1].numpy().astype(np.uint8)
        rec[f"post{k}"] = np.asarray(ri[3])
        gn, gs, gh = checksums(r["grads"])
        rec[f"grad_names{k}"], rec[f"grad_stats{k}"], rec[f"grad_heads{k}"] = gn, gs, gh
        _, ps, ph = checksums(lp.model.named_parameters())
        rec[f"param_stats{k}"], rec[f"param_heads{k}"] = ps, ph
    np.savez_compressed(os.path.join(HERE, "cdm_joint_tiny.npz"), L=L, B=B, p=p, nsteps=nsteps,
                        param_names=init[0], init_stats=init[1], init_heads=init[2], **rec)
    print("wrote cdm_joint_tiny.npz", [rec[f"ploss{k}"] for k in range(nsteps)])


def guided_fixture(L=9, B=4, nsteps=2, p=0.2, curve_steps=30):
    """exp_cdm_guidedTF.sh (--guide=True, penalty 0.1, lr 1e-2 -> 1e-5): the tiny
    case's batches, guided targets, predictions, losses and gradient checksums, and
    the default config's first curve_steps losses."""
    lp = Loop(p, L, B, lr_max=1e-2, lr_min=1e-5, guide=True)
    init = checksums(lp.model.named_parameters())
    rec = {}
    for k in range(nsteps):
        r = lp.step()
        for key in ("ploss", "loss", "compare"):
            rec[f"{key}{k}"] = r[key]
        rec[f"pred{k}"] = r["pred"].numpy()
        rt, ri = r["batch"]
        rec[f"t_leaves{k}"] = rt[0].numpy().astype(np.uint8)
        rec[f"z{k}"] = ri[0].numpy()
        rec[f"i_leaves{k}"] = ri[1].numpy().astype(np.uint8)
        for j, g in enumerate(rt[2]):
            rec[f"t_guide{k}_{j}"] = g.numpy()
        for j, g in enumerate(ri[2]):
            rec[f"i_guide{k}_{j}"] = g.numpy()
        gn, gs, gh = checksums(r["grads"])
        rec[f"grad_names{k}"], rec[f"grad_stats{k}"], rec[f"grad_heads{k}"] = gn, gs, gh
    np.savez_compressed(os.path.join(HERE, "cdm_guided_tiny.npz"), L=L, B=B, p=p, nsteps=nsteps,
                        param_names=init[0], init_stats=init[1], init_heads=init[2], **rec)
    print("wrote cdm_guided_tiny.npz", [rec[f"ploss{k}"] for k in range(nsteps)])
    lp = Loop(p, 9, 128, lr_max=1e-2, lr_min=1e-5, guide=True)
    hist = np.zeros((3, curve_steps))
    for k in range(curve_steps):
        r = lp.step()
        hist[:, k] = (r["ploss"], r["loss"], r["compare"])
    np.savez_compressed(os.path.join(HERE, "cdm_guided_curve.npz"), p=p, L=9, B=128, total_iters=30000, lr_max=1e-2,
                        lr_min=1e-5, penalty=0.1, ploss=hist[0], loss=hist[1], compare=hist[2],
                        threads=torch.get_num_threads())
    print("wrote cdm_guided_curve.npz", hist[0, :3])


def guided_curve(steps, p=0.2, out="cdm_guided_curve.npz"):
    lp = Loop(p, 9, 128, lr_max=1e-2, lr_min=1e-5, guide=True)
    hist = np.zeros((3, steps))
    for k in range(steps):
        r = lp.step()
        hist[:, k] = (r["ploss"], r["loss"], r["compare"])
    np.savez_compressed(os.path.join(HERE, out), p=p, L=9, B=128, total_iters=30000, lr_max=1e-2,
                        lr_min=1e-5, penalty=0.1, ploss=hist[0], loss=hist[1], compare=hist[2],
                        threads=torch.get_num_threads())
    print("wrote", out, hist[0, :3])


def curve_fixture(steps, p=0.2, L=9, B=128, out="cdm_joint_curve.npz"):
    lp = Loop(p, L, B)
    hist = np.zeros((3, steps))
    t0 = time.time()
    for k in range(steps):
        r = lp.step()
        hist[:, k] = (r["ploss"], r["loss"], r["compare"])
        if k % 10 == 0:
            print(f"step {k} ploss {r['ploss']:.6f} compare {r['compare']:.6f} ({time.time() - t0:.1f}s)", flush=True)
    np.savez_compressed(os.path.join(HERE, out), p=p, L=L, B=B, total_iters=30000, lr_max=1e-3,
                        lr_min=1e-6, ploss=hist[0], loss=hist[1], compare=hist[2], threads=torch.get_num_threads())
    print("wrote", out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--curve-steps", type=int, default=30)
    ap.add_argument("--only", default="")
    ap.add_argument("--spread", action="store_true",
                    help="write the 2-thread curves (*_t2.npz) next to the 8-thread fixtures")
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else None
    if a.spread:
        torch.set_num_threads(2)
        curve_fixture(a.curve_steps, out="cdm_joint_curve_t2.npz")
        guided_curve(a.curve_steps, out="cdm_guided_curve_t2.npz")
        sys.exit(0)
    if not only or "tiny" in only:
        tiny_fixture()
    if not only or "curve" in only:
        curve_fixture(a.curve_steps)
    if not only or "guided" in only:
        guided_fixture(curve_steps=a.curve_steps)
