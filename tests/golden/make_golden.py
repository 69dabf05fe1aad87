"""Generate the golden fixtures that pin the oracle to the real reference.

Run ONLY in the build container, where the read-only reference is mounted:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--curve-steps 200]

It imports the reference package from /root/reference/src (never copied) and
records inputs/outputs as small .npz/.json files next to this script.  The GPU
box never runs this script; it only reads the committed fixtures.

Fixtures
--------
sampler_p20.npz     transitions (seedtree=42, p=0.2) + first 3 ClipSampler.get_batch
                    draws after seed_everything(224) (B=128, K=4) as uint8.
                    Mirrors train_CLIP.py:67-76,83,145 (data_random_GHM.py:645-658,753-784).
sampler_p40_b16.npz same for p=0.4, B=16 (another shape/probability).
clip_tiny.npz       tiny CLIP config (L=2, d=16, B=4): init weights, embeddings, loss,
                    raw grads, clip norm, weights after 2 AdamW steps.
clip_d128.npz       d=128, L=2, B=8 single step: embeddings, loss, grad checksums.
clip_d64.npz / clip_d256.npz  the same at d = 64 (the reference CLI's default
                    clip_{t,i}model_deb) and d = 256 (--only d64,d256).
clip_default_curve.npz  the default CLIP config (p=0.2, L=5, d=128, B=128) loss_history
                    for the first --curve-steps steps of the 3001-step schedule.
bayes.json          the 20 published Bayes CLIP risks (figures/data/ghm-data/clip-risk.json:90-110).
guide_bp.npz        get_batch(guide=True) at B=8 (p=0.2) after seed_everything(224): leaves,
                    the 4 guided targets per tower stored compactly per tree node
                    (GHMTree.guided_info, data_random_GHM.py:526-549, repeats checked
                    here) and the BP_CLS posteriors (:185-221).
guide_tiny.npz      guided CLIP (clip_guide=True, exp_clip_guidedTF.sh: lr 1e-3 -> 1e-6,
                    penalty 1e-3) at L=5, d=16, B=4 for 2 steps: loss, loss_nop, penalty,
                    raw grads, weights after each step.
guide_nonti_tiny.npz  the same at d=128 (the HIP encoder's width) on
                    --translation_invariance=False trees (--only guide_nonti_tiny), with
                    (sum, sum of squares, abs-max) checksums of the weight / gradient
                    tensors, plus every edge's transition matrix of both trees.
guide_curve.npz     the guided default config (L=5, d=128, B=128) ploss/loss history
                    for the first --guide-steps steps.

The long reference runs (hours on this container's CPU) were made with:
  clip_default_curve3001.npz   --only curve --curve-steps 3001 --curve-out clip_default_curve3001.npz --threads 6
  clip_shallow_curve3001.npz   --only curve --curve-steps 3001 --curve-layers 1 --curve-out ... --threads 3
  clip_guided_curve3001.npz    --only guide_curve --guide-steps 3001 --guide-out ... --threads 5
  clip_guided_curve3001_t2.npz --only guide_curve --guide-steps 1101 --guide-out ... --threads 2
  clip_guided_curve3001_avx2.npz  ATEN_CPU_CAPABILITY=avx2 MKL_CBWR=AVX2 (the same command,
                    --guide-steps 1101 --threads 5): the reference's own code on the kernels a
                    host without AVX-512 runs -- with the 2-thread run, the spread of the
                    reference's own fp32 arithmetic (tests/conftest.py curve_bound).
  clip_guided_curve3001_scalar.npz  ATEN_CPU_CAPABILITY=default (--guide-steps 1101 --threads 4,
                    69 min): the same code on ATen's scalar (non-SIMD) kernels -- LayerNorm,
                    softmax, GELU and the reductions summed in another order, the GEMMs
                    unchanged (MKL).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REF, "src"))

import torch  # noqa: E402
from ghmclip.models.model import EncoderTransformer, GuidedClipLoss, seed_everything  # noqa: E402
from ghmclip.models.optimizer import AdamW, get_lr_cosine_schedule  # noqa: E402
from ghmclip.data.data_random_GHM import ClipSampler  # noqa: E402

P_Y = np.ones(10) / 10


def make_sampler(p, seedtree=42, K=4, ti=True):
    return ClipSampler([4, 4], [3, 3], [P_Y, P_Y], [p, p], K=K, flip_scale=1,
                       variable_type=10, translation_invariance=ti, seedtree=seedtree)


def distinct_transitions(trans):
    # translation invariance: per layer the list repeats the n_child templates
    return np.stack([np.stack(layer[:3]) for layer in trans])


def sampler_fixture(p, B, nb, name):
    s = make_sampler(p)
    seed_everything(224)
    tl, il, tr, ir = [], [], [], []
    for _ in range(nb):
        t, i = s.get_batch(device="cpu", batch_size=B, guide=False)
        tl.append(t[0].numpy().astype(np.uint8)); il.append(i[0].numpy().astype(np.uint8))
        tr.append(t[1].numpy().astype(np.uint8)); ir.append(i[1].numpy().astype(np.uint8))
    np.savez_compressed(os.path.join(HERE, name), p=p, B=B, K=4,
                        t_transition=distinct_transitions(s.t_transition),
                        i_transition=distinct_transitions(s.i_transition),
                        t_leaves=np.stack(tl), i_leaves=np.stack(il),
                        t_root=np.stack(tr), i_root=np.stack(ir))
    print("wrote", name)


def build_models(T, L, d, activation="softmax"):
    kw = dict(n_token=T, num_class=10, n_embd=d, n_layer=L, n_guided_layer=4, n_head=4,
              n_mlp_multiplier=4, activation=activation, mlp=True, normalize_attn=True,
              layernorm=True, guide=False)
    return EncoderTransformer(**kw), EncoderTransformer(**kw)


def flat_state(model, prefix):
    return {f"{prefix}.{k}": v.detach().clone().numpy() for k, v in model.state_dict().items()}


def step_fixture(name, L, d, B, nsteps, p=0.2, total_iters=3000, checksum_only=False, activation="softmax"):
    """Mirror of train_CLIP.py:83-167 for a few steps on a small config
    (activation: train_CLIP --clip_activation, models/model.py:121-130)."""
    s = make_sampler(p)
    seed_everything(224)
    tm, im = build_models(81, L, d, activation)
    loss = GuidedClipLoss(4, B, penalty=1e-3, guide=False)
    loss_nop = GuidedClipLoss(4, B, penalty=0, guide=False)
    params = list(tm.parameters()) + list(im.parameters())
    opt = AdamW(params=params, lr=None)
    out = {}
    out.update({"init." + k: v for k, v in flat_state(tm, "t").items()})
    out.update({"init." + k: v for k, v in flat_state(im, "i").items()})
    for it in range(nsteps):
        opt.zero_grad()
        rt, ri = s.get_batch(device="cpu", batch_size=B, guide=False)
        to = tm(rt[0]); io = im(ri[0])
        o = loss(to, io, [rt[2], ri[2]])
        onop = loss_nop(to, io, [rt[2], ri[2]])
        o[0].backward()
        out[f"s{it}.t_leaves"] = rt[0].numpy().astype(np.uint8)
        out[f"s{it}.i_leaves"] = ri[0].numpy().astype(np.uint8)
        out[f"s{it}.t_emb"] = to[0].detach().numpy()
        out[f"s{it}.i_emb"] = io[0].detach().numpy()
        out[f"s{it}.loss"] = np.float64(o[0].item())
        out[f"s{it}.loss_nop"] = np.float64(onop[0].item())
        for pref, m in (("t", tm), ("i", im)):
            for k, prm in m.named_parameters():
                out[f"s{it}.grad.{pref}.{k}"] = prm.grad.detach().clone().numpy()
        tot = torch.nn.utils.clip_grad_norm_(params, 1.0, norm_type=2)
        out[f"s{it}.total_norm"] = np.float64(tot.item())
        lr = get_lr_cosine_schedule(it, 3e-4, 3e-7, 0, total_iters)
        out[f"s{it}.lr"] = np.float64(lr)
        opt.set_lr(lr)
        opt.step()
        out.update({f"s{it}.post.{k}": v for k, v in flat_state(tm, "t").items()})
        out.update({f"s{it}.post.{k}": v for k, v in flat_state(im, "i").items()})
    out["meta"] = np.array([L, d, B, nsteps, total_iters], dtype=np.int64)
    out["p"] = np.float64(p)
    out["activation"] = np.array(activation)
    if checksum_only:
        # keep big configs small on disk: per-tensor (sum, sum of squares, abs-max)
        # for weight/grad tensors; full arrays for leaves, embeddings and scalars.
        slim = {}
        for k, v in out.items():
            if (".grad." in k or k.startswith("init.") or ".post." in k) and v.size > 64:
                v64 = v.astype(np.float64)
                slim[k + ".cks"] = np.array([v64.sum(), (v64 * v64).sum(), np.abs(v64).max()])
            else:
                slim[k] = v
        out = slim
    np.savez_compressed(os.path.join(HERE, name), **out)
    print("wrote", name)


def curve_fixture(steps, p=0.2, B=128, total_iters=3000, out="clip_default_curve.npz", n_layer=5):
    """Default CLIP config (scripts/experiments/exp_clip_standardTF.sh:15-40).
    With steps = total_iters + 1 this is the whole reference run (F5): its final
    risk is mean(loss_history[-100:]) (figures/eval-clip-risk.py:29).
    n_layer=1 is the Shallow TF architecture (exp_clip_shallowTF.sh:19-36)."""
    s = make_sampler(p)
    seed_everything(224)
    tm, im = build_models(81, n_layer, 128)
    loss_nop = GuidedClipLoss(4, B, penalty=0, guide=False)
    loss = GuidedClipLoss(4, B, penalty=1e-3, guide=False)
    params = list(tm.parameters()) + list(im.parameters())
    opt = AdamW(params=params, lr=None)
    hist = np.zeros(steps)
    norms = np.zeros(steps)
    t0 = time.time()
    for it in range(steps):
        opt.zero_grad()
        rt, ri = s.get_batch(device="cpu", batch_size=B, guide=False)
        to = tm(rt[0]); io = im(ri[0])
        o = loss(to, io, [rt[2], ri[2]])
        onop = loss_nop(to, io, [rt[2], ri[2]])
        o[0].backward()
        hist[it] = onop[0].item()
        norms[it] = torch.nn.utils.clip_grad_norm_(params, 1.0, norm_type=2).item()
        lr = get_lr_cosine_schedule(it, 3e-4, 3e-7, 0, total_iters)
        opt.set_lr(lr)
        opt.step()
        if it % 20 == 0:
            print(f"curve step {it} loss {hist[it]:.6f} ({time.time()-t0:.0f}s)", flush=True)
        if it % 200 == 0 and steps > 1000:  # checkpoint the long run
            np.savez_compressed(os.path.join(HERE, out), loss_history=hist[:it + 1], grad_norm=norms[:it + 1],
                                p=p, B=B, total_iters=total_iters, n_layer=n_layer,
                                threads=torch.get_num_threads())
    np.savez_compressed(os.path.join(HERE, out), loss_history=hist,
                        grad_norm=norms, p=p, B=B, total_iters=total_iters, n_layer=n_layer,
                        threads=torch.get_num_threads())
    print("wrote", out)


def build_guided(T, L, d):
    kw = dict(n_token=T, num_class=10, n_embd=d, n_layer=L, n_guided_layer=4, n_head=4,
              n_mlp_multiplier=4, activation="softmax", mlp=True, normalize_attn=True,
              layernorm=True, guide=True)
    return EncoderTransformer(**kw), EncoderTransformer(**kw)


def compact_targets(gl):
    """[N,81,10] guided target k (ancestor at depth 3-k repeated over its 3^(k+1)
    leaves) -> [N, 81/3^(k+1), 10], checking the repeats are exact."""
    out = []
    for k, g in enumerate(gl):
        g = g.numpy()
        ext = 3 ** (k + 1)
        c = g[:, ::ext, :]
        assert np.array_equal(np.repeat(c, ext, axis=1), g)
        out.append(c.astype(np.float32))
    return out


def guide_bp_fixture(B=8, p=0.2):
    s = make_sampler(p)
    seed_everything(224)
    rt, ri = s.get_batch(device="cpu", batch_size=B, guide=True)
    out = {"p": p, "B": B, "t_transition": distinct_transitions(s.t_transition),
           "i_transition": distinct_transitions(s.i_transition),
           "t_leaves": rt[0].numpy().astype(np.uint8), "i_leaves": ri[0].numpy().astype(np.uint8),
           "t_pp": np.asarray(rt[3], dtype=np.float64), "i_pp": np.asarray(ri[3], dtype=np.float64)}
    for pref, r in (("t", rt), ("i", ri)):
        for k, c in enumerate(compact_targets(r[2])):
            out[f"{pref}_msg{k}"] = c
    np.savez_compressed(os.path.join(HERE, "guide_bp.npz"), **out)
    print("wrote guide_bp.npz")


def guide_step_fixture(name, L=5, d=16, B=4, nsteps=2, p=0.2, total_iters=3000, penalty=1e-3,
                       lr_max=1e-3, lr_min=1e-6, ti=True, checksum_only=False):
    """train_CLIP.py:83-167 with clip_guide=True (exp_clip_guidedTF.sh); ti=False:
    --translation_invariance=False trees (one transition matrix per edge)."""
    s = make_sampler(p, ti=ti)
    seed_everything(224)
    tm, im = build_guided(81, L, d)
    loss = GuidedClipLoss(4, B, penalty=penalty, guide=True)
    loss_nop = GuidedClipLoss(4, B, penalty=0, guide=False)
    params = list(tm.parameters()) + list(im.parameters())
    opt = AdamW(params=params, lr=None)
    out = {}
    out.update({"init." + k: v for k, v in flat_state(tm, "t").items()})
    out.update({"init." + k: v for k, v in flat_state(im, "i").items()})
    for it in range(nsteps):
        opt.zero_grad()
        rt, ri = s.get_batch(device="cpu", batch_size=B, guide=True)
        to = tm(rt[0]); io = im(ri[0])
        o = loss(to, io, [rt[2], ri[2]])
        onop = loss_nop(to, io, [rt[2], ri[2]])
        o[0].backward()
        out[f"s{it}.t_leaves"] = rt[0].numpy().astype(np.uint8)
        out[f"s{it}.i_leaves"] = ri[0].numpy().astype(np.uint8)
        out[f"s{it}.loss"] = np.float64(o[0].item())
        out[f"s{it}.loss_nop"] = np.float64(onop[0].item())
        out[f"s{it}.penalty"] = np.float64(o[1])
        for pref, m in (("t", tm), ("i", im)):
            for k, prm in m.named_parameters():
                out[f"s{it}.grad.{pref}.{k}"] = prm.grad.detach().clone().numpy()
        tot = torch.nn.utils.clip_grad_norm_(params, 1.0, norm_type=2)
        out[f"s{it}.total_norm"] = np.float64(tot.item())
        lr = get_lr_cosine_schedule(it, lr_max, lr_min, 0, total_iters)
        opt.set_lr(lr)
        opt.step()
        out.update({f"s{it}.post.{k}": v for k, v in flat_state(tm, "t").items()})
        out.update({f"s{it}.post.{k}": v for k, v in flat_state(im, "i").items()})
    out["meta"] = np.array([L, d, B, nsteps, total_iters], dtype=np.int64)
    out["hyper"] = np.array([p, penalty, lr_max, lr_min])
    if checksum_only:  # as step_fixture: (sum, sum of squares, abs-max) of the big tensors
        out = {k + ".cks" if (".grad." in k or k.startswith("init.") or ".post." in k) and v.size > 64 else k:
               np.array([v.astype(np.float64).sum(), (v.astype(np.float64) ** 2).sum(), np.abs(v).max()])
               if (".grad." in k or k.startswith("init.") or ".post." in k) and v.size > 64 else v
               for k, v in out.items()}
    if not ti:
        out["t_edges"] = np.concatenate([np.stack(layer) for layer in s.t_transition])
        out["i_edges"] = np.concatenate([np.stack(layer) for layer in s.i_transition])
    np.savez_compressed(os.path.join(HERE, name), **out)
    print("wrote", name)


def guide_curve_fixture(steps, p=0.2, B=128, total_iters=3000, penalty=1e-3, lr_max=1e-3, lr_min=1e-6,
                        out="guide_curve.npz"):
    """Guided default config (exp_clip_guidedTF.sh) ploss/loss history.  With
    steps = total_iters + 1 this is the whole reference run (final risk =
    mean(loss_history[-100:]), figures/eval-clip-risk.py:29)."""
    s = make_sampler(p)
    seed_everything(224)
    tm, im = build_guided(81, 5, 128)
    loss = GuidedClipLoss(4, B, penalty=penalty, guide=True)
    loss_nop = GuidedClipLoss(4, B, penalty=0, guide=False)
    params = list(tm.parameters()) + list(im.parameters())
    opt = AdamW(params=params, lr=None)
    hist, phist, pen = np.zeros(steps), np.zeros(steps), np.zeros(steps)
    t0 = time.time()
    for it in range(steps):
        opt.zero_grad()
        rt, ri = s.get_batch(device="cpu", batch_size=B, guide=True)
        to = tm(rt[0]); io = im(ri[0])
        o = loss(to, io, [rt[2], ri[2]])
        onop = loss_nop(to, io, [rt[2], ri[2]])
        o[0].backward()
        phist[it], hist[it], pen[it] = o[0].item(), onop[0].item(), o[1]
        torch.nn.utils.clip_grad_norm_(params, 1.0, norm_type=2)
        opt.set_lr(get_lr_cosine_schedule(it, lr_max, lr_min, 0, total_iters))
        opt.step()
        if it % 20 == 0:
            print(f"guide curve step {it} ploss {phist[it]:.6f} loss {hist[it]:.6f} ({time.time()-t0:.0f}s)",
                  flush=True)
        if it % 100 == 0 and steps > 1000:  # checkpoint the long run (partial prefix)
            np.savez_compressed(os.path.join(HERE, out), loss_history=hist[:it + 1], ploss_history=phist[:it + 1],
                                penalty=pen[:it + 1], p=p, B=B, total_iters=total_iters,
                                hyper=np.array([penalty, lr_max, lr_min]), threads=torch.get_num_threads())
    np.savez_compressed(os.path.join(HERE, out), loss_history=hist, ploss_history=phist,
                        penalty=pen, p=p, B=B, total_iters=total_iters,
                        hyper=np.array([penalty, lr_max, lr_min]), threads=torch.get_num_threads())
    print("wrote", out)


def bayes_fixture():
    with open(os.path.join(REF, "figures/data/ghm-data/clip-risk.json")) as f:
        d = json.load(f)
    out = {"p_flip": [p / 100 for p in d["p_flip"]], "Bayes": d["Bayes"],
           "Standard TF": d["Standard TF"],
           "source": "figures/data/ghm-data/clip-risk.json:90-110"}
    with open(os.path.join(HERE, "bayes.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote bayes.json")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--curve-steps", type=int, default=200)
    ap.add_argument("--curve-out", default="clip_default_curve.npz")
    ap.add_argument("--curve-layers", type=int, default=5)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--only", default="")
    ap.add_argument("--guide-steps", type=int, default=100)
    ap.add_argument("--guide-out", default="guide_curve.npz")
    a = ap.parse_args()
    if a.threads:
        torch.set_num_threads(a.threads)
    jobs = a.only.split(",") if a.only else ["sampler", "tiny", "d128", "bayes", "curve"]
    if "sampler" in jobs:
        sampler_fixture(0.2, 128, 3, "sampler_p20.npz")
        sampler_fixture(0.4, 16, 2, "sampler_p40_b16.npz")
    if "tiny" in jobs:
        step_fixture("clip_tiny.npz", L=2, d=16, B=4, nsteps=2)
    if "d128" in jobs:
        step_fixture("clip_d128.npz", L=2, d=128, B=8, nsteps=2, checksum_only=True)
    if "d64" in jobs:  # the reference CLI's default width (utils/config.py:58-59)
        step_fixture("clip_d64.npz", L=2, d=64, B=8, nsteps=2, checksum_only=True)
    if "d256" in jobs:
        step_fixture("clip_d256.npz", L=2, d=256, B=8, nsteps=2, checksum_only=True)
    if "bayes" in jobs:
        bayes_fixture()
    if "curve" in jobs:
        curve_fixture(a.curve_steps, out=a.curve_out, n_layer=a.curve_layers)
    if "guide_bp" in jobs:
        guide_bp_fixture()
    if "guide_tiny" in jobs:
        guide_step_fixture("guide_tiny.npz")
    if "guide_nonti_tiny" in jobs:
        guide_step_fixture("guide_nonti_tiny.npz", d=128, ti=False, checksum_only=True)
    if "guide_curve" in jobs:
        guide_curve_fixture(a.guide_steps, out=a.guide_out)
