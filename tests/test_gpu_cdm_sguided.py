"""Guided sequential CDM (train_sequential_DNS.py --guide=True, scripts/examples/
eg_sdns.sh: p = 0.04, L = 9, n_guided_layers [1, 4], penalty 0.1, lr 3e-4 -> 3e-7)
on the HIP path vs the reference's own numbers (tests/golden/make_golden_cdm.py
--only sguided_tiny,sguided_curve).

The model is the sequential CDM (81 noisy image leaves + the frozen CLIP text
feature as one token).  Guided outputs (model.py:448-527): 9 image-guided layers
(h / q blocks, then h / q / u blocks of the image tree's BP_DNS messages) and 2
text-guided layers whose one conditioning token's 10-column block is pulled to the
CLIP feature itself (train_sequential_DNS.py:145: guided_layers =
[[clip_text_output, clip_text_output], res_image[2]]).

What is pinned, and against what:
  * the device BP messages gathered through cdm_guide_blocks == the sampler's
    guided targets (data_random_GHM.py:551-592), 1e-5 relative to the max-abs;
  * two fused steps (B = 4): penalised loss, loss, compare, the four penalty groups
    of ConditionalGuidedLsLoss (model.py:1023-1040), predictions, per-tensor
    clipped-gradient sums of squares (1e-3) and (f32) post-step parameter sums of
    squares (1e-3);
  * the first 30 steps at eg_sdns.sh's B = 128: ploss / loss / compare within
    max(1e-4, 2 x the reference's own 1-vs-2-thread spread) (f32) or 1e-3 (x3).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, curve_bound

pytestmark = pytest.mark.gpu

DEV = "cuda"
P_Y = np.ones(10) / 10
PENALTY, LR_MAX, LR_MIN = 0.1, 3e-4, 3e-7


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ghmclip import _native
    assert _native.hip_lib().ghm_device_ok() == 1, "libghm_hip.so not usable on this device"


def _trainer(B, precision, L=9, total_iters=30000):
    """train_sequential_DNS.py:62-127 order: seed, sampler (seedtree 42), get_Bayes,
    the frozen CLIP text encoder, the guided denoiser."""
    from ghmclip import (ConditionalDenoiseEncoderTransformer, ConditionalDenoiseSampler, EncoderTransformer,
                         get_lr_cosine_schedule, seed_everything)
    from ghmclip.training.cdm_trainer import CdmTrainer
    seed_everything(224)
    s = ConditionalDenoiseSampler([4, 4], [3, 3], [P_Y, P_Y], [0.04, 0.04], sigma=1)
    s.get_Bayes(n_eval=10000)
    clip = EncoderTransformer(81, 10, 128, 5).to(DEV)
    model = ConditionalDenoiseEncoderTransformer(82, 81, 10, 128, L, [1, 4], 4, 512, sequential=True,
                                                 guide=True).to(DEV)
    sched = [get_lr_cosine_schedule(k, LR_MAX, LR_MIN, 0, total_iters) for k in range(total_iters + 1)]
    tr = CdmTrainer(model, clip, B, sched, s.t_templ, s.i_templ, sigma=1.0, device=DEV, precision=precision,
                    penalty=PENALTY)
    return s, tr


def _draw(s, tr, B):
    tl, _, z, il = s.draw_numpy(B)
    tr.set_batch(torch.from_numpy(tl), torch.from_numpy(il), torch.from_numpy(z))


def _gather(tr, blk):
    """The [B, ntok, V] target a guided block reads on the device."""
    src, tok0, ntok, col, moff, ext = blk
    msgs = {"i": tr.imsgs, "c": tr.clip_plan.emb}[src].reshape(tr.B, -1)
    V = tr.tree[4]
    t = torch.arange(ntok, device=msgs.device)
    idx = moff + (t // ext)[:, None] * V + torch.arange(V, device=msgs.device)[None, :]
    return msgs[:, idx]


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-12)


@pytest.mark.parametrize("precision", ["f32", "x3"])
def test_sguided_steps_vs_reference_fixture(precision):
    f = np.load(os.path.join(GOLDEN, "cdm_sguided_tiny.npz"))
    assert bool(f["guide"]) and int(f["L"]) == 9
    B = int(f["B"])
    s, tr = _trainer(B, precision)
    for (n, p), want in zip(tr.model.named_parameters(), f["init_stats"]):
        assert abs((p.double() ** 2).sum().item() - want[1]) <= 1e-12 * want[1] + 1e-12, n
    for (n, p), want in zip(tr.clip.named_parameters(), f["clip_stats"]):
        assert abs((p.double() ** 2).sum().item() - want[1]) <= 1e-12 * want[1] + 1e-12, n
    ig = [l for l, fl in enumerate(tr.model.i_guided_layer_flag) if fl]
    ftol = {"f32": 2e-5, "x3": 1e-4}[precision]
    for k in range(int(f["nsteps"])):
        _draw(s, tr, B)
        tr.step()
        torch.cuda.synchronize()
        for j, l in enumerate(ig):
            blks = [b for b in tr.gblocks[l] if b[0] == "i"]
            got = torch.cat([_gather(tr, b) for b in blks], dim=2)
            want = f[f"i_guide{k}_{j}"]
            assert got.shape == want.shape, (j, got.shape, want.shape)
            assert _rel(got, want) < 1e-5, ("image", k, j)
        assert _rel(tr.clip_plan.emb, f[f"feat{k}"]) < ftol
        for l in (0, 3):  # the text blocks read the CLIP feature itself
            blk = [b for b in tr.gblocks[l] if b[0] == "c"][0]
            assert torch.equal(_gather(tr, blk)[:, 0], tr.clip_plan.emb)
        assert _rel(tr.plan.pred, f[f"pred{k}"]) < ftol * 5
        pen = tr.penalty_groups()
        want = f[f"pen{k}"]
        assert np.all(np.abs(pen - want) <= 1e-4 * np.abs(want) + 1e-6), (k, pen, want)
        coef = tr.hyper[1].item()
        gstats = {n: st for n, st in zip(f[f"grad_names{k}"], f[f"grad_stats{k}"])}
        for n, g in tr.gd.items():  # the fixture's are clipped in place; the trainer's raw, coef in hyper[1]
            got = ((g.double() * coef) ** 2).sum().item()
            want = gstats[n][1]
            assert abs(got - want) <= 1e-3 * want + 1e-12, (k, n, got, want)
        assert 0 < coef <= 1
    ph, h, ch = tr.ploss_history(), tr.loss_history(), tr.compare_history()
    for k in range(int(f["nsteps"])):
        assert abs(ph[k] - float(f[f"ploss{k}"])) <= 2e-5 * float(f[f"ploss{k}"]), (k, ph[k])
        assert abs(h[k] - float(f[f"loss{k}"])) <= 1e-4 * float(f[f"loss{k}"]), (k, h[k])
        assert abs(ch[k] - float(f[f"compare{k}"])) <= 1e-4 * float(f[f"compare{k}"]), (k, ch[k])
    if precision == "x3":  # (split-bf16: Adam's first steps turn noise-level gradients into +-lr moves)
        return
    # post-step parameters of the last step (AdamW after the clip)
    names = list(f["param_names"])
    last = int(f["nsteps"]) - 1
    sd = dict(tr.model.named_parameters())
    for n, st in zip(names, f[f"param_stats{last}"]):
        got = (sd[n].double() ** 2).sum().item()
        assert abs(got - st[1]) <= 1e-3 * st[1] + 1e-9, (n, got, st[1])


def test_sguided_graph_replay_matches_eager():
    hs = []
    for graph in (False, True):
        s, tr = _trainer(4, "x3")
        for k in range(5):
            _draw(s, tr, 4)
            tr.step()
            if graph and k == 1:
                tr.capture()
        torch.cuda.synchronize()
        hs.append((tr.ploss_history(), tr.compare_history()))
    np.testing.assert_array_equal(hs[0][0], hs[1][0])
    np.testing.assert_array_equal(hs[0][1], hs[1][1])


@pytest.mark.parametrize("precision", ["f32", "x3"])
def test_sguided_curve_vs_reference(precision):
    """eg_sdns.sh at B = 128: the first 30 steps vs the reference's CPU run
    (cdm_sguided_curve.npz, 1 thread) and its 2-thread rerun (*_t2.npz)."""
    g = np.load(os.path.join(GOLDEN, "cdm_sguided_curve.npz"))
    g2 = np.load(os.path.join(GOLDEN, "cdm_sguided_curve_t2.npz"))
    n = len(g["ploss"])
    s, tr = _trainer(128, precision)
    for k in range(n):
        _draw(s, tr, 128)
        tr.step()
        if k == 2:
            tr.capture()
    torch.cuda.synchronize()
    ph, h, ch = tr.ploss_history(), tr.loss_history(), tr.compare_history()
    msg, ok = [], True
    for key, got in (("ploss", ph), ("loss", h), ("compare", ch)):
        d = np.abs(got - g[key]) / np.abs(g[key])
        b, w, sp = curve_bound(g[key], g2[key])
        msg.append(f"{key} {d.max():.3e} (spread {sp[-1]:.3e})")
        ok = ok and bool((d <= b).all() if precision == "f32" else d.max() <= 1e-3)
    print(f"guided sequential CDM curve ({precision}), {n} steps: " + "; ".join(msg))
    assert ok
