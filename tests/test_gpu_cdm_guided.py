"""Guided joint CDM (train_CDNS.py --guide=True, scripts/experiments/exp_cdm_guidedTF.sh:
penalty 0.1, lr 1e-2 -> 1e-5, L=9, n_guided_layers [4, 4]) on the HIP path vs the
reference's own numbers (tests/golden/make_golden_cdm_joint.py --only guided).

What is pinned, and against what:
  * the device BP messages, gathered through cdm_guide_blocks, equal the sampler's
    guided targets (data_random_GHM.py:526-592) element for element (f32 of the
    same f64 recursion: 1e-5 relative to the target's max-abs);
  * the penalised loss, the loss and the compare value of two fused steps (1e-4
    relative), which also pins the column blocks (model.py:502-527);
  * per-tensor gradient sums of squares of both steps (1e-3 relative);
  * the first 30 steps of the guided default config (B=128): penalised loss within
    1e-3 relative, loss and compare within 2e-3 (measured 1.4e-4 / 6.9e-4 / 9.6e-4).
Split-bf16 (x3) matrix products throughout (162-token sequences)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, curve_bound

pytestmark = pytest.mark.gpu

DEV = "cuda"
P_Y = np.ones(10) / 10


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ghmclip import _native
    assert _native.hip_lib().ghm_device_ok() == 1, "libghm_hip.so not usable on this device"


def _trainer(L, B, total_iters=30000, precision="x3"):
    """train_CDNS.py order: sampler (seedtree 42), seed_everything(224), the model."""
    from ghmclip import (ConditionalDenoiseEncoderTransformer, ConditionalDenoiseSampler, get_lr_cosine_schedule,
                         seed_everything)
    from ghmclip.training.cdm_trainer import CdmTrainer
    s = ConditionalDenoiseSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2], sigma=1)
    seed_everything(224)
    model = ConditionalDenoiseEncoderTransformer(162, 81, 10, 128, L, [4, 4], 4, 512, sequential=False,
                                                 guide=True).to(DEV)
    sched = [get_lr_cosine_schedule(k, 1e-2, 1e-5, 0, total_iters) for k in range(total_iters + 1)]
    tr = CdmTrainer(model, None, B, sched, s.t_templ, s.i_templ, sigma=1.0, device=DEV, precision=precision,
                    penalty=0.1)
    return s, tr


def _draw(s, tr, B):
    tl, _, z, il = s.draw_numpy(B)
    tr.set_batch(torch.from_numpy(tl), torch.from_numpy(il), torch.from_numpy(z))


def _gather(tr, blk):
    """The [B, ntok, V] target a guided block reads from the device messages."""
    src, tok0, ntok, col, moff, ext = blk
    msgs = (tr.imsgs if src == "i" else tr.tmsgs).reshape(tr.B, -1)
    V = tr.tree[4]
    t = torch.arange(ntok, device=msgs.device)
    idx = moff + (t // ext)[:, None] * V + torch.arange(V, device=msgs.device)[None, :]
    return msgs[:, idx]


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-12)


def test_guided_flags_match_reference_layout():
    from ghmclip import ConditionalDenoiseEncoderTransformer
    m = ConditionalDenoiseEncoderTransformer(162, 81, 10, 128, 9, [4, 4], 4, 512, sequential=False, guide=True)
    assert m.i_guided_layer_flag == [True] * 9  # gap 9 // 9 = 1 (model.py:372, :407-416)
    assert m.t_guided_layer_flag == [True] * 4 + [False] * 5


def test_guided_targets_losses_and_grads_vs_reference_fixture():
    f = np.load(os.path.join(GOLDEN, "cdm_guided_tiny.npz"))
    B = int(f["B"])
    s, tr = _trainer(int(f["L"]), B)
    for (n, p), want in zip(tr.model.named_parameters(), f["init_stats"]):
        assert abs((p.double() ** 2).sum().item() - want[1]) <= 1e-12 * want[1] + 1e-12, n
    ig = [l for l, fl in enumerate(tr.model.i_guided_layer_flag) if fl]
    tg = [l for l, fl in enumerate(tr.model.t_guided_layer_flag) if fl]
    for k in range(int(f["nsteps"])):
        _draw(s, tr, B)
        tr.step()
        torch.cuda.synchronize()
        # guided targets: image counter j uses the image blocks of layer ig[j]
        for j, l in enumerate(ig):
            blks = [b for b in tr.gblocks[l] if b[0] == "i"]
            got = torch.cat([_gather(tr, b) for b in blks], dim=2)
            want = f[f"i_guide{k}_{j}"]
            assert got.shape == want.shape, (j, got.shape, want.shape)
            assert _rel(got, want) < 1e-5, ("image", k, j)
        for j, l in enumerate(tg):
            blk = [b for b in tr.gblocks[l] if b[0] == "t"][0]
            assert _rel(_gather(tr, blk), f[f"t_guide{k}_{j}"]) < 1e-5, ("text", k, j)
        assert _rel(tr.plan.pred, f[f"pred{k}"]) < 1e-4
        coef = tr.hyper[1].item()
        stats = {n: st for n, st in zip(f[f"grad_names{k}"], f[f"grad_stats{k}"])}
        for n, g in tr.gd.items():
            want = stats[n][1]
            got = ((g.double() * coef) ** 2).sum().item()
            assert abs(got - want) <= 1e-3 * want + 1e-12, (k, n, got, want)
    ph, h, ch = tr.ploss_history(), tr.loss_history(), tr.compare_history()
    for k in range(int(f["nsteps"])):
        assert abs(ph[k] - float(f[f"ploss{k}"])) <= 1e-4 * float(f[f"ploss{k}"]), (k, ph[k])
        assert abs(h[k] - float(f[f"loss{k}"])) <= 1e-4 * float(f[f"loss{k}"]), (k, h[k])
        assert abs(ch[k] - float(f[f"compare{k}"])) <= 1e-4 * float(f[f"compare{k}"]), (k, ch[k])
        assert ph[k] > h[k]


def test_guided_graph_replay_matches_eager():
    hs = []
    for graph in (False, True):
        s, tr = _trainer(9, 4)
        for k in range(5):
            _draw(s, tr, 4)
            tr.step()
            if graph and k == 1:
                tr.capture()
        torch.cuda.synchronize()
        hs.append((tr.ploss_history(), tr.compare_history()))
    np.testing.assert_array_equal(hs[0][0], hs[1][0])
    np.testing.assert_array_equal(hs[0][1], hs[1][1])


@pytest.mark.parametrize("precision", ["x3", "f32", "f32fwd", "f32x6"])
def test_guided_default_config_curve_vs_reference(precision):
    """exp_cdm_guidedTF.sh (lr 1e-2, penalty 0.1, B=128): ploss / loss / compare vs
    the reference's 8-thread CPU run.  f32: within 1e-4 or twice the reference's
    own 2-vs-8-thread spread up to that step (conftest.curve_bound); x3: 2e-3."""
    g = np.load(os.path.join(GOLDEN, "cdm_guided_curve.npz"))
    g2 = np.load(os.path.join(GOLDEN, "cdm_guided_curve_t2.npz"))
    n = len(g["ploss"])
    s, tr = _trainer(9, 128, precision=precision)
    for k in range(n):
        _draw(s, tr, 128)
        tr.step()
        if k == 2:
            tr.capture()
    torch.cuda.synchronize()
    ph, h, ch = tr.ploss_history(), tr.loss_history(), tr.compare_history()
    msg = []
    ok = True
    for key, got in (("ploss", ph), ("loss", h), ("compare", ch)):
        d = np.abs(got - g[key]) / np.abs(g[key])
        b, w, sp = curve_bound(g[key], g2[key])
        msg.append(f"{key} {d.max():.3e} (spread {sp[-1]:.3e}, window {w}, in-window {d[:w].max() if w else 0:.3e})")
        # f32 and f32x6 (the x6 forward, the exact-f32 backward: the guided joint
        # default since round 6, measured 3.8e-6 / 1.7e-5 / 2.1e-5) are the parity
        # claim; x3 is opt-in: lr 1e-2 grows its rounding to ~1e-3 over 30 steps
        # (measured 1.3e-4 / 6.6e-4 / 9.3e-4); f32fwd (f32-accurate forward, x3
        # backward) behaves as x3 here (8.1e-5 / 6.8e-4 / 9.5e-4): the lr-1e-2 run
        # amplifies the backward's rounding, so it is held to x3's envelope
        ok = ok and bool((d <= b).all() if precision in ("f32", "f32x6") else d.max() <= 2e-3)
    print(f"guided CDM curve ({precision}), {n} steps: " + "; ".join(msg))
    assert ok
