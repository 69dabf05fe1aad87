"""Guided joint VLM (train_NWP.py --guide=True, exp_vlm_guidedTF.sh: L = 9, d = 256,
all 9 layers text-guided, layers 0-3 image-guided, penalty 0.001) on the HIP path
vs the reference's own fixtures (tests/golden/make_golden_vlm_guided.py).
Targets come from the host BP (bp_nwp_posterior(guide=True), pinned against the
reference in tests/test_vlm_guided_host.py); the penalties and their gradients
run in the fused step.  Tolerances as the other split-bf16 VLM tests: losses 1e-4
relative, gradient / parameter checksums 5e-4."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DEV = "cuda"
P_Y = np.ones(10) / 10


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _trainer(B, total_iters=30000):
    """train_NWP.py order: sampler (seedtree 42), seed_everything(224), the model."""
    from ghmclip import AutoRegressiveTransformer, NextWordPredictSampler, get_lr_cosine_schedule, seed_everything
    from ghmclip.training.vlm_trainer import VlmTrainer
    s = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2])
    seed_everything(224)
    model = AutoRegressiveTransformer(161, 81, 10, 256, 9, [4, 4], 4, 1024, auto_regressive=True,
                                      sequential=False, guide=True).to(DEV)
    sched = [get_lr_cosine_schedule(k, 1e-3, 1e-6, 0, total_iters) for k in range(total_iters)]
    tr = VlmTrainer(model, None, B, sched, device=DEV, precision="x3", penalty=0.001)
    return s, tr


def _stage(s, trs, B):
    """Draw one batch (the sampler uses numpy's global stream, as the reference)
    and stage it on every trainer in `trs`."""
    from ghmclip.data.data_random_GHM import vlm_guide_planes
    tl, il, _ = s.draw_numpy(B)
    post, _, tg, ig = s.posterior(tl, il, guide=True)
    planes = vlm_guide_planes(tg, ig, 10)
    for tr in (trs if isinstance(trs, (list, tuple)) else [trs]):
        tr.set_batch(torch.from_numpy(np.ascontiguousarray(tl[:, :-1])), torch.from_numpy(np.ascontiguousarray(tl[:, 1:])),
                     torch.from_numpy(post), torch.from_numpy(il), torch.from_numpy(planes))
    return tl, il


def test_guided_vlm_steps_vs_reference_fixture():
    f = np.load(os.path.join(GOLDEN, "vlm_guided_tiny.npz"))
    B = int(f["B"])
    s, tr = _trainer(B)
    assert tr.model.t_guided_layer_flag == [True] * 9 and tr.model.i_guided_layer_flag == [True] * 4 + [False] * 5
    for k in range(2):
        tl, il = _stage(s, tr, B)
        np.testing.assert_array_equal(tl[:, :-1], f[f"xt{k}"])
        np.testing.assert_array_equal(il, f[f"i_leaves{k}"])
        tr.step()
        torch.cuda.synchronize()
        pen = tr.guide_penalties()
        want_pen = f[f"pen{k}"]
        np.testing.assert_allclose(pen, want_pen, rtol=1e-4, err_msg=f"penalty groups step {k}")
        names = list(f["param_names"])
        sd = dict(tr.model.named_parameters())
        for n, st in zip(names, f[f"param_stats{k}"]):
            got = (sd[n].detach().double() ** 2).sum().item()
            assert abs(got - st[1]) <= 5e-4 * st[1] + 1e-12, (k, n, got, st[1])
    ph, h, c = tr.ploss_history(), tr.loss_history(), tr.compare_history()
    for k in range(2):
        assert abs(ph[k] - float(f[f"ploss{k}"])) <= 1e-4 * float(f[f"ploss{k}"]), (k, ph[k])
        assert abs(h[k] - float(f[f"loss{k}"])) <= 1e-4 * float(f[f"loss{k}"]), (k, h[k])
        assert abs(c[k] - float(f[f"compare{k}"])) <= 1e-4 * float(f[f"compare{k}"]), (k, c[k])


def test_guided_vlm_module_api_first_step_gradients():
    """AutoRegressiveTransformer(guide=True).forward returns the reference's guided
    outputs ([9 text, 4 image]); ConditionalGuidedCELoss(guide=True) on them
    gives the fixture's step-0 penalised loss and gradients (through the module's
    autograd: guided-output gradients enter the residual stream before each
    layer's backward)."""
    from ghmclip import AutoRegressiveTransformer, NextWordPredictSampler, seed_everything
    from ghmclip.models.vlm import ConditionalGuidedCELoss
    f = np.load(os.path.join(GOLDEN, "vlm_guided_tiny.npz"))
    B = int(f["B"])
    s = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2])
    seed_everything(224)
    model = AutoRegressiveTransformer(161, 81, 10, 256, 9, [4, 4], 4, 1024, auto_regressive=True,
                                      sequential=False, guide=True).to(DEV)
    model.precision = "x3"
    rt, ri = s.get_batch(batch_size=B, device=DEV, guide=True)
    out = model(rt[0], ri[0])
    assert len(out[1][0]) == 9 and len(out[1][1]) == 4
    assert [tuple(t.shape) for t in out[1][0]] == [(B, 80, 10)] + [(B, 80, 20)] * 4 + [(B, 80, 10)] * 4
    assert all(tuple(t.shape) == (B, 81, 10) for t in out[1][1])
    loss = ConditionalGuidedCELoss(penalty=0.001, guide=True)
    res = loss(out, [rt[1], [rt[2], ri[2]]])
    res[0].backward()
    torch.cuda.synchronize()
    assert abs(res[0].item() - float(f["ploss0"])) <= 1e-4 * float(f["ploss0"])
    np.testing.assert_allclose(res[1:], f["pen0"], rtol=1e-4)
    sd = dict(model.named_parameters())
    # the fixture's gradients are recorded after clip_grad_norm_(max_norm=1) (in place)
    tot = sum((p.grad.detach().double() ** 2).sum().item() for p in sd.values() if p.grad is not None) ** 0.5
    coef = min(1.0, 1.0 / (tot + 1e-6))
    for n, st in zip(list(f["grad_names0"]), f["grad_stats0"]):
        got = (sd[n].grad.detach().double() ** 2).sum().item() * coef ** 2
        assert abs(got - st[1]) <= 5e-4 * st[1] + 1e-20, (n, got, st[1])


def test_guided_vlm_graph_replay_bit_identical():
    _, t1 = _trainer(4)
    s2, t2 = _trainer(4)
    for k in range(4):
        _stage(s2, [t1, t2], 4)
        t1.step()
        t2.step()
        if k == 1:
            t2.capture()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(t1.ploss_history(), t2.ploss_history())
    np.testing.assert_array_equal(t1.compare_history(), t2.compare_history())


@pytest.mark.parametrize("steps", [20])
def test_guided_vlm_curve_vs_reference(steps):
    path = os.path.join(GOLDEN, "vlm_guided_curve.npz")
    if not os.path.exists(path):
        pytest.skip("vlm_guided_curve.npz not generated")
    f = np.load(path)
    n = min(steps, len(f["ploss"]))
    s, tr = _trainer(128)
    for k in range(n):
        _stage(s, tr, 128)
        tr.step()
        if k == 1:
            tr.capture()
    torch.cuda.synchronize()
    ph, h, c = tr.ploss_history(), tr.loss_history(), tr.compare_history()
    rel = lambda a, b: np.abs(a[:n] - b[:n]) / np.abs(b[:n])  # noqa: E731
    print(f"guided VLM curve {n} steps: ploss {rel(ph, f['ploss']).max():.2e} loss {rel(h, f['loss']).max():.2e} "
          f"compare {rel(c, f['compare']).max():.2e}")
    assert rel(ph, f["ploss"]).max() < 1e-4
    assert rel(h, f["loss"]).max() < 1e-4
    assert rel(c, f["compare"]).max() < 1e-4
