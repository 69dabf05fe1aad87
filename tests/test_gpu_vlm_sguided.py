"""Guided sequential VLM (train_sequential_NWP.py --guide=True: L = 9, d = 256,
n_guided_layers = [4, 1], penalty 0.001), the relu-attention VLM
(AutoRegressiveTransformer(activation="relu"), model.py:121-130, 287) and the VLM
without LayerNorm (layernorm=False, model.py:269-277, 294-301) on the HIP path vs
the reference's own fixtures (tests/golden/make_golden_vlm.py).

Guided sequential: every layer is text-guided (gap 9 // 9 = 1) and layers 0 and 3
image-guided (model.py:207-216: counter < 1, and counter == n_t - 1 with n_i < n_t);
the text targets come from the host BP (bp_nwp_posterior(guide=True)), the two image
blocks H[:, 0, 0:10] / H[:, 0, 10:20] target the frozen CLIP feature itself
(train_sequential_NWP.py:165), which the fused trainer reads from the CLIP
encoder's output on the device.  Tolerances as the other split-bf16 VLM tests:
losses and penalties 1e-4 relative, gradient / parameter checksums 5e-4."""
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


def _trainer(B, L=9, guide=True, activation="softmax", total_iters=30000, layernorm=True, precision="x3"):
    """train_sequential_NWP.py order (raw=True): sampler, the CLIP image encoder
    (torch.manual_seed(7), as the fixtures), seed_everything(224), the model."""
    from ghmclip import AutoRegressiveTransformer, EncoderTransformer, NextWordPredictSampler, seed_everything
    from ghmclip import get_lr_cosine_schedule
    from ghmclip.training.vlm_trainer import VlmTrainer
    s = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2])
    torch.manual_seed(7)
    clip = EncoderTransformer(81, 10, 128, 5).to(DEV)
    seed_everything(224)
    model = AutoRegressiveTransformer(81, 1, 10, 256, L, [4, 1], 4, 1024, auto_regressive=True, sequential=True,
                                      guide=guide, activation=activation, layernorm=layernorm).to(DEV)
    sched = [get_lr_cosine_schedule(k, 1e-3, 1e-6, 0, total_iters) for k in range(total_iters)]
    tr = VlmTrainer(model, clip, B, sched, device=DEV, precision=precision, penalty=0.001)
    return s, clip, tr


def _stage(s, trs, B, guide=True):
    from ghmclip.data.data_random_GHM import vlm_guide_planes
    tl, il, _ = s.draw_numpy(B)
    if guide:
        post, _, tg, _ = s.posterior(tl, il, guide=True)
        extra = (torch.from_numpy(vlm_guide_planes(tg, [], 10)),)
    else:
        post = s.posterior(tl, il)[0]
        extra = ()
    for tr in (trs if isinstance(trs, (list, tuple)) else [trs]):
        tr.set_batch(torch.from_numpy(np.ascontiguousarray(tl[:, :-1])), torch.from_numpy(np.ascontiguousarray(tl[:, 1:])),
                     torch.from_numpy(post), torch.from_numpy(il), *extra)
    return tl, il


def _check_params(tr, f, k):
    sd = dict(tr.model.named_parameters())
    for n, st in zip(list(f["param_names"]), f[f"param_stats{k}"]):
        got = (sd[n].detach().double() ** 2).sum().item()
        assert abs(got - st[1]) <= 5e-4 * st[1] + 1e-12, (k, n, got, st[1])


def test_sguided_flags_and_plane_layout():
    _, _, tr = _trainer(4)
    m = tr.model
    assert m.t_guided_layer_flag == [True] * 9
    assert m.i_guided_layer_flag == [True, False, False, True] + [False] * 5
    assert tr.n_gelems == 80 * 10 * 13
    img = [(l, b) for l, b in tr.gitems if b[4] == "loss3"]
    assert [(l, b[0], b[1], b[2]) for l, b in img] == [(0, 0, 1, 0), (3, 0, 1, 10)]


def test_sguided_vlm_steps_vs_reference_fixture():
    f = np.load(os.path.join(GOLDEN, "vlm_sguided_tiny.npz"))
    assert bool(f["guide"]) and int(f["L"]) == 9
    B = int(f["B"])
    s, _, tr = _trainer(B)
    for (n, p), want in zip(tr.model.named_parameters(), f["init_stats"]):
        assert abs((p.double() ** 2).sum().item() - want[1]) <= 1e-12 * want[1] + 1e-12, n
    for k in range(2):
        tl, il = _stage(s, tr, B)
        np.testing.assert_array_equal(tl[:, :-1], f[f"xt{k}"])
        np.testing.assert_array_equal(il, f[f"i_leaves{k}"])
        tr.step()
        torch.cuda.synchronize()
        np.testing.assert_allclose(tr.clip_plan.emb.cpu().numpy(), f[f"feat{k}"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(tr.guide_penalties(), f[f"penalties{k}"], rtol=1e-4,
                                   err_msg=f"penalty groups (loss2, loss4, loss5, loss3) step {k}")
        _check_params(tr, f, k)
    ph, h, c = tr.ploss_history(), tr.loss_history(), tr.compare_history()
    for k in range(2):
        assert abs(ph[k] - float(f[f"ploss{k}"])) <= 1e-4 * float(f[f"ploss{k}"]), (k, ph[k])
        assert abs(h[k] - float(f[f"loss{k}"])) <= 1e-4 * float(f[f"loss{k}"]), (k, h[k])
        assert abs(c[k] - float(f[f"compare{k}"])) <= 1e-4 * float(f[f"compare{k}"]), (k, c[k])


def test_sguided_vlm_module_api_first_step_gradients():
    """AutoRegressiveTransformer(sequential=True, guide=True).forward returns the
    reference's guided outputs ([9 text, 2 image]); ConditionalGuidedCELoss on them
    with the CLIP feature as both image targets gives the fixture's step-0
    penalised loss, penalties and (clipped) gradients."""
    from ghmclip.models.vlm import ConditionalGuidedCELoss
    f = np.load(os.path.join(GOLDEN, "vlm_sguided_tiny.npz"))
    B = int(f["B"])
    s, clip, tr = _trainer(B)
    model = tr.model
    rt, ri = s.get_batch(batch_size=B, device=DEV, guide=True)
    feat = clip(ri[0])[0].unsqueeze(1).detach()
    out = model(rt[0], feat)
    assert len(out[1][0]) == 9 and len(out[1][1]) == 2
    assert all(tuple(t.shape) == (B, 1, 10) for t in out[1][1])
    for p in model.parameters():
        p.grad = None
    res = ConditionalGuidedCELoss(penalty=0.001, guide=True)(out, [rt[1], [rt[-2], [feat, feat]]])
    res[0].backward()
    torch.cuda.synchronize()
    assert abs(res[0].item() - float(f["ploss0"])) <= 1e-4 * float(f["ploss0"])
    np.testing.assert_allclose(res[1:], f["penalties0"], rtol=1e-4)
    sd = dict(model.named_parameters())
    tot = sum((p.grad.detach().double() ** 2).sum().item() for p in sd.values() if p.grad is not None) ** 0.5
    coef = min(1.0, 1.0 / (tot + 1e-6))
    for n, st in zip(list(f["grad_names0"]), f["grad_stats0"]):
        got = (sd[n].grad.detach().double() ** 2).sum().item() * coef ** 2
        assert abs(got - st[1]) <= 5e-4 * st[1] + 1e-20, (n, got, st[1])


def test_sguided_vlm_graph_replay_bit_identical():
    s1, _, t1 = _trainer(4)
    s2, _, t2 = _trainer(4)
    for k in range(4):
        _stage(s2, [t1, t2], 4)
        t1.step()
        t2.step()
        if k == 1:
            t2.capture()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(t1.ploss_history(), t2.ploss_history())
    np.testing.assert_array_equal(t1.compare_history(), t2.compare_history())


def test_sguided_vlm_curve_vs_reference():
    f = np.load(os.path.join(GOLDEN, "vlm_sguided_curve.npz"))
    n = len(f["ploss"])
    s, _, tr = _trainer(128)
    pen = []
    for k in range(n):
        _stage(s, tr, 128)
        tr.step()
        pen.append(tr.guide_penalties())
        if k == 1:
            tr.capture()
    torch.cuda.synchronize()
    ph, h, c = tr.ploss_history(), tr.loss_history(), tr.compare_history()
    rel = lambda a, b: np.abs(a[:n] - b[:n]) / np.abs(b[:n])  # noqa: E731
    pr = np.abs(np.array(pen) - f["penalties"]) / np.abs(f["penalties"])
    print(f"guided sequential VLM curve {n} steps: ploss {rel(ph, f['ploss']).max():.2e} "
          f"loss {rel(h, f['loss']).max():.2e} compare {rel(c, f['compare']).max():.2e} penalties {pr.max():.2e}")
    assert rel(ph, f["ploss"]).max() < 1e-4
    assert rel(h, f["loss"]).max() < 1e-4
    assert rel(c, f["compare"]).max() < 1e-4
    assert pr.max() < 1e-3


def test_relu_vlm_steps_vs_reference_fixture():
    """activation="relu" (model.py:287: relu of the masked, scaled scores, masked
    entries 0), d=256, L=1, B=4, two fused steps (vlm_relu_tiny.npz)."""
    f = np.load(os.path.join(GOLDEN, "vlm_relu_tiny.npz"))
    assert str(f["activation"]) == "relu"
    B = int(f["B"])
    s, _, tr = _trainer(B, L=1, guide=False, activation="relu")
    assert tr.plan.act == 1
    for k in range(2):
        tl, il = _stage(s, tr, B, guide=False)
        np.testing.assert_array_equal(tl[:, :-1], f[f"xt{k}"])
        tr.step()
        torch.cuda.synchronize()
        got = tr.plan.logits.view(B, 81, 10)[:, 1:].cpu().numpy()
        want = f[f"logits{k}"]
        assert np.abs(got - want).max() <= 1e-4 * np.abs(want).max(), k
        _check_params(tr, f, k)
    h, c = tr.loss_history(), tr.compare_history()
    for k in range(2):
        assert abs(h[k] - float(f[f"ploss{k}"])) <= 1e-4 * float(f[f"ploss{k}"]), (k, h[k])
        assert abs(c[k] - float(f[f"compare{k}"])) <= 1e-4 * float(f[f"compare{k}"]), (k, c[k])


@pytest.mark.parametrize("B", [3, 5])
def test_relu_vlm_module_vs_oracle(B):
    """Module forward / backward with relu attention vs the oracle restatement
    (oracle/vlm_oracle.py OracleVlm(activation="relu"), pinned by vlm_relu_tiny.npz
    in tests/test_cdm_host.py): logits, parameter and prefix-feature gradients."""
    import oracle.vlm_oracle as VO
    from ghmclip import AutoRegressiveTransformer
    torch.manual_seed(13)
    prod = AutoRegressiveTransformer(81, 1, 10, 256, 2, [4, 1], 4, 1024, auto_regressive=True, sequential=True,
                                     activation="relu")
    torch.manual_seed(13)
    ref = VO.OracleVlm(81, 1, 10, 256, 2, 1024, activation="relu")
    prod.precision = "x3"
    prod = prod.to(DEV)
    g = torch.Generator().manual_seed(B)
    xt = torch.randint(0, 10, (B, 80), generator=g)
    feat = torch.randn(B, 1, 10, generator=g)
    R = torch.randn(B, 80, 10, generator=g)
    fd = feat.to(DEV).requires_grad_(True)
    logits, _ = prod(xt.to(DEV), fd)
    (logits * R.to(DEV)).sum().backward()
    fr = feat.clone().requires_grad_(True)
    want = ref(xt, fr)
    (want * R).sum().backward()
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.detach().cpu().double() - b.detach().double()).abs().max()  # noqa: E731
                        / b.detach().double().abs().max()).item()
    assert rel(logits, want) < 1e-4
    for (k, pp), (_, pr) in zip(prod.named_parameters(), ref.named_parameters()):
        if pr.grad is None:
            assert pp.grad is None, k
            continue
        assert rel(pp.grad, pr.grad) < 5e-4, k
    assert rel(fd.grad, fr.grad) < 5e-4


TOL = {"f32": (2e-5, 1e-4), "x3": (1e-4, 5e-4)}  # (losses, parameter checksums) relative, as test_gpu_vlm.py


@pytest.mark.parametrize("precision", ["f32", "x3"])
def test_noln_vlm_steps_vs_reference_fixture(precision):
    """layernorm=False, d=256, L=2, B=4: two fused steps (vlm_noln_tiny.npz); the
    LayerNorm parameters stay untouched (no gradient, no AdamW step)."""
    f = np.load(os.path.join(GOLDEN, "vlm_noln_tiny.npz"))
    assert not bool(f["layernorm"])
    tl_, tp = TOL[precision]
    B = int(f["B"])
    s, _, tr = _trainer(B, L=2, guide=False, layernorm=False, precision=precision)
    assert not tr.plan.layernorm and all("_lns_" not in n for n in tr.gd)
    ln0 = {n: p.detach().clone() for n, p in tr.model.named_parameters() if "_lns_" in n}
    for k in range(2):
        tl, il = _stage(s, tr, B, guide=False)
        np.testing.assert_array_equal(tl[:, :-1], f[f"xt{k}"])
        tr.step()
        torch.cuda.synchronize()
        sd = dict(tr.model.named_parameters())
        for n, st in zip(list(f["param_names"]), f[f"param_stats{k}"]):
            got = (sd[n].detach().double() ** 2).sum().item()
            assert abs(got - st[1]) <= tp * st[1] + 1e-12, (k, n, got, st[1])
    for n, v in ln0.items():
        assert torch.equal(dict(tr.model.named_parameters())[n].detach(), v), n
    h, c = tr.loss_history(), tr.compare_history()
    for k in range(2):
        assert abs(h[k] - float(f[f"ploss{k}"])) <= tl_ * float(f[f"ploss{k}"]), (k, h[k])
        assert abs(c[k] - float(f[f"compare{k}"])) <= tl_ * float(f[f"compare{k}"]), (k, c[k])


@pytest.mark.parametrize("precision", ["f32", "x3"])
def test_noln_vlm_module_vs_oracle(precision):
    """Module forward / backward with layernorm=False vs OracleVlm(layernorm=False)
    (pinned by vlm_noln_tiny.npz in tests/test_cdm_host.py): logits, gradients, no
    LayerNorm gradients."""
    import oracle.vlm_oracle as VO
    from ghmclip import AutoRegressiveTransformer
    tf, tg = TOL[precision]
    torch.manual_seed(17)
    prod = AutoRegressiveTransformer(81, 1, 10, 256, 2, [4, 1], 4, 1024, auto_regressive=True, sequential=True,
                                     layernorm=False)
    torch.manual_seed(17)
    ref = VO.OracleVlm(81, 1, 10, 256, 2, 1024, layernorm=False)
    prod.precision = precision
    prod = prod.to(DEV)
    g = torch.Generator().manual_seed(5)
    xt = torch.randint(0, 10, (4, 80), generator=g)
    feat = torch.randn(4, 1, 10, generator=g)
    R = torch.randn(4, 80, 10, generator=g)
    fd = feat.to(DEV).requires_grad_(True)
    logits, _ = prod(xt.to(DEV), fd)
    (logits * R.to(DEV)).sum().backward()
    fr = feat.clone().requires_grad_(True)
    want = ref(xt, fr)
    (want * R).sum().backward()
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.detach().cpu().double() - b.detach().double()).abs().max()  # noqa: E731
                        / b.detach().double().abs().max()).item()
    assert rel(logits, want) < tf
    for (k, pp), (_, pr) in zip(prod.named_parameters(), ref.named_parameters()):
        if pr.grad is None:
            assert pp.grad is None, k
            continue
        assert rel(pp.grad, pr.grad) < tg, k
    assert rel(fd.grad, fr.grad) < tg
