"""Sequential VLM (BASELINE config 5) on the HIP path vs the CPU oracle and the
reference's own fixtures (tests/golden/make_golden_vlm.py).

Every VLM projection runs on the hand-written GEMM template of csrc/ghm_gemm.hip
(`ghm_gemm_x3` split-bf16, or `ghm_gemm_f32` exact-f32 MFMA in the f32 mode; no
library GEMM), attention and the other operators on csrc/ghm_vlm.hip /
ghm_vlm_x3.hip; tolerances: forward 2e-5 and gradients 1e-4 relative to the
tensor's max-abs, losses 2e-5 relative (f32 mode; x3 as stated per test)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import vlm_oracle as VO

pytestmark = pytest.mark.gpu

DEV = "cuda"
P_Y = np.ones(10) / 10


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    scale = max(b.abs().max().item(), 1e-12)
    return (a - b).abs().max().item() / scale


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ghmclip import _native
    assert _native.hip_lib().ghm_device_ok() == 1, "libghm_hip.so not usable on this device"


TOL = {"f32": (2e-5, 1e-4), "x3": (1e-4, 5e-4)}  # (forward / loss, gradients), relative


def _pair(L=2, d=256, seed=13, precision="f32"):
    from ghmclip import AutoRegressiveTransformer
    torch.manual_seed(seed)
    prod = AutoRegressiveTransformer(81, 1, 10, d, L, [4, 1], 4, 4 * d, auto_regressive=True, sequential=True)
    torch.manual_seed(seed)
    ref = VO.OracleVlm(81, 1, 10, d, L, 4 * d)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for (kp, vp), (_, vr) in zip(prod.named_parameters(), ref.named_parameters()):
            assert torch.equal(vp, vr), kp
            if "_lns_" in kp or kp.endswith("bias"):
                dd = 0.1 * torch.randn(vp.shape, generator=g)
                vp.add_(dd)
                vr.add_(dd)
    prod.precision = precision
    return prod.to(DEV), ref


@pytest.mark.parametrize("precision", ["f32", "x3"])
@pytest.mark.parametrize("B,d", [(5, 256), (3, 128)])
def test_vlm_module_forward_backward(B, d, precision):
    """AutoRegressiveTransformer logits, parameter and prefix-feature gradients vs
    the oracle restatement of model.py:132-335 (mask, double residual)."""
    tf, tg = TOL[precision]
    prod, ref = _pair(d=d, precision=precision)
    g = torch.Generator().manual_seed(B)
    xt = torch.randint(0, 10, (B, 80), generator=g)
    feat = torch.randn(B, 1, 10, generator=g)
    R = torch.randn(B, 80, 10, generator=g)
    fd = feat.to(DEV).requires_grad_(True)
    logits, gl = prod(xt.to(DEV), fd)
    assert gl == [[], []]
    (logits * R.to(DEV)).sum().backward()
    fr = feat.clone().requires_grad_(True)
    want = ref(xt, fr)
    (want * R).sum().backward()
    torch.cuda.synchronize()
    assert _rel(logits, want) < tf
    for (k, pp), (_, pr) in zip(prod.named_parameters(), ref.named_parameters()):
        if pr.grad is None:
            assert pp.grad is None, k
            continue
        assert _rel(pp.grad, pr.grad) < tg, k
    assert _rel(fd.grad, fr.grad) < tg


def _trainer(L, B, total_iters=30000, d=256, precision="f32"):
    """train_sequential_NWP.py order (raw=True): sampler, CLIP image encoder
    (torch.manual_seed(7), as the fixtures), seed_everything(224), the model."""
    from ghmclip import AutoRegressiveTransformer, EncoderTransformer, NextWordPredictSampler, seed_everything
    from ghmclip import get_lr_cosine_schedule
    from ghmclip.training.vlm_trainer import VlmTrainer
    s = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2])
    torch.manual_seed(7)
    clip = EncoderTransformer(81, 10, 128, 5).to(DEV)
    seed_everything(224)
    model = AutoRegressiveTransformer(81, 1, 10, d, L, [4, 1], 4, 4 * d, auto_regressive=True,
                                      sequential=True).to(DEV)
    sched = [get_lr_cosine_schedule(k, 1e-3, 1e-6, 0, total_iters) for k in range(total_iters)]
    tr = VlmTrainer(model, clip, B, sched, device=DEV, precision=precision)
    return s, tr


def _batch(s, B):
    tl, il, _ = s.draw_numpy(B)
    post, _ = s.posterior(tl, il)
    return tl, il, post


def _run(s, tr, B, steps, graph_after=None):
    for k in range(steps):
        tl, il, post = _batch(s, B)
        tr.set_batch(torch.from_numpy(np.ascontiguousarray(tl[:, :-1])),
                     torch.from_numpy(np.ascontiguousarray(tl[:, 1:])), torch.from_numpy(post),
                     torch.from_numpy(il))
        tr.step()
        if graph_after is not None and k + 1 == graph_after:
            tr.capture()
    torch.cuda.synchronize()
    return tr.loss_history(), tr.compare_history()


def test_vlm_steps_vs_reference_fixture():
    """Two fused steps (d=256, L=1, B=4) against the reference's numbers (vlm_tiny.npz)."""
    f = np.load(os.path.join(GOLDEN, "vlm_tiny.npz"))
    s, tr = _trainer(1, 4)
    for (n, p), want in zip(tr.model.named_parameters(), f["init_stats"]):
        assert abs((p.double() ** 2).sum().item() - want[1]) <= 1e-12 * want[1] + 1e-12, n
    hist, chist = _run(s, tr, 4, 2)
    for k in range(2):
        assert abs(hist[k] - float(f[f"ploss{k}"])) <= 2e-5 * float(f[f"ploss{k}"]), (k, hist[k])
        assert abs(chist[k] - float(f[f"compare{k}"])) <= 2e-5 * float(f[f"compare{k}"]), (k, chist[k])


@pytest.mark.parametrize("precision", ["f32", "x3"])
def test_vlm_steps_vs_oracle(precision):
    """Fused step == the oracle's step on identical draws: logits, losses and the
    unclipped gradients (clip coefficient hyper[1])."""
    tf, tg = TOL[precision]
    s, tr = _trainer(2, 6, precision=precision)
    ref = VO.OracleVlmTrainer(B=6, L=2)
    rparams = dict(ref.model.named_parameters())
    for it in range(2):
        tl, il, post = _batch(s, 6)
        tr.set_batch(torch.from_numpy(np.ascontiguousarray(tl[:, :-1])),
                     torch.from_numpy(np.ascontiguousarray(tl[:, 1:])), torch.from_numpy(post),
                     torch.from_numpy(il))
        tr.step()
        ploss, _, cmp = ref.step(batch=(tl[:, :-1].astype(np.int64), tl[:, 1:].astype(np.int64), post,
                                        il.astype(np.int64)))
        torch.cuda.synchronize()
        assert abs(tr.loss_history()[it] - ploss) <= tf * ploss
        assert abs(tr.compare_history()[it] - cmp) <= tf * cmp
        coef = tr.hyper[1].item()
        for n, p in tr.model.named_parameters():
            if n in tr.gd:
                assert _rel(p.grad * coef, rparams[n].grad) < tg, n


@pytest.mark.parametrize("precision", ["f32", "x3"])
def test_vlm_graph_replay_matches_eager(precision):
    s1, t1 = _trainer(1, 4, precision=precision)
    h1 = _run(s1, t1, 4, 5)
    s2, t2 = _trainer(1, 4, precision=precision)
    h2 = _run(s2, t2, 4, 5, graph_after=2)
    np.testing.assert_array_equal(h1[0], h2[0])
    np.testing.assert_array_equal(h1[1], h2[1])


@pytest.mark.parametrize("precision", ["f32", "x3"])
def test_vlm_default_config_curve_vs_reference(precision):
    """BASELINE config 5 parity: the default VLM config (p=0.2, L=9, d=256, B=128,
    lr 1e-3 -> 1e-6) loss and Compare histories vs the reference PyTorch-CPU run."""
    g = np.load(os.path.join(GOLDEN, "vlm_curve.npz"))
    n = len(g["loss"])
    s, tr = _trainer(9, 128, precision=precision)
    hist, chist = _run(s, tr, 128, n, graph_after=3)
    dev = np.abs(hist - g["loss"]) / g["loss"]
    cdev = np.abs(chist - g["compare"]) / g["compare"]
    print(f"VLM curve ({precision}): {n} steps, max rel dloss {dev.max():.3e} (first 20: {dev[:20].max():.3e}), dcompare "
          f"{cdev.max():.3e} (first 20: {cdev[:20].max():.3e}), final {hist[-1]:.5f} vs {g['loss'][-1]:.5f}")
    # f32: measured 2.4e-7 (loss) / 1.0e-6 (compare) over all 40 steps; x3: budget 1e-4
    lim = 1e-5 if precision == "f32" else 1e-4
    assert dev.max() <= lim and cdev.max() <= lim


def test_nwp_pipeline_matches_sampler_draws():
    """NwpBatchPipeline (producer thread, pinned slots) yields the sampler's own
    reference-order draws and BP posteriors (train_sequential_NWP.py:159)."""
    from ghmclip import NextWordPredictSampler
    from ghmclip.training.pipeline import NwpBatchPipeline
    s = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2])
    np.random.seed(224)
    want = [_batch(s, 6) for _ in range(3)]
    np.random.seed(224)
    s.native.pull_numpy_state()

    class Rec:
        def __init__(self):
            self.got = []

        def set_batch(self, xt, yt, post, il):
            self.got.append([t.clone() for t in (xt, yt, post, il)])

    rec = Rec()
    pipe = NwpBatchPipeline(s, 6, n_slots=2)
    try:
        for _ in range(3):
            pipe.next_into(rec)
    finally:
        pipe.close()
    for (tl, il, post), (xt, yt, p, i) in zip(want, rec.got):
        np.testing.assert_array_equal(xt.numpy(), tl[:, :-1])
        np.testing.assert_array_equal(yt.numpy(), tl[:, 1:])
        np.testing.assert_array_equal(i.numpy(), il)
        np.testing.assert_array_equal(p.numpy(), post)


@pytest.mark.parametrize("d", [256, 128])
def test_presplit_weight_images_bit_identical(d, monkeypatch):
    """x3: the weight products on pre-split images (ghm_split_pack once per
    forward + ghm_gemm_x3p, GHM_VLM_PACK=1) give logits and every gradient bit for
    bit as the GEMMs that split the weights per tile (the default): the same
    split, the same products in the same order -- and a second forward after a
    weight update re-splits (the images follow the weights)."""
    from ghmclip import AutoRegressiveTransformer
    B = 4
    g = torch.Generator().manual_seed(d)
    xt = torch.randint(0, 10, (B, 80), generator=g).to(DEV)
    feat = torch.randn(B, 1, 10, generator=g).to(DEV)
    R = torch.randn(B, 80, 10, generator=g).to(DEV)
    outs = []
    for pack in ("0", "1"):
        monkeypatch.setenv("GHM_VLM_PACK", pack)
        torch.manual_seed(5)
        m = AutoRegressiveTransformer(81, 1, 10, d, 2, [4, 1], 4, 4 * d, auto_regressive=True,
                                      sequential=True).to(DEV)
        m.precision = "x3"
        res = []
        for it in range(2):
            fd = feat.clone().requires_grad_(True)
            logits, _ = m(xt, fd)
            (logits * R).sum().backward()
            torch.cuda.synchronize()
            res.append([logits.detach().cpu(), fd.grad.cpu()] + [p.grad.cpu().clone() for p in m.parameters()
                                                                  if p.grad is not None])
            with torch.no_grad():  # a weight update between the two forwards
                for p in m.parameters():
                    if p.grad is not None:
                        p.sub_(1e-2 * p.grad)
                        p.grad = None
        plan = next(iter(m._plans.values())) if hasattr(m, "_plans") else None
        if plan is not None and hasattr(plan, "pack_on"):
            assert plan.pack_on == (pack == "1")
        outs.append(res)
    for a, b in zip(outs[0], outs[1]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


@pytest.mark.parametrize("vec", ["1", "0"])
@pytest.mark.parametrize("D", [128, 256, 512])
def test_ln_rows_kernels_vs_float64(D, vec, monkeypatch):
    """ghm_ln_rows_fwd / ghm_ln_rows_bwd (the VLM's and CDM's row LayerNorms,
    model.py:340-343 nn.LayerNorm) against float64 torch: Y and the (mean, rstd)
    statistics, dX = dres + the LN backward (dres aliasing dX, as the VLM calls
    it) and the fixed-order dgamma / dbeta partials, on a ragged token count.
    GHM_LN_VEC=1 (default) is the float4-per-lane form for D = 256 / 512, 0 the
    one-float-per-lane kernels; tolerance 2e-5 of each tensor's max-abs."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    monkeypatch.setenv("GHM_LN_VEC", vec)
    g = torch.Generator().manual_seed(5)
    M, eps = 1037, 1e-5
    X = (torch.randn(M, D, generator=g) * 3 + 0.5).double()
    w, b = torch.randn(D, generator=g).double(), torch.randn(D, generator=g).double()
    dY, dres = torch.randn(M, D, generator=g).double(), torch.randn(M, D, generator=g).double()
    import ctypes
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    Xd, wd, bd = X.float().to(DEV), w.float().to(DEV), b.float().to(DEV)
    Y, st = torch.empty(M, D, device=DEV), torch.empty(M, 2, device=DEV)
    _native.call("ghm_ln_rows_fwd", _ptr(Xd), _ptr(wd), _ptr(bd), _ptr(Y), _ptr(st), M, D, eps, s)
    nblk = int(_native.hip_lib().ghm_ln_rows_blocks(M))
    part = torch.empty(nblk, 2, D, device=DEV)
    dX = dres.float().to(DEV)  # dres aliases dX
    _native.call("ghm_ln_rows_bwd", _ptr(dY.float().to(DEV)), _ptr(Xd), _ptr(st), _ptr(wd), _ptr(dX), _ptr(dX),
                 _ptr(part), M, D, s)
    torch.cuda.synchronize()
    Xr = X.float().double().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(Xr, (D,), w.float().double(), b.float().double(), eps)
    ref.backward(dY.float().double())
    mean = Xr.detach().mean(1)
    rstd = 1 / (Xr.detach().var(1, unbiased=False) + eps).sqrt()
    xhat = (Xr.detach() - mean[:, None]) * rstd[:, None]
    assert _rel(Y, ref) < 2e-5
    assert _rel(st[:, 0], mean) < 2e-5 and _rel(st[:, 1], rstd) < 2e-5
    assert _rel(dX, dres.float().double() + Xr.grad) < 2e-5
    dYf = dY.float().double()
    assert _rel(part[:, 0].sum(0), (dYf * xhat).sum(0)) < 2e-5
    assert _rel(part[:, 1].sum(0), dYf.sum(0)) < 2e-5
