"""EncoderTransformer at widths other than 128 on the GEMM path
(models/gemm_encoder.py): n_embd = 64, the reference CLI's default
clip_{t,i}model_deb (utils/config.py:58-59), and 256.  Pinned to the reference's
own two training steps (tests/golden/clip_d64.npz / clip_d256.npz, make_golden.py
--only d64,d256; the oracle is checked against the same fixtures in
tests/test_oracle_golden.py) and to the oracle's float64 gradients."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ghm_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-12)


def _trainer(d, L, B, total_iters=3000, activation="softmax"):
    from ghmclip import ClipSampler, EncoderTransformer, get_lr_cosine_schedule, seed_everything
    from ghmclip.training.clip_trainer import ClipTrainer
    p_y = np.ones(10) / 10
    sampler = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
    seed_everything(224)
    tm = EncoderTransformer(81, 10, d, L, activation=activation).to(DEV)
    im = EncoderTransformer(81, 10, d, L, activation=activation).to(DEV)
    sched = [get_lr_cosine_schedule(s, 3e-4, 3e-7, 0, total_iters) for s in range(total_iters + 1)]
    return sampler, ClipTrainer(tm, im, 4, B, sched, device=DEV, precision="x3")


def _run(sampler, tr, B, steps, graph_after=None):
    for s in range(steps):
        tl, _, il, _ = sampler.draw_numpy(B)
        tr.set_tokens(torch.from_numpy(tl), torch.from_numpy(il))
        tr.step()
        if graph_after is not None and s + 1 == graph_after:
            tr.capture(graphs=True)
    torch.cuda.synchronize()
    return tr.loss_history()


@pytest.mark.parametrize("d", [64, 256])
def test_train_steps_vs_reference_fixture_width(d):
    """Two full ClipTrainer steps (both towers on the GEMM path, the K-way loss
    gradient recomputed per tower, clip, AdamW) against the reference's own run at
    n_embd = d, L = 2, B = 8: losses within 1e-5, every post-step parameter's sum
    of squares within 1e-5 relative (the bounds of the d = 128 fixture test)."""
    from ghmclip.models.gemm_encoder import GemmEncoderPlan
    gfx = np.load(os.path.join(GOLDEN, f"clip_d{d}.npz"))
    assert int(gfx["meta"][1]) == d
    sampler, tr = _trainer(d, 2, 8)
    assert all(isinstance(pl, GemmEncoderPlan) for pl in tr.plans)
    hist = _run(sampler, tr, 8, 2)
    for it in range(2):
        assert abs(hist[it] - float(gfx[f"s{it}.loss"])) < 1e-5, (it, hist[it], float(gfx[f"s{it}.loss"]))
    worst = []
    for pref, m in (("t", tr.tm), ("i", tr.im)):
        for k, v in m.state_dict().items():
            key = f"s1.post.{pref}.{k}"
            got = (v.double().cpu() ** 2).sum().item()
            want = float(gfx[key + ".cks"][1]) if key + ".cks" in gfx else float((gfx[key].astype(np.float64) ** 2).sum())
            worst.append((abs(got - want) / (want + 1e-12), f"{pref}.{k}"))
    worst.sort(reverse=True)
    print(f"d={d}: post-step sum-of-squares deviations, worst 3: {worst[:3]}")
    assert worst[0][0] <= 1e-5, worst[:3]


def _pair(d, L=2, T=81, seed=7, activation="softmax"):
    from ghmclip import EncoderTransformer
    torch.manual_seed(seed)
    prod = EncoderTransformer(T, 10, d, L, activation=activation)
    torch.manual_seed(seed)
    ref = O.OracleEncoder(T, 10, d, L, activation=activation)
    for (kp, vp), (kr, vr) in zip(prod.state_dict().items(), ref.state_dict().items()):
        assert kp == kr and torch.equal(vp, vr)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for (kp, vp), (_, vr) in zip(prod.named_parameters(), ref.named_parameters()):
            if "_lns_" in kp or kp.endswith("bias"):
                dd = 0.1 * torch.randn(vp.shape, generator=g)
                vp.add_(dd)
                vr.add_(dd)
    prod.precision = "x3"
    return prod.to(DEV), ref.double()


@pytest.mark.parametrize("d", [64, 256])
@pytest.mark.parametrize("activation", ["softmax", "relu", "gelu"])
@pytest.mark.parametrize("T,nseq", [(81, 20), (27, 7)])
def test_encoder_module_width(d, activation, T, nseq):
    """EncoderTransformer(n_embd=d) forward and every parameter gradient against the
    float64 oracle, at the split-bf16 bounds of the d = 128 module tests (1e-4
    forward, 5e-4 gradients, relative to each tensor's max); relu against the
    oracle taken with the kernels' own masks (a score inside the rounding band of
    zero can flip)."""
    from conftest import kernel_relu_masks
    prod, ref = _pair(d, T=T, activation=activation)
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 10, (nseq, T), generator=g)
    R = torch.randn(nseq, 10, generator=g, dtype=torch.float64)
    emb, _ = prod(x.to(DEV))
    (emb * R.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()
    if activation == "relu":  # the kernels' masks, checked to be relu's own but for near-zero scores
        masks = kernel_relu_masks(prod)
        ref.scores = []
        with torch.no_grad():
            ref(x)
        for s, m in zip(ref.scores, masks):
            assert int(((s > 0) != m).sum()) <= 16
        ref.scores, ref.relu_masks = None, masks
    want = ref(x)[0]
    (want * R).sum().backward()
    assert _rel(emb, want) < 1e-4
    for (k, pp), (_, pr) in zip(prod.named_parameters(), ref.named_parameters()):
        assert _rel(pp.grad, pr.grad) < 5e-4, k


def test_width_graph_replay_matches_eager():
    """Captured piece graphs of the GEMM-path step replay bit-identically to eager
    steps (d = 64)."""
    s1, t1 = _trainer(64, 2, 16)
    h1 = _run(s1, t1, 16, 5)
    p1 = t1.pflat.cpu().clone()
    s2, t2 = _trainer(64, 2, 16)
    h2 = _run(s2, t2, 16, 5, graph_after=2)
    np.testing.assert_array_equal(h1, h2)
    assert torch.equal(p1, t2.pflat.cpu())


def test_train_clip_cli_default_width(tmp_path, monkeypatch):
    """python -m ghmclip.training.train_CLIP with the reference's default model flags
    (clip_{t,i}model_deb = 64, clip_{t,i}model_nlayer = 10, clip_layernorm default;
    utils/config.py:53-64) -- only the run length and logging shortened -- trains
    on the GEMM path and writes its D64 run folder and checkpoint."""
    from ghmclip.training import train_CLIP
    monkeypatch.chdir(tmp_path)
    hist = train_CLIP.main(["--batch_size=16", "--total_iters=4", "--raw=False", "--log_interval=2",
                            "--eval_interval=2"])
    assert len(hist) == 5 and np.isfinite(hist).all()
    ck = glob.glob("logs/clip/*/TF_L10H4D64_L10H4D64/*/checkpoint.pth")  # job_name default "clip"
    assert len(ck) == 1, glob.glob("logs/*/*/*")
