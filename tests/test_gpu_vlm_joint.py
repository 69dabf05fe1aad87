"""Joint VLM (train_NWP.py, exp_vlm_jointtrain.sh: sequential=False, the 81 image
leaves through i_embedding as the prefix of the 80 text tokens, T = 161) on the HIP
path vs the CPU oracle and the reference's own fixtures
(tests/golden/make_golden_vlm_joint.py).  Sequences past 96 tokens run on the
split-bf16 kernels only: tolerances as the x3 VLM tests (forward / losses 1e-4,
gradients 5e-4 relative)."""
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


@pytest.mark.parametrize("B,d", [(4, 256), (3, 128)])
def test_joint_vlm_module_forward_backward(B, d):
    from ghmclip import AutoRegressiveTransformer
    torch.manual_seed(21)
    prod = AutoRegressiveTransformer(161, 81, 10, d, 2, [4, 4], 4, 4 * d, auto_regressive=True, sequential=False)
    torch.manual_seed(21)
    ref = VO.OracleVlm(161, 81, 10, d, 2, 4 * d, sequential=False)
    g = torch.Generator().manual_seed(B)
    with torch.no_grad():
        for (kp, vp), (_, vr) in zip(prod.named_parameters(), ref.named_parameters()):
            assert torch.equal(vp, vr), kp
            if "_lns_" in kp or kp.endswith("bias"):
                dd = 0.1 * torch.randn(vp.shape, generator=g)
                vp.add_(dd)
                vr.add_(dd)
    prod.precision = "x3"
    prod = prod.to(DEV)
    xt = torch.randint(0, 10, (B, 80), generator=g)
    il = torch.randint(0, 10, (B, 81), generator=g)
    R = torch.randn(B, 80, 10, generator=g)
    logits, gl = prod(xt.to(DEV), il.to(DEV))
    assert gl == [[], []]
    (logits * R.to(DEV)).sum().backward()
    want = ref(xt, il)
    (want * R).sum().backward()
    torch.cuda.synchronize()
    assert _rel(logits, want) < 1e-4
    for (k, pp), (_, pr) in zip(prod.named_parameters(), ref.named_parameters()):
        if pr.grad is None:
            assert pp.grad is None, k
            continue
        assert _rel(pp.grad, pr.grad) < 5e-4, k


def _trainer(L, B, total_iters=30000):
    """train_NWP.py order: sampler (seedtree 42), seed_everything(224), the model."""
    from ghmclip import AutoRegressiveTransformer, NextWordPredictSampler, get_lr_cosine_schedule, seed_everything
    from ghmclip.training.vlm_trainer import VlmTrainer
    s = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2])
    seed_everything(224)
    model = AutoRegressiveTransformer(161, 81, 10, 256, L, [4, 4], 4, 1024, auto_regressive=True,
                                      sequential=False).to(DEV)
    sched = [get_lr_cosine_schedule(k, 1e-3, 1e-6, 0, total_iters) for k in range(total_iters)]
    tr = VlmTrainer(model, None, B, sched, device=DEV, precision="x3")
    return s, tr


def _run(s, tr, B, steps, graph_after=None):
    for k in range(steps):
        tl, il, _ = s.draw_numpy(B)
        post, _ = s.posterior(tl, il)
        tr.set_batch(torch.from_numpy(np.ascontiguousarray(tl[:, :-1])),
                     torch.from_numpy(np.ascontiguousarray(tl[:, 1:])), torch.from_numpy(post),
                     torch.from_numpy(il))
        tr.step()
        if graph_after is not None and k + 1 == graph_after:
            tr.capture()
    torch.cuda.synchronize()
    return tr.loss_history(), tr.compare_history()


def test_joint_vlm_steps_vs_reference_fixture():
    f = np.load(os.path.join(GOLDEN, "vlm_joint_tiny.npz"))
    s, tr = _trainer(1, 4)
    for (n, p), want in zip(tr.model.named_parameters(), f["init_stats"]):
        assert abs((p.double() ** 2).sum().item() - want[1]) <= 1e-12 * want[1] + 1e-12, n
    hist, chist = _run(s, tr, 4, 2)
    for k in range(2):
        assert abs(hist[k] - float(f[f"ploss{k}"])) <= 1e-4 * float(f[f"ploss{k}"]), (k, hist[k])
        assert abs(chist[k] - float(f[f"compare{k}"])) <= 1e-4 * float(f[f"compare{k}"]), (k, chist[k])


def test_joint_vlm_steps_vs_oracle():
    s, tr = _trainer(2, 6)
    ref = VO.OracleVlmJointTrainer(B=6, L=2)
    rparams = dict(ref.model.named_parameters())
    for it in range(2):
        tl, il, _ = s.draw_numpy(6)
        post, _ = s.posterior(tl, il)
        tr.set_batch(torch.from_numpy(np.ascontiguousarray(tl[:, :-1])),
                     torch.from_numpy(np.ascontiguousarray(tl[:, 1:])), torch.from_numpy(post),
                     torch.from_numpy(il))
        tr.step()
        ploss, _, cmp = ref.step(batch=(tl[:, :-1].astype(np.int64), tl[:, 1:].astype(np.int64), post,
                                        il.astype(np.int64)))
        torch.cuda.synchronize()
        assert abs(tr.loss_history()[it] - ploss) <= 1e-4 * ploss
        assert abs(tr.compare_history()[it] - cmp) <= 1e-4 * cmp
        coef = tr.hyper[1].item()
        for n, p in tr.model.named_parameters():
            if n in tr.gd:
                assert _rel(p.grad * coef, rparams[n].grad) < 5e-4, n
        assert "i_embedding.weight" in tr.gd


def test_joint_vlm_graph_replay_matches_eager():
    s1, t1 = _trainer(1, 4)
    h1 = _run(s1, t1, 4, 5)
    s2, t2 = _trainer(1, 4)
    h2 = _run(s2, t2, 4, 5, graph_after=2)
    np.testing.assert_array_equal(h1[0], h2[0])
    np.testing.assert_array_equal(h1[1], h2[1])


def test_joint_vlm_default_config_curve_vs_reference():
    """exp_vlm_jointtrain.sh config (p=0.2, L=9, d=256, B=128, lr 1e-3 -> 1e-6):
    loss and Compare histories vs the reference PyTorch-CPU run."""
    g = np.load(os.path.join(GOLDEN, "vlm_joint_curve.npz"))
    n = len(g["loss"])
    s, tr = _trainer(9, 128)
    hist, chist = _run(s, tr, 128, n, graph_after=3)
    dev = np.abs(hist - g["loss"]) / g["loss"]
    cdev = np.abs(chist - g["compare"]) / g["compare"]
    print(f"joint VLM curve (x3): {n} steps, max rel dloss {dev.max():.3e}, dcompare {cdev.max():.3e}, "
          f"final {hist[-1]:.5f} vs {g['loss'][-1]:.5f}")
    assert dev.max() <= 1e-4 and cdev.max() <= 1e-4
