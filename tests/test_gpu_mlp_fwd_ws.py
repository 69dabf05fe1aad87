"""The wave-specialised MLP forward (k_ln_mlp_fwd_x3w, GHM_MLP_FWD_WS=1; review
item 3; =1: 8-wave workgroups, two per CU; =2: 16-wave, 256-token workgroups, one
per CU) against the default k_ln_mlp_fwd_x3b: the same products in the same
order, only scheduled differently (waves 4-7 one interval behind waves 0-3), so
the outputs, the LN2 statistics and a whole training step's gradients are
bit-identical.  Replaces model.py:784-788 (LN2 + Linear-GELU-Linear + residual)."""
import ctypes
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _trainer():
    from ghmclip import ClipSampler, EncoderTransformer, get_lr_cosine_schedule, seed_everything
    from ghmclip.training.clip_trainer import ClipTrainer
    p_y = np.ones(10) / 10
    sampler = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
    seed_everything(224)
    tm = EncoderTransformer(81, 10, 128, 5).to(DEV)
    im = EncoderTransformer(81, 10, 128, 5).to(DEV)
    sched = [get_lr_cosine_schedule(s, 3e-4, 3e-7, 0, 3000) for s in range(3001)]
    return sampler, ClipTrainer(tm, im, 4, 128, sched, device=DEV, precision="x3")


def _run(plan, p, Hmid, M, ws):
    from ghmclip import _native
    os.environ["GHM_MLP_FWD_WS"] = str(ws)
    try:
        H = torch.full((M, 128), float("nan"), device=DEV)
        st = torch.full((M, 2), float("nan"), device=DEV)
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _native.call("ghm_ln_mlp_fwd_x3b", P(Hmid), P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]),
                     P(plan.pack[0]), P(p["_mlps.0.0.bias"]), P(p["_mlps.0.2.bias"]), P(H), P(st), M, 128, 512,
                     plan.eps, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
    finally:
        os.environ.pop("GHM_MLP_FWD_WS", None)
    return H, st


@pytest.mark.parametrize("ws", [1, 2, 3, 4])
@pytest.mark.parametrize("M", [51840, 40001, 32768])
def test_ws_forward_bit_identical(M, ws):
    """Every M that takes the 128-token workgroups (>= 256 of them), ragged tails included."""
    sampler, tr = _trainer()
    tl, _, il, _ = sampler.draw_numpy(128)
    tr.set_tokens(torch.from_numpy(tl), torch.from_numpy(il))
    tr.step()
    torch.cuda.synchronize()
    plan, p = tr.plans[0], tr.views[0][0]
    g = torch.Generator(device=DEV).manual_seed(M)
    Hmid = torch.randn(M, 128, device=DEV, generator=g) * 1.5 + 0.25
    H0, s0 = _run(plan, p, Hmid, M, 0)
    H1, s1 = _run(plan, p, Hmid, M, ws)
    assert torch.isfinite(H0).all() and torch.isfinite(s0).all()
    assert torch.equal(H0, H1)
    assert torch.equal(s0, s1)


@pytest.mark.parametrize("mode", ["1", "2", "3", "4"])
def test_ws_step_gradients_bit_identical(mode):
    grads = []
    for ws in (mode, "0"):
        os.environ["GHM_MLP_FWD_WS"] = ws
        try:
            sampler, tr = _trainer()
            for _ in range(2):
                tl, _, il, _ = sampler.draw_numpy(128)
                tr.set_tokens(torch.from_numpy(tl), torch.from_numpy(il))
                tr.step()
            torch.cuda.synchronize()
            grads.append(tr.gflat.clone())
            del tr
        finally:
            os.environ.pop("GHM_MLP_FWD_WS", None)
    assert torch.equal(grads[0], grads[1])
