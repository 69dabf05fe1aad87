"""The ring weight-gradient kernel (ghm_wgrad_ring_x3, csrc/ghm_wgrad.hip) against
float64 references of the products it replaces (the autograd weight / bias
gradients of model.py:773-775 and :787-788): every operand-format pairing the
encoder step uses (dW2 = dY^T G with db2, dW1 = dU^T LN2(Hmid) with db1,
dWq|k|v = dqkv^T LN1(H)) plus the two fallback pairings, on the encoder's own
token count and on ragged ones (splits whose last step is partial, M not a
multiple of 32).  Tolerance: split-bf16 products carry ~2^-16 relative error each,
so the bound is 3e-5 of sum |a||b| per output element (the same budget as
tests/test_gpu_gemm.py)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _perm32_index(n):
    from ghmclip.models.hip_encoder import perm32
    return torch.tensor([perm32(q) for q in range(n)], dtype=torch.long)


def _split_planes(x):
    """f32 [M][n] -> (bf16 planes [2][M][n] in perm32 column order, the f32 value hi + lo)."""
    idx = _perm32_index(x.shape[1]).to(x.device)
    xp = x[:, idx]
    hi = xp.to(torch.bfloat16)
    lo = (xp - hi.float()).to(torch.bfloat16)
    planes = torch.stack([hi, lo]).contiguous()
    val = torch.empty_like(x)
    val[:, idx] = hi.float() + lo.float()
    return planes, val


def _ln(x, st, w, b):
    return (x - st[:, :1]) * st[:, 1:] * w + b


CASES = [  # (name, a_fmt, a_cols, b_fmt, b_cols, bias)
    ("dW2", 0, 128, 2, 512, True),
    ("dW1", 2, 512, 1, 128, True),
    ("dWqkv", 0, 384, 1, 128, False),
    ("split_x_f32", 2, 256, 0, 128, True),
    ("f32_x_f32", 0, 128, 0, 256, True),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("M,tps", [(51840, 832), (1000, 96), (333, 64), (40, 32)])
def test_wgrad_ring_matches_float64(case, M, tps):
    from ghmclip import _native
    _, af, ac, bf, bc, with_bias = case
    g = torch.Generator(device=DEV).manual_seed(M + 7 * ac + bc)
    A = torch.randn(M, ac, device=DEV, generator=g)
    B = torch.randn(M, bc, device=DEV, generator=g) * 2 + 0.5
    st = torch.stack([B.mean(1), torch.rsqrt(B.var(1, unbiased=False) + 1e-5)], 1).contiguous()
    lw = 1 + 0.1 * torch.randn(bc, device=DEV, generator=g)
    lb = 0.1 * torch.randn(bc, device=DEV, generator=g)
    if af == 2:
        a_buf, A_val = _split_planes(A)
        a_plane = M * ac
    else:
        a_buf, A_val, a_plane = A, A, 0
    if bf == 2:
        b_buf, B_val = _split_planes(B)
        b_plane = M * bc
    else:
        b_buf, B_val, b_plane = B, B, 0
    if bf == 1:
        B_val = _ln(B, st, lw, lb)
    nsplit = -(-M // tps)
    part = torch.full((nsplit, ac, bc), float("nan"), device=DEV)
    bias = torch.full((nsplit, ac), float("nan"), device=DEV) if with_bias else None
    P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _native.call("ghm_wgrad_ring_x3", P(a_buf), ac, ac, af, a_plane, P(b_buf), bc, bc, bf, b_plane,
                 P(st) if bf == 1 else None, P(lw) if bf == 1 else None, P(lb) if bf == 1 else None,
                 P(part), P(bias), M, tps, s)
    torch.cuda.synchronize()
    a64, b64 = A_val.double(), B_val.double()
    want = a64.t() @ b64
    scale = a64.abs().t() @ b64.abs()
    got = part.double().sum(0)
    assert torch.isfinite(got).all()
    err = ((got - want).abs() / scale.clamp_min(1e-30)).max().item()
    assert err < 3e-5, err
    # each split's partial is its own token range's product
    z = nsplit // 2
    lo_, hi_ = z * tps, min(M, (z + 1) * tps)
    wz = a64[lo_:hi_].t() @ b64[lo_:hi_]
    sz = a64[lo_:hi_].abs().t() @ b64[lo_:hi_].abs()
    assert ((part[z].double() - wz).abs() / sz.clamp_min(1e-30)).max().item() < 3e-5
    if with_bias:
        bw = a64.sum(0)
        bs = a64.abs().sum(0)
        berr = ((bias.double().sum(0) - bw).abs() / bs).max().item()
        assert berr < 1e-6, berr


def test_wgrad_ring_close_to_round4_kernel_on_the_encoder_step():
    """On a real training step's operands (default config, 51,840 tokens per
    tower) the product path's three ring launches give the gradients of the
    round-4 kernels (ghm_wgrad_x3 on f32 G / dU) to the x3 rounding: the two
    EncoderPlan paths (GHM_WGRAD_RING=7 every weight gradient on the ring / =0 the
    default) after one identical step."""
    import os
    import numpy as np
    from ghmclip import ClipSampler, EncoderTransformer, get_lr_cosine_schedule, seed_everything
    from ghmclip.training.clip_trainer import ClipTrainer
    grads = []
    for ring in ("7", "0"):
        os.environ["GHM_WGRAD_RING"] = ring
        try:
            p_y = np.ones(10) / 10
            sampler = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
            seed_everything(224)
            tm = EncoderTransformer(81, 10, 128, 5).to(DEV)
            im = EncoderTransformer(81, 10, 128, 5).to(DEV)
            sched = [get_lr_cosine_schedule(s, 3e-4, 3e-7, 0, 3000) for s in range(3001)]
            tr = ClipTrainer(tm, im, 4, 128, sched, device=DEV, precision="x3")
            assert tr.plans[0].wgrad_ring == (ring == "7") and tr.plans[0].wgrad_ring_qkv == (ring == "7")
            tl, _, il, _ = sampler.draw_numpy(128)
            tr.set_tokens(torch.from_numpy(tl), torch.from_numpy(il))
            tr.step()
            torch.cuda.synchronize()
            grads.append(tr.gflat.double().cpu().clone())
            del tr
        finally:
            os.environ.pop("GHM_WGRAD_RING", None)
    a, b = grads
    rel = ((a - b).abs().max() / b.abs().max()).item()
    assert rel < 2e-5, rel
