"""Numerics of the split-bf16 ("x3") path, restated on the CPU.

The HIP kernels (multimodal-ghm_amd/csrc/ghm_split.h) evaluate every f32
product a*b as hi_a*hi_b + hi_a*lo_b + lo_a*hi_b with hi = bf16(x),
lo = bf16(x - hi), each bf16 x bf16 product exact in f32, and GELU / GELU'
through a fitted erfc polynomial.  These tests pin the error bounds the GPU
parity tolerances (tests/test_gpu_parity.py FWD_TOL / GRAD_TOL) rely on.
"""
import numpy as np
import pytest
import torch

# gelu_fast coefficients, copied from ghm_split.h (degree-8 fit of erfc(z) e^{z^2} / (2t))
GELU_R = [-0.02965068817138672, 0.14285887777805328, -0.24479423463344574, 0.1404150128364563,
          -0.014276500791311264, 0.10175687074661255, 0.12144583463668823, 0.14120244979858398,
          0.14104235172271729]


def _bf16(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(torch.bfloat16).float().numpy()


def split(x):
    hi = _bf16(x)
    lo = _bf16(x - hi)
    return hi, lo


def gemm_x3(a, b):
    """A[m,k] @ B[k,n] the way the kernels do it (f32 accumulation of exact products)."""
    ah, al = split(a)
    bh, bl = split(b)
    f = np.float32
    return (al.astype(f) @ bh.astype(f)) + (ah.astype(f) @ bl.astype(f)) + (ah.astype(f) @ bh.astype(f))


def test_split_reconstructs_to_2e16():
    x = np.random.default_rng(0).standard_normal(100000).astype(np.float32) * 10
    hi, lo = split(x)
    rel = np.abs((hi.astype(np.float64) + lo) - x) / np.abs(x)
    assert rel.max() < 2.0 ** -16


@pytest.mark.parametrize("k", [16, 128, 512])
def test_gemm_x3_error_bound(k):
    rng = np.random.default_rng(k)
    a = rng.standard_normal((64, k)).astype(np.float32)
    b = rng.standard_normal((k, 48)).astype(np.float32)
    exact = a.astype(np.float64) @ b.astype(np.float64)
    scale = np.abs(a).astype(np.float64) @ np.abs(b).astype(np.float64)
    err = np.abs(gemm_x3(a, b) - exact) / scale
    # dropped lo*lo term and bf16 truncation of lo: <= ~2^-15 of sum |a||b| per element
    assert err.max() < 2.0 ** -15
    f32 = np.abs(a @ b - exact) / scale
    assert err.max() < 64 * max(f32.max(), 2.0 ** -24)


def gelu_fast(x):
    """f32 restatement of gelu_fast (ghm_split.h)."""
    f = np.float32
    x = x.astype(f)
    z = (np.abs(x) * f(0.70710678118654752440)).astype(f)
    t = (f(1) / (f(0.5) * z + f(1))).astype(f)
    r = np.full_like(t, f(GELU_R[0]))
    for c in GELU_R[1:]:
        r = (r * t + f(c)).astype(f)
    e = np.exp2(((x * x).astype(f) * f(-0.72134752044448170368)).astype(np.float64)).astype(f)
    half = ((t * e).astype(f) * r).astype(f)
    phi = np.where(x >= 0, (f(1) - half).astype(f), half)
    g = (x * phi).astype(f)
    d = (phi + x * (e * f(0.39894228040143267794)).astype(f)).astype(f)
    return g, d


def test_gelu_fast_matches_erf_gelu():
    from scipy.special import erfc
    x = np.linspace(-12, 12, 400001).astype(np.float32)
    g, d = gelu_fast(x)
    xd = x.astype(np.float64)
    phi = 0.5 * erfc(-xd / np.sqrt(2))
    g_ref = xd * phi
    d_ref = phi + xd * np.exp(-0.5 * xd * xd) / np.sqrt(2 * np.pi)
    assert np.abs(g - g_ref).max() < 5e-7
    assert np.abs(d - d_ref).max() < 3e-7
    # and against the reference's own op (torch GELU, approximate='none', fp32)
    tg = torch.nn.functional.gelu(torch.from_numpy(x)).numpy()
    assert np.abs(g - tg).max() < 2e-6
