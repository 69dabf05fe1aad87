"""Split-bf16 (x3) GEMM (csrc/ghm_gemm.hip), its exact-f32 variant (ghm_gemm_f32:
the VLM's precision "f32" mode) and the VLM's split-bf16 attention
(csrc/ghm_vlm_x3.hip) against float64 torch references of the same ops.

Tolerance of a split-bf16 product: every bf16 x bf16 partial product is exact in
f32; the dropped lo*lo term and the bf16 rounding of lo bound the error at about
2^-16 of sum_k |a||b| per element (tests/test_split_numerics.py pins that bound on
the CPU), so each element is checked against 4e-5 * (|A| |B|)[m][n]; the f32
variant (f32 products, f32 accumulation over K <= 1024) against 4e-6."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
EPI_STORE, EPI_GELU, EPI_RESID, EPI_MUL, EPI_SLAB = range(5)
REL = 4e-5
RELS = {False: 4e-5, True: 4e-6}  # f32=False: split-bf16; True: exact-f32 products


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ghmclip import _native
    assert _native.hip_lib().ghm_device_ok() == 1


def _gemm(*a, **k):
    from ghmclip.models.vlm import _gemm as g
    g(*a, **k)


def _gelu64(u):
    return u * 0.5 * (1 + torch.erf(u / math.sqrt(2)))


def _dgelu64(u):
    return 0.5 * (1 + torch.erf(u / math.sqrt(2))) + u * torch.exp(-0.5 * u * u) / math.sqrt(2 * math.pi)


def _check(got, want, bound, what):
    err = (got.double().cpu() - want).abs()
    bad = err > bound
    assert not bad.any(), f"{what}: max err {err.max().item():.3e}, worst ratio {(err / bound).max().item():.2f}"


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("M", [405, 1280])
@pytest.mark.parametrize("K,N", [(256, 256), (256, 1024), (128, 512), (1024, 256)])
def test_forward_shapes(M, K, N, f32):
    """Y = X W^T (ta=0, tb=1) with the store, GELU and bias+residual epilogues."""
    REL = RELS[f32]
    g = torch.Generator().manual_seed(M + K + N)
    X = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    Xd, Wd, bd, Rd = X.to(DEV), W.to(DEV), b.to(DEV), R.to(DEV)
    acc = X.double() @ W.double().t()
    bound = REL * (X.double().abs() @ W.double().abs().t()) + 1e-6
    C = torch.empty(M, N, device=DEV)
    _gemm(0, 1, EPI_STORE, Xd, K, (Wd,), K, 0, C, N, M, N, K, f32=f32)
    torch.cuda.synchronize()
    _check(C, acc, bound, "store")
    C2 = torch.empty(M, N, device=DEV)
    _gemm(0, 1, EPI_GELU, Xd, K, (Wd,), K, 0, C, N, M, N, K, C2=C2, bias=bd, f32=f32)
    torch.cuda.synchronize()
    u = acc + b.double()
    _check(C, _gelu64(u), 1.2 * bound + 1e-6, "gelu")
    _check(C2, _dgelu64(u), 0.5 * bound + 1e-6, "gelu'")
    _gemm(0, 1, EPI_RESID, Xd, K, (Wd,), K, 0, C, N, M, N, K, bias=bd, R=Rd, ldr=N, f32=f32)
    torch.cuda.synchronize()
    _check(C, acc + b.double() + R.double(), bound + 1e-6, "resid")


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("D", [128, 256])
def test_stacked_qkv_forward_and_data_grad(D, f32):
    """The fused QKV product over three separate weights, and its data gradient
    dX = [dq|dk|dv] [Wq; Wk; Wv] (B stacked along k)."""
    REL = RELS[f32]
    M = 3 * 81
    g = torch.Generator().manual_seed(D)
    X = torch.randn(M, D, generator=g)
    Ws = [torch.randn(D, D, generator=g) / math.sqrt(D) for _ in range(3)]
    Wd = [w.to(DEV) for w in Ws]
    Wcat = torch.cat(Ws, 0).double()
    C = torch.empty(M, 3 * D, device=DEV)
    _gemm(0, 1, EPI_STORE, X.to(DEV), D, Wd, D, D, C, 3 * D, M, 3 * D, D, f32=f32)
    torch.cuda.synchronize()
    _check(C, X.double() @ Wcat.t(), REL * (X.double().abs() @ Wcat.abs().t()) + 1e-6, "qkv")
    dY = torch.randn(M, 3 * D, generator=g)
    dX = torch.empty(M, D, device=DEV)
    _gemm(0, 0, EPI_STORE, dY.to(DEV), 3 * D, Wd, D, D, dX, D, M, D, 3 * D, f32=f32)
    torch.cuda.synchronize()
    _check(dX, dY.double() @ Wcat, REL * (dY.double().abs() @ Wcat.abs()) + 1e-6, "dX")


@pytest.mark.parametrize("f32", [False, True])
def test_data_grad_product_epilogue(f32):
    """dU = (dY W2) * GELU'(U) (ta=0, tb=0, product epilogue)."""
    REL = RELS[f32]
    M, D, F = 700, 256, 1024
    g = torch.Generator().manual_seed(5)
    dY = torch.randn(M, D, generator=g)
    W2 = torch.randn(D, F, generator=g) / 16
    R = torch.rand(M, F, generator=g)
    C = torch.empty(M, F, device=DEV)
    _gemm(0, 0, EPI_MUL, dY.to(DEV), D, (W2.to(DEV),), F, 0, C, F, M, F, D, R=R.to(DEV), ldr=F, f32=f32)
    torch.cuda.synchronize()
    want = (dY.double() @ W2.double()) * R.double()
    bound = REL * (dY.double().abs() @ W2.double().abs()) * R.double() + 1e-6
    _check(C, want, bound, "mul")


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("M_tok,nsplit", [(405, 1), (2000, 7), (10368, 32), (10368 + 5, 32)])
def test_wgrad_split_k(M_tok, nsplit, f32):
    """dW = dY^T X over tokens (ta=1, tb=0) in split-k slabs and the fixed-order
    reduce into three stacked destinations; bit-identical when repeated."""
    REL = RELS[f32]
    D = 256
    g = torch.Generator().manual_seed(M_tok)
    dY = torch.randn(M_tok, 3 * D, generator=g)
    X = torch.randn(M_tok, D, generator=g)
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    slab = torch.empty(nsplit * 3 * D * D, device=DEV)
    outs = [torch.empty(D, D, device=DEV) for _ in range(3)]
    want = dY.double().t() @ X.double()
    bound = REL * (dY.double().abs().t() @ X.double().abs()) + 1e-6
    # NaN guard rows after both operands: any read past the last token (e.g. by an
    # empty trailing split) would turn the result into NaN
    dY_big = torch.full((M_tok + 64, 3 * D), float("nan"), device=DEV)
    X_big = torch.full((M_tok + 64, D), float("nan"), device=DEV)
    dY_big[:M_tok] = dY.to(DEV)
    X_big[:M_tok] = X.to(DEV)
    res = []
    for _ in range(2):
        _gemm(1, 0, EPI_SLAB, dY_big, 3 * D, (X_big,), D, 0, slab, D, 3 * D, D, M_tok, nsplit=nsplit, f32=f32)
        _native.call("ghm_gemm_reduce", _ptr(slab), nsplit, 3 * D, D, _ptr(outs[0]), _ptr(outs[1]), _ptr(outs[2]), D,
                     ctypes_stream())
        torch.cuda.synchronize()
        res.append(torch.cat(outs, 0).cpu())
    _check(res[0], want, bound, "wgrad")
    assert torch.equal(res[0], res[1])


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("m,n", [(256, 1024), (1024, 256)])  # 128- and 64-row tiles (launch_tm)
@pytest.mark.parametrize("M_tok,nsplit", [(2000, 7), (10368 + 5, 16)])
def test_wgrad_split_k_bias_rows(m, n, M_tok, nsplit, f32):
    """The slab GEMM's C2 row sums + ghm_gemm_reduce_bias: the MLP bias gradient
    (sum over tokens of dY, model.py:344-347 autograd) from the weight-gradient
    launch, beside the weight gradient itself; split tails zeroed, bit-identical
    when repeated."""
    REL = RELS[f32]
    g = torch.Generator().manual_seed(M_tok + m)
    dY = torch.randn(M_tok, m, generator=g)
    X = torch.randn(M_tok, n, generator=g)
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    slab = torch.empty(nsplit * m * n, device=DEV)
    bslab = torch.full((nsplit * m,), float("nan"), device=DEV)
    out, bias = torch.empty(m, n, device=DEV), torch.empty(m, device=DEV)
    dY_big = torch.full((M_tok + 64, m), float("nan"), device=DEV)
    X_big = torch.full((M_tok + 64, n), float("nan"), device=DEV)
    dY_big[:M_tok] = dY.to(DEV)
    X_big[:M_tok] = X.to(DEV)
    res = []
    for _ in range(2):
        _gemm(1, 0, EPI_SLAB, dY_big, m, (X_big,), n, 0, slab, n, m, n, M_tok, C2=bslab, nsplit=nsplit, f32=f32)
        _native.call("ghm_gemm_reduce_bias", _ptr(slab), nsplit, m, n, _ptr(out), None, None, 0, _ptr(bslab),
                     _ptr(bias), ctypes_stream())
        torch.cuda.synchronize()
        res.append((out.cpu(), bias.cpu()))
    _check(res[0][0], dY.double().t() @ X.double(), REL * (dY.double().abs().t() @ X.double().abs()) + 1e-6, "wgrad")
    want_b = dY.double().sum(0)
    bound_b = 1e-6 * dY.double().abs().sum(0) + 1e-6  # f32 sums in a fixed order
    _check(res[0][1], want_b, bound_b, "bias rows")
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("K,stacked,nsplit", [(1024, False, 2), (1024, False, 3), (768, True, 2)])
def test_dgrad_split_k(K, stacked, nsplit, f32):
    """dX = dY W (ta = 0, tb = 0) in split-k slabs + the fixed-order reduce (the
    VLM's GHM_VLM_DSPLIT path), W as one tensor or three stacked along k."""
    REL = RELS[f32]
    D, M = 256, 10368 + 5
    g = torch.Generator().manual_seed(K + nsplit)
    dY = torch.randn(M, K, generator=g)
    W = torch.randn(K, D, generator=g) * 0.05
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    Bs = tuple(W[i * D:(i + 1) * D].to(DEV) for i in range(3)) if stacked else (W.to(DEV),)
    slab = torch.empty(nsplit * M * D, device=DEV)
    out = torch.empty(M, D, device=DEV)
    _gemm(0, 0, EPI_SLAB, dY.to(DEV), K, Bs, D, D if stacked else 0, slab, D, M, D, K, nsplit=nsplit, f32=f32)
    _native.call("ghm_gemm_reduce", _ptr(slab), nsplit, M, D, _ptr(out), None, None, 0, ctypes_stream())
    torch.cuda.synchronize()
    _check(out, dY.double() @ W.double(), REL * (dY.double().abs() @ W.double().abs()) + 1e-6, "dgrad split")


def ctypes_stream():
    import ctypes
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _attn_ref(q, k, v, H, npre, D, dbl=None):
    """float64 restatement of model.py:329-341 on one batch: mask, softmax,
    double residual (dbl = 1/D; 0 for the plain residual of model.py:474-478)."""
    N, T, _ = q.shape
    i = torch.arange(T).view(T, 1)
    j = torch.arange(T).view(1, T)
    allowed = torch.where(i < npre, j < npre, j <= i)
    S = (q @ k.transpose(1, 2)).masked_fill(~allowed, float("-inf")) / math.sqrt(D)
    A = torch.softmax(S, -1)
    o = A @ v
    return H + o + o * (1.0 / D if dbl is None else dbl), A


@pytest.mark.parametrize("D,T", [(256, 81), (128, 81), (256, 40)])
def test_attention_x3_forward_backward(D, T):
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    N = 6
    g = torch.Generator().manual_seed(D + T)
    qkv = torch.randn(N, T, 3 * D, generator=g) * 0.5
    H = torch.randn(N, T, D, generator=g)
    dHm = torch.randn(N, T, D, generator=g)
    q64, k64, v64 = (qkv[..., i * D:(i + 1) * D].double().requires_grad_(True) for i in range(3))
    want, A = _attn_ref(q64, k64, v64, H.double(), 1, D)
    (want * dHm.double()).sum().backward()
    qkv_d, H_d = qkv.to(DEV), H.to(DEV)
    Hm = torch.empty(N * T, D, device=DEV)
    P = torch.zeros(N, 96, 96, device=DEV)
    _native.call("ghm_vlm_attn_fwd_x3", _ptr(qkv_d), _ptr(H_d), _ptr(Hm), _ptr(P), N, T, D, 1, math.sqrt(D),
                 ctypes_stream())
    dS = torch.zeros(N, 96, 96, device=DEV)
    dqkv = torch.empty(N * T, 3 * D, device=DEV)
    _native.call("ghm_vlm_attn_bwd_x3", _ptr(qkv_d), _ptr(P), _ptr(dHm.to(DEV)), _ptr(dS), _ptr(dqkv), N, T, D,
                 math.sqrt(D), ctypes_stream())
    torch.cuda.synchronize()
    scale = lambda t: t.abs().max().item()  # noqa: E731
    assert (Hm.cpu().view(N, T, D).double() - want.detach()).abs().max().item() <= 1e-4 * scale(want)
    assert (P.cpu()[:, :T, :T].double() - A.detach()).abs().max().item() <= 2e-5
    assert P.cpu()[:, :T, T:].abs().max().item() == 0.0
    got = dqkv.cpu().view(N, T, 3 * D).double()
    for i, ref in enumerate((q64.grad, k64.grad, v64.grad)):
        assert (got[..., i * D:(i + 1) * D] - ref).abs().max().item() <= 2e-4 * scale(ref), "dq dk dv"[3 * i:3 * i + 2]


@pytest.mark.parametrize("M,N", [(10368, 1024), (10368, 256), (405, 256), (128, 81 * 256), (7, 16)])
def test_colsum(M, N):
    """ghm_colsum (bias / position-embedding gradients): fp32 sums in a fixed order,
    within fp32 summation error of the float64 sum and bit-identical on repeat."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    g = torch.Generator().manual_seed(M + N)
    X = torch.randn(M, N, generator=g)
    Xd = X.to(DEV)
    part = torch.empty(_native.hip_lib().ghm_colsum_part_elems(M, N), device=DEV)
    outs = []
    for _ in range(2):
        out = torch.empty(N, device=DEV)
        _native.call("ghm_colsum", _ptr(Xd), M, N, _ptr(out), _ptr(part), ctypes_stream())
        torch.cuda.synchronize()
        outs.append(out.cpu())
    want = X.double().sum(0)
    bound = 1e-6 * X.double().abs().sum(0) + 1e-7
    assert ((outs[0].double() - want).abs() <= bound).all()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("C,D,tok,rowmap", [(10, 256, False, None), (10, 128, True, (35, 41, 6)),
                                             (33, 128, False, None), (64, 256, True, (9, 17, 8)),
                                             (3, 16, True, (5, 5, 0))])
def test_wcolsum(C, D, tok, rowmap):
    """ghm_wcolsum (readout weight / bias and token-embedding gradients): dense
    weights or token ids, text-row maps inside each sequence, several class blocks;
    fp32 against the float64 product, bit-identical on repeat."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    g = torch.Generator().manual_seed(C * D)
    n_seq = 300
    rps, seq_rows, off = rowmap if rowmap else (1, 1, 0)
    Mrows = n_seq * seq_rows if rowmap else 10_368
    M = n_seq * rps if rowmap else Mrows
    X = torch.randn(Mrows, D, generator=g)
    rows = torch.arange(M)
    xrow = (rows // rps) * seq_rows + off + rows % rps
    if tok:
        ids = torch.randint(0, C, (M,), generator=g, dtype=torch.uint8)
        Wm = torch.nn.functional.one_hot(ids.long(), C).double()
    else:
        Wm = torch.randn(M, C, generator=g).double()
    want = Wm.t() @ X[xrow].double()
    want_w = Wm.sum(0)
    Xd = X.to(DEV)
    if tok:
        idd = ids.to(DEV)
        src = (None, _ptr(idd))
    else:
        wd = Wm.float().to(DEV)
        src = (_ptr(wd), None)
    part = torch.empty(_native.hip_lib().ghm_wcolsum_part_elems(M, D, C), device=DEV)
    outs = []
    for _ in range(2):
        out, ws = torch.full((C, D), float("nan"), device=DEV), torch.full((C,), float("nan"), device=DEV)
        _native.call("ghm_wcolsum", src[0], src[1], C, _ptr(Xd), rps, seq_rows, off, M, D, _ptr(out),
                     None if tok else _ptr(ws), _ptr(part), ctypes_stream())
        torch.cuda.synchronize()
        outs.append((out.cpu(), ws.cpu()))
    bound = 1e-6 * (Wm.abs().t() @ X[xrow].double().abs()) + 1e-6
    assert ((outs[0][0].double() - want).abs() <= bound).all()
    assert torch.equal(outs[0][0], outs[1][0])
    if not tok:
        assert ((outs[0][1].double() - want_w).abs() <= 1e-6 * Wm.abs().sum(0) + 1e-6).all()
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("C,D,M", [(10, 256, 10_368), (10, 128, 1000), (64, 256, 333), (17, 128, 77)])
def test_rows_linear(C, D, M):
    """ghm_rows_linear / _t (the VLM readout, model.py:332): logits = X W^T + b and
    dX = dZ W against the float64 products."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    g = torch.Generator().manual_seed(C + D + M)
    X, W, b = torch.randn(M, D, generator=g), torch.randn(C, D, generator=g) * 0.1, torch.randn(C, generator=g)
    dZ = torch.randn(M, C, generator=g)
    Xd, Wd, bd, dZd = X.to(DEV), W.to(DEV), b.to(DEV), dZ.to(DEV)
    Y, dX = torch.empty(M, C, device=DEV), torch.empty(M, D, device=DEV)
    _native.call("ghm_rows_linear", _ptr(Xd), _ptr(Wd), _ptr(bd), _ptr(Y), M, D, C, ctypes_stream())
    _native.call("ghm_rows_linear_t", _ptr(dZd), _ptr(Wd), _ptr(dX), M, D, C, ctypes_stream())
    torch.cuda.synchronize()
    want_y = X.double() @ W.double().t() + b.double()
    want_dx = dZ.double() @ W.double()
    by = 1e-6 * (X.double().abs() @ W.double().abs().t() + b.double().abs()) + 1e-6
    bx = 1e-6 * (dZ.double().abs() @ W.double().abs()) + 1e-6
    assert ((Y.cpu().double() - want_y).abs() <= by).all()
    assert ((dX.cpu().double() - want_dx).abs() <= bx).all()


@pytest.mark.parametrize("T,npre,dbl", [(162, 162, 0.0), (130, 1, 1 / 128), (81, 81, 0.0), (100, 100, 0.0)])
def test_attention_ext_long_sequences(T, npre, dbl):
    """ghm_attn_ext_*_x3 at D = 128: sequences past 96 tokens (the joint CDM's 162,
    train_CDNS.py) with P / dS padded to 192, unmasked (n_prefix = T) and plain
    residual (dbl = 0), plus a masked double-residual case."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    N, D = 5, 128
    pad = 96 if T <= 96 else 192
    g = torch.Generator().manual_seed(T)
    qkv = torch.randn(N, T, 3 * D, generator=g) * 0.5
    H = torch.randn(N, T, D, generator=g)
    dHm = torch.randn(N, T, D, generator=g)
    q64, k64, v64 = (qkv[..., i * D:(i + 1) * D].double().requires_grad_(True) for i in range(3))
    want, A = _attn_ref(q64, k64, v64, H.double(), npre, D, dbl)
    (want * dHm.double()).sum().backward()
    qkv_d = qkv.to(DEV)
    Hm = torch.empty(N * T, D, device=DEV)
    P = torch.zeros(N, pad, pad, device=DEV)
    dS = torch.zeros(N, pad, pad, device=DEV)
    dqkv = torch.empty(N * T, 3 * D, device=DEV)
    _native.call("ghm_attn_ext_fwd_x3", _ptr(qkv_d), _ptr(H.to(DEV)), _ptr(Hm), _ptr(P), N, T, D, npre, math.sqrt(D),
                 dbl, ctypes_stream())
    _native.call("ghm_attn_ext_bwd_x3", _ptr(qkv_d), _ptr(P), _ptr(dHm.to(DEV)), _ptr(dS), _ptr(dqkv), N, T, D,
                 npre, math.sqrt(D), dbl, ctypes_stream())
    torch.cuda.synchronize()
    scale = lambda t: t.abs().max().item()  # noqa: E731
    assert (Hm.cpu().view(N, T, D).double() - want.detach()).abs().max().item() <= 1e-4 * scale(want)
    assert (P.cpu()[:, :T, :T].double() - A.detach()).abs().max().item() <= 2e-5
    assert P.cpu()[:, :T, T:].abs().max().item() == 0.0
    got = dqkv.cpu().view(N, T, 3 * D).double()
    for i, ref in enumerate((q64.grad, k64.grad, v64.grad)):
        assert (got[..., i * D:(i + 1) * D] - ref).abs().max().item() <= 2e-4 * scale(ref), "dq dk dv"[3 * i:3 * i + 2]


@pytest.mark.parametrize("T,act", [(162, 1), (162, 2), (130, 2), (81, 1)])
def test_attention_ext_activation(T, act):
    """ghm_attn_ext_*_x3_act at D = 128 (the joint CDM's T = 162 under
    train_CDNS.py --activation): relu / gelu of the scaled scores, no row
    normalisation, plain residual; P, the output and dq / dk / dv against float64
    autograd of model.py:485-486."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    N, D = 5, 128
    pad = 96 if T <= 96 else 192
    g = torch.Generator().manual_seed(T + act)
    qkv = torch.randn(N, T, 3 * D, generator=g) * 0.5
    H = torch.randn(N, T, D, generator=g)
    dHm = torch.randn(N, T, D, generator=g)
    q64, k64, v64 = (qkv[..., i * D:(i + 1) * D].double().requires_grad_(True) for i in range(3))
    S = (q64 @ k64.transpose(1, 2)) / math.sqrt(D)
    A = torch.relu(S) if act == 1 else torch.nn.functional.gelu(S)
    want = H.double() + A @ v64
    (want * dHm.double()).sum().backward()
    qkv_d = qkv.to(DEV)
    Hm = torch.empty(N * T, D, device=DEV)
    P = torch.zeros(N, pad, pad, device=DEV)
    Pd = torch.zeros(N, pad, pad, device=DEV)
    dS = torch.zeros(N, pad, pad, device=DEV)
    dqkv = torch.empty(N * T, 3 * D, device=DEV)
    _native.call("ghm_attn_ext_fwd_x3_act", _ptr(qkv_d), _ptr(H.to(DEV)), _ptr(Hm), _ptr(P), _ptr(Pd), N, T, D, T,
                 math.sqrt(D), 0.0, act, ctypes_stream())
    _native.call("ghm_attn_ext_bwd_x3_act", _ptr(qkv_d), _ptr(P), _ptr(Pd), _ptr(dHm.to(DEV)), _ptr(dS), _ptr(dqkv),
                 N, T, D, T, math.sqrt(D), 0.0, act, ctypes_stream())
    torch.cuda.synchronize()
    scale = lambda t: t.abs().max().item()  # noqa: E731
    assert (Hm.cpu().view(N, T, D).double() - want.detach()).abs().max().item() <= 1e-4 * scale(want)
    assert (P.cpu()[:, :T, :T].double() - A.detach()).abs().max().item() <= 1e-4 * scale(A)
    assert P.cpu()[:, :T, T:].abs().max().item() == 0.0
    got = dqkv.cpu().view(N, T, 3 * D).double()
    for i, ref in enumerate((q64.grad, k64.grad, v64.grad)):
        assert (got[..., i * D:(i + 1) * D] - ref).abs().max().item() <= 2e-4 * scale(ref), "dq dk dv"[3 * i:3 * i + 2]



@pytest.mark.parametrize("T,act", [(81, 1), (81, 2), (40, 2), (17, 1)])
def test_attention_f32_activation(T, act):
    """ghm_attn_{fwd,bwd}_act (exact-f32 one-sequence kernels; the guided CLIP's
    default precision under train_CLIP --clip_activation): relu / gelu of the
    scaled scores, no row normalisation; P, the output and dq / dk / dv against
    float64 autograd of model.py:778-782 with get_activation (:121-130)."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    N, D, pad = 5, 128, 96
    g = torch.Generator().manual_seed(T + 10 * act)
    qkv = torch.randn(N, T, 3 * D, generator=g) * 0.5
    H = torch.randn(N, T, D, generator=g)
    dHm = torch.randn(N, T, D, generator=g)
    q64, k64, v64 = (qkv[..., i * D:(i + 1) * D].double().requires_grad_(True) for i in range(3))
    S = (q64 @ k64.transpose(1, 2)) / math.sqrt(D)
    A = torch.relu(S) if act == 1 else torch.nn.functional.gelu(S)
    want = H.double() + A @ v64
    (want * dHm.double()).sum().backward()
    qkv_d = qkv.to(DEV)
    Hm = torch.empty(N * T, D, device=DEV)
    P = torch.zeros(N, pad, pad, device=DEV)
    Pd = torch.zeros(N, pad, pad, device=DEV)
    dS = torch.zeros(N, pad, pad, device=DEV)
    dqkv = torch.empty(N * T, 3 * D, device=DEV)
    _native.call("ghm_attn_fwd_act", _ptr(qkv_d), _ptr(H.to(DEV)), _ptr(Hm), _ptr(P), _ptr(Pd), N, T, D,
                 math.sqrt(D), act, ctypes_stream())
    _native.call("ghm_attn_bwd_act", _ptr(qkv_d), _ptr(P), _ptr(Pd), _ptr(dHm.to(DEV)), _ptr(dS), _ptr(dqkv),
                 N, T, D, math.sqrt(D), act, ctypes_stream())
    torch.cuda.synchronize()
    scale = lambda t: t.abs().max().item()  # noqa: E731
    # exact f32 products (k-ordered fmaf chains): f32-rounding-level bounds
    assert (Hm.cpu().view(N, T, D).double() - want.detach()).abs().max().item() <= 5e-6 * scale(want)
    assert (P.cpu()[:, :T, :T].double() - A.detach()).abs().max().item() <= 5e-6 * scale(A)
    assert P.cpu()[:, :T, T:].abs().max().item() == 0.0 and P.cpu()[:, T:, :].abs().max().item() == 0.0
    got = dqkv.cpu().view(N, T, 3 * D).double()
    for i, ref in enumerate((q64.grad, k64.grad, v64.grad)):
        assert (got[..., i * D:(i + 1) * D] - ref).abs().max().item() <= 1e-5 * scale(ref), "dq dk dv"[3 * i:3 * i + 2]


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("variant", ["1", "3", "bn64", "bn128", "sb", "sb0"])
def test_buffer_load_staging_bit_identical(variant, f32, monkeypatch):
    """GHM_GEMM_BUF=1 (buffer-load staging: rows past M, past a split's last
    token or past K read as hardware zeros instead of clamped re-reads + zeroing
    selects) and =3 (the same with the next tile's split store interleaved into
    the current tile's MFMAs) change only how and when tiles are loaded and
    stored (GHM_GEMM_BUF=0 is the pointer-load staging; the default is 1, and 3
    for the weight gradients), and so do both tile widths (GHM_GEMM_BN=64 / 128) and one or two LDS
    tiles (GHM_GEMM_SB=1 / 0): every
    shape class -- forward
    store / GELU / residual, data gradient store / product / split-k, split-k
    weight gradient with bias rows, token tails and an empty trailing split, both
    tile heights -- is bit-identical to the pointer-load staging.  The guard rows
    past every operand are NaN, so a read past the end would show."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    g = torch.Generator().manual_seed(77)
    M = 10368 + 5
    cases = []

    def nan_pad(t):
        big = torch.full((t.shape[0] + 64, t.shape[1]), float("nan"), device=DEV)
        big[:t.shape[0]] = t.to(DEV)
        return big

    for K, N in [(256, 1024), (256, 256), (1024, 256)]:
        X = nan_pad(torch.randn(M, K, generator=g))
        W, W2 = (torch.randn(N, K, generator=g) / 16).to(DEV), (torch.randn(K, N, generator=g) / 16).to(DEV)
        b, R = torch.randn(N, generator=g).to(DEV), torch.randn(M, N, generator=g).to(DEV)

        def run(X=X, W=W, b=b, R=R, W2=W2, K=K, N=N):
            C, C2, C3, C4, C5 = (torch.empty(M, N, device=DEV) for _ in range(5))
            _gemm(0, 1, EPI_STORE, X, K, (W,), K, 0, C, N, M, N, K, f32=f32)
            _gemm(0, 1, EPI_GELU, X, K, (W,), K, 0, C2, N, M, N, K, C2=C3, bias=b, f32=f32)
            _gemm(0, 1, EPI_RESID, X, K, (W,), K, 0, C4, N, M, N, K, bias=b, R=R, ldr=N, f32=f32)
            _gemm(0, 0, EPI_MUL, X, K, (W2,), N, 0, C5, N, M, N, K, R=R, ldr=N, f32=f32)
            return C, C2, C3, C4, C5
        cases.append(run)
    Wq = [(torch.randn(256, 256, generator=g) / 16).to(DEV) for _ in range(3)]
    dQ = nan_pad(torch.randn(M, 768, generator=g))

    def run_dsplit():
        slab = torch.empty(3 * M * 256, device=DEV)
        out = torch.empty(M, 256, device=DEV)
        _gemm(0, 0, EPI_SLAB, dQ, 768, Wq, 256, 256, slab, 256, M, 256, 768, nsplit=3, f32=f32)
        _native.call("ghm_gemm_reduce", _ptr(slab), 3, M, 256, _ptr(out), None, None, 0, ctypes_stream())
        return (out,)
    cases.append(run_dsplit)
    for m, n, Mt, ns in [(1024, 256, 10368 + 5, 16), (256, 1024, 2000, 7), (768, 256, 405, 4), (256, 256, 40, 3)]:
        dY = nan_pad(torch.randn(Mt, m, generator=g))
        Xw = nan_pad(torch.randn(Mt, n, generator=g))

        def runw(dY=dY, Xw=Xw, m=m, n=n, Mt=Mt, ns=ns):
            slab = torch.empty(ns * m * n, device=DEV)
            bslab = torch.empty(ns * m, device=DEV)
            out, bias = torch.empty(m, n, device=DEV), torch.empty(m, device=DEV)
            _gemm(1, 0, EPI_SLAB, dY, m, (Xw,), n, 0, slab, n, m, n, Mt, C2=bslab, nsplit=ns, f32=f32)
            _native.call("ghm_gemm_reduce_bias", _ptr(slab), ns, m, n, _ptr(out), None, None, 0, _ptr(bslab),
                         _ptr(bias), ctypes_stream())
            return out, bias
        cases.append(runw)
    monkeypatch.setenv("GHM_GEMM_BUF", "0")
    base = [[t.cpu() for t in c()] for c in cases]
    if variant.startswith("sb"):  # one LDS tile for the N >= 768 products (default; three workgroups per CU, x3 only) or two
        monkeypatch.delenv("GHM_GEMM_BUF", raising=False)
        monkeypatch.setenv("GHM_GEMM_SB", "1" if variant == "sb" else "0")
    elif variant.startswith("bn"):  # the default staging, one tile width for the N < 768 products (x3 only)
        monkeypatch.delenv("GHM_GEMM_BUF", raising=False)
        monkeypatch.setenv("GHM_GEMM_BN", variant[2:])
    else:
        monkeypatch.setenv("GHM_GEMM_BUF", variant)
    got = [[t.cpu() for t in c()] for c in cases]
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(base, got)):
        for j, (x, y) in enumerate(zip(a, b)):
            assert torch.isfinite(x).all(), (i, j)
            assert torch.equal(x, y), (i, j)


def _split_ref(x):
    hi = x.float().bfloat16()
    lo = (x.float() - hi.float()).bfloat16()
    return hi, lo


def test_split_pack_and_presplit_gemm(monkeypatch):
    """ghm_split_pack writes split1's (hi, lo) of f32 matrices -- plain and
    transposed, ragged 64 x 64 tiles, into column / row offsets of a wider image
    -- equal to torch's round-to-nearest-even bf16 split; ghm_gemm_x3p on those
    images equals ghm_gemm_x3 on the f32 weights bit for bit in every epilogue
    (GELU with GELU', bias + residual, product, store, split-k slabs) and both tile
    heights."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    g = torch.Generator().manual_seed(3)
    # split kernel: W [100][70] into columns 8.. of a [100][88] image (plain) and
    # rows 8.. of a [88][100] image (transposed)
    W = torch.randn(100, 70, generator=g).to(DEV)
    img = torch.zeros(2, 100, 88, dtype=torch.bfloat16, device=DEV)
    imgT = torch.zeros(2, 88, 100, dtype=torch.bfloat16, device=DEV)
    jobs = torch.tensor([[W.data_ptr(), 70, 100, 70, img.data_ptr() + 2 * 8, 88, 100 * 88, 0],
                         [W.data_ptr(), 70, 100, 70, imgT.data_ptr() + 2 * 8 * 100, 100, 88 * 100, 1]],
                        dtype=torch.int64).to(DEV)
    _native.call("ghm_split_pack", _ptr(jobs), 2, 4, ctypes_stream())
    torch.cuda.synchronize()
    hi, lo = _split_ref(W)
    assert torch.equal(img[0, :, 8:78].cpu(), hi.cpu()) and torch.equal(img[1, :, 8:78].cpu(), lo.cpu())
    assert torch.equal(imgT[0, 8:78, :].cpu(), hi.t().cpu()) and torch.equal(imgT[1, 8:78, :].cpu(), lo.t().cpu())
    assert (img[:, :, :8] == 0).all() and (img[:, :, 78:] == 0).all()

    def pack(Bkn):  # B(k, n) -> pre-split image [n][k] (hi, lo planes)
        K, N = Bkn.shape
        out = torch.empty(2, N, K, dtype=torch.bfloat16, device=DEV)
        src = Bkn.t().contiguous()
        j = torch.tensor([[src.data_ptr(), K, N, K, out.data_ptr(), K, N * K, 0]], dtype=torch.int64).to(DEV)
        _native.call("ghm_split_pack", _ptr(j), 1, -(-N // 64) * -(-K // 64), ctypes_stream())
        torch.cuda.synchronize()
        return out, src

    M = 10368 + 5
    for K, N in [(256, 1024), (256, 768), (1024, 256), (256, 256)]:
        X = torch.randn(M, K, generator=g).to(DEV)
        Wnk = (torch.randn(N, K, generator=g) / 16).to(DEV)  # forward weight W[n][k]: B(k,n) = W[n][k]
        b = torch.randn(N, generator=g).to(DEV)
        R = torch.randn(M, N, generator=g).to(DEV)
        img, _ = pack(Wnk.t())
        for epi in (EPI_STORE, EPI_GELU, EPI_RESID, EPI_MUL):
            kw = {"C2": torch.empty(M, N, device=DEV), "bias": b} if epi == EPI_GELU else (
                {"bias": b, "R": R, "ldr": N} if epi == EPI_RESID else ({"R": R, "ldr": N} if epi == EPI_MUL else {}))
            C0, C1 = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
            if epi == EPI_MUL:  # (ta, tb) = (0, 0) is the product epilogue's shape: B = W^T stored [K][N]
                _gemm(0, 0, epi, X, K, (Wnk.t().contiguous(),), N, 0, C0, N, M, N, K, **kw)
            else:
                _gemm(0, 1, epi, X, K, (Wnk,), K, 0, C0, N, M, N, K, **kw)
            c2 = kw.get("C2")
            ref2 = c2.clone() if c2 is not None else None
            pp = lambda t: None if t is None else _ptr(t)  # noqa: E731
            _native.call("ghm_gemm_x3p", epi, _ptr(X), K, _ptr(img), K, N * K, _ptr(C1), N, pp(c2), pp(kw.get("bias")),
                         pp(kw.get("R")), kw.get("ldr", 0), M, N, K, 1, ctypes_stream())
            torch.cuda.synchronize()
            assert torch.equal(C0.cpu(), C1.cpu()), (K, N, epi)
            if c2 is not None:
                assert torch.equal(ref2.cpu(), c2.cpu())
    # split-k data gradient dX = dY W over K = 1024 in 2 slabs
    K, N = 1024, 256
    dY = torch.randn(M, K, generator=g).to(DEV)
    Wkn = (torch.randn(K, N, generator=g) * 0.05).to(DEV)
    img, _ = pack(Wkn)
    s0, s1 = torch.empty(2 * M * N, device=DEV), torch.empty(2 * M * N, device=DEV)
    _gemm(0, 0, EPI_SLAB, dY, K, (Wkn,), N, 0, s0, N, M, N, K, nsplit=2)
    _native.call("ghm_gemm_x3p", EPI_SLAB, _ptr(dY), K, _ptr(img), K, N * K, _ptr(s1), N, None, None, None, 0, M, N,
                 K, 2, ctypes_stream())
    torch.cuda.synchronize()
    assert torch.equal(s0.cpu(), s1.cpu())


@pytest.mark.parametrize("D,T,npre,act", [(256, 81, 1, 0), (256, 161, 81, 0), (128, 162, 162, 0), (256, 40, 1, 0),
                                          (256, 81, 1, 1), (128, 130, 130, 2)])
@pytest.mark.parametrize("split", ["2", "4"])
def test_attention_forward_column_split_bit_identical(D, T, npre, act, split, monkeypatch):
    """GHM_VX_SPLIT (the split-bf16 attention kernels' output column blocks over 2
    or 4 workgroups: the forward and the dQ kernel recompute their query tiles'
    scores / dS, the dK / dV kernel only reloads P and dS) leaves the output, P,
    GELU', dS and dq / dk / dv bit-identical: the same products per element in the
    same order."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    N = 7
    pad = 96 if T <= 96 else 192
    g = torch.Generator().manual_seed(D + T + act)
    qkv = (torch.randn(N, T, 3 * D, generator=g) * 0.5).to(DEV)
    H = torch.randn(N, T, D, generator=g).to(DEV)
    dHm = torch.randn(N, T, D, generator=g).to(DEV)
    out = []
    for sp in ("1", split):
        monkeypatch.setenv("GHM_VX_SPLIT", sp)
        monkeypatch.setenv("GHM_VX_SPLIT_KV", sp)
        Hm = torch.full((N * T, D), float("nan"), device=DEV)
        P = torch.zeros(N, pad, pad, device=DEV)
        Pd = torch.zeros(N, pad, pad, device=DEV)
        dS = torch.zeros(N, pad, pad, device=DEV)
        dqkv = torch.full((N * T, 3 * D), float("nan"), device=DEV)
        if act == 0:
            _native.call("ghm_attn_ext_fwd_x3", _ptr(qkv), _ptr(H), _ptr(Hm), _ptr(P), N, T, D, npre, math.sqrt(D),
                         1.0 / D, ctypes_stream())
            _native.call("ghm_attn_ext_bwd_x3", _ptr(qkv), _ptr(P), _ptr(dHm), _ptr(dS), _ptr(dqkv), N, T, D, npre,
                         math.sqrt(D), 1.0 / D, ctypes_stream())
        else:
            _native.call("ghm_attn_ext_fwd_x3_act", _ptr(qkv), _ptr(H), _ptr(Hm), _ptr(P), _ptr(Pd), N, T, D, npre,
                         math.sqrt(D), 0.0, act, ctypes_stream())
            _native.call("ghm_attn_ext_bwd_x3_act", _ptr(qkv), _ptr(P), _ptr(Pd), _ptr(dHm), _ptr(dS), _ptr(dqkv),
                         N, T, D, npre, math.sqrt(D), 0.0, act, ctypes_stream())
        torch.cuda.synchronize()
        out.append((Hm.cpu(), P.cpu(), Pd.cpu(), dS.cpu(), dqkv.cpu()))
    assert torch.isfinite(out[0][0]).all() and torch.isfinite(out[0][4]).all()
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("ns", [1, 3, 8, 9, 16, 17])
def test_slab_reduce_is_the_z_ordered_sum(ns):
    """ghm_gemm_reduce_bias (the split-k slabs and the bias row-sum partials,
    loads of 8 slabs in flight): bit-identical to s[0] + s[1] + ... in z order in
    f32, signed zeros included, for split counts around the batch of 8."""
    from ghmclip import _native
    from ghmclip.models.vlm import _ptr
    g = torch.Generator().manual_seed(ns)
    m, n = 96, 256
    slab = torch.randn(ns, m, n, generator=g)
    slab[0, 0, :8] = -0.0
    slab[:, 1, :4] = 0.0
    slab[0, 1, :4] = -0.0
    bslab = torch.randn(ns, m, generator=g)
    want, bwant = slab[0].clone(), bslab[0].clone()
    for z in range(1, ns):
        want += slab[z]
        bwant += bslab[z]
    out, bias = torch.empty(m, n, device=DEV), torch.empty(m, device=DEV)
    sd, bd = slab.to(DEV), bslab.to(DEV)
    _native.call("ghm_gemm_reduce_bias", _ptr(sd), ns, m, n, _ptr(out), None, None, 0, _ptr(bd), _ptr(bias),
                 ctypes_stream())
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), want) and torch.equal(torch.signbit(out.cpu()), torch.signbit(want))
    assert torch.equal(bias.cpu(), bwant)
