"""Zero-shot classification evaluation on the HIP path
(ghmclip.evaluation.zsc_loss, figures/eval-zsc-risk.py:62-121): the
ghm_zsc_logits kernel against the oracle restatement, and the whole
evaluation against the numbers the reference's own zsc_loss produced
(tests/golden/zsc_{small,full}.npz, tests/golden/make_golden_zsc.py).
Tolerances: logits 1e-5 absolute (f32 exp and sums in another order), the
kernel on the reference's own embeddings 1e-6 relative in the risk, the full
evaluation (HIP encoders in split-bf16 vs the reference's CPU encoders)
1e-4 relative."""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT
from oracle import zsc_oracle as Z

pytestmark = pytest.mark.gpu
DEV = "cuda"
P_Y = np.ones(10) / 10


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _logits(i_emb, t_emb, idx, n_list):
    from ghmclip.evaluation.zsc import zsc_logits
    out = zsc_logits(torch.from_numpy(np.ascontiguousarray(i_emb, np.float32)).to(DEV),
                     torch.from_numpy(np.ascontiguousarray(t_emb, np.float32)).to(DEV),
                     torch.from_numpy(np.ascontiguousarray(idx, np.int32)).to(DEV), n_list)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def test_kernel_on_reference_embeddings():
    f = np.load(os.path.join(GOLDEN, "zsc_small.npz"))
    n_list = [int(n) for n in f["n_list"]]
    ie, te = Z.reference_rows(f["i_emb"]), Z.reference_rows(f["t_emb"])
    got = _logits(ie, te, f["proto_idx"], n_list)
    want = Z.zsc_logits(ie, te, f["proto_idx"], n_list)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-5)
    risks = [Z.cross_entropy(got[q], f["first"]) for q in range(len(n_list))]
    np.testing.assert_allclose(risks, f["loss"], rtol=1e-6)


@pytest.mark.parametrize("n_rows,n_proto,D,n_class,n_list", [(333, 45, 10, 3, [1, 7, 45]),
                                                             (128, 32, 7, 10, [32]),
                                                             (1, 70, 16, 2, [3, 64, 70]),
                                                             (4097, 250, 10, 10, [5, 10, 50, 100, 250])])
def test_kernel_edge_shapes(n_rows, n_proto, D, n_class, n_list):
    """Ragged row counts (not a multiple of the 128-row workgroup), prototype
    counts that are not a multiple of the 32-prototype tile, odd and maximal
    embedding widths, several support sizes per launch."""
    g = np.random.default_rng(n_rows * 31 + D)
    n_t = max(n_proto * n_class, 8)
    ie = g.standard_normal((n_rows, D)).astype(np.float32) * 0.7
    te = g.standard_normal((n_t, D)).astype(np.float32) * 0.7
    idx = np.stack([g.permutation(n_t)[:n_proto] for _ in range(n_class)]).astype(np.int32)
    got = _logits(ie, te, idx, n_list)
    want = Z.zsc_logits(ie, te, idx, n_list)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-5)


def _pairs(spec):
    from ghmclip import EncoderTransformer
    return {name: (EncoderTransformer(81, 10, 128, L).to(DEV), EncoderTransformer(81, 10, 128, L).to(DEV))
            for name, L in spec}


def _sampler():
    from ghmclip.data.data_random_GHM import DoubleSampler
    return DoubleSampler(n_layers=[4, 4], n_childs=[3, 3], variable_type=10, p_ys=[P_Y, P_Y], p_flips=[0.2, 0.2],
                         seedtree=42)


def test_zsc_loss_full_vs_reference():
    """The figure's setting (num_samples_list [250], N = 7500) with the
    fixture's random-init Standard (L = 5) and Shallow (L = 1) pairs, in the
    fixture's order: seed_everything(224) -> encoders -> DoubleSampler(42)."""
    from ghmclip import seed_everything
    from ghmclip.evaluation import zsc_loss
    f = np.load(os.path.join(GOLDEN, "zsc_full.npz"))
    seed_everything(224)
    pairs = _pairs([("Standard TF", 5), ("Shallow TF", 1)])
    s = _sampler()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = zsc_loss(s, pairs, np.array([250]), device=DEV)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"zsc_loss N=7500, 2 encoder pairs: {dt * 1e3:.1f} ms; Bayes {res['Bayes'][0]:.7f} vs {f['bayes'][0]:.7f}; "
          f"Standard {res['Standard TF'][0]:.7f} vs {f['standard'][0]:.7f}; "
          f"Shallow {res['Shallow TF'][0]:.7f} vs {f['shallow'][0]:.7f}")
    assert res["num_samples_list"] == [250]
    assert abs(res["Bayes"][0] - f["bayes"][0]) <= 1e-6 * f["bayes"][0]
    assert abs(res["Standard TF"][0] - f["standard"][0]) <= 1e-4 * f["standard"][0]
    assert abs(res["Shallow TF"][0] - f["shallow"][0]) <= 1e-4 * f["shallow"][0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-ghm_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ghmclip import seed_everything
        from ghmclip.evaluation import zsc_loss
        seed_everything(224)
        pairs = _pairs([("pair", 1)])
        res = zsc_loss(_sampler(), pairs, np.array([5, 10]), device=DEV)
        q.put((rank, dict(res), None))
    except Exception as e:  # noqa: BLE001 — surfaced in the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def test_zsc_loss_two_ranks_equals_one():
    """Two ranks (gloo, sharing the GPU): each embeds half of the rows, the text
    embeddings are all-gathered, the loss sums all-reduced; the result equals
    the one-process evaluation, which equals the reference's (zsc_small.npz)."""
    from ghmclip import seed_everything
    from ghmclip.evaluation import zsc_loss
    f = np.load(os.path.join(GOLDEN, "zsc_small.npz"))
    seed_everything(224)
    one = zsc_loss(_sampler(), _pairs([("pair", 1)]), np.array([5, 10]), device=DEV)
    np.testing.assert_allclose(one["pair"], f["loss"], rtol=1e-4)
    np.testing.assert_allclose(one["Bayes"], f["bayes"], rtol=1e-6)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        out = [q.get(timeout=120) for _ in range(2)]
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, res, err in out:
        assert err is None, f"rank {rank}: {err}"
        np.testing.assert_allclose(res["pair"], one["pair"], rtol=1e-6)
        np.testing.assert_allclose(res["Bayes"], one["Bayes"], rtol=1e-7)
