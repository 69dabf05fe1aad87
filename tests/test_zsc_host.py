"""Zero-shot classification evaluation (figures/eval-zsc-risk.py), host side:
the shared-root draw against the reference's own draw, the oracle restatement
against the losses the reference's zsc_loss returned (tests/golden/zsc_small.npz,
made by tests/golden/make_golden_zsc.py), and the data-parallel row sharding /
text-embedding all-gather under two gloo ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN
from oracle import zsc_oracle as Z

P_Y = np.ones(10) / 10


def _sampler():
    from ghmclip.data.data_random_GHM import DoubleSampler
    return DoubleSampler(n_layers=[4, 4], n_childs=[3, 3], variable_type=10, p_ys=[P_Y, P_Y], p_flips=[0.2, 0.2],
                         seedtree=42)


def test_zeroshot_batch_equals_reference_draw():
    """DoubleSampler.get_zeroshot_batch (data_random_GHM.py:670-683): leaves and
    roots bit-exact, BP_CLS root posteriors to 1e-12, after the same
    seed_everything(224) -> DoubleSampler(seedtree=42) order as the fixture."""
    from ghmclip import seed_everything
    f = np.load(os.path.join(GOLDEN, "zsc_small.npz"))
    seed_everything(224)
    tl, il, tp, ip, root = _sampler().get_zeroshot_batch(batch_size=300)
    np.testing.assert_array_equal(tl, f["t_leaves"])
    np.testing.assert_array_equal(il, f["i_leaves"])
    np.testing.assert_array_equal(root, f["root"])
    np.testing.assert_allclose(tp, f["t_pp"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(ip, f["i_pp"], rtol=0, atol=1e-12)
    assert tl.dtype == np.int64 and tp.shape == (300, 10)


def test_oracle_matches_reference_losses():
    """The oracle's ZSC risks from the reference's own embeddings equal the
    losses the reference's zsc_loss returned (float32 sums in another order:
    1e-6 relative), and its Bayes risk the reference's."""
    f = np.load(os.path.join(GOLDEN, "zsc_small.npz"))
    n_list = [int(n) for n in f["n_list"]]
    got = Z.zsc_risks(f["i_emb"], f["t_emb"], f["first"], n_list)
    np.testing.assert_allclose(got, f["loss"], rtol=1e-6)
    idx = Z.prototype_index(f["first"], 10, max(n_list))
    np.testing.assert_array_equal(idx, f["proto_idx"])
    s = _sampler()
    np.testing.assert_allclose(Z.bayes_risk(f["i_pp"], s.t_transition, f["first"]), f["bayes"][0], rtol=1e-6)


def test_zsc_logits_refuses_host_tensors():
    """The product path has no CPU fallback."""
    from ghmclip.evaluation.zsc import zsc_logits
    with pytest.raises(RuntimeError):
        zsc_logits(torch.zeros(4, 10), torch.zeros(4, 10), torch.zeros(10, 2, dtype=torch.int32), [1])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_worker(rank, world, port, n, q):
    import torch.distributed as dist
    from ghmclip.evaluation.zsc import gather_rows, shard_rows
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.arange(n * 10, dtype=torch.float32).reshape(n, 10)
        lo, hi, per = shard_rows(n, rank, world)
        got = gather_rows(full[lo:hi].clone(), n, per)
        q.put((rank, bool(torch.equal(got, full)), hi - lo))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(300, 2), (301, 2), (7, 4)])
def test_dp_shard_and_gather_rows_gloo(n, world):
    """Each rank embeds a contiguous ceil(n/world) shard; the all-gather of the
    text embeddings rebuilds all n rows in order on every rank (n not divisible
    by the world size, and a rank with a short shard)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=60) for _ in range(world)]
    for p in ps:
        p.join(timeout=30)
    assert all(ok for _, ok, _ in res)
    assert sum(k for _, _, k in res) == n
