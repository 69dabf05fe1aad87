"""Data-parallel sharding on CPU (gloo, world_size 2): the product's row
sharding (ghmclip.training.pipeline.shard_rows) + an AVG all-reduce of the
per-rank gradients reproduce the full-batch loss and gradients.
The per-rank forward/backward is the CPU oracle (no GPU here)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, K, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-ghm_amd")]
    from ghmclip.training.pipeline import shard_rows
    from oracle import ghm_oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    s = O.ClipSamplerOracle([3, 3], [3, 3], [0.2, 0.2], K=K, seedtree=42)
    O.seed_everything(224)
    tm, im = O.build_encoders(27, 1, 16)
    batch = s.get_batch(B)  # every rank draws the same global batch
    idx = shard_rows(B, K + 1, rank, world)
    t = tm(torch.as_tensor(batch[0][idx]))[0]
    i = im(torch.as_tensor(batch[2][idx]))[0]
    loss = O.clip_loss(t, i, K, B // world)
    loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in list(tm.parameters()) + list(im.parameters())])
    dist.all_reduce(g, op=dist.ReduceOp.SUM)
    g /= world
    lt = loss.detach().reshape(1).clone()
    dist.all_reduce(lt, op=dist.ReduceOp.SUM)
    if rank == 0:
        out.put((g.numpy(), float(lt.item() / world)))
    dist.destroy_process_group()


def test_sharded_grads_equal_full_batch():
    from oracle import ghm_oracle as O
    B, K, world = 8, 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, B, K, q)) for r in range(world)]
    for p in ps:
        p.start()
    g_dp, loss_dp = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    s = O.ClipSamplerOracle([3, 3], [3, 3], [0.2, 0.2], K=K, seedtree=42)
    O.seed_everything(224)
    tm, im = O.build_encoders(27, 1, 16)
    batch = s.get_batch(B)
    loss = O.clip_loss(tm(torch.as_tensor(batch[0]))[0], im(torch.as_tensor(batch[2]))[0], K, B)
    loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in list(tm.parameters()) + list(im.parameters())]).numpy()
    assert abs(loss_dp - loss.item()) < 1e-6
    np.testing.assert_allclose(g_dp, g, rtol=1e-4, atol=1e-7)


def test_shard_rows_partition():
    from ghmclip.training.pipeline import shard_rows
    B, K = 16, 4
    parts = [shard_rows(B, K + 1, r, 4) for r in range(4)]
    allrows = np.sort(np.concatenate(parts))
    np.testing.assert_array_equal(allrows, np.arange(B * (K + 1)))
    # each shard keeps the block structure: block b of the shard = rows b*B + [r*B/4, (r+1)*B/4)
    np.testing.assert_array_equal(parts[1][:4], [4, 5, 6, 7])
    np.testing.assert_array_equal(parts[1][4:8], [20, 21, 22, 23])


def _cdm_worker(rank, world, port, B, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-ghm_amd")]
    from ghmclip.training.pipeline import shard_samples
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    model, batch, cond = _cdm_setup(B)
    a, b = shard_samples(B, rank, world)
    loss = _cdm_loss(model, batch, cond, slice(a, b))
    loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in model.parameters() if p.grad is not None])
    dist.all_reduce(g, op=dist.ReduceOp.SUM)
    g /= world
    lt = loss.detach().reshape(1).clone()
    dist.all_reduce(lt, op=dist.ReduceOp.SUM)
    if rank == 0:
        out.put((g.numpy(), float(lt.item() / world)))
    dist.destroy_process_group()


def _cdm_setup(B):
    """Small CDM (27-leaf trees, d=16, L=1) on one global batch, conditioning
    features standing in for the frozen CLIP embedding."""
    from oracle import cdm_oracle as CO
    CO.seed_everything(224)
    s = CO.CdmSamplerOracle([3, 3], [3, 3], [0.2, 0.2])
    batch = s.get_batch(B)
    model = CO.OracleCdm(28, 27, 10, 16, 1, 64)
    cond = torch.randn(B, 1, 10, generator=torch.Generator().manual_seed(1))
    return model, batch, cond


def _cdm_loss(model, batch, cond, rows):
    from oracle import cdm_oracle as CO
    _, _, z, il, _ = batch
    pred = model(cond[rows], torch.as_tensor(z[rows]))
    return CO.ls_loss(pred, torch.as_tensor(il[rows], dtype=torch.long))


def test_cdm_sharded_grads_equal_full_batch():
    """Sequential CDM data parallel: each rank's contiguous sample shard
    (pipeline.shard_samples) + an AVG all-reduce == the full-batch gradient."""
    B, world = 8, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_cdm_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in ps:
        p.start()
    g_dp, loss_dp = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    model, batch, cond = _cdm_setup(B)
    loss = _cdm_loss(model, batch, cond, slice(0, B))
    loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in model.parameters() if p.grad is not None]).numpy()
    assert abs(loss_dp - loss.item()) <= 1e-6 * loss.item()
    np.testing.assert_allclose(g_dp, g, rtol=1e-4, atol=1e-6)


def _bucket_worker(rank, world, port, out):
    """Every rank: the product's flat layout of two 5-layer towers, a rank-seeded
    gradient, then (a) one flat all-reduce, (b) the two buckets ClipTrainer.step
    issues (A = top layers, B = the rest), each through distributed.py."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-ghm_amd")]
    from ghmclip.training import distributed
    from ghmclip.training.clip_trainer import dp_bucket_ranges, flat_layout
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    tm, im = _towers()
    _, bucket_a, n = flat_layout([tm, im], 3)
    g = torch.randn(n, generator=torch.Generator().manual_seed(100 + rank)) * 10.0 ** torch.randint(
        -6, 3, (n,), generator=torch.Generator().manual_seed(7 + rank))
    flat = distributed.allreduce_mean_(g.clone())
    a, b = dp_bucket_ranges(bucket_a, n)
    bucketed = g.clone()
    distributed.allreduce_ranges_mean_(bucketed, a)
    distributed.allreduce_ranges_mean_(bucketed, b)
    if rank == 0:
        out.put((flat.numpy(), bucketed.numpy()))
    dist.destroy_process_group()


def _towers():
    from ghmclip.models.model import EncoderTransformer
    torch.manual_seed(0)
    return EncoderTransformer(81, 10, n_embd=128, n_layer=5), EncoderTransformer(27, 10, n_embd=128, n_layer=5)


def test_bucketed_allreduce_equals_flat_bit_for_bit():
    """SURVEY §5 / DP=8 prep: the per-layer-bucket all-reduce (bucket A issued
    while the lower layers' backward runs) gives exactly the flat all-reduce's
    gradient at world 2."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    flat, bucketed = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert flat.tobytes() == bucketed.tobytes()


def test_flat_layout_buckets_cover_top_layers():
    """Bucket A of each tower holds exactly its top dp_top layers' parameters
    and A + B tile [0, n) once."""
    from ghmclip.training.clip_trainer import _layer_of, dp_bucket_ranges, flat_layout
    tm, im = _towers()
    for top in range(0, 6):
        layout, bucket_a, n = flat_layout([tm, im], top)
        assert n == sum(p.numel() for m in (tm, im) for p in m.parameters())
        a, b = dp_bucket_ranges(bucket_a, n)
        cover = np.zeros(n, dtype=np.int64)
        for lo, hi in a + b:
            cover[lo:hi] += 1
        assert (cover == 1).all()
        for m, slots, (lo, hi) in zip((tm, im), layout, bucket_a):
            for name, (off, k) in slots.items():
                ly = _layer_of(name)
                in_a = lo <= off and off + k <= hi
                assert in_a == (ly is not None and ly >= m.n_layer - top), (top, name)


def test_flat_layout_unequal_towers():
    """--clip_tmodel_nlayer=4 --clip_imodel_nlayer=1 (the reference takes separate
    layer counts, utils/config.py): the bucket depth is clamped per tower, so the
    1-layer tower's bucket A is its one layer and A + B still tile [0, n) once."""
    from ghmclip.models.model import EncoderTransformer
    from ghmclip.training.clip_trainer import _layer_of, dp_bucket_ranges, flat_layout
    torch.manual_seed(0)
    tm, im = EncoderTransformer(81, 10, n_embd=128, n_layer=4), EncoderTransformer(81, 10, n_embd=128, n_layer=1)
    for top in range(0, 5):
        layout, bucket_a, n = flat_layout([tm, im], top)
        a, b = dp_bucket_ranges(bucket_a, n)
        cover = np.zeros(n, dtype=np.int64)
        for lo, hi in a + b:
            cover[lo:hi] += 1
        assert (cover == 1).all()
        for m, slots, (lo, hi) in zip((tm, im), layout, bucket_a):
            for name, (off, k) in slots.items():
                ly = _layer_of(name)
                in_a = lo <= off and off + k <= hi
                assert in_a == (ly is not None and ly >= m.n_layer - min(top, m.n_layer)), (top, name)


def _world4_worker(rank, world, port, B, K, out):
    """A strong split of the global batch over `world` ranks (B / world rows of
    every block per rank, pipeline.shard_rows), the per-rank oracle gradient, and
    the product's bucketed asynchronous all-reduce (distributed.allreduce_ranges_start
    / allreduce_finish: both buckets started before either is waited for, as
    ClipTrainer.step issues bucket A while the lower layers' backward runs)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-ghm_amd")]
    from ghmclip.training import distributed
    from ghmclip.training.pipeline import shard_rows
    from oracle import ghm_oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    s = O.ClipSamplerOracle([3, 3], [3, 3], [0.2, 0.2], K=K, seedtree=42)
    O.seed_everything(224)
    tm, im = O.build_encoders(27, 1, 16)
    batch = s.get_batch(B)  # every rank draws the same global batch
    idx = shard_rows(B, K + 1, rank, world)
    t = tm(torch.as_tensor(batch[0][idx]))[0]
    i = im(torch.as_tensor(batch[2][idx]))[0]
    loss = O.clip_loss(t, i, K, B // world)
    loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in list(tm.parameters()) + list(im.parameters())])
    n = g.numel()
    pa = distributed.allreduce_ranges_start(g, [(0, n // 3)])
    pb = distributed.allreduce_ranges_start(g, [(n // 3, n)])
    lt = loss.detach().reshape(1).clone()
    distributed.allreduce_mean_(lt)
    distributed.allreduce_finish(pa + pb)
    allg = [torch.empty_like(g) for _ in range(world)]
    dist.all_gather(allg, g)
    if rank == 0:
        out.put((g.numpy(), float(lt.item()), [x.numpy() for x in allg]))
    dist.destroy_process_group()


def test_world4_strong_split_equals_one_rank():
    """World 4, global B = 128 split into 32 rows per rank (review
    item 5): the mean over ranks of the shard losses and gradients equals the
    1-rank full-batch loss and gradient to the ring-order bound (4-term sums in a
    rank-order-dependent association: 1e-5 relative per element, 2e-7 on the
    loss), and every rank ends with the same bytes."""
    from oracle import ghm_oracle as O
    B, K, world = 128, 4, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_world4_worker, args=(r, world, port, B, K, q)) for r in range(world)]
    for p in ps:
        p.start()
    g_dp, loss_dp, per_rank = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for x in per_rank:
        assert x.tobytes() == g_dp.tobytes()
    s = O.ClipSamplerOracle([3, 3], [3, 3], [0.2, 0.2], K=K, seedtree=42)
    O.seed_everything(224)
    tm, im = O.build_encoders(27, 1, 16)
    batch = s.get_batch(B)
    loss = O.clip_loss(tm(torch.as_tensor(batch[0]))[0], im(torch.as_tensor(batch[2]))[0], K, B)
    loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in list(tm.parameters()) + list(im.parameters())]).numpy()
    assert abs(loss_dp - loss.item()) <= 2e-7 * abs(loss.item())
    scale = np.abs(g).max()
    assert np.abs(g_dp - g).max() <= 1e-5 * scale
