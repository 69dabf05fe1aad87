"""Guided VLM host targets (train_NWP.py --guide=True): the vectorised
BP_NWP_autoregressive(guide_info=True) restatement and the image guided_info,
against the reference's own NextWordPredictSampler.get_batch(guide=True) draw
(tests/golden/vlm_guided_bp.npz, tests/golden/make_golden_vlm_guided.py)."""
import os

import numpy as np

from conftest import GOLDEN


def _sampler():
    from ghmclip import NextWordPredictSampler
    p_y = np.ones(10) / 10
    return NextWordPredictSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2])


def test_bp_nwp_guide_targets_match_reference():
    from ghmclip.data.data_random_GHM import bp_cls_root_message, bp_nwp_posterior, guided_targets
    g = np.load(os.path.join(GOLDEN, "vlm_guided_bp.npz"))
    s = _sampler()
    tl, il = g["t_leaves"], g["i_leaves"]
    ext = bp_cls_root_message(s.i_templ, il)
    post, tg = bp_nwp_posterior(s.t_templ, tl, ext, guide=True)
    np.testing.assert_allclose(post, g["post"], rtol=1e-6, atol=1e-7)
    assert len(tg) == 9
    for k, t in enumerate(tg):
        want = g[f"text{k}"]
        assert t.shape == want.shape, k
        np.testing.assert_allclose(t, want, rtol=1e-6, atol=1e-5, err_msg=f"text target {k}")
    ig = guided_targets(s.i_templ, il)
    assert len(ig) == 4
    for k, t in enumerate(ig):
        np.testing.assert_allclose(t.numpy(), g[f"image{k}"], rtol=1e-6, atol=1e-5, err_msg=f"image target {k}")


def test_get_batch_guide_draws_reference_batch():
    """get_batch(guide=True) after seed_everything(224) = the reference's draw."""
    from ghmclip import seed_everything
    g = np.load(os.path.join(GOLDEN, "vlm_guided_bp.npz"))
    s = _sampler()
    seed_everything(224)
    rt, ri = s.get_batch(batch_size=int(g["B"]), guide=True)
    np.testing.assert_array_equal(rt[0].numpy(), g["t_leaves"][:, :-1])
    np.testing.assert_array_equal(ri[0].numpy(), g["i_leaves"])
    assert len(rt[2]) == 9 and len(ri[2]) == 4
    for k in range(9):
        np.testing.assert_allclose(rt[2][k].numpy(), g[f"text{k}"], rtol=1e-6, atol=1e-5)


def test_guide_planes_layout():
    """vlm_guide_planes: 13 text blocks (the (hd, qd) / (hd, bu) targets split in two)
    then 4 image blocks, per sample."""
    from ghmclip.data.data_random_GHM import vlm_guide_planes
    B, n, V = 2, 80, 10
    rng = np.random.default_rng(0)
    tg = [rng.standard_normal((B, n, V if k in (0, 5, 6, 7, 8) else 2 * V)).astype(np.float32) for k in range(9)]
    ig = [rng.standard_normal((B, 81, V)).astype(np.float32) for _ in range(4)]
    pl = vlm_guide_planes(tg, ig, V)
    assert pl.shape == (B, 13 * n * V + 4 * 81 * V)
    blk = pl[:, :13 * n * V].reshape(B, 13, n, V)
    np.testing.assert_array_equal(blk[:, 0], tg[0])
    np.testing.assert_array_equal(blk[:, 1], tg[1][:, :, :V])
    np.testing.assert_array_equal(blk[:, 2], tg[1][:, :, V:])
    np.testing.assert_array_equal(blk[:, 7], tg[4][:, :, :V])
    np.testing.assert_array_equal(blk[:, 9], tg[5])
    np.testing.assert_array_equal(pl[:, 13 * n * V:].reshape(B, 4, 81, V)[:, 3], ig[3])


def test_sequential_guided_blocks_and_planes():
    """train_sequential_NWP.py --guide=True (n_guided_layers = [n_ttree_layer, 1],
    L = 9): every layer text-guided, layers 0 and 3 image-guided (model.py:207-216);
    text blocks start at token 1 (one prefix token), the two image blocks are
    columns 0:10 / 10:20 of the prefix row; the packed planes hold the 13 text
    blocks only (the image targets are the CLIP feature, read on the device)."""
    from ghmclip import AutoRegressiveTransformer
    from ghmclip.models.vlm import vlm_guide_blocks, vlm_guide_plane_elems
    from ghmclip.training.pipeline import NwpBatchPipeline
    m = AutoRegressiveTransformer(81, 1, 10, 256, 9, [4, 1], 4, 1024, auto_regressive=True, sequential=True,
                                  guide=True)
    assert m.t_guided_layer_flag == [True] * 9
    assert m.i_guided_layer_flag == [True, False, False, True] + [False] * 5
    blocks = vlm_guide_blocks(m, 80, 10)
    assert sorted(blocks) == list(range(9))
    img = [(l, b[:3]) for l in sorted(blocks) for b in blocks[l] if b[4] == "loss3"]
    assert img == [(0, (0, 1, 0)), (3, (0, 1, 10))]
    text = [b for l in sorted(blocks) for b in blocks[l] if b[4] != "loss3"]
    assert all(b[0] == 1 and b[1] == 80 for b in text) and len(text) == 13
    assert sorted(b[3] for b in text) == [800 * k for k in range(13)]
    assert vlm_guide_plane_elems(m, 80, 10) == 13 * 800
    # the joint model keeps one plane per image-guided layer
    mj = AutoRegressiveTransformer(161, 81, 10, 256, 9, [4, 4], 4, 1024, auto_regressive=True, sequential=False,
                                   guide=True)
    assert vlm_guide_plane_elems(mj, 80, 10) == 13 * 800 + 4 * 810
    pipe = NwpBatchPipeline.__new__(NwpBatchPipeline)
    pipe.sampler, pipe.guide, pipe.image_guide = _sampler(), True, False
    pipe.B, pipe.slice = 2, None
    pipe.s = pipe.sampler.native
    pipe._make_slots(1)
    assert tuple(pipe.slots[0][4].shape) == (2, 13 * 800)
    pipe._fill(0)
    xt, _, post, il, gt = pipe.slots[0]
    from ghmclip.data.data_random_GHM import vlm_guide_planes
    _, _, tg, _ = pipe.sampler.posterior(pipe.tl, il.numpy(), guide=True)
    np.testing.assert_array_equal(gt.numpy(), vlm_guide_planes(tg, [], 10))
