"""Non-translation-invariant GHM trees and unequal text / image trees on the host
(GenTransition translation_invariance=False, data_random_GHM.py:43-89; the tree
draw :145-165; ClipSampler n_layers / n_childs :645-658), against the
reference's own draws (tests/golden/make_golden_ti.py): per-edge transitions,
the native sampler's batches, get_Bayes (host BP_CLS on per-edge tables) and the
guided next-word-prediction targets of scripts/examples/eg_nwp.sh's trees."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

P_Y = np.ones(10) / 10


def _edges(transition):
    return np.concatenate([np.stack(layer) for layer in transition])


def test_clip_sampler_nonti_unequal_trees_bit_exact():
    from ghmclip import ClipSampler, seed_everything
    g = np.load(os.path.join(GOLDEN, "clip_nonti.npz"))
    s = ClipSampler([4, 3], [3, 2], [P_Y, P_Y], [0.3, 0.2], K=4, translation_invariance=False, seedtree=42)
    np.testing.assert_array_equal(_edges(s.t_transition), g["t_edges"])
    np.testing.assert_array_equal(_edges(s.i_transition), g["i_edges"])
    assert s.t_templ is None and s.i_templ is None  # per-edge matrices: no templates
    assert (s.T_t, s.T_i) == (81, 8)
    seed_everything(224)
    for k in range(2):
        rt, ri = s.get_batch(batch_size=int(g["B"]))
        np.testing.assert_array_equal(rt[0].numpy(), g[f"t_leaves{k}"])
        np.testing.assert_array_equal(ri[0].numpy(), g[f"i_leaves{k}"])
        np.testing.assert_array_equal(rt[1].numpy(), g[f"t_root{k}"])
        np.testing.assert_array_equal(ri[1].numpy(), g[f"i_root{k}"])
    m, se = s.get_Bayes(n_eval=300)
    np.testing.assert_allclose([m, se], g["bayes"], rtol=1e-12)


def test_device_tree_nonti_per_edge_tables():
    """device_templates of a non-invariant tree: every edge's matrix, layer by
    layer in child order (the per_edge layout of ghm_bp_cls / ghm_bp_dns), and
    host BP on it == host BP on the reference's transition lists."""
    from ghmclip import ClipSampler
    from ghmclip.data.data_random_GHM import DeviceTree, _bp_levels
    s = ClipSampler([2, 3], [3, 2], [P_Y, P_Y], [0.3, 0.3], K=4, translation_invariance=False, seedtree=42)
    t, i = s.device_templates("guided CLIP")
    assert isinstance(t, DeviceTree) and t.per_edge == 1 and (t.L, t.C, t.V) == (2, 3, 10)
    assert isinstance(i, DeviceTree) and i.per_edge == 1 and (i.L, i.C, i.V) == (3, 2, 10)
    assert t.trans.shape == (3 + 9, 10, 10) and i.trans.shape == (2 + 4 + 8, 10, 10)
    np.testing.assert_array_equal(t.trans, _edges(s.t_transition))
    leaves = np.random.default_rng(0).integers(0, 10, size=(5, 8))
    for a, b in zip(_bp_levels(i, leaves), _bp_levels(s.i_transition, leaves)):
        np.testing.assert_array_equal(a, b)
    ti = ClipSampler([2, 2], [3, 3], [P_Y, P_Y], [0.3, 0.3], K=4, seedtree=42)
    t0, _ = ti.device_templates()
    assert DeviceTree.of(t0).per_edge == 0 and t0.shape == (2, 3, 10, 10)


def test_nwp_nonti_guided_batch_matches_reference():
    """eg_nwp.sh's trees (p = 0.4, translation_invariance=False): get_batch(guide=True)
    draws, BP_NWP posteriors and the 9 text / 4 image guide targets."""
    from ghmclip import NextWordPredictSampler, seed_everything
    g = np.load(os.path.join(GOLDEN, "nwp_nonti.npz"))
    s = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.4, 0.4], translation_invariance=False, seedtree=42)
    np.testing.assert_array_equal(_edges(s.t_transition), g["t_edges"])
    seed_everything(224)
    rt, ri = s.get_batch(batch_size=int(g["B"]), guide=True)
    np.testing.assert_array_equal(rt[0].numpy(), g["t_leaves"][:, :-1])
    np.testing.assert_array_equal(rt[1].numpy(), g["t_leaves"][:, 1:])
    np.testing.assert_array_equal(ri[0].numpy(), g["i_leaves"])
    np.testing.assert_array_equal(ri[1].numpy(), g["root"])
    np.testing.assert_allclose(rt[3].numpy(), g["post"], rtol=1e-6, atol=1e-7)
    assert len(rt[2]) == 9 and len(ri[2]) == 4
    for k in range(9):
        np.testing.assert_allclose(rt[2][k].numpy(), g[f"text{k}"], rtol=1e-6, atol=1e-5, err_msg=f"text {k}")
    for k in range(4):
        np.testing.assert_allclose(ri[2][k].numpy(), g[f"image{k}"], rtol=1e-6, atol=1e-5, err_msg=f"image {k}")


def test_nwp_pipeline_nonti_matches_sampler():
    """The train_NWP producer (NwpBatchPipeline, guide=True) on non-invariant trees
    fills its slots with the sampler's own draws and posteriors."""
    from ghmclip import NextWordPredictSampler, seed_everything
    from ghmclip.data.data_random_GHM import vlm_guide_planes
    from ghmclip.training.pipeline import NwpBatchPipeline
    B = 4
    ref = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.4, 0.4], translation_invariance=False)
    s = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.4, 0.4], translation_invariance=False)
    seed_everything(224)
    tl, il, _ = ref.draw_numpy(B)
    post, _, tg, ig = ref.posterior(tl, il, guide=True)
    seed_everything(224)
    s.native.pull_numpy_state()
    pipe = NwpBatchPipeline(s, B, n_slots=2, guide=True)
    try:
        assert pipe.ready[0].wait(timeout=60)
        xt, yt, p, im, gt = pipe.slots[0]
        np.testing.assert_array_equal(xt.numpy(), tl[:, :-1])
        np.testing.assert_array_equal(im.numpy(), il)
        np.testing.assert_array_equal(p.numpy(), post)
        np.testing.assert_array_equal(gt.numpy(), vlm_guide_planes(tg, ig, 10))
    finally:
        pipe.close()


def _tree(edges, L, C):
    from ghmclip.data.data_random_GHM import DeviceTree
    return DeviceTree(edges, L, C, edges.shape[-1], 1)


def test_guided_targets_nonti_host_matches_reference():
    """Host BP_CLS guided targets on per-edge tables == GHMTree.guided_info of the
    reference's non-invariant trees (clip_nonti_guide.npz)."""
    from ghmclip.data.data_random_GHM import guided_targets
    g = np.load(os.path.join(GOLDEN, "clip_nonti_guide.npz"))
    for pref, L, C in (("t", 4, 3), ("i", 3, 2)):
        got = guided_targets(_tree(g[f"{pref}_edges"], L, C), g[f"{pref}_leaves"])
        assert len(got) == L
        for k, m in enumerate(got):
            np.testing.assert_allclose(m.numpy()[:, ::C ** (k + 1)], g[f"{pref}_msg{k}"], rtol=1e-6, atol=1e-6)


def test_bp_dns_nonti_host_matches_reference():
    """Host BP_DNS posterior means on per-edge tables == the reference's
    posterior_mean_DNS on a non-invariant tree (cdm_nonti.npz)."""
    from ghmclip.data.data_random_GHM import _bp_levels, bp_dns_posterior
    g = np.load(os.path.join(GOLDEN, "cdm_nonti.npz"))
    ext = _bp_levels(_tree(g["t_edges"], 4, 3), g["t_leaves"])[-1][0]
    post = bp_dns_posterior(_tree(g["i_edges"], 4, 3), g["z"].T, 1.0, ext)
    np.testing.assert_allclose(post.T, g["post"], rtol=1e-12, atol=1e-12)


def test_cdm_sampler_unequal_trees_matches_reference():
    """ConditionalDenoiseSampler on the trees of the reference's own unit tests
    (tests/test_data_randomghm.py: n_layers [3, 4], sigma 0.1): text and image
    leaf counts differ (27 / 81); draws, BP_DNS posterior means and get_Bayes
    against the reference (cdm_unequal.npz)."""
    from ghmclip import ConditionalDenoiseSampler, seed_everything
    g = np.load(os.path.join(GOLDEN, "cdm_unequal.npz"))
    s = ConditionalDenoiseSampler([3, 4], [3, 3], [P_Y, P_Y], [0.1, 0.1], sigma=0.1)
    assert (s.T_t, s.T_i) == (27, 81)
    seed_everything(3)
    for k in range(2):
        rt, ri = s.get_batch(batch_size=int(g["B"]))
        np.testing.assert_array_equal(rt[0].numpy(), g[f"t_leaves{k}"])
        np.testing.assert_array_equal(rt[1].numpy(), g[f"root{k}"])
        np.testing.assert_array_equal(ri[0].numpy(), g[f"z{k}"])
        np.testing.assert_array_equal(ri[1].numpy(), g[f"i_leaves{k}"])
        np.testing.assert_allclose(ri[3], g[f"post{k}"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(s.get_Bayes(n_eval=500), g["bayes"], rtol=1e-8)


def test_conditional_denoising_posterior_identity():
    """The reference's own unit test (tests/test_data_randomghm.py:38-45) on this
    package, as written there: with exact posterior means x_hat, E[x_hat^2] =
    E[x_hat x] over a 10,000-sample guide=True batch, |difference| < 3e-3."""
    from ghmclip import ConditionalDenoiseSampler
    s = ConditionalDenoiseSampler([3, 4], [3, 3], [P_Y, P_Y], [0.1, 0.1], sigma=0.1, flip_scale=1,
                                  translation_invariance=True, variable_type=10)
    _, res_image = s.get_batch(batch_size=10000, guide=True)
    assert len(res_image[2]) == 2 * 4 + 1
    true, pred = np.asarray(res_image[1]), np.asarray(res_image[-1])
    err = abs(np.mean(np.mean(pred ** 2, 1)) - np.mean(np.mean(pred * true, 1)))
    assert err < 3e-3, err


def test_cdm_guided_info_nonti_matches_reference():
    """ConditionalDenoiseSampler.get_batch(guide=True) on non-invariant trees: the
    text BP_CLS and image BP_DNS guided_info levels (data_random_GHM.py:526-592)
    against the reference's own batch (cdm_nonti.npz, stored one column per node)."""
    from ghmclip import ConditionalDenoiseSampler, seed_everything
    g = np.load(os.path.join(GOLDEN, "cdm_nonti.npz"))
    s = ConditionalDenoiseSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2], sigma=1, translation_invariance=False)
    seed_everything(5)
    rt, ri = s.get_batch(batch_size=int(g["B"]), guide=True)
    np.testing.assert_array_equal(rt[0].numpy(), g["t_leaves"])
    np.testing.assert_allclose(ri[3], g["post"], rtol=1e-10, atol=1e-12)
    assert len(rt[2]) == 4 and len(ri[2]) == 9
    for k, m in enumerate(rt[2]):
        np.testing.assert_allclose(m.numpy()[:, ::3 ** (k + 1)], g[f"text{k}"], rtol=1e-6, atol=1e-6)
    for k, m in enumerate(ri[2]):
        depth = 4 - k if k <= 4 else k - 4
        np.testing.assert_allclose(m.numpy()[:, ::3 ** (4 - depth)], g[f"image{k}"], rtol=1e-6, atol=1e-5,
                                   err_msg=f"image level {k}")
