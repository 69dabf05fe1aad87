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


def test_device_paths_refuse_nonti_templates():
    from ghmclip import ClipSampler
    s = ClipSampler([2, 2], [3, 3], [P_Y, P_Y], [0.3, 0.3], K=4, translation_invariance=False, seedtree=42)
    with pytest.raises(NotImplementedError):
        s.device_templates("guided CLIP")


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
