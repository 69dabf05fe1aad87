"""CPU tests of the sequential CDM path: the oracle against the reference's own
fixtures (tests/golden/make_golden_cdm.py) and the product's host side (native
ConditionalDenoiseSampler draws, host BP_DNS, module construction)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import cdm_oracle as CO

P_Y = np.ones(10) / 10


def _fix(name):
    return np.load(os.path.join(GOLDEN, name))


def test_oracle_sampler_and_bayes_match_reference():
    f = _fix("cdm_sampler.npz")
    CO.seed_everything(224)
    s = CO.CdmSamplerOracle([4, 4], [3, 3], [0.2, 0.2])
    np.testing.assert_array_equal(s.t_trans, f["t_transition"])
    np.testing.assert_array_equal(s.i_trans, f["i_transition"])
    bayes = s.get_Bayes(10000)
    np.testing.assert_allclose(bayes, f["bayes"], rtol=1e-12)
    for k in range(2):
        tl, root, z, il, post = s.get_batch(int(f["B"]))
        np.testing.assert_array_equal(tl, f["t_leaves"][k])
        np.testing.assert_array_equal(root, f["t_root"][k])
        np.testing.assert_array_equal(z, f["z"][k])
        np.testing.assert_array_equal(il, f["i_leaves"][k])
        np.testing.assert_allclose(post, f["post"][k], rtol=0, atol=1e-12)


def test_native_sampler_matches_reference():
    """ConditionalDenoiseSampler (native MT19937 + legacy Gaussians) == the reference's
    draws bit-for-bit, numpy's global state (incl. the cached Gaussian) left as the
    reference leaves it; host BP posteriors within 1e-12."""
    from ghmclip import ConditionalDenoiseSampler, seed_everything
    f = _fix("cdm_sampler.npz")
    seed_everything(224)
    s = ConditionalDenoiseSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2], sigma=1)
    bayes = s.get_Bayes(n_eval=10000)
    np.testing.assert_allclose(bayes, f["bayes"], rtol=1e-12)
    for k in range(2):
        (t, r, tg, tpp), (z, i, ig, post) = s.get_batch(int(f["B"]))
        assert tg is None and ig is None
        np.testing.assert_array_equal(t.numpy(), f["t_leaves"][k])
        np.testing.assert_array_equal(r.numpy(), f["t_root"][k])
        np.testing.assert_array_equal(z.numpy(), f["z"][k])
        np.testing.assert_array_equal(i.numpy(), f["i_leaves"][k])
        np.testing.assert_allclose(post, f["post"][k], rtol=0, atol=1e-12)
        np.testing.assert_allclose(tpp, f["t_pp"][k], rtol=0, atol=1e-12)
    # numpy's global state (MT key, position, cached Gaussian) ends where the
    # reference's per-node loops + randn leave it
    mine = np.random.get_state()
    CO.seed_everything(224)
    o = CO.CdmSamplerOracle([4, 4], [3, 3], [0.2, 0.2])
    o.get_Bayes(10000)
    o.get_batch(int(f["B"]))
    o.get_batch(int(f["B"]))
    want = np.random.get_state()
    np.testing.assert_array_equal(mine[1], want[1])
    assert mine[2] == want[2] and mine[3] == want[3] and mine[4] == want[4]


def test_native_randn_stream():
    """ghm_sampler_randn == numpy.random.randn, including the cached second deviate."""
    from ghmclip import ConditionalDenoiseSampler
    s = ConditionalDenoiseSampler([2, 2], [3, 3], [P_Y, P_Y], [0.2, 0.2])
    np.random.seed(5)
    np.random.randn(1)  # leave a cached Gaussian behind
    nat = s.native
    nat.pull_numpy_state()
    out = np.empty(7)
    from ghmclip import _native
    assert _native.host_lib().ghm_sampler_randn(nat._h, out.ctypes.data, 7) == 0
    want = np.random.randn(7)
    np.testing.assert_array_equal(out, want)
    np.random.seed(5)
    np.random.randn(1)
    nat.pull_numpy_state()
    nat.push_numpy_state()
    assert _native.host_lib().ghm_sampler_randn(nat._h, out.ctypes.data, 7) == 0
    nat.push_numpy_state()  # the native stream hands back to numpy mid-pair
    np.testing.assert_array_equal(np.random.randn(3), _after(5, 8, 3))


def _after(seed, skip, n):
    np.random.seed(seed)
    np.random.randn(skip)
    return np.random.randn(n)


def test_oracle_two_steps_match_reference():
    """Two full training steps at L=1, d=128, B=4 (cdm_tiny.npz): initial weights of
    both models, predictions, losses, compare and post-step parameters."""
    g = _fix("cdm_tiny.npz")
    tr = CO.OracleCdmTrainer(B=4, L=1)
    assert [n for n, _ in tr.model.named_parameters()] == list(g["param_names"])
    st = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
    np.testing.assert_array_equal(st, g["init_stats"])
    cst = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.clip.parameters()])
    np.testing.assert_array_equal(cst, g["clip_stats"])
    for k in range(2):
        ploss, loss, cmp = tr.step()
        assert ploss == float(g[f"ploss{k}"]) and loss == float(g[f"loss{k}"])
        assert abs(cmp - float(g[f"compare{k}"])) <= 1e-6 * cmp
        np.testing.assert_array_equal(tr.last_pred.numpy(), g[f"pred{k}"])
        np.testing.assert_array_equal(tr.last_feat[:, 0].numpy(), g[f"feat{k}"])
        ps = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
        np.testing.assert_allclose(ps, g[f"param_stats{k}"], rtol=1e-12, atol=1e-12)


def test_noln_oracle_two_steps_match_reference():
    """ConditionalDenoiseEncoderTransformer(layernorm=False) (model.py:470-477,
    488-498; the ModelConfig default): two full training steps at L=2, B=4
    (cdm_noln_tiny.npz); the unused LayerNorms get no gradient."""
    g = _fix("cdm_noln_tiny.npz")
    assert not bool(g["layernorm"])
    tr = CO.OracleCdmTrainer(B=4, L=2, layernorm=False)
    for k in range(2):
        ploss, loss, cmp = tr.step()
        assert abs(ploss - float(g[f"ploss{k}"])) <= 1e-6 * ploss
        assert abs(cmp - float(g[f"compare{k}"])) <= 1e-6 * cmp
        np.testing.assert_allclose(tr.last_pred.numpy(), g[f"pred{k}"], rtol=1e-5, atol=1e-4)
        ps = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
        np.testing.assert_allclose(ps[:, 1], g[f"param_stats{k}"][:, 1], rtol=1e-9)
    assert not any("_lns_" in n for n in g["grad_names0"])


def test_joint_oracle_two_steps_match_reference():
    """Joint model (train_CDNS.py, sequential=False, T = 162), two full training steps
    at L=1, B=4 (cdm_joint_tiny.npz): initial weights, predictions, losses, compare
    and post-step parameters."""
    g = _fix("cdm_joint_tiny.npz")
    tr = CO.OracleCdmJointTrainer(B=4, L=1)
    assert [n for n, _ in tr.model.named_parameters()] == list(g["param_names"])
    st = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
    np.testing.assert_array_equal(st, g["init_stats"])
    for k in range(2):
        batch = (g[f"t_leaves{k}"], None, g[f"z{k}"], g[f"i_leaves{k}"], g[f"post{k}"])
        drawn = tr.sampler.get_batch(tr.B)
        np.testing.assert_array_equal(np.asarray(drawn[0]), g[f"t_leaves{k}"])
        np.testing.assert_array_equal(np.asarray(drawn[2], dtype=np.float32), g[f"z{k}"])
        ploss, loss, cmp = tr.step(batch=batch)
        assert abs(ploss - float(g[f"ploss{k}"])) <= 1e-6 * ploss
        assert abs(cmp - float(g[f"compare{k}"])) <= 1e-6 * cmp
        np.testing.assert_allclose(tr.last_pred.numpy(), g[f"pred{k}"], rtol=1e-5, atol=1e-5)
        ps = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
        np.testing.assert_allclose(ps, g[f"param_stats{k}"], rtol=1e-6, atol=1e-9)


@pytest.mark.slow
def test_oracle_curve_head_matches_reference():
    """First 5 steps of the default CDM config (cdm_curve.npz)."""
    g = _fix("cdm_curve.npz")
    tr = CO.OracleCdmTrainer(B=128, L=9)
    np.testing.assert_allclose(tr.bayes, g["bayes"], rtol=1e-12)
    for k in range(5):
        ploss, _, cmp = tr.step()
        assert abs(ploss - g["ploss"][k]) <= 1e-6 * g["ploss"][k]
        assert abs(cmp - g["compare"][k]) <= 1e-6 * g["compare"][k]


def test_cdm_module_api_matches_reference_construction():
    """Same parameter names, shapes, registration order and seeded initial values
    as the reference constructor (via the oracle, itself pinned by cdm_tiny.npz)."""
    from ghmclip import ConditionalDenoiseEncoderTransformer
    from ghmclip.models.cdm import cdm_param_names
    torch.manual_seed(3)
    m = ConditionalDenoiseEncoderTransformer(82, 81, 10, 128, 3, [1, 4], 4, 512, sequential=True)
    torch.manual_seed(3)
    o = CO.OracleCdm(82, 81, 10, 128, 3, 512)
    assert list(m.state_dict().keys()) == list(o.state_dict().keys()) == cdm_param_names(3)
    for (k, a), (_, b) in zip(m.state_dict().items(), o.state_dict().items()):
        assert torch.equal(a, b), k
    # the joint model (sequential=False, train_CDNS.py) is built too, same construction
    torch.manual_seed(3)
    mj = ConditionalDenoiseEncoderTransformer(162, 81, 10, 128, 3, [4, 4], 4, 512, sequential=False)
    torch.manual_seed(3)
    oj = CO.OracleCdm(162, 81, 10, 128, 3, 512, sequential=False)
    for (k, a), (_, b) in zip(mj.state_dict().items(), oj.state_dict().items()):
        assert torch.equal(a, b), k
    with pytest.raises(ValueError):  # guided-layer gap 3 // 7 == 0 (the reference divides by it)
        ConditionalDenoiseEncoderTransformer(162, 81, 10, 128, 3, sequential=False, guide=True)
    # guided sequential model (eg_sdns.sh): same construction (RNG order) as unguided
    torch.manual_seed(3)
    ms = ConditionalDenoiseEncoderTransformer(82, 81, 10, 128, 9, [1, 4], 4, 512, sequential=True, guide=True)
    torch.manual_seed(3)
    os_ = CO.OracleCdm(82, 81, 10, 128, 9, 512)
    for (k, a), (_, b) in zip(ms.state_dict().items(), os_.state_dict().items()):
        assert torch.equal(a, b), k
    # guided joint model (exp_cdm_guidedTF.sh): flags and guide blocks as model.py:392-416, 458-527
    from ghmclip.models.cdm import cdm_guide_blocks
    torch.manual_seed(3)
    mg = ConditionalDenoiseEncoderTransformer(162, 81, 10, 128, 9, [4, 4], 4, 512, sequential=False, guide=True)
    torch.manual_seed(3)
    og = CO.OracleCdm(162, 81, 10, 128, 9, 512, sequential=False)
    for (k, a), (_, b) in zip(mg.state_dict().items(), og.state_dict().items()):
        assert torch.equal(a, b), k  # the flags draw no random numbers
    assert mg.i_guided_layer_flag == [True] * 9 and mg.t_guided_layer_flag == [True] * 4 + [False] * 5
    blocks = cdm_guide_blocks(mg, (4, 3), (4, 3), 10)
    cols = {l: [(b[0], b[3]) for b in blocks[l]] for l in blocks}
    assert cols[0] == [("i", 0), ("i", 40), ("t", 0)]      # leaves h / q, text depth 3
    assert cols[4] == [("i", 40), ("i", 80)]                # root hd / bu
    assert cols[5] == [("i", 40), ("i", 80), ("i", 80)]     # first upward layer: q and u share a slice
    assert cols[8] == [("i", 10), ("i", 50), ("i", 110)]
    assert [b[5] for b in blocks[0]] == [1, 1, 3] and blocks[4][0][5] == 81 and blocks[8][0][5] == 1
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, 1, 10), torch.zeros(2, 81))  # CPU tensors: no fallback


def test_checkpoint_loader_accepts_numpy_scalars(tmp_path):
    """The weights-only loader reads the checkpoint dicts the CLIs write (numpy
    histories, the numpy-scalar Bayes risk, the data-only loss descriptor)."""
    from ghmclip.training.train_CLIP import load_checkpoint
    p = tmp_path / "checkpoint.pth"
    torch.save({"bayes": np.mean(np.ones(3)), "loss_history": np.zeros(4), "iter": 3,
                "loss": {"type": "ConditionalGuidedLsLoss", "penalty": 0.1, "guide": False}}, p)
    d = load_checkpoint(str(p), "cpu")
    assert d["bayes"] == 1.0 and d["iter"] == 3 and d["loss"]["penalty"] == 0.1


# ---------------------------------------------------------------------------
# sequential VLM (BASELINE config 5): oracle and product sampler vs the reference
# ---------------------------------------------------------------------------
def test_vlm_oracle_sampler_and_bayes_match_reference():
    from oracle import vlm_oracle as VO
    f = _fix("vlm_sampler.npz")
    s = VO.NwpSamplerOracle([4, 4], [3, 3], [0.2, 0.2])
    np.testing.assert_array_equal(s.t_trans, f["t_transition"])
    np.testing.assert_allclose(s.get_Bayes(int(f["n_bayes"])), f["bayes"], rtol=1e-6)
    np.random.seed(224)
    for k in range(2):
        xt, yt, post, il, root = s.get_batch(int(f["B"]))
        np.testing.assert_array_equal(xt, f["xt"][k])
        np.testing.assert_array_equal(yt, f["yt"][k])
        np.testing.assert_array_equal(il, f["i_leaves"][k])
        np.testing.assert_array_equal(root, f["i_root"][k])
        np.testing.assert_allclose(post, f["post"][k], rtol=0, atol=1e-7)


def test_vlm_native_sampler_matches_reference():
    """NextWordPredictSampler: native paired trees bit-exact, host BP_NWP_autoregressive
    posteriors equal to the reference's float32 tensor, Bayes risk."""
    from ghmclip import NextWordPredictSampler
    f = _fix("vlm_sampler.npz")
    s = NextWordPredictSampler([4, 4], [3, 3], [P_Y, P_Y], [0.2, 0.2])
    bayes = s.get_Bayes(int(f["n_bayes"]))
    np.testing.assert_allclose([float(bayes[0]), float(bayes[1])], f["bayes"], rtol=1e-6)
    np.random.seed(224)
    for k in range(2):
        (xt, yt, tg, post), (il, root, ig, ipp) = s.get_batch(int(f["B"]))
        assert tg is None and ig is None
        np.testing.assert_array_equal(xt.numpy(), f["xt"][k])
        np.testing.assert_array_equal(yt.numpy(), f["yt"][k])
        np.testing.assert_array_equal(il.numpy(), f["i_leaves"][k])
        np.testing.assert_array_equal(root.numpy(), f["i_root"][k])
        np.testing.assert_allclose(post.numpy(), f["post"][k], rtol=0, atol=1e-7)
        np.testing.assert_allclose(ipp, f["i_pp"][k], rtol=0, atol=1e-12)


def test_vlm_oracle_two_steps_match_reference():
    """Two full training steps at d=256, L=1, B=4 (vlm_tiny.npz)."""
    from oracle import vlm_oracle as VO
    g = _fix("vlm_tiny.npz")
    tr = VO.OracleVlmTrainer(B=4, L=1)
    assert [n for n, _ in tr.model.named_parameters()] == list(g["param_names"])
    st = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
    np.testing.assert_array_equal(st, g["init_stats"])
    cst = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.clip.parameters()])
    np.testing.assert_array_equal(cst, g["clip_stats"])
    for k in range(2):
        ploss, loss, cmp = tr.step()
        assert ploss == float(g[f"ploss{k}"]) and loss == float(g[f"loss{k}"])
        assert abs(cmp - float(g[f"compare{k}"])) <= 1e-6 * cmp
        np.testing.assert_array_equal(tr.last_logits.numpy(), g[f"logits{k}"])
        ps = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
        np.testing.assert_allclose(ps, g[f"param_stats{k}"], rtol=1e-12, atol=1e-12)


def test_vlm_relu_oracle_two_steps_match_reference():
    """AutoRegressiveTransformer(activation="relu") (model.py:121-130, 287): two full
    training steps at d=256, L=1, B=4 (vlm_relu_tiny.npz)."""
    from oracle import vlm_oracle as VO
    g = _fix("vlm_relu_tiny.npz")
    assert str(g["activation"]) == "relu"
    tr = VO.OracleVlmTrainer(B=4, L=1, activation="relu")
    for k in range(2):
        ploss, loss, cmp = tr.step()
        assert abs(ploss - float(g[f"ploss{k}"])) <= 1e-6 * ploss
        assert abs(cmp - float(g[f"compare{k}"])) <= 1e-5 * cmp
        np.testing.assert_allclose(tr.last_logits.numpy(), g[f"logits{k}"], rtol=1e-5, atol=1e-5)
        ps = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
        np.testing.assert_allclose(ps[:, 1], g[f"param_stats{k}"][:, 1], rtol=1e-9)


def test_vlm_noln_oracle_two_steps_match_reference():
    """AutoRegressiveTransformer(layernorm=False) (model.py:269-277, 294-301): two
    full training steps at d=256, L=2, B=4 (vlm_noln_tiny.npz); the unused
    LayerNorms get no gradient and no AdamW update."""
    from oracle import vlm_oracle as VO
    g = _fix("vlm_noln_tiny.npz")
    assert not bool(g["layernorm"])
    tr = VO.OracleVlmTrainer(B=4, L=2, layernorm=False)
    for k in range(2):
        ploss, loss, cmp = tr.step()
        assert abs(ploss - float(g[f"ploss{k}"])) <= 1e-6 * ploss
        assert abs(cmp - float(g[f"compare{k}"])) <= 1e-5 * cmp
        np.testing.assert_allclose(tr.last_logits.numpy(), g[f"logits{k}"], rtol=1e-5, atol=1e-5)
        ps = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
        np.testing.assert_allclose(ps[:, 1], g[f"param_stats{k}"][:, 1], rtol=1e-9)
    assert not any("_lns_" in n for n in g["grad_names0"])


def test_vlm_joint_oracle_two_steps_match_reference():
    """Joint VLM (train_NWP.py, sequential=False, T = 161), two full training steps at
    d=256, L=1, B=4 (vlm_joint_tiny.npz): draws, initial weights, logits, losses."""
    from oracle import vlm_oracle as VO
    g = _fix("vlm_joint_tiny.npz")
    tr = VO.OracleVlmJointTrainer(B=4, L=1)
    assert [n for n, _ in tr.model.named_parameters()] == list(g["param_names"])
    st = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
    np.testing.assert_array_equal(st, g["init_stats"])
    for k in range(2):
        drawn = tr.sampler.get_batch(tr.B)
        np.testing.assert_array_equal(np.asarray(drawn[0]), g[f"xt{k}"])
        np.testing.assert_array_equal(np.asarray(drawn[3]), g[f"i_leaves{k}"])
        ploss, loss, cmp = tr.step(batch=drawn)
        assert abs(ploss - float(g[f"ploss{k}"])) <= 1e-6 * ploss
        assert abs(cmp - float(g[f"compare{k}"])) <= 1e-5 * cmp
        np.testing.assert_allclose(tr.last_logits.numpy(), g[f"logits{k}"], rtol=1e-5, atol=1e-5)
        ps = np.array([[p.double().sum().item(), (p.double() ** 2).sum().item()] for p in tr.model.parameters()])
        np.testing.assert_allclose(ps, g[f"param_stats{k}"], rtol=1e-6, atol=1e-9)


def test_oracle_guided_targets_match_reference():
    """The oracle's BP_DNS / BP_CLS message restatement, assembled as guided_info
    (data_random_GHM.py:526-592), equals the reference sampler's guided targets of
    cdm_guided_tiny.npz (z stored as float32 there; the reference ran BP on the f64
    draw, hence 1e-5 relative).  Includes the root's aliased hd (= bu) target."""
    f = np.load(os.path.join(GOLDEN, "cdm_guided_tiny.npz"))
    s = CO.CdmSamplerOracle([4, 4], [3, 3], [0.2, 0.2])
    for k in range(int(f["nsteps"])):
        tt, it = CO.cdm_guided_targets(s.t_trans, s.i_trans, f[f"t_leaves{k}"].astype(np.int64),
                                       f[f"z{k}"].astype(np.float64), 1.0)
        assert len(tt) == 4 and len(it) == 9
        for j, g in enumerate(tt):
            want = f[f"t_guide{k}_{j}"]
            assert g.shape == want.shape
            assert np.abs(g.numpy() - want).max() <= 1e-5 * np.abs(want).max(), ("text", k, j)
        for j, g in enumerate(it):
            want = f[f"i_guide{k}_{j}"]
            assert g.shape == want.shape, (j, g.shape, want.shape)
            assert np.abs(g.numpy() - want).max() <= 1e-5 * np.abs(want).max() + 1e-6, ("image", k, j)


def test_sguided_flags_and_blocks_match_reference_layout():
    """Guided sequential CDM (eg_sdns.sh, model.py:372, :407-416, :448-527 with
    n_guided_layers [1, 4], L = 9): every layer image-guided; text-guided at
    counter 0 and n_i - 1 = 3, their blocks (index_i = 0, 10) on the conditioning
    token (index 81) against the CLIP feature ("c"); index_q starts at n_t V = 10
    and index_u at 2 n_t V = 20 (model.py:455-457)."""
    from ghmclip import ConditionalDenoiseEncoderTransformer
    from ghmclip.models.cdm import cdm_guide_blocks
    m = ConditionalDenoiseEncoderTransformer(82, 81, 10, 128, 9, [1, 4], 4, 512, sequential=True, guide=True)
    assert m.i_guided_layer_flag == [True] * 9
    assert m.t_guided_layer_flag == [True, False, False, True] + [False] * 5
    blocks = cdm_guide_blocks(m, (4, 3), (4, 3), 10)
    assert [b for b in blocks[0] if b[0] == "c"] == [("c", 81, 1, 0, 0, 1)]
    assert [b for b in blocks[3] if b[0] == "c"] == [("c", 81, 1, 10, 0, 1)]
    assert sum(b[0] == "c" for v in blocks.values() for b in v) == 2
    # downward layers k = 0..4: h at k V, q at (n_t + k) V (the root's q plane is bu)
    assert [[b[3] for b in blocks[k] if b[0] == "i"] for k in range(5)] == [[0, 10], [10, 20], [20, 30],
                                                                            [30, 40], [40, 50]]
    # upward layers: h, q one block back, u from 2 n_t V = 20 upwards
    assert [[b[3] for b in blocks[k] if b[0] == "i"] for k in range(5, 9)] == [[40, 50, 20], [30, 40, 30],
                                                                               [20, 30, 40], [10, 20, 50]]


@pytest.mark.parametrize("kind", ["cdm", "vlm", "clip"])
def test_cls_posteriors_use_each_trees_root_prior(kind):
    """The BP_CLS posteriors a sampler returns use the tree's own root prior p_ys[0]
    (text) / p_ys[1] (image), as the reference's GHMTree(p_ys[k]) + BP_CLS
    (data_random_GHM.py:213, 665-666, 860-861, 908-909): with a non-uniform prior
    the posterior is the uniform-prior one reweighted by p_y and renormalised, on
    the same draws (the roots are drawn uniformly either way)."""
    from ghmclip import ClipSampler, ConditionalDenoiseSampler, NextWordPredictSampler, seed_everything
    rng = np.random.RandomState(3)
    pt, pi = rng.dirichlet(np.ones(10)), rng.dirichlet(np.ones(10))

    def draw(p_ys):
        seed_everything(11)
        if kind == "cdm":
            s = ConditionalDenoiseSampler([3, 3], [3, 3], p_ys, [0.2, 0.2], sigma=1)
            (_, _, _, tpp), _ = s.get_batch(6)
            return [(tpp, 0)]
        if kind == "vlm":
            s = NextWordPredictSampler([3, 3], [3, 3], p_ys, [0.2, 0.2])
            _, (_, _, _, ipp) = s.get_batch(6)
            return [(ipp.T, 1)]
        s = ClipSampler([3, 3], [3, 3], p_ys, [0.2, 0.2], K=2)
        (_, _, _, tp), (_, _, _, ip) = s.get_batch("cpu", 6, guide=True)
        return [(tp, 0), (ip, 1)]

    uni = draw([P_Y, P_Y])
    non = draw([pt, pi])
    for (u, k), (n, _) in zip(uni, non):
        u, n = np.asarray(u, np.float64), np.asarray(n, np.float64)
        prior = (pt, pi)[k].reshape(-1, 1) if u.shape[0] == 10 else (pt, pi)[k].reshape(1, -1)
        w = u * prior
        axis = 0 if u.shape[0] == 10 else 1
        np.testing.assert_allclose(n, w / w.sum(axis=axis, keepdims=True), rtol=1e-9, atol=1e-12)
