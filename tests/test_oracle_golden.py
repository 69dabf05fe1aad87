"""Pin the CPU oracle to the reference: every check here compares oracle/ against
fixtures produced by the real reference (tests/golden/make_golden.py)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ghm_oracle as O


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.mark.parametrize("name", ["sampler_p20.npz", "sampler_p40_b16.npz"])
def test_sampler_bit_exact(name):
    g = _load(name)
    p, B = float(g["p"]), int(g["B"])
    s = O.ClipSamplerOracle([4, 4], [3, 3], [p, p], K=4, seedtree=42)
    np.testing.assert_array_equal(s.t_trans, g["t_transition"])
    np.testing.assert_array_equal(s.i_trans, g["i_transition"])
    O.seed_everything(224)
    for b in range(g["t_leaves"].shape[0]):
        tl, tr, il, ir = s.get_batch(B)
        np.testing.assert_array_equal(tl, g["t_leaves"][b])
        np.testing.assert_array_equal(il, g["i_leaves"][b])
        np.testing.assert_array_equal(tr, g["t_root"][b])
        np.testing.assert_array_equal(ir, g["i_root"][b])


def _check_steps(g, full):
    L, d, B, nsteps, total = [int(x) for x in g["meta"]]
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    act = str(g["activation"]) if "activation" in g else "softmax"
    tr = O.OracleTrainer(p=float(g["p"]), B=B, L=L, d=d, total_iters=total, activation=act)
    keys_t = list(tr.tm.state_dict().keys())
    for k in keys_t:  # initial weights identical => same init RNG order & key layout
        for pref, m in (("t", tr.tm), ("i", tr.im)):
            v = m.state_dict()[k].numpy()
            if full:
                np.testing.assert_array_equal(v, g[f"init.{pref}.{k}"])
            else:
                ck = g[f"init.{pref}.{k}.cks"] if f"init.{pref}.{k}.cks" in g else None
                if ck is not None:
                    np.testing.assert_allclose(v.astype(np.float64).sum(), ck[0], rtol=1e-9, atol=1e-9)
    for it in range(nsteps):
        batch = tr.sampler.get_batch(B)
        np.testing.assert_array_equal(batch[0], g[f"s{it}.t_leaves"])
        np.testing.assert_array_equal(batch[2], g[f"s{it}.i_leaves"])
        # forward pieces
        for p in tr.params:
            p.grad = None
        t = tr.tm(torch.as_tensor(batch[0]))[0]
        i = tr.im(torch.as_tensor(batch[2]))[0]
        np.testing.assert_allclose(t.detach().numpy(), g[f"s{it}.t_emb"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(i.detach().numpy(), g[f"s{it}.i_emb"], rtol=1e-5, atol=1e-5)
        loss = O.clip_loss(t, i, 4, B)
        np.testing.assert_allclose(loss.item(), float(g[f"s{it}.loss"]), rtol=1e-6)
        loss.backward()
        for pref, m in (("t", tr.tm), ("i", tr.im)):
            for k, prm in m.named_parameters():
                gr = prm.grad.numpy()
                key = f"s{it}.grad.{pref}.{k}"
                if key in g:
                    np.testing.assert_allclose(gr, g[key], rtol=1e-4, atol=1e-6)
                else:
                    ck = g[key + ".cks"]
                    np.testing.assert_allclose(gr.astype(np.float64).sum(), ck[0], rtol=1e-3, atol=1e-5)
                    np.testing.assert_allclose((gr.astype(np.float64) ** 2).sum(), ck[1], rtol=1e-4)
        norm = torch.nn.utils.clip_grad_norm_(tr.params, 1.0, norm_type=2)
        np.testing.assert_allclose(norm.item(), float(g[f"s{it}.total_norm"]), rtol=1e-5)
        lr = O.lr_cosine(tr.it, *tr.sched)
        assert lr == float(g[f"s{it}.lr"])
        tr.opt.set_lr(lr)
        tr.opt.step()
        tr.it += 1
        for pref, m in (("t", tr.tm), ("i", tr.im)):
            for k, v in m.state_dict().items():
                key = f"s{it}.post.{pref}.{k}"
                if key in g:
                    np.testing.assert_allclose(v.numpy(), g[key], rtol=1e-5, atol=1e-7)
                else:
                    ck = g[key + ".cks"]
                    np.testing.assert_allclose((v.numpy().astype(np.float64) ** 2).sum(), ck[1], rtol=1e-6)


def test_tiny_training_steps():
    _check_steps(_load("clip_tiny.npz"), full=True)


def test_d128_training_steps():
    _check_steps(_load("clip_d128.npz"), full=False)


@pytest.mark.parametrize("d", [64, 256])
def test_other_width_training_steps(d):
    """n_embd = 64 (the reference CLI's default clip_{t,i}model_deb,
    utils/config.py:58-59) and 256: the widths the GEMM encoder path runs."""
    _check_steps(_load(f"clip_d{d}.npz"), full=False)


@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_d128_training_steps_attention_activation(act):
    """train_CLIP --clip_activation=relu|gelu (model.py:121-130, :781), pinned to
    the reference's own run (make_golden_act.py)."""
    _check_steps(_load(f"clip_d128_{act}.npz"), full=False)


@pytest.mark.parametrize("p", [0.2, 0.4])
def test_bayes_matches_published(p):
    with open(os.path.join(GOLDEN, "bayes.json")) as f:
        d = json.load(f)
    idx = [round(x, 2) for x in d["p_flip"]].index(p)
    s = O.ClipSamplerOracle([4, 4], [3, 3], [p, p], K=4, seedtree=42)
    bayes, _ = O.clip_bayes(s, n_eval=10000)
    np.testing.assert_allclose(bayes, d["Bayes"][idx], rtol=1e-12)


@pytest.mark.slow
def test_default_curve_prefix():
    """Oracle reproduces the reference's default-config loss curve (first 10 steps)."""
    path = os.path.join(GOLDEN, "clip_default_curve.npz")
    if not os.path.exists(path):
        pytest.skip("curve fixture not generated")
    g = np.load(path)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    tr = O.OracleTrainer()
    for it in range(3):
        loss, _ = tr.step()
        assert abs(loss - g["loss_history"][it]) < 1e-5


# ----------------------------------------------------------------------------
# guided CLIP (clip_guide=True): BP guide targets and the Frobenius penalty
# ----------------------------------------------------------------------------
def test_guide_bp_messages_match_reference():
    """bp_cls_messages == GHMTree.BP_CLS + guided_info (data_random_GHM.py:185-221,
    526-549) on the reference's own draws, and the posteriors match BP_CLS."""
    g = _load("guide_bp.npz")
    for pref in ("t", "i"):
        trans = g[f"{pref}_transition"]
        leaves = g[f"{pref}_leaves"].astype(np.int64)
        msgs = O.bp_cls_messages(trans, leaves)
        assert len(msgs) == 4
        for k, m in enumerate(msgs):
            want = g[f"{pref}_msg{k}"]
            assert m.shape == want.shape
            np.testing.assert_allclose(m.astype(np.float32), want, rtol=1e-6, atol=1e-6)
        pp = O.bp_cls_posterior(trans, leaves, np.ones(10) / 10)
        np.testing.assert_allclose(pp, g[f"{pref}_pp"], rtol=1e-10, atol=1e-12)


def test_guided_training_steps():
    """Two guided CLIP steps (exp_clip_guidedTF.sh hyper-parameters, L=5, d=16, B=4)."""
    g = _load("guide_tiny.npz")
    L, d, B, nsteps, total = [int(x) for x in g["meta"]]
    p, penalty, lr_max, lr_min = [float(x) for x in g["hyper"]]
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    tr = O.OracleTrainer(p=p, B=B, L=L, d=d, total_iters=total, lr_max=lr_max, lr_min=lr_min,
                         guide=True, penalty=penalty)
    assert tr.tm.guided_layer_flag == [True, True, True, True, False]
    for pref, m in (("t", tr.tm), ("i", tr.im)):
        for k, v in m.state_dict().items():
            np.testing.assert_array_equal(v.numpy(), g[f"init.{pref}.{k}"])
    for it in range(nsteps):
        batch = tr.sampler.get_batch(B)
        np.testing.assert_array_equal(batch[0], g[f"s{it}.t_leaves"])
        ploss, _ = tr.step(batch=batch)
        np.testing.assert_allclose(tr.last_loss_nop, float(g[f"s{it}.loss_nop"]), rtol=1e-6)
        np.testing.assert_allclose(ploss, float(g[f"s{it}.loss"]), rtol=1e-6)
        np.testing.assert_allclose(tr.last_penalty, float(g[f"s{it}.penalty"]), rtol=1e-5)
        for pref, m in (("t", tr.tm), ("i", tr.im)):
            for k, v in m.state_dict().items():
                np.testing.assert_allclose(v.numpy(), g[f"s{it}.post.{pref}.{k}"], rtol=1e-5, atol=1e-7)


def test_get_activation_names():
    """models/model.py:121-130: softmax, relu and gelu resolve (the HIP kernels
    apply them); any other name raises NotImplementedError, as the reference."""
    from ghmclip.models.model import get_activation
    for a in ("softmax", "relu", "gelu"):
        assert get_activation(a) == a
    with pytest.raises(NotImplementedError):
        get_activation("tanh")
