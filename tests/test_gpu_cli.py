"""The drop-in CLIs end to end on a HIP device: train_CLIP writes a checkpoint
under logs/CLIP/<tree folder>/TF_L5.../<timestamp>/ (train_CLIP.py:43-60,193-211),
and train_sequential_DNS discovers it as its frozen text encoder
(train_sequential_DNS.py:99-111) and trains the CDM, with the flags of
scripts/experiments/exp_clip_standardTF.sh / exp_cdm_standardTF.sh (shortened)."""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CLIP_FLAGS = ["--job_name=CLIP", "--n_ttree_layer=4", "--n_itree_layer=4", "--n_ttree_child=3", "--n_itree_child=3",
              "--p_ttree_flip=0.2", "--p_itree_flip=0.2", "--flip_scale=1", "--K=4", "--batch_size=8",
              "--variable_type=10", "--clip_tmodel_nlayer=5", "--clip_imodel_nlayer=5", "--clip_tmodel_nhead=4",
              "--clip_imodel_nhead=4", "--clip_tmodel_deb=128", "--clip_imodel_deb=128", "--clip_layernorm=True",
              "--clip_attennorm=True", "--clip_guide=False", "--lr_max=3e-4", "--lr_min=3e-7", "--total_iters=4",
              "--penalty=1e-3", "--raw=False", "--log_interval=2", "--eval_interval=2"]
CDM_FLAGS = ["--clip_feature=TF", "--job_name=CDM", "--model_type=TF", "--n_ttree_layer=4", "--n_itree_layer=4",
             "--n_ttree_child=3", "--n_itree_child=3", "--p_ttree_flip=0.2", "--p_itree_flip=0.2", "--flip_scale=1",
             "--sigma=1", "--batch_size=8", "--variable_type=10", "--d_eb=128", "--n_model_layer=2", "--n_head=4",
             "--layernorm=True", "--normalize_attn=True", "--lr_max=1e-3", "--lr_min=1e-6", "--guide=False",
             "--total_iters=5", "--penalty=0.1", "--raw=False", "--log_interval=2", "--eval_interval=2"]


VLM_FLAGS = ["--job_name=VLM", "--clip_feature=TF", "--model_type=TF", "--n_ttree_layer=4", "--n_itree_layer=4",
             "--n_ttree_child=3", "--n_itree_child=3", "--p_ttree_flip=0.2", "--p_itree_flip=0.2", "--flip_scale=1",
             "--batch_size=8", "--variable_type=10", "--d_eb=256", "--n_model_layer=2", "--n_head=4",
             "--layernorm=True", "--normalize_attn=True", "--lr_max=1e-3", "--lr_min=1e-6", "--guide=False",
             "--total_iters=5", "--penalty=0.001", "--raw=False", "--log_interval=2", "--eval_interval=2"]


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_clip_then_sequential_cdm_and_vlm_cli(tmp_path, monkeypatch):
    """exp_vlm_standardTF.sh flags (shortened): train_sequential_NWP finds the same
    CLIP run and loads its image tower (train_sequential_NWP.py:99-117)."""
    from ghmclip.training import train_CLIP, train_sequential_DNS, train_sequential_NWP
    from ghmclip.training.train_CLIP import load_checkpoint
    monkeypatch.chdir(tmp_path)
    hist = train_CLIP.main(CLIP_FLAGS)
    assert len(hist) == 5 and np.isfinite(hist).all()
    ck_clip = glob.glob("logs/CLIP/K4_L4C3p20_L4C3p20sc10/TF_L5H4D128_L5H4D128/*/checkpoint.pth")
    assert len(ck_clip) == 1
    loss, compare = train_sequential_DNS.main(CDM_FLAGS)
    assert len(loss) == 5 and np.isfinite(loss).all() and np.isfinite(compare).all()
    ck = glob.glob("logs/CDM/K4_L4C3p20_L4C3p20sc10/StT_L2H4D128/*/checkpoint.pth")
    assert len(ck) == 1
    d = load_checkpoint(ck[0], "cpu")
    assert set(d) == {"model_state_dict", "optimizer_state_dict", "loss", "iter", "loss_history", "ploss_history",
                      "bayes"}
    assert d["iter"] == 5
    np.testing.assert_allclose(d["loss_history"], loss)
    assert os.path.exists(os.path.join(os.path.dirname(ck[0]), "training.log"))
    loss, compare = train_sequential_NWP.main(VLM_FLAGS)
    assert len(loss) == 5 and np.isfinite(loss).all() and np.isfinite(compare).all()
    ck = glob.glob("logs/VLM/K4_L4C3p20_L4C3p20sc10/StT_L2H4D256/*/checkpoint.pth")
    assert len(ck) == 1
    d = load_checkpoint(ck[0], "cpu")
    assert set(d) == {"model_state_dict", "optimizer_state_dict", "loss", "iter", "loss_history", "ploss_history",
                      "bayes", "compare"}
    assert d["iter"] == 5
    np.testing.assert_allclose(d["loss_history"], loss)
    np.testing.assert_allclose(d["compare"], compare)


CDNS_FLAGS = ["--job_name=CDM", "--model_type=TF", "--n_ttree_layer=4", "--n_itree_layer=4", "--n_ttree_child=3",
              "--n_itree_child=3", "--p_ttree_flip=0.2", "--p_itree_flip=0.2", "--flip_scale=1", "--sigma=1",
              "--batch_size=8", "--variable_type=10", "--d_eb=128", "--n_model_layer=2", "--n_head=4",
              "--layernorm=True", "--normalize_attn=True", "--lr_max=1e-3", "--lr_min=1e-6", "--guide=False",
              "--total_iters=5", "--penalty=0.1", "--raw=False", "--log_interval=2", "--eval_interval=2"]


def test_joint_cdm_cli(tmp_path, monkeypatch):
    """exp_cdm_jointtrain.sh flags (shortened): train_CDNS writes logs/CDM/<tree>/JT_L2H4D128/."""
    from ghmclip.training import train_CDNS
    from ghmclip.training.train_CLIP import load_checkpoint
    monkeypatch.chdir(tmp_path)
    loss, compare = train_CDNS.main(CDNS_FLAGS)
    assert len(loss) == 5 and np.isfinite(loss).all() and np.isfinite(compare).all()
    ck = glob.glob("logs/CDM/K4_L4C3p20_L4C3p20sc10/JT_L2H4D128/*/checkpoint.pth")
    assert len(ck) == 1
    d = load_checkpoint(ck[0], "cpu")
    assert set(d) == {"model_state_dict", "optimizer_state_dict", "loss", "iter", "loss_history", "ploss_history",
                      "bayes"}
    assert d["iter"] == 5
    np.testing.assert_allclose(d["loss_history"], loss)
    assert d["model_state_dict"]["position_embeddings.weight"].shape == (162, 128)


def test_cdm_and_vlm_cli_layernorm_default(tmp_path, monkeypatch):
    """train_CDNS / train_NWP without --layernorm: ModelConfig's default
    layernorm=False (utils/config.py:46) runs the models without LayerNorm
    (model.py:269-301, 470-498); the unused LayerNorms stay at their initial values
    in the saved state dict."""
    from ghmclip.training import train_CDNS, train_NWP
    from ghmclip.training.train_CLIP import load_checkpoint
    monkeypatch.chdir(tmp_path)
    flags = [f for f in CDNS_FLAGS if not f.startswith("--layernorm")]
    loss, compare = train_CDNS.main(flags)
    assert len(loss) == 5 and np.isfinite(loss).all() and np.isfinite(compare).all()
    ck = glob.glob("logs/CDM/K4_L4C3p20_L4C3p20sc10/JT_L2H4D128/*/checkpoint.pth")
    sd = load_checkpoint(ck[0], "cpu")["model_state_dict"]
    assert torch.equal(sd["_lns_1.0.weight"], torch.ones(128)) and torch.equal(sd["_lns_2.1.bias"], torch.zeros(128))
    loss, compare = train_NWP.main([f for f in NWP_FLAGS if not f.startswith("--layernorm")])
    assert len(loss) == 5 and np.isfinite(loss).all() and np.isfinite(compare).all()


def test_guided_cdm_cli(tmp_path, monkeypatch):
    """exp_cdm_guidedTF.sh flags (shortened, L=9 for the 9 guided layers): train_CDNS
    --guide=True writes logs/CDM/<tree>/GT_L9H4D128/ with the penalised loss in
    ploss_history (above the plain loss)."""
    from ghmclip.training import train_CDNS
    from ghmclip.training.train_CLIP import load_checkpoint
    monkeypatch.chdir(tmp_path)
    flags = [f for f in CDNS_FLAGS if not f.startswith(("--guide", "--n_model_layer", "--lr_max", "--lr_min"))]
    flags += ["--guide=True", "--n_model_layer=9", "--lr_max=1e-2", "--lr_min=1e-5"]
    loss, compare = train_CDNS.main(flags)
    assert len(loss) == 5 and np.isfinite(loss).all() and np.isfinite(compare).all()
    ck = glob.glob("logs/CDM/K4_L4C3p20_L4C3p20sc10/GT_L9H4D128/*/checkpoint.pth")
    assert len(ck) == 1
    d = load_checkpoint(ck[0], "cpu")
    assert d["loss"]["guide"] is True and d["iter"] == 5
    np.testing.assert_allclose(d["loss_history"], loss)
    assert (d["ploss_history"] > d["loss_history"]).all()


NWP_FLAGS = ["--job_name=VLM", "--model_type=TF", "--n_ttree_layer=4", "--n_itree_layer=4", "--n_ttree_child=3",
             "--n_itree_child=3", "--p_ttree_flip=0.2", "--p_itree_flip=0.2", "--flip_scale=1", "--batch_size=8",
             "--variable_type=10", "--d_eb=256", "--n_model_layer=2", "--n_head=4", "--layernorm=True",
             "--normalize_attn=True", "--lr_max=1e-3", "--lr_min=1e-6", "--guide=False", "--total_iters=5",
             "--penalty=0.001", "--raw=False", "--log_interval=2", "--eval_interval=2"]


def test_joint_vlm_cli(tmp_path, monkeypatch):
    """exp_vlm_jointtrain.sh flags (shortened): train_NWP writes logs/VLM/<tree>/JT_L2H4D256/."""
    from ghmclip.training import train_NWP
    from ghmclip.training.train_CLIP import load_checkpoint
    monkeypatch.chdir(tmp_path)
    loss, compare = train_NWP.main(NWP_FLAGS)
    assert len(loss) == 5 and np.isfinite(loss).all() and np.isfinite(compare).all()
    ck = glob.glob("logs/VLM/K4_L4C3p20_L4C3p20sc10/JT_L2H4D256/*/checkpoint.pth")
    assert len(ck) == 1
    d = load_checkpoint(ck[0], "cpu")
    assert set(d) == {"model_state_dict", "optimizer_state_dict", "loss", "iter", "loss_history", "ploss_history",
                      "bayes", "compare"}
    assert d["model_state_dict"]["position_embeddings.weight"].shape == (161, 256)


CLIP_CKPT_KEYS = {"tmodel_state_dict", "imodel_state_dict", "optimizer_state_dict", "iter", "loss_history",
                  "ploss_history", "bayes"}  # /root/reference/src/ghmclip/training/train_CLIP.py:193-211


def test_clip_checkpoint_contract_and_resume(tmp_path, monkeypatch):
    """The CLIP checkpoint dict (train_CLIP.py:193-211): exactly the reference's keys,
    state dicts with the reference's key names, loss_history of length
    total_iters + 1 (what figures/eval-clip-risk.py:29 averages the last 100 of),
    iter = total_iters + 1 after the final save.  Resume (--init_from) from the
    eval-interval save at iter 4 reproduces the uninterrupted run bit for bit
    (weights, AdamW moments and step count, the sampler stream and both histories)."""
    import shutil

    from ghmclip import EncoderTransformer
    from ghmclip.training import train_CLIP
    from ghmclip.training.train_CLIP import load_checkpoint
    flags = [f for f in CLIP_FLAGS if not f.startswith(("--total_iters", "--eval_interval"))]
    flags += ["--total_iters=8", "--eval_interval=4"]
    real_save = torch.save
    snap = str(tmp_path / "ck_iter4.pth")

    def save(obj, path, *a, **k):
        real_save(obj, path, *a, **k)
        if isinstance(obj, dict) and obj.get("iter") == 4:
            shutil.copy(path, snap)
    monkeypatch.setattr(torch, "save", save)
    (tmp_path / "a").mkdir()
    monkeypatch.chdir(tmp_path / "a")
    full = train_CLIP.main(flags)
    ck = glob.glob("logs/CLIP/*/*/*/checkpoint.pth")
    assert len(ck) == 1
    d = load_checkpoint(ck[0], "cpu")
    assert set(d) == CLIP_CKPT_KEYS
    assert d["iter"] == 9 and len(d["loss_history"]) == 9 and len(d["ploss_history"]) == 9
    np.testing.assert_array_equal(d["loss_history"], full)
    ref_keys = set(EncoderTransformer(81, 10, 128, 5).state_dict())
    assert set(d["tmodel_state_dict"]) == ref_keys and set(d["imodel_state_dict"]) == ref_keys
    assert len(d["optimizer_state_dict"]["state"]) == 2 * len(ref_keys)
    assert float(d["loss_history"][-100:].mean()) == float(np.mean(full))  # eval-clip-risk.py:29

    d4 = load_checkpoint(snap, "cpu")
    assert d4["iter"] == 4
    (tmp_path / "b").mkdir()
    monkeypatch.chdir(tmp_path / "b")
    resumed = train_CLIP.main(flags + [f"--init_from={snap}"])
    np.testing.assert_array_equal(resumed, full)
    d2 = load_checkpoint(glob.glob("logs/CLIP/*/*/*/checkpoint.pth")[0], "cpu")
    for k in ("tmodel_state_dict", "imodel_state_dict"):
        for n, v in d[k].items():
            assert torch.equal(v, d2[k][n]), n
    for pid, st in d["optimizer_state_dict"]["state"].items():
        st2 = d2["optimizer_state_dict"]["state"][pid]
        assert st["t"] == st2["t"] and torch.equal(st["m"], st2["m"]) and torch.equal(st["v"], st2["v"])


def test_eg_nwp_nontranslation_invariant_cli(tmp_path, monkeypatch):
    """scripts/examples/eg_nwp.sh (shortened): train_NWP --guide=True
    --translation_invariance=False --p_*_flip=0.4 --raw=True — the per-edge
    GHM trees (native sampler + host BP_NWP / guided targets, pinned by
    tests/test_nonti_host.py) through the guided joint VLM step."""
    from ghmclip.training import train_NWP
    monkeypatch.chdir(tmp_path)
    flags = ["--model_type=TF", "--n_ttree_layer=4", "--n_itree_layer=4", "--n_ttree_child=3", "--n_itree_child=3",
             "--p_ttree_flip=0.4", "--p_itree_flip=0.4", "--flip_scale=1", "--batch_size=8", "--variable_type=10",
             "--d_eb=256", "--n_model_layer=9", "--n_head=4", "--layernorm=True", "--normalize_attn=True",
             "--lr_max=1e-3", "--lr_min=1e-6", "--guide=True", "--translation_invariance=False", "--total_iters=4",
             "--penalty=0.001", "--raw=True", "--log_interval=2"]
    loss, compare = train_NWP.main(flags)
    assert len(loss) == 4 and np.isfinite(loss).all() and np.isfinite(compare).all()


def test_guided_sequential_cdm_cli(tmp_path, monkeypatch, capsys):
    """scripts/examples/eg_sdns.sh (shortened: batch 8, 5 iterations, log every 2):
    train_sequential_DNS --guide=True with the default --clip_feature=GT finds a
    guided CLIP run (train_CLIP --clip_guide=True writes GT_L5...) as its frozen text
    encoder (train_sequential_DNS.py:99-111), trains the guided denoiser and writes
    logs/Sequential_CDNS/<tree>/GT_L9H4D128/ with the penalised loss in
    ploss_history and the four penalty groups in the log line (:160)."""
    from ghmclip.training import train_CLIP, train_sequential_DNS
    from ghmclip.training.train_CLIP import load_checkpoint
    monkeypatch.chdir(tmp_path)
    clip_flags = [f for f in CLIP_FLAGS if not f.startswith(("--p_ttree_flip", "--p_itree_flip", "--clip_guide",
                                                              "--lr_max", "--lr_min"))]
    clip_flags += ["--p_ttree_flip=0.04", "--p_itree_flip=0.04", "--clip_guide=True", "--lr_max=1e-3",
                   "--lr_min=1e-6"]
    train_CLIP.main(clip_flags)
    assert len(glob.glob("logs/CLIP/K4_L4C3p4_L4C3p4sc10/GT_L5H4D128_L5H4D128/*/checkpoint.pth")) == 1
    flags = ["--model_type=TF", "--n_ttree_layer=4", "--n_itree_layer=4", "--n_ttree_child=3", "--n_itree_child=3",
             "--p_ttree_flip=0.04", "--p_itree_flip=0.04", "--flip_scale=1", "--sigma=1", "--batch_size=8",
             "--variable_type=10", "--d_eb=128", "--n_model_layer=9", "--n_head=4", "--layernorm=True",
             "--normalize_attn=True", "--lr_max=3e-4", "--lr_min=3e-7", "--guide=True", "--total_iters=5",
             "--penalty=0.1", "--raw=False", "--log_interval=2", "--eval_interval=2"]
    loss, compare = train_sequential_DNS.main(flags)
    assert len(loss) == 5 and np.isfinite(loss).all() and np.isfinite(compare).all()
    ck = glob.glob("logs/Sequential_CDNS/K4_L4C3p4_L4C3p4sc10/GT_L9H4D128/*/checkpoint.pth")
    assert len(ck) == 1
    d = load_checkpoint(ck[0], "cpu")
    assert d["iter"] == 5
    np.testing.assert_allclose(d["loss_history"], loss)
    assert (d["ploss_history"] > d["loss_history"]).all()
    with open(os.path.join(os.path.dirname(ck[0]), "training.log")) as f:
        lines = [ln for ln in f if "Penalty: [" in ln]
    assert lines and "Penalty: [0.00,0.00,0.00,0.00]" not in lines[-1], lines[-1:]


def test_guided_sequential_vlm_cli(tmp_path, monkeypatch):
    """scripts/examples/eg_snwp.sh with --guide=True (shortened: batch 8, 5
    iterations, log every 2): train_sequential_NWP finds the standard CLIP run
    (--clip_feature=TF) as its frozen image encoder, trains the guided next-word
    model (n_guided_layers = [4, 1]: text BP guides, the CLIP feature as the image
    guide) and writes logs/exp_snwp/<tree>/GT_L9H4D256/ with the penalised loss in
    ploss_history and the four penalty groups in the log line."""
    from ghmclip.training import train_CLIP, train_sequential_NWP
    from ghmclip.training.train_CLIP import load_checkpoint
    monkeypatch.chdir(tmp_path)
    clip_flags = [f for f in CLIP_FLAGS if not f.startswith(("--p_ttree_flip", "--p_itree_flip"))]
    train_CLIP.main(clip_flags + ["--p_ttree_flip=0.02", "--p_itree_flip=0.02"])
    assert len(glob.glob("logs/CLIP/K4_L4C3p2_L4C3p2sc10/TF_L5H4D128_L5H4D128/*/checkpoint.pth")) == 1
    flags = ["--job_name=exp_snwp", "--clip_feature=TF", "--model_type=TF", "--n_ttree_layer=4", "--n_itree_layer=4",
             "--n_ttree_child=3", "--n_itree_child=3", "--p_ttree_flip=0.02", "--p_itree_flip=0.02", "--flip_scale=1",
             "--batch_size=8", "--variable_type=10", "--d_eb=256", "--n_model_layer=9", "--n_head=4",
             "--layernorm=True", "--normalize_attn=True", "--lr_max=1e-3", "--lr_min=1e-6", "--guide=True",
             "--total_iters=5", "--penalty=0.001", "--raw=False", "--log_interval=2", "--eval_interval=2"]
    loss, compare = train_sequential_NWP.main(flags)
    assert len(loss) == 5 and np.isfinite(loss).all() and np.isfinite(compare).all()
    ck = glob.glob("logs/exp_snwp/K4_L4C3p2_L4C3p2sc10/GT_L9H4D256/*/checkpoint.pth")
    assert len(ck) == 1
    d = load_checkpoint(ck[0], "cpu")
    assert d["iter"] == 5 and d["loss"]["guide"] is True
    np.testing.assert_allclose(d["loss_history"], loss)
    assert (d["ploss_history"] > d["loss_history"]).all()
    with open(os.path.join(os.path.dirname(ck[0]), "training.log")) as f:
        lines = [ln for ln in f if "Penalty: [" in ln]
    assert lines and "Penalty: [0.0000, 0.0000, 0.0000, 0.0000]" not in lines[-1], lines[-1:]
