"""The CDM and VLM data-parallel PRODUCT paths on one MI355X (BASELINE configs 4
and 5, their multi-GPU part): each CLI's main() under 2 ranks sharing the GPU
over gloo (RCCL refuses two ranks on one device; distributed.py keeps the code
path identical otherwise: SUM + 1/world scale, every collective on every rank)
against the same CLI under 1 rank.

The objective is a sample mean (ConditionalGuidedLsLoss, model.py:989-1041;
ConditionalGuidedCELoss, model.py:1080-1149, in the loops of train_CDNS.py:
124-149 / train_NWP.py:125-149 and the sequential twins): rank r trains on the
contiguous 1/world of every global batch's samples (CdmBatchPipeline /
NwpBatchPipeline row_slice) and the flat gradient is averaged, so rank 0's
loss_history (the rank mean of the shard losses) equals the single-rank run's
up to reduction order (measured: <= 2.4e-7 absolute for the VLM CLIs, <= 2e-7
relative for the CDM CLIs, whose losses are 1e2..1e5).  --raw=False --eval_interval=2 exercises the collective
schedule that deadlocked in round 1 (history syncs before each rank-0 save).

Also the bench line: bench.py --workload cdm --gpus 2 under torch.distributed.run.
"""
import glob
import json
import os
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TREE = ["--n_ttree_layer=4", "--n_itree_layer=4", "--n_ttree_child=3", "--n_itree_child=3", "--p_ttree_flip=0.2",
        "--p_itree_flip=0.2", "--flip_scale=1", "--variable_type=10"]
LOOP = ["--total_iters=6", "--raw=False", "--log_interval=2", "--eval_interval=2"]
CLIP_FLAGS = ["--job_name=CLIP", "--K=4", "--batch_size=8", "--clip_tmodel_nlayer=5", "--clip_imodel_nlayer=5",
              "--clip_tmodel_deb=128", "--clip_imodel_deb=128", "--lr_max=3e-4", "--lr_min=3e-7",
              "--total_iters=2", "--raw=False"] + TREE
CDM = ["--job_name=CDM", "--model_type=TF", "--sigma=1", "--batch_size=8", "--d_eb=128", "--n_head=4",
       "--layernorm=True", "--normalize_attn=True", "--penalty=0.1"] + TREE + LOOP
VLM = ["--job_name=VLM", "--model_type=TF", "--batch_size=8", "--d_eb=256", "--n_head=4", "--layernorm=True",
       "--normalize_attn=True", "--penalty=0.001"] + TREE + LOOP
CASES = {
    # exp_cdm_jointtrain.sh (shortened)
    "cdns": ("train_CDNS", CDM + ["--n_model_layer=2", "--lr_max=1e-3", "--lr_min=1e-6", "--guide=False"]),
    # exp_cdm_guidedTF.sh (shortened; L = 9 for the 9 guided layers)
    "cdns_guided": ("train_CDNS", CDM + ["--n_model_layer=9", "--lr_max=1e-2", "--lr_min=1e-5", "--guide=True"]),
    # exp_cdm_standardTF.sh (shortened): needs the CLIP run's checkpoint
    "seq_dns": ("train_sequential_DNS", CDM + ["--clip_feature=TF", "--n_model_layer=2", "--lr_max=1e-3",
                                                 "--lr_min=1e-6", "--guide=False"]),
    # exp_vlm_jointtrain.sh / exp_vlm_guidedTF.sh (shortened)
    "nwp": ("train_NWP", VLM + ["--n_model_layer=2", "--lr_max=1e-3", "--lr_min=1e-6", "--guide=False"]),
    "nwp_guided": ("train_NWP", VLM + ["--n_model_layer=9", "--lr_max=1e-3", "--lr_min=1e-6", "--guide=True"]),
    # exp_vlm_standardTF.sh (shortened): needs the CLIP run's checkpoint
    "seq_nwp": ("train_sequential_NWP", VLM + ["--clip_feature=TF", "--n_model_layer=2", "--lr_max=1e-3",
                                                "--lr_min=1e-6", "--guide=False"]),
}


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tmp, cli, flags, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-ghm_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), GHM_DIST_BACKEND="gloo")
    os.chdir(tmp)
    try:
        import importlib
        out = importlib.import_module(f"ghmclip.training.{cli}").main(flags)
        q.put((rank, [np.asarray(h) for h in (out if isinstance(out, tuple) else (out,))], None))
    except Exception as e:  # noqa: BLE001 — surfaced in the parent
        q.put((rank, None, repr(e)))


def _run(cli, flags, world, tmp):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, str(tmp), cli, flags, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, h, err = q.get(timeout=150)
            assert err is None, f"{cli} rank {r}/{world}: {err}"
            res[r] = h
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return res


@pytest.fixture(scope="module")
def clip_logs(tmp_path_factory):
    """One short CLIP run whose checkpoint the sequential CLIs discover
    (train_sequential_DNS.py:99-111, train_sequential_NWP.py:99-117)."""
    d = tmp_path_factory.mktemp("clip")
    _run("train_CLIP", CLIP_FLAGS, 1, d)
    assert len(glob.glob(str(d / "logs/CLIP/*/*/*/checkpoint.pth"))) == 1
    return d / "logs"


@pytest.mark.parametrize("case", list(CASES))
def test_cli_dp2_equals_single_rank(case, tmp_path, clip_logs):
    from ghmclip.training.train_CLIP import load_checkpoint
    cli, flags = CASES[case]
    for sub in ("one", "two"):
        (tmp_path / sub).mkdir()
        if cli.startswith("train_sequential"):
            shutil.copytree(clip_logs, tmp_path / sub / "logs")
    one = _run(cli, flags, 1, tmp_path / "one")[0]
    two = _run(cli, flags, 2, tmp_path / "two")
    loss1, loss2 = one[0], two[0][0]
    assert len(loss1) == 6 and np.isfinite(loss1).all()
    for a, b in zip(two[0], two[1]):  # every rank holds the same (averaged) histories
        np.testing.assert_array_equal(a, b)
    dev = [float(np.abs(a - b).max()) for a, b in zip(two[0], one)]
    print(f"{case}: dp2 vs single-rank max |d| per history (loss, compare) = {dev}")
    # 1e-6 relative: the CDM's LS losses run to 1e5 (guided, lr 1e-2), where one
    # float32 ulp of the shard-mean order is ~1e-7 relative (measured <= 2e-7)
    np.testing.assert_allclose(loss2, loss1, rtol=1e-6, atol=1e-6)
    if len(one) > 1:  # Compare (the BP-posterior gap) is a sample mean too
        np.testing.assert_allclose(two[0][1], one[1], rtol=1e-6, atol=1e-6)
    job = "CDM" if "DNS" in cli else "VLM"
    ck = glob.glob(str(tmp_path / f"two/logs/{job}/*/*/*/checkpoint.pth"))
    assert len(ck) == 1, ck  # rank 0 saves, rank 1 is raw
    d = load_checkpoint(ck[0], "cpu")
    assert d["iter"] == 6
    np.testing.assert_array_equal(d["loss_history"], loss2)


def test_bench_cdm_dp2_weak_scaling_line():
    env = dict(os.environ, GHM_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"), "--workload", "cdm", "--gpus", "2",
           "--steps", "4", "--warmup", "3", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and out["value"] > 0
