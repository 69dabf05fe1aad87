"""The data-parallel CLI loop's collective schedule, on CPU (gloo, world size 2).

Every collective of train_CLIP / train_CDNS's loop (the per-step gradient
all-reduce inside trainer.step(), the history all-reduce before each log line,
each checkpoint save and at the end) must be issued by every rank at the same
point: the checkpoint itself is rank-0 only (raw = c.raw or rank != 0), the
history mean before it is not.  Here the HIP trainer and the pinned-memory
pipeline are replaced by CPU fakes that do the same collectives as the real ones
(distributed.allreduce_mean_ of a flat gradient per step), so a mismatched
schedule shows up as a gloo size mismatch or a hang (timeout), and the saved
loss_history must be the mean of the ranks' shard losses.  The real product path
(ClipTrainer + BatchPipeline on a GPU) is tests/test_gpu_dp.py.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeTrainer:
    """Stands in for ClipTrainer / CdmTrainer: one gradient all-reduce per step,
    per-rank shard losses loss(step) = step + 0.25 * rank."""
    N_GRAD = 1000

    def __init__(self, *a, **k):
        import torch.distributed as dist
        self.rank = dist.get_rank()
        self.steps_done = 0
        self.g = torch.zeros(self.N_GRAD)
        self.hist = []

    def step(self):
        from ghmclip.training import distributed
        self.g.fill_(float(self.rank))
        distributed.allreduce_mean_(self.g)
        assert float(self.g[0]) == 0.5, "gradient all-reduce paired with a different collective"
        self.hist.append(self.steps_done + 0.25 * self.rank)
        self.steps_done += 1

    def capture(self):
        pass

    def loss_history(self, upto=None):
        n = self.steps_done if upto is None else upto
        return np.asarray(self.hist[:n], np.float64)

    ploss_history = loss_history
    compare_history = loss_history

    def fill_optimizer_state(self, opt):
        pass

    def load_optimizer_state(self, opt):
        pass


class _FakePipe:
    def __init__(self, *a, **k):
        pass

    def next_into(self, trainer):
        pass

    def close(self):
        pass


def _worker(rank, world, port, tmp, cli, flags, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-ghm_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), GHM_DIST_BACKEND="gloo")
    os.chdir(tmp)
    torch.set_num_threads(1)
    import importlib

    import torch.distributed as dist
    from ghmclip.training import distributed
    mod = importlib.import_module(f"ghmclip.training.{cli}")

    def setup():
        dist.init_process_group("gloo", rank=rank, world_size=world)
        return world, rank, torch.device("cpu")
    distributed.setup = setup
    for name in ("ClipTrainer", "CdmTrainer"):
        if hasattr(mod, name):
            setattr(mod, name, _FakeTrainer)
    for name in ("BatchPipeline", "CdmBatchPipeline"):
        if hasattr(mod, name):
            setattr(mod, name, _FakePipe)
    try:
        out = mod.main(flags)
        hist = out[0] if isinstance(out, tuple) else out
        q.put((rank, np.asarray(hist), None))
    except Exception as e:  # noqa: BLE001 — surfaced in the parent
        q.put((rank, None, repr(e)))


def _run(cli, flags, tmp_path, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), cli, flags, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, h, err = q.get(timeout=240)
            assert err is None, f"rank {r}: {err}"
            res[r] = h
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return res


CLIP_FLAGS = ["--job_name=CLIP", "--n_ttree_layer=2", "--n_itree_layer=2", "--n_ttree_child=3", "--n_itree_child=3",
              "--K=4", "--batch_size=8", "--clip_tmodel_nlayer=1", "--clip_imodel_nlayer=1", "--clip_tmodel_deb=16",
              "--clip_imodel_deb=16", "--total_iters=6", "--raw=False", "--log_interval=2", "--eval_interval=2",
              "--device=cpu"]


def test_clip_cli_dp_collective_schedule(tmp_path):
    """train_CLIP --raw=False --eval_interval=2 under 2 ranks: no mismatched
    collective, the histories are the rank means, and rank 0's checkpoint holds
    them (len == total_iters + 1, the length figures/eval-clip-risk.py reads)."""
    import glob
    sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-ghm_amd")]
    from ghmclip.training.train_CLIP import load_checkpoint
    res = _run("train_CLIP", CLIP_FLAGS, tmp_path)
    want = np.arange(7) + 0.125  # mean over ranks of step + 0.25 * rank
    for r in (0, 1):
        np.testing.assert_allclose(res[r], want, rtol=0, atol=1e-12)
    ck = glob.glob(str(tmp_path / "logs/CLIP/*/*/*/checkpoint.pth"))
    assert len(ck) == 1, ck  # rank 0 only
    d = load_checkpoint(ck[0], "cpu")
    assert d["iter"] == 7
    np.testing.assert_allclose(d["loss_history"], want, atol=1e-12)


CDNS_FLAGS = ["--job_name=CDM", "--n_ttree_layer=2", "--n_itree_layer=2", "--n_ttree_child=3", "--n_itree_child=3",
              "--batch_size=8", "--d_eb=16", "--n_model_layer=1", "--layernorm=True", "--total_iters=6", "--raw=False",
              "--log_interval=2", "--eval_interval=2", "--device=cpu"]


@pytest.mark.parametrize("cli", ["train_CDNS"])
def test_cdm_cli_dp_collective_schedule(tmp_path, cli):
    res = _run(cli, CDNS_FLAGS, tmp_path)
    want = np.arange(6) + 0.125
    for r in (0, 1):
        np.testing.assert_allclose(res[r], want, rtol=0, atol=1e-12)
