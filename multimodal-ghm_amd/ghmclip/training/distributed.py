"""Process-group plumbing shared by the data-parallel CLIs and trainers.

The reference is single-process (one run per GPU, exp_clip_standardTF.sh:1); the
data-parallel mode is new here and must give the same objective as one GPU:
each rank takes an equal shard of the batch, the loss is a mean over that batch
(model.py:906-907 CLIP, :998 CDM, :1087-1098 VLM), so the full-batch gradient
and loss are the MEAN of the shard values.

Two rules every caller follows:
  * collectives are issued by EVERY rank at the same program points (never inside
    a rank-conditional branch: checkpoint saving and logging are rank-0 only, the
    history all-reduce that precedes them is not);
  * the mean is SUM followed by a 1/world scale, so the same code runs on RCCL
    (backend "nccl") and on gloo (CPU tests; two ranks sharing one GPU), which has
    no ReduceOp.AVG.

Backend: $GHM_DIST_BACKEND (default "nccl" = RCCL over xGMI on ROCm).
"""
import os

import numpy as np
import torch


def world():
    """(world_size, rank) of the torchrun environment (1, 0 without one)."""
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))


def backend():
    return os.environ.get("GHM_DIST_BACKEND", "nccl")


def setup():
    """Initialise the process group when WORLD_SIZE > 1 and pick this rank's HIP
    device.  Returns (world_size, rank, device).  Ranks beyond the visible device
    count share devices round-robin (only meaningful with gloo: RCCL refuses two
    ranks on one GPU)."""
    ws, rank = world()
    if not torch.cuda.is_available():
        raise RuntimeError("ghmclip (MI355X build) needs a HIP device")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1:
        import torch.distributed as dist
        if dist.is_initialized():  # e.g. bench.py's group, reused by train_CLIP.run
            dev = torch.cuda.current_device()
            return ws, rank, torch.device("cuda", dev)
        dev = local % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        device = torch.device("cuda", dev)
        be = backend()
        if be == "nccl":
            dist.init_process_group(be, device_id=device)
        else:
            dist.init_process_group(be)
        return ws, rank, device
    return 1, 0, torch.device("cuda", torch.cuda.current_device())


def teardown():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def is_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def allreduce_mean_(t, group=None):
    """In-place mean over ranks: SUM, then scale by 1/world (gloo has no AVG)."""
    import torch.distributed as dist
    n = dist.get_world_size(group)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    t.mul_(1.0 / n)
    return t


def allreduce_ranges_start(flat, ranges, group=None):
    """Start the mean over ranks of flat[a:b] for each (a, b) of `ranges`, in order
    (the bucketed gradient all-reduce of ClipTrainer.step): one SUM collective per
    bucket with async_op=True, issued by every rank with the same ranges.  Returns
    the pending (work, view, world) triples for allreduce_finish, which waits for
    each and applies the 1/world scale.  Overlap: RCCL enqueues the collective on
    its own stream behind the caller's current (comm) stream and the host returns
    at once; gloo runs it on a background thread and returns at once too, so the
    towers' later launches are issued (and run) while it is in flight in both
    backends.  Each element is the SUM of the ranks' values times 1/world; at world
    2 that sum is one addition, so bucketed == flat bit for bit
    (tests/test_dp_gloo.py); beyond 2 ranks a ring may add an element's terms in an
    order that depends on its chunk, which can change its last bit (the same on
    every rank; the world-4 test bounds it)."""
    import torch.distributed as dist
    n = dist.get_world_size(group)
    return [(dist.all_reduce(flat[a:b], op=dist.ReduceOp.SUM, group=group, async_op=True), flat[a:b], n)
            for a, b in ranges]


def allreduce_finish(pending):
    """Wait for allreduce_ranges_start's collectives (the current stream is ordered
    after each) and scale each bucket by 1/world, on the current stream."""
    for work, view, n in pending:
        work.wait()
        view.mul_(1.0 / n)


def allreduce_ranges_mean_(flat, ranges, group=None):
    """allreduce_mean_ of flat[a:b] for each (a, b) of `ranges`: start + finish."""
    allreduce_finish(allreduce_ranges_start(flat, ranges, group))
    return flat


def mean_histories(arrays, device):
    """Average equal-length float64 host arrays over ranks (every rank calls
    this at the same iteration).  Returns the averaged arrays; identity with one
    rank.  The reduction runs in float64."""
    if not is_on():
        return list(arrays)
    t = torch.from_numpy(np.stack([np.asarray(a, np.float64) for a in arrays]))
    if backend() == "nccl":
        t = t.to(device)
    allreduce_mean_(t)
    return list(t.cpu().numpy())
