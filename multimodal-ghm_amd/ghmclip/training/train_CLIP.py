"""CLIP training on MI355X — drop-in for ``python -m ghmclip.training.train_CLIP``.

Same flags (HfArgumentParser over the same dataclasses), same run-folder naming,
same log line and the same checkpoint.pth keys as the reference
(src/ghmclip/training/train_CLIP.py:17-220), so scripts/experiments/exp_clip_*.sh
and figures/eval-clip-*.py work unchanged.  The hot loop (:139-201) runs as the
fused, HIP-graph-replayed ClipTrainer step with the native sampler overlapped
in a producer thread.  Differences, by design:
  * --device must be a HIP device (there is no CPU path);
  * clip_guide=True computes the BP guide targets on the device from the staged
    leaves (ghm_bp_cls) inside the captured step instead of in the sampler;
  * resume (--init_from=<checkpoint.pth>) actually resumes: weights, AdamW
    moments, step count and loss histories (the reference's resume is broken,
    :126-137);
  * wandb/s3fs are optional (skipped with a warning when not installed);
  * with torchrun (WORLD_SIZE > 1) each rank takes a contiguous slice of the
    within-block index i of the SAME global batch (all ranks run the same
    sampler stream), and gradients are averaged with one RCCL all-reduce —
    identical objective to the single-GPU run.
"""
import os
import sys
import time
from dataclasses import asdict, dataclass, field
from typing import Optional

import numpy as np
import torch

from ..data import ClipSampler
from ..models import AdamW, EncoderTransformer, GuidedClipLoss, get_lr_cosine_schedule, seed_everything  # noqa: F401
from ..utils import ClipModelConfig, DoubleTreeConfig, GenLogger, UtilConfig, logging
from . import distributed
from .clip_trainer import ClipTrainer
from .pipeline import BatchPipeline


@dataclass
class TrainingConfig(UtilConfig, DoubleTreeConfig, ClipModelConfig):
    """CLI configuration for CLIP training on paired GHM trees (train_CLIP.py:17-21)."""
    job_name: Optional[str] = field(default='clip')


def parse(argv=None):
    from transformers import HfArgumentParser
    parser = HfArgumentParser(TrainingConfig)
    if argv is None:
        return parser.parse_args_into_dataclasses()[0]
    return parser.parse_args_into_dataclasses(args=argv)[0]


def load_checkpoint(path, device):
    """checkpoint.pth of train_CLIP / train_sequential_DNS (state dicts, numpy
    histories, numpy scalars) with the weights-only unpickler: numpy arrays and
    scalars are allow-listed, nothing else runs."""
    from numpy._core import multiarray as npm
    allow = [npm._reconstruct, npm.scalar, np.ndarray, np.dtype, type(np.dtype(np.float64)), np.float64]
    with torch.serialization.safe_globals(allow):
        return torch.load(path, map_location=device, weights_only=True)


def run_names(c):
    """Folder naming of train_CLIP.py:43-52 (figure evaluators depend on it)."""
    tree_folder = (f'K{c.K}_L{c.n_ttree_layer}C{c.n_ttree_child}p{int(c.p_ttree_flip*100)}'
                   f'_L{c.n_itree_layer}C{c.n_itree_child}p{int(c.p_itree_flip*100)}sc{int(c.flip_scale*10)}')
    model_name = (f'L{c.clip_tmodel_nlayer}H{c.clip_tmodel_nhead}D{c.clip_tmodel_deb}'
                  f'_L{c.clip_imodel_nlayer}H{c.clip_imodel_nhead}D{c.clip_imodel_deb}')
    model_name = ('GT_' if c.clip_guide else 'TF_') + model_name
    return tree_folder, model_name


def main(argv=None):
    """The CLI entry point: returns loss_history (length total_iters + 1)."""
    return run(parse(argv))["loss_history"]


def run(c, teardown=True):
    """Train with configuration c; returns the histories, the Bayes loss, the
    final CLIP risk (figures/eval-clip-risk.py:29: mean of the last 100
    loss_history entries) and the wall time of the training loop (sampler,
    H2D staging and every step included)."""
    ws, rank, device = distributed.setup()
    if ws == 1:
        print(f"Using GPU: {torch.cuda.get_device_name(0)}", file=sys.stderr if c.raw else sys.stdout)
    if c.batch_size % ws:
        raise ValueError(f"batch_size {c.batch_size} must be divisible by the world size {ws}")

    tree_folder, model_name = run_names(c)
    timestamp = time.strftime('%Y%m%d-%H%M%S', time.localtime())
    directory = os.path.join("./logs", c.job_name, tree_folder, model_name, timestamp)
    raw = c.raw or rank != 0
    logger = GenLogger(directory, c, raw=raw)
    checkpoint_path = os.path.join(directory, 'checkpoint.pth')
    wandb = None
    if not raw:
        try:
            import wandb as _wandb
            wandb = _wandb
            wandb.init(project=c.wandb_project, name=timestamp + '-' + model_name,
                       tags=[c.job_name, tree_folder], dir=c.wandb_path)
            wandb.config.update(asdict(c))
        except ImportError:
            logger.warning("wandb not installed: skipping wandb logging")

    p_y = np.ones(c.variable_type) / c.variable_type
    sampler = ClipSampler([c.n_ttree_layer, c.n_itree_layer], [c.n_ttree_child, c.n_itree_child], [p_y, p_y],
                          [c.p_ttree_flip, c.p_itree_flip], K=c.K, flip_scale=c.flip_scale,
                          variable_type=c.variable_type, translation_invariance=True, seedtree=42)
    Bayes_loss, Bayes_std = sampler.get_Bayes(n_eval=10000)
    logger.info(f'Bayes Loss: {Bayes_loss}, Bayes Std: {Bayes_std}')
    if wandb:
        wandb.log({'Bayes_loss': Bayes_loss, 'Bayes_std': Bayes_std})

    seed_everything(c.seed)
    d_t = c.n_ttree_child ** c.n_ttree_layer
    d_i = c.n_itree_child ** c.n_itree_layer
    mk = lambda T, deb, nl, nh, ng: EncoderTransformer(  # noqa: E731
        n_token=T, num_class=c.variable_type, n_embd=deb, n_layer=nl, n_guided_layer=ng, n_head=nh,
        n_mlp_multiplier=4, activation=c.clip_activation, mlp=True, normalize_attn=c.clip_attennorm,
        layernorm=c.clip_layernorm, guide=c.clip_guide)
    tmodel = mk(d_t, c.clip_tmodel_deb, c.clip_tmodel_nlayer, c.clip_tmodel_nhead, c.n_ttree_layer).to(device)
    imodel = mk(d_i, c.clip_imodel_deb, c.clip_imodel_nlayer, c.clip_imodel_nhead, c.n_itree_layer).to(device)
    optimizer = AdamW(params=list(tmodel.parameters()) + list(imodel.parameters()), lr=None)

    total = c.total_iters + 1
    ploss_history = np.zeros(total)
    loss_history = np.zeros(total)
    start = 0
    if c.init_from != 'scratch':
        ck = load_checkpoint(c.init_from, device)
        tmodel.load_state_dict(ck['tmodel_state_dict'])
        imodel.load_state_dict(ck['imodel_state_dict'])
        optimizer.load_state_dict(ck['optimizer_state_dict'])
        # eval-interval saves record the last completed step, the final save total_iters+1
        start = min(int(ck['iter']) + 1, total)
        loss_history[:start] = ck['loss_history'][:start]
        ploss_history[:start] = ck['ploss_history'][:start]
    sched = [get_lr_cosine_schedule(i, c.lr_max, c.lr_min, c.warmup_iters, c.total_iters) for i in range(start, total)]
    B_local = c.batch_size // ws
    trainer = ClipTrainer(tmodel, imodel, c.K, B_local, sched, max_norm=c.max_norm, device=device, t_offset=start,
                          penalty=c.penalty,
                          guide_trans=sampler.device_templates("guided CLIP (--clip_guide=True)") if c.clip_guide
                          else None)
    if start:
        trainer.load_optimizer_state(optimizer)

    # sampler: the producer owns numpy's global MT stream from here on
    sampler.native.pull_numpy_state()
    if start:  # replay the consumed draws on resume
        tmp_t = np.empty((c.batch_size * (c.K + 1), d_t), np.uint8)
        tmp_i = np.empty((c.batch_size * (c.K + 1), d_i), np.uint8)
        for _ in range(start):
            sampler.native.next_into(c.batch_size, tmp_t, tmp_i)
    row_slice = (c.batch_size, rank, ws) if ws > 1 else None
    pipe = BatchPipeline(sampler.native, c.batch_size, n_slots=3, row_slice=row_slice)

    def save(iter_num):
        trainer.fill_optimizer_state(optimizer)
        torch.save({'tmodel_state_dict': tmodel.state_dict(), 'imodel_state_dict': imodel.state_dict(),
                    'optimizer_state_dict': optimizer.state_dict(), 'iter': iter_num,
                    'loss_history': loss_history, 'ploss_history': ploss_history, 'bayes': Bayes_loss},
                   checkpoint_path)

    def sync_hist(upto):
        h = trainer.loss_history(upto - start)
        ph = trainer.ploss_history(upto - start)  # == h without guidance
        h, ph = distributed.mean_histories([h, ph], device)  # every rank
        loss_history[start:upto] = h
        ploss_history[start:upto] = ph

    def guided_penalty(i):
        """GuidedClipLoss's second output at step i: loss3.mean() / penalty."""
        return (ploss_history[i] - loss_history[i]) / c.penalty if c.clip_guide else 0.0

    curr_time = time.time()
    lr = sched[0]
    loop_t0 = time.perf_counter()
    try:
        for iter_num in range(start, total):
            pipe.next_into(trainer)
            trainer.step()
            if iter_num == start + 1:
                trainer.capture()
            lr = sched[iter_num - start]
            if iter_num > 0 and iter_num % c.log_interval == 0:
                sync_hist(iter_num + 1)
                finish_time = time.time()
                logger.info((f'Iter: {iter_num}, '
                             f'Penalty train loss: {np.mean(ploss_history[iter_num//2:iter_num]):.4f}, '
                             f'Train loss: {np.mean(loss_history[iter_num//2:iter_num]):.4f}, '
                             f'Guided penalty: [{guided_penalty(iter_num):.4f}],'
                             f'Bayes: {Bayes_loss:.4f}, '
                             f'LR: {lr:.6f}, '
                             f'Time: {(finish_time - curr_time):.2f}s'))
                if wandb:
                    wandb.log({'train_loss': loss_history[iter_num], 'penalty_train_loss': ploss_history[iter_num],
                               'lr': lr, 'Bayes_loss': Bayes_loss, 'Bayes_std': Bayes_std, 'iter': iter_num})
            if iter_num % c.eval_interval == 0:
                sync_hist(iter_num + 1)  # a collective: every rank, not only the saving one
                if not raw:
                    save(iter_num)
    finally:
        pipe.close()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    loop_s = time.perf_counter() - loop_t0
    sync_hist(total)
    if not raw:
        save(total)
    logging.shutdown()
    if c.S3_upload and rank == 0:
        import s3fs
        s3fs.S3FileSystem().put(directory, c.S3_bucket_name + f'/GHM/{c.job_name}/{tree_folder}/{model_name}/{timestamp}',
                                recursive=True)
    if teardown:
        distributed.teardown()
    return {"loss_history": loss_history, "ploss_history": ploss_history, "bayes": Bayes_loss,
            "final_risk": float(np.mean(loss_history[-100:])), "loop_seconds": loop_s, "steps": total - start,
            "world_size": ws, "batch_size": c.batch_size}


if __name__ == "__main__":
    main(sys.argv[1:])
