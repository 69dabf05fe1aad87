"""Sequential next-word-prediction (VLM) training on MI355X — drop-in for
``python -m ghmclip.training.train_sequential_NWP`` (BASELINE config 5,
scripts/experiments/exp_vlm_{standard,shallow}TF.sh).

Same flags, run-folder naming, CLIP-checkpoint discovery (the IMAGE tower,
``imodel_state_dict``), RNG order, log line and checkpoint.pth keys as the
reference (src/ghmclip/training/train_sequential_NWP.py:17-222).  The hot loop
(:157-185) runs as the fused, HIP-graph-replayed VlmTrainer step: frozen CLIP
image encoder, AutoRegressiveTransformer forward/backward, next-token cross
entropy, KL "Compare" against the exact BP posterior, clip and AdamW; the
native sampler and the host BP posteriors run in a producer thread.
Differences, by design:
  * --device must be a HIP device;
  * --guide=True: the producer thread computes the text BP guide targets on the
    host (bp_nwp_posterior(guide=True)) and stages them with the batch; the image
    guides target the frozen CLIP feature on the device (:165); penalties and
    their gradients run inside the fused step (VlmTrainer guide branch);
  * checkpoints are read with the weights-only unpickler, and the saved 'loss'
    entry is a plain dict (type, penalty, guide) instead of the pickled module;
  * wandb/s3fs are optional (skipped with a warning when not installed);
  * with torchrun (WORLD_SIZE > 1) each rank takes a contiguous 1/world of the
    samples of the SAME global batch and gradients are averaged with one RCCL
    all-reduce (the loss is a mean over samples);
  * init_from resumes AdamW's step count (the reference restarts at iteration 0).
"""
import os
import sys
import time
from dataclasses import asdict, dataclass, field
from typing import Optional

import numpy as np
import torch

from ..data import NextWordPredictSampler
from ..models import (AdamW, AutoRegressiveTransformer, ConditionalGuidedCELoss, EncoderTransformer,
                      get_lr_cosine_schedule, seed_everything)
from ..utils import DoubleTreeConfig, GenLogger, ModelConfig, UtilConfig, logging
from . import distributed
from .pipeline import NwpBatchPipeline
from .train_CLIP import load_checkpoint
from .train_sequential_DNS import find_clip_checkpoint, run_names
from .vlm_trainer import VlmTrainer


@dataclass
class TrainingConfig(UtilConfig, DoubleTreeConfig, ModelConfig):
    """CLI configuration for sequential next-word prediction (train_sequential_NWP.py:17-22)."""
    clip_feature: Optional[str] = field(default='GT')
    job_name: Optional[str] = field(default='Sequential_NWP')


def parse(argv=None):
    from transformers import HfArgumentParser
    parser = HfArgumentParser(TrainingConfig)
    if argv is None:
        return parser.parse_args_into_dataclasses()[0]
    return parser.parse_args_into_dataclasses(args=argv)[0]


def main(argv=None):
    c = parse(argv)
    ws, rank, device = distributed.setup()
    if ws == 1:
        print(f"Using GPU: {torch.cuda.get_device_name(0)}")
    if c.batch_size % ws:
        raise ValueError(f"batch_size {c.batch_size} must be divisible by the world size {ws}")

    d_tmodel = c.n_ttree_child ** c.n_ttree_layer
    d_imodel = c.n_itree_child ** c.n_itree_layer
    d_model = d_tmodel  # :36-38: one image prefix token + T-1 text inputs
    tree_folder, model_name = run_names(c)  # :40-52 (same naming as the CDM script)
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
            wandb.init(project=c.wandb_project, name=timestamp + '-' + model_name, tags=[c.job_name, tree_folder],
                       dir=c.wandb_path)
            wandb.config.update(asdict(c))
        except ImportError:
            logger.warning("wandb not installed: skipping wandb logging")

    p_y = np.ones(c.variable_type) / c.variable_type
    sampler = NextWordPredictSampler([c.n_ttree_layer, c.n_itree_layer], [c.n_ttree_child, c.n_itree_child],
                                     [p_y, p_y], [c.p_ttree_flip, c.p_itree_flip], flip_scale=c.flip_scale,
                                     variable_type=c.variable_type, translation_invariance=True, seedtree=42)
    if not c.raw:  # :78-84 (the reference draws the Bayes batch only when logging)
        Bayes_loss, Bayes_std = sampler.get_Bayes(n_eval=10000)
        Bayes_loss, Bayes_std = float(Bayes_loss), float(Bayes_std)
        logger.info(f'Bayes Loss: {Bayes_loss}, Bayes Std: {Bayes_std}')
        if wandb:
            wandb.log({'Bayes_loss': Bayes_loss, 'Bayes_std': Bayes_std})
    else:
        Bayes_loss, Bayes_std = 0, 0

    # frozen CLIP image encoder (:86-117), then seed_everything and the model (:120-136)
    clip_image_model = EncoderTransformer(n_token=d_imodel, num_class=c.variable_type, n_embd=128, n_layer=5,
                                          n_head=4, n_mlp_multiplier=4, activation=c.activation, mlp=True,
                                          normalize_attn=True, layernorm=True, maxnorm=False, guide=False)
    ck = load_checkpoint(find_clip_checkpoint(tree_folder, c.clip_feature), device)
    clip_image_model.load_state_dict(ck['imodel_state_dict'])
    clip_image_model = clip_image_model.to(device)
    seed_everything(c.seed)
    model = AutoRegressiveTransformer(n_token=d_model, n_i_token=1, num_class=c.variable_type, n_embd=c.d_eb,
                                      n_layer=c.n_model_layer, n_guided_layers=[c.n_ttree_layer, 1], n_head=c.n_head,
                                      n_mlp_hidden=4 * c.d_eb, auto_regressive=True, activation="softmax", mlp=True,
                                      normalize_attn=c.normalize_attn, layernorm=c.layernorm, sequential=True,
                                      guide=c.guide).to(device)
    loss = ConditionalGuidedCELoss(penalty=c.penalty, guide=c.guide)
    optimizer = AdamW(params=model.parameters(), lr=None)
    ploss_history = np.zeros(c.total_iters)
    loss_history = np.zeros(c.total_iters)
    compare_history = np.zeros(c.total_iters)
    t_offset = 0
    if c.init_from != 'scratch':  # :143-149
        ckm = load_checkpoint(c.init_from, device)
        model.load_state_dict(ckm['model_state_dict'])
        optimizer.load_state_dict(ckm['optimizer_state_dict'])
        st = next(iter(optimizer.state.values()), None)
        t_offset = int(st['t']) if st else 0

    sched = [get_lr_cosine_schedule(i, c.lr_max, c.lr_min, c.warmup_iters, c.total_iters)
             for i in range(c.total_iters)]
    trainer = VlmTrainer(model, clip_image_model, c.batch_size // ws, sched, max_norm=c.max_norm, device=device,
                         t_offset=t_offset, penalty=c.penalty)
    if t_offset:
        trainer.load_optimizer_state(optimizer)
    sampler.native.pull_numpy_state()  # the producer owns numpy's MT stream from here on
    pipe = NwpBatchPipeline(sampler, c.batch_size, n_slots=3, row_slice=(rank, ws) if ws > 1 else None,
                            guide=c.guide, image_guide=False)

    def sync_hist(upto):
        h, ph, ch = trainer.loss_history(upto), trainer.ploss_history(upto), trainer.compare_history(upto)
        h, ph, ch = distributed.mean_histories([h, ph, ch], device)  # every rank
        loss_history[:upto] = h
        ploss_history[:upto] = ph  # equals the loss without guidance
        compare_history[:upto] = ch

    def save(iter_num):
        trainer.fill_optimizer_state(optimizer)
        torch.save({'model_state_dict': model.state_dict(), 'optimizer_state_dict': optimizer.state_dict(),
                    'loss': {'type': type(loss).__name__, 'penalty': loss.penalty, 'guide': loss.guide},
                    'iter': iter_num, 'loss_history': loss_history, 'ploss_history': ploss_history,
                    'bayes': Bayes_loss, 'compare': compare_history}, checkpoint_path)

    curr_time = time.time()
    try:
        for iter_num in range(c.total_iters):
            pipe.next_into(trainer)
            trainer.step()
            if iter_num == 1:
                trainer.capture()
            lr = sched[iter_num]
            if iter_num > 0 and iter_num % c.log_interval == 0:
                sync_hist(iter_num + 1)
                finish_time = time.time()
                h = iter_num // 2
                # the last step's output[1:5] (a collective under DP: every rank logs)
                pen = distributed.mean_histories([trainer.guide_penalties()], device)[0] if c.guide \
                    else [0.0, 0.0, 0.0, 0.0]
                logger.info(f"Iter: {iter_num}, "
                            f"Penalty train loss: {np.mean(ploss_history[h:iter_num]):.4f}, "
                            f"Train loss: {np.mean(loss_history[h:iter_num]):.4f}, "
                            f"Penalty: [{pen[0]:.4f}, {pen[1]:.4f}, {pen[2]:.4f}, {pen[3]:.4f}], "
                            f"Compare: {np.mean(compare_history[h:iter_num]):.4f},"
                            f"Bayes: {Bayes_loss:.4f}, "
                            f"LR: {lr:.6f}, "
                            f"Time: {(finish_time - curr_time):.2f}s")
                if wandb:
                    wandb.log({'train_loss': loss_history[iter_num], 'penalty_train_loss': ploss_history[iter_num],
                               'Compare': compare_history[iter_num], 'lr': lr, 'Bayes_loss': Bayes_loss,
                               'Bayes_std': Bayes_std, 'iter': iter_num})
            if iter_num % c.eval_interval == 0:
                sync_hist(iter_num + 1)  # a collective: every rank, not only the saving one
                if not raw:
                    save(iter_num)
    finally:
        pipe.close()
    sync_hist(c.total_iters)
    logging.shutdown()
    if not raw:
        save(c.total_iters)
    if c.S3_upload and rank == 0:
        import s3fs
        s3fs.S3FileSystem().put(directory, c.S3_bucket_name + f'/GHM/{c.job_name}/{tree_folder}/{model_name}/{timestamp}',
                                recursive=True)
    distributed.teardown()
    return loss_history, compare_history


if __name__ == "__main__":
    main(sys.argv[1:])
