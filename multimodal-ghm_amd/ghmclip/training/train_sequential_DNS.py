"""Sequential conditional-denoising (CDM) training on MI355X — drop-in for
``python -m ghmclip.training.train_sequential_DNS`` (BASELINE config 4,
scripts/experiments/exp_cdm_{standard,shallow}TF.sh).

Same flags, run-folder naming, CLIP-checkpoint discovery, log line and
checkpoint.pth keys as the reference (src/ghmclip/training/train_sequential_DNS.py:
19-211).  The hot loop (:141-168) runs as the fused, HIP-graph-replayed CdmTrainer
step: frozen CLIP text encoder, denoiser forward/backward, loss, Compare against
the exact BP posterior (computed on the device), clip and AdamW; the native
sampler runs in a producer thread.  Differences, by design:
  * --device must be a HIP device;
  * --guide=True (scripts/examples/eg_sdns.sh) computes the image tree's BP guide
    targets on the device and adds the guided penalties (text blocks against the
    frozen CLIP feature, :145) inside the fused step;
  * the CLIP checkpoint is read with the weights-only unpickler;
  * wandb/s3fs are optional (skipped with a warning when not installed);
  * with torchrun (WORLD_SIZE > 1) each rank takes a contiguous 1/world of the
    samples of the SAME global batch and gradients are averaged with one RCCL
    all-reduce (the loss is a mean over samples).
"""
import os
import sys
import time
from dataclasses import asdict, dataclass, field
from typing import Optional

import numpy as np
import torch

from ..data import ConditionalDenoiseSampler
from ..models import (AdamW, ConditionalDenoiseEncoderTransformer, ConditionalGuidedLsLoss, EncoderTransformer,
                      get_lr_cosine_schedule, seed_everything)
from ..utils import DoubleTreeConfig, GenLogger, ModelConfig, UtilConfig, logging
from . import distributed
from .cdm_trainer import CdmTrainer
from .pipeline import CdmBatchPipeline
from .train_CLIP import load_checkpoint


@dataclass
class TrainingConfig(UtilConfig, DoubleTreeConfig, ModelConfig):
    """CLI configuration for sequential conditional denoising (train_sequential_DNS.py:19-24)."""
    clip_feature: Optional[str] = field(default='GT')
    job_name: Optional[str] = field(default='Sequential_CDNS')


def parse(argv=None):
    from transformers import HfArgumentParser
    parser = HfArgumentParser(TrainingConfig)
    if argv is None:
        return parser.parse_args_into_dataclasses()[0]
    return parser.parse_args_into_dataclasses(args=argv)[0]


def run_names(c):
    """Folder naming of train_sequential_DNS.py:43-55."""
    tree_folder = (f'K{c.K}_L{c.n_ttree_layer}C{c.n_ttree_child}p{int(c.p_ttree_flip*100)}'
                   f'_L{c.n_itree_layer}C{c.n_itree_child}p{int(c.p_itree_flip*100)}sc{int(c.flip_scale*10)}')
    model_name = f'L{c.n_model_layer}H{c.n_head}D{c.d_eb}'
    if c.guide:
        model_name = 'GT_' + model_name
    elif c.n_model_layer == 1:
        model_name = 'ShT_' + model_name
    else:
        model_name = 'StT_' + model_name
    return tree_folder, model_name


def find_clip_checkpoint(tree_folder, clip_feature, root="logs"):
    """CLIP checkpoint discovery of train_sequential_DNS.py:99-111: the first
    run folder under logs/CLIP/<tree_folder> whose name matches the feature kind
    (GT: guided; TF: standard 5-layer), then its first timestamp folder."""
    clip_path = os.path.join(root, "CLIP", tree_folder)
    for folder in os.listdir(clip_path):
        if "GT" in folder and clip_feature == "GT":
            clip_path = os.path.join(clip_path, folder)
            break
        elif "TF" in folder and "L5" in folder and clip_feature == "TF":
            clip_path = os.path.join(clip_path, folder)
            break
    clip_path = os.path.join(clip_path, os.listdir(clip_path)[0])
    return os.path.join(clip_path, "checkpoint.pth")


def main(argv=None):
    c = parse(argv)
    ws, rank, device = distributed.setup()
    if ws == 1:
        print(f"Using GPU: {torch.cuda.get_device_name(0)}")
    if c.batch_size % ws:
        raise ValueError(f"batch_size {c.batch_size} must be divisible by the world size {ws}")

    d_tmodel = c.n_ttree_child ** c.n_ttree_layer
    d_model = c.n_itree_child ** c.n_itree_layer + 1
    d_i_model = d_model - 1
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
            wandb.init(project=c.wandb_project, name=timestamp + '-' + model_name, tags=[c.job_name, tree_folder],
                       dir=c.wandb_path)
            wandb.config.update(asdict(c))
        except ImportError:
            logger.warning("wandb not installed: skipping wandb logging")

    seed_everything(c.seed)  # :62
    p_y = np.ones(c.variable_type) / c.variable_type
    sampler = ConditionalDenoiseSampler([c.n_ttree_layer, c.n_itree_layer], [c.n_ttree_child, c.n_itree_child],
                                        [p_y, p_y], [c.p_ttree_flip, c.p_itree_flip], sigma=c.sigma,
                                        flip_scale=c.flip_scale, variable_type=c.variable_type,
                                        translation_invariance=True, seedtree=42)
    Bayes_loss, Bayes_std = sampler.get_Bayes(n_eval=10000)
    logger.info(f'Bayes Loss: {Bayes_loss}, Bayes Std: {Bayes_std}')
    if wandb:
        wandb.log({'Bayes_loss': Bayes_loss, 'Bayes_std': Bayes_std})

    # frozen CLIP text encoder (:84-111), then the denoiser (:113-127): same RNG order
    clip_text_model = EncoderTransformer(n_token=d_tmodel, num_class=c.variable_type, n_embd=128, n_layer=5,
                                         n_head=4, n_mlp_multiplier=4, activation="softmax", mlp=True,
                                         normalize_attn=True, layernorm=True, maxnorm=False, guide=False)
    ck = load_checkpoint(find_clip_checkpoint(tree_folder, c.clip_feature), device)
    clip_text_model.load_state_dict(ck['tmodel_state_dict'])
    clip_text_model = clip_text_model.to(device)
    model = ConditionalDenoiseEncoderTransformer(n_token=d_model, n_i_token=d_i_model, num_class=c.variable_type,
                                                 n_embd=c.d_eb, n_layer=c.n_model_layer,
                                                 n_guided_layers=[1, c.n_itree_layer], n_head=c.n_head,
                                                 n_mlp_hidden=4 * c.d_eb, activation="softmax", mlp=True,
                                                 normalize_attn=c.normalize_attn, layernorm=c.layernorm,
                                                 maxnorm=False, sequential=True, guide=c.guide).to(device)
    loss = ConditionalGuidedLsLoss(penalty=c.penalty, guide=c.guide)
    optimizer = AdamW(params=model.parameters(), lr=None)
    ploss_history = np.zeros(c.total_iters)
    loss_history = np.zeros(c.total_iters)
    compare_history = np.zeros(c.total_iters)
    t_offset = 0
    if c.init_from != 'scratch':  # :132-138 (the reference restarts the loop at iteration 0)
        ckm = load_checkpoint(c.init_from, device)
        model.load_state_dict(ckm['model_state_dict'])
        optimizer.load_state_dict(ckm['optimizer_state_dict'])
        st = next(iter(optimizer.state.values()), None)
        t_offset = int(st['t']) if st else 0  # AdamW's step count continues (optimizer.py:58-66)

    sched = [get_lr_cosine_schedule(i, c.lr_max, c.lr_min, c.warmup_iters, c.total_iters)
             for i in range(c.total_iters)]
    trainer = CdmTrainer(model, clip_text_model, c.batch_size // ws,
                         sched, *sampler.device_templates("the CDM trainer (BP_DNS on the device)"),
                         sigma=c.sigma, max_norm=c.max_norm, device=device, t_offset=t_offset,
                         penalty=c.penalty)
    if t_offset:
        trainer.load_optimizer_state(optimizer)
    sampler.native.pull_numpy_state()  # the producer owns numpy's MT stream from here on
    pipe = CdmBatchPipeline(sampler.native, c.batch_size, c.sigma, n_slots=3,
                            row_slice=(rank, ws) if ws > 1 else None)

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
                    'bayes': Bayes_loss}, checkpoint_path)

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
                pen = distributed.mean_histories([trainer.penalty_groups()], device)[0]  # (loss2, 4, 5, 3)
                finish_time = time.time()
                h = iter_num // 2
                logger.info(f'Iter: {iter_num},Penalty train loss: {np.mean(ploss_history[h:iter_num]):.4f}, '
                            f'Penalty: [{pen[0]:.2f},{pen[1]:.2f},{pen[2]:.2f},{pen[3]:.2f}],  '
                            f'Train loss: {np.mean(loss_history[h:iter_num]):.4f}, '
                            f'Compare: {np.mean(compare_history[h:iter_num]):.4f},  Bayes:{Bayes_loss:.4f}, '
                            f'LR: {lr:.6f}, Time: {(finish_time - curr_time):.2f}s')
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
