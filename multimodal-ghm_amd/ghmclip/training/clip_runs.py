"""The reference's CLIP experiment configurations as flag lists, run through the
drop-in CLI code path (train_CLIP.run): the three architectures of
scripts/experiments/exp_clip_{standard,guided,shallow}TF.sh, each swept over the
20 p_flip values 0.02 .. 0.40 (:6) with total_iters = 3000.  The published
result of each run is its final CLIP risk, mean(loss_history[-100:])
(figures/eval-clip-risk.py:29), in figures/data/ghm-data/clip-risk.json.
"""
P_FLIPS = [round(0.02 * k, 2) for k in range(1, 21)]

_COMMON = ["--job_name=CLIP", "--n_ttree_layer=4", "--n_itree_layer=4", "--n_ttree_child=3", "--n_itree_child=3",
           "--flip_scale=1", "--K=4", "--batch_size=128", "--variable_type=10", "--clip_tmodel_nhead=4",
           "--clip_imodel_nhead=4", "--clip_tmodel_deb=128", "--clip_imodel_deb=128", "--clip_layernorm=True",
           "--clip_attennorm=True", "--penalty=1e-3"]

ARCHS = {  # exp_clip_*.sh:15-40
    "Standard TF": ["--clip_tmodel_nlayer=5", "--clip_imodel_nlayer=5", "--clip_guide=False", "--lr_max=3e-4",
                    "--lr_min=3e-7"],
    "Guided TF": ["--clip_tmodel_nlayer=5", "--clip_imodel_nlayer=5", "--clip_guide=True", "--lr_max=1e-3",
                  "--lr_min=1e-6"],
    "Shallow TF": ["--clip_tmodel_nlayer=1", "--clip_imodel_nlayer=1", "--clip_guide=False", "--lr_max=3e-4",
                   "--lr_min=3e-7"],
}


def clip_flags(arch, p_flip, total_iters=3000, raw=True, extra=()):
    """CLI flags of one run of exp_clip_<arch>.sh at p_flip (raw: no checkpoint)."""
    return (_COMMON + ARCHS[arch] + [f"--p_ttree_flip={p_flip}", f"--p_itree_flip={p_flip}",
                                     f"--total_iters={total_iters}", f"--raw={raw}"] + list(extra))


def run_clip(arch, p_flip, total_iters=3000, raw=True, extra=(), teardown=True):
    """One reference run through train_CLIP.run; returns its result dict
    (loss_history, bayes, final_risk, loop_seconds, ...)."""
    from . import train_CLIP
    return train_CLIP.run(train_CLIP.parse(clip_flags(arch, p_flip, total_iters, raw, extra)), teardown=teardown)
