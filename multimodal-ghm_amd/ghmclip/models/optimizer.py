"""Optimizer API of the reference (src/ghmclip/models/optimizer.py) on the HIP path.

``AdamW`` keeps the reference's update order — bias correction folded into the
learning rate, eps added to sqrt(v), weight decay applied AFTER the Adam step to
the already-updated weights, on every parameter (optimizer.py:46-75) — and runs
it in the fused native kernel ``ghm_adamw``.  State keys per parameter are the
reference's ('t', 'm', 'v'), so optimizer.state_dict() round-trips.
"""
import ctypes
from collections.abc import Callable
from typing import Optional

import numpy as np
import torch

from .. import _native
from .hip_encoder import require_hip

__all__ = ["AdamW", "get_lr_cosine_schedule"]


def adam_consts(betas, eps):
    """The fp32 scalars torch would use for `beta*m + (1-beta)*g` etc."""
    b1, b2 = betas
    return (float(np.float32(b1)), float(np.float32(1 - b1)), float(np.float32(b2)),
            float(np.float32(1 - b2)), float(np.float32(eps)))


def adam_lr_t(lr, t, betas):
    """optimizer.py:66 — lr * sqrt(1 - beta2**t) / (1 - beta1**t), in double."""
    b1, b2 = betas
    return lr * (1 - b2 ** t) ** 0.5 / (1 - b1 ** t)


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=None, weight_decay=0.001, betas=(0.9, 0.999), eps=1e-8, **kwargs):
        defaults = dict(lr=lr, weight_decay=weight_decay, betas=betas, eps=eps)
        super().__init__(params, defaults)

    def set_lr(self, lr):
        for group in self.param_groups:
            group["lr"] = lr

    @torch.no_grad()
    def step(self, closure: Optional[Callable] = None):
        loss = None if closure is None else closure()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        work = []  # (param, state, t, consts, hyper row)
        for group in self.param_groups:
            lr, wd = group["lr"], group["weight_decay"]
            consts = adam_consts(group["betas"], group["eps"])
            for p in group["params"]:
                if p.grad is None:
                    continue
                require_hip(p)
                if p.dtype != torch.float32 or not p.is_contiguous() or not p.grad.is_contiguous():
                    raise RuntimeError("HIP AdamW takes contiguous fp32 parameters and grads")
                state = self.state[p]
                if len(state) == 0:
                    state["t"] = 0
                    state["m"] = torch.zeros_like(p.data)
                    state["v"] = torch.zeros_like(p.data)
                t = state["t"] + 1
                work.append((p, state, t, consts, [0.0, 1.0, adam_lr_t(lr, t, group["betas"]), lr * wd]))
        if not work:
            return loss
        # every parameter's step scalars in one pinned buffer and one H2D copy (the
        # caching host allocator keeps a pinned block alive until its copy is done)
        host = torch.tensor([w[4] for w in work], dtype=torch.float32).pin_memory()
        hyper = host.to(work[0][0].device, non_blocking=True)
        for k, (p, state, t, (b1, omb1, b2, omb2, eps), _) in enumerate(work):
            _native.call("ghm_adamw", p.data.data_ptr(), p.grad.data_ptr(), state["m"].data_ptr(),
                         state["v"].data_ptr(), p.numel(), hyper[k].data_ptr(), b1, omb1, b2, omb2, eps, stream)
            state["t"] = t
        return loss


def get_lr_cosine_schedule(t, lr_max, lr_min, warmup_iters, total_iters, **kwargs):
    """optimizer.py:78-85 (warmup + cosine, then lr_min)."""
    if t < warmup_iters:
        return lr_max * t / warmup_iters
    elif t < total_iters:
        return lr_min + 0.5 * (lr_max - lr_min) * (
            1 + np.cos((t - warmup_iters) / (total_iters - warmup_iters) * 3.141592653589793))
    else:
        return lr_min
