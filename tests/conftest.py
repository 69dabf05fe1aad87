"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic (native
sampler, configs, schedule, checkpoint format), C-ABI library load + exports.
`-m gpu` runs on an MI355X and calls the HIP path through the C-ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multimodal-ghm_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def curve_bound(ref, ref_t2, floor=1e-4, factor=2.0):
    """Per-step relative tolerance of a curve against the reference's PyTorch-CPU
    run `ref`: floor, or `factor` x the largest relative disagreement up to that
    step between that run and the reference's own reruns `ref_t2` (one curve or a
    list: another thread count, *_t2.npz; another CPU dispatch of the same code,
    *_avx2.npz) -- the spread of the reference's own arithmetic.  `ref` is cut to
    the reruns' length.  Also returns the self-consistent window: the leading
    steps whose spread stays under `floor`."""
    import numpy as np
    alts = [ref_t2] if np.ndim(ref_t2[0] if len(ref_t2) else 0) == 0 else list(ref_t2)
    n = min(len(a) for a in alts)
    ref = np.asarray(ref, np.float64)[:n]
    dev = np.max([np.abs(ref - np.asarray(a, np.float64)[:n]) / np.abs(ref) for a in alts], axis=0)
    spread = np.maximum.accumulate(dev)
    bound = np.maximum(floor, factor * spread)
    window = int(np.argmax(spread > floor)) if (spread > floor).any() else len(spread)
    return bound, window, spread


def kernel_relu_masks(module):
    """The relu masks the split-bf16 attention kernels used in a module's last
    forward: P > 0 of each layer's saved scores ([L] x bool [N, T, T], on the CPU;
    the backward takes relu's derivative from the same P)."""
    (plan,) = module._plans.values()
    return [(plan.probs_dense(l) > 0).cpu() for l in range(plan.L)]


def masked_relu_oracle(ref, masks, loss):
    """A float64 copy of an oracle module with relu replaced by the given masks
    (OracleCdm.relu_masks), its gradients from loss(model).backward() in float64.
    Checks first that the masks are relu's own up to near-zero scores: they agree
    with the float64 scores' signs everywhere but a handful of entries."""
    import copy

    import torch
    dt = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        r64 = copy.deepcopy(ref).double()
        r64.zero_grad()
        S = []
        orig = torch.einsum

        def capture(eq, *a):
            y = orig(eq, *a)
            if eq == "bid,bjd->bij":
                S.append(y.detach())
            return y
        torch.einsum = capture
        try:
            with torch.no_grad():
                loss(r64)
        finally:
            torch.einsum = orig
        assert len(S) == len(masks)
        for s, m in zip(S, masks):
            assert s.shape == m.shape
            assert int(((s > 0) != m).sum()) <= 16, "kernel masks differ from relu(S > 0) beyond near-zero scores"
        r64.relu_masks = [m.double() for m in masks]
        loss(r64).backward()
    finally:
        torch.set_default_dtype(dt)
    return r64
