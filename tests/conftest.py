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
