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
    run `ref` (8 threads): floor, or `factor` x the largest relative disagreement
    between that run and the reference's own 2-thread run `ref_t2` up to that
    step (the reference's reduction-order spread, committed as *_t2.npz
    fixtures).  Also returns the self-consistent window: the leading steps whose
    spread stays under `floor`."""
    import numpy as np
    ref, ref_t2 = np.asarray(ref, np.float64), np.asarray(ref_t2, np.float64)
    spread = np.maximum.accumulate(np.abs(ref - ref_t2) / np.abs(ref))
    bound = np.maximum(floor, factor * spread)
    window = int(np.argmax(spread > floor)) if (spread > floor).any() else len(spread)
    return bound, window, spread
