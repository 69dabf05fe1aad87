"""Diagnostic: the guided CLIP 3001-step run (exp_clip_guidedTF.sh) at a given
precision against the reference's CPU run and the spread of the reference's own
reruns (2 threads; AVX2 dispatch), steps 0-1100.
Usage: python tools/guided_spread.py f32|x3"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import GOLDEN, curve_bound  # noqa: E402
from test_gpu_parity import _guided_trainer, _run  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "x3"
ref = np.load(os.path.join(GOLDEN, "clip_guided_curve3001.npz"))["loss_history"].astype(np.float64)
alts = [np.load(os.path.join(GOLDEN, f"clip_guided_curve3001_{k}.npz"))["loss_history"] for k in ("t2", "avx2")]
sampler, tr = _guided_trainer(5, 128, prec)
hist = _run(sampler, tr, 128, 3001, graph_after=3).astype(np.float64)
rel = np.abs(hist - ref) / np.abs(ref)
bound, window, spread = curve_bound(ref, alts)
n2 = len(bound)
over = np.nonzero(rel[:n2] > bound)[0]
print(f"{prec}: final risk {hist[-100:].mean():.7f} vs {ref[-100:].mean():.7f}; rel |dloss| max {rel.max():.2e} "
      f"(step {rel.argmax()}), steps 0-{n2 - 1}: max {rel[:n2].max():.2e} vs spread max {spread.max():.2e}, "
      f"{len(over)} steps over max(1e-4, 2 x spread) (first {over[0] if len(over) else None})")
