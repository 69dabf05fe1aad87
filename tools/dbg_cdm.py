"""Debug: CDM module forward/backward with every native launch synchronised and logged."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-ghm_amd"))
from ghmclip import _native, ConditionalDenoiseEncoderTransformer
log = open(os.path.join(ROOT, "gpurun_out", "dbg_cdm.log"), "w")
_orig = _native.call


def call(name, *args):
    log.write(f"launch {name} {[a if isinstance(a, (int, float)) else '' for a in args]}\n")
    log.flush()
    _orig(name, *args)
    torch.cuda.synchronize()
    log.write("  ok\n")
    log.flush()


_native.call = call
import ghmclip.models.hip_encoder as he  # noqa: E402
import ghmclip.models.cdm as cd  # noqa: E402
he._native.call = call
torch.manual_seed(11)
m = ConditionalDenoiseEncoderTransformer(82, 81, 10, 128, 2, [1, 4], 4, 512, sequential=True)
m.precision = sys.argv[1] if len(sys.argv) > 1 else "f32"
m = m.cuda()
B = 7
z = (torch.randint(0, 10, (B, 81)).float() + torch.randn(B, 81)).cuda()
c = torch.randn(B, 1, 10).cuda().requires_grad_(True)
pred, _ = m(c, z)
log.write(f"pred finite {bool(torch.isfinite(pred).all())}\n")
pred.sum().backward()
torch.cuda.synchronize()
log.write("backward done\n")
log.close()
