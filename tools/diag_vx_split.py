"""Where GHM_VX_SPLIT's attention forward differs from the unsplit one (diagnostic)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multimodal-ghm_amd"))
from ghmclip import _native  # noqa: E402
from ghmclip.models.vlm import _ptr  # noqa: E402
import ctypes  # noqa: E402

N, D, T, npre = 7, 256, 81, 1
g = torch.Generator().manual_seed(D + T)
qkv = (torch.randn(N, T, 3 * D, generator=g) * 0.5).cuda()
H = torch.randn(N, T, D, generator=g).cuda()
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
dbl = float(os.environ.get("DIAG_DBL", str(1.0 / D)))
H0 = torch.zeros_like(H) if os.environ.get("DIAG_H0") else H
print("dbl", dbl, "H zero" if os.environ.get("DIAG_H0") else "")
res = []
for sp in ("1", "1", "2", "4"):
    os.environ["GHM_VX_SPLIT"] = sp
    Hm = torch.full((N * T, D), float("nan"), device="cuda")
    P = torch.zeros(N, 96, 96, device="cuda")
    _native.call("ghm_attn_ext_fwd_x3", _ptr(qkv), _ptr(H0), _ptr(Hm), _ptr(P), N, T, D, npre, math.sqrt(D), dbl, s)
    torch.cuda.synchronize()
    res.append((Hm.cpu().view(N, T, D), P.cpu()))
for k, sp in ((1, "1 again"), (2, "2"), (3, "4")):
    d = (res[k][0] - res[0][0]).abs()
    nan = torch.isnan(res[k][0])
    print(sp, "Hm max diff", d[~nan].max().item() if (~nan).any() else None, "nan count", int(nan.sum()),
          "P max diff", (res[k][1] - res[0][1]).abs().max().item())
    if int(nan.sum()):
        idx = nan.nonzero()
        print("  nan at seq", sorted(set(idx[:, 0].tolist()))[:8], "tokens", sorted(set(idx[:, 1].tolist()))[:10],
              "cols", sorted(set((idx[:, 2] // 32).tolist())))
    bad = (d > 0) & ~nan
    if bad.any():
        idx = bad.nonzero()
        print("  diff at tokens", sorted(set(idx[:, 1].tolist()))[:10], "col blocks", sorted(set((idx[:, 2] // 32).tolist())))
