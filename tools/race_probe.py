"""Cross-stream interference probe: one kernel (victim) runs repeatedly on fixed
inputs on stream A while another kernel (aggressor) runs on stream B; the
victim's outputs must be bit-identical across repetitions.

    python tools/race_probe.py [victim] [aggressor] [reps]
    victim: qkv_bwd | qkv_load | qkv_dev | mlp_bwd | wgrad | attn_bwd ; aggressor: mlp_bwd | wgrad | attn_bwd | fwd_mlp | none
"""
import ctypes
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multimodal-ghm_amd"))
import bench  # noqa: E402
from ghmclip import _native  # noqa: E402


def digest(t):
    t = t.detach().contiguous()
    if t.dtype == torch.bfloat16:
        t = t.view(torch.int16)
    return hashlib.sha1(t.cpu().numpy().tobytes()).hexdigest()[:10]


QKV_MODES = {"qkv_load": 1, "qkv_dev": 2, "qkv_sc1": 3, "qkv_dbg": 4, "qkv_dbgu": 5}


def main():
    victim = sys.argv[1] if len(sys.argv) > 1 else "qkv_bwd"
    aggr = sys.argv[2] if len(sys.argv) > 2 else "mlp_bwd"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    sampler, tr = bench.build(0, 128, 5, 0.2, 3000, "x3")
    ring = bench.make_ring(sampler, 128, 2)
    tr.set_tokens(ring[0, 0], ring[0, 1])
    tr.step()
    torch.cuda.synchronize()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    c = _native.call
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    A = ctypes.c_void_p(sa.cuda_stream)
    B = ctypes.c_void_p(sb.cuda_stream)
    l = 2
    p0, p1 = tr.plans
    w0, w1 = tr.views[0][0], tr.views[1][0]
    M = p0.M
    # victim inputs: plan 0 buffers as left by the step; outputs into fresh tensors
    dHmid = torch.randn(M, 128, device="cuda") * 1e-3
    dqkv = torch.randn(M, 384, device="cuda") * 1e-3
    outH = torch.empty(M, 128, device="cuda")
    outP = torch.empty_like(p0.part_ln2)
    outG, outU = torch.empty(M, 512, device="cuda"), torch.randn(M, 512, device="cuda") * 1e-3
    vpart, vpb = torch.empty_like(p0.part_w1), torch.empty_like(p0.part_b1)
    vdS, outQ = torch.zeros_like(p0.dS), torch.empty(M, 384, device="cuda")
    xH, xP = torch.empty(M, 128, device="cuda"), torch.empty_like(p1.part_ln2)
    dbg = torch.zeros(M, 4, device="cuda")
    n_dbg = 0
    xa, xb, xc = (torch.randn(4096, 4096, device="cuda") for _ in range(3))

    def run_victim():
        if victim == "qkv_bwd":
            c("ghm_qkv_bwd_x3", P(dqkv), P(p0.H[l]), P(p0.st1[l]), P(w0[f"_lns_1.{l}.weight"]), P(p0.pack[l]),
              P(dHmid), P(outH), P(outP), M, 128, p0.eps, A)
            return [outH, outP]
        if victim in QKV_MODES:  # the statistics read from p0.st1 (ghm_qkv_bwd_x3_probe)
            c("ghm_qkv_bwd_x3_probe", P(dqkv), P(p0.H[l]), P(p0.st1[l]), P(w0[f"_lns_1.{l}.weight"]),
              P(p0.pack[l]), P(dHmid), P(outH), P(outP), P(dbg), M, 128, p0.eps, QKV_MODES[victim], A)
            return [outH, outP]
        if victim == "wgrad":
            tps, ns = p0.wg["w1"]
            c("ghm_wgrad_x3", P(outU), 512, 512, P(p0.Hmid[l]), 128, 128, 2, P(p0.st2[l]),
              P(w0[f"_lns_2.{l}.weight"]), P(w0[f"_lns_2.{l}.bias"]), P(vpart), P(vpb), M, tps, A)
            return [vpart, vpb]
        if victim == "attn_bwd":
            c("ghm_attn_bwd_x3", P(p0.qkv[l]), P(p0.P[l]), P(dHmid), P(vdS), P(outQ), p0.N, p0.T, 128,
              p0.scale_div, A)
            return [outQ]
        c("ghm_mlp_bwd_rc_x3", P(dHmid), P(p0.Hmid[l]), P(p0.st2[l]), P(w0[f"_lns_2.{l}.weight"]),
          P(w0[f"_lns_2.{l}.bias"]), P(p0.pack[l]), P(w0[f"_mlps.{l}.0.bias"]), P(outG), P(outU), P(outH), P(outP),
          M, 128, 512, A)
        return [outG, outU, outH, outP]

    def run_aggr():
        if aggr == "mlp_bwd":
            c("ghm_mlp_bwd_rc_x3", P(p1.H[l + 1]), P(p1.Hmid[l]), P(p1.st2[l]), P(w1[f"_lns_2.{l}.weight"]),
              P(w1[f"_lns_2.{l}.bias"]), P(p1.pack[l]), P(w1[f"_mlps.{l}.0.bias"]), P(p1.G), P(p1.dU), P(xH), P(xP),
              M, 128, 512, B)
        elif aggr == "fwd_mlp":
            c("ghm_ln_mlp_fwd_x3b", P(p1.Hmid[l]), P(w1[f"_lns_2.{l}.weight"]), P(w1[f"_lns_2.{l}.bias"]),
              P(p1.pack[l]), P(w1[f"_mlps.{l}.0.bias"]), P(w1[f"_mlps.{l}.2.bias"]), P(xH),
              P(p1.st2[l + 1 if l + 1 < p1.L else l]), M, 128, 512, p1.eps, B)
        elif aggr == "wgrad0":
            tps, ns = p1.wg["w2"]
            c("ghm_wgrad_x3", P(p1.H[l + 1]), 128, 128, P(p1.G), 512, 512, 0, None, None, None, P(p1.part_w2),
              P(p1.part_b2), M, tps, B)
        elif aggr == "wgrad_nb":
            tps, ns = p1.wg["w1"]
            c("ghm_wgrad_x3", P(p1.dU), 512, 512, P(p1.Hmid[l]), 128, 128, 2, P(p1.st2[l]),
              P(w1[f"_lns_2.{l}.weight"]), P(w1[f"_lns_2.{l}.bias"]), P(p1.part_w1), None, M, tps, B)
        elif aggr == "mm":
            with torch.cuda.stream(sb):
                torch.mm(xa, xb, out=xc)
        elif aggr == "copy":
            xG = p1.G.view(-1)
            xG2 = p1.dU.view(-1)
            with torch.cuda.stream(sb):
                xG2.copy_(xG)
        elif aggr == "wgrad":
            tps, ns = p1.wg["w1"]
            c("ghm_wgrad_x3", P(p1.dU), 512, 512, P(p1.Hmid[l]), 128, 128, 2, P(p1.st2[l]),
              P(w1[f"_lns_2.{l}.weight"]), P(w1[f"_lns_2.{l}.bias"]), P(p1.part_w1), P(p1.part_b1), M, tps, B)
        elif aggr == "attn_bwd":
            c("ghm_attn_bwd_x3", P(p1.qkv[l]), P(p1.P[l]), P(p1.H[l + 1]), P(p1.dS), P(p1.dqkv), p1.N, p1.T, 128,
              p1.scale_div, B)

    ref = [digest(t) for t in run_victim()]
    torch.cuda.synchronize()
    ref = None
    # aggressor alone: every other buffer of both plans and the victim's inputs must be untouched
    watch = {"dHmid": dHmid, "dqkv": dqkv, "outH": outH, "outP": outP}
    for i, pl in enumerate((p0, p1)):
        for k, v in vars(pl).items():
            if isinstance(v, torch.Tensor) and v.is_cuda and k not in ("part_w1", "part_b1", "part_w2", "part_b2",
                                                                         "part_w", "part_b", "G", "dU", "dqkv", "dS"):
                watch[f"p{i}.{k}"] = v
    before = {k: digest(v) for k, v in watch.items()}
    before_p = digest(tr.pflat)
    for _ in range(5):
        if aggr != "none":
            run_aggr()
    torch.cuda.synchronize()
    changed = [k for k, v in watch.items() if digest(v) != before[k]]
    print(f"aggressor {aggr} alone changed: {changed} pflat changed: {digest(tr.pflat) != before_p}")
    bad = 0
    for r in range(reps):
        sb.wait_stream(torch.cuda.current_stream())
        sa.wait_stream(torch.cuda.current_stream())
        for _ in range(3):
            if aggr != "none":
                run_aggr()
        outs = run_victim()
        for _ in range(3):
            if aggr != "none":
                run_aggr()
        torch.cuda.synchronize()
        if victim in ("qkv_dbg", "qkv_dbgu"):  # loaded (and used) vs the buffer's statistics, per token
            bad_rows = torch.nonzero((dbg[:, :2] != p0.st1[l]).any(1)).flatten()
            if len(bad_rows):
                n_dbg += 1
                rows = bad_rows.tolist()
                print(f"  rep {r}: loaded stats differ from the buffer's for {len(rows)} tokens "
                      f"(first {rows[:4]}, last {rows[-1]}; 16-aligned groups "
                      f"{sorted(set(x // 16 * 16 for x in rows))[:8]})")
                st_all = {"p0.st1": p0.st1, "p0.st2": p0.st2, "p1.st1": p1.st1, "p1.st2": p1.st2}
                for m in rows[:3]:
                    v = dbg[m, :2]
                    hits = []
                    for name, t in st_all.items():
                        flat = t.reshape(-1, 2)
                        idx = torch.nonzero((flat == v).all(1)).flatten().tolist()
                        if idx:
                            hits.append(f"{name}[flat {idx[:3]} = (layer, token) "
                                        f"{[(i // M, i % M) for i in idx[:3]]}]")
                    print(f"    token {m}: loaded {v.tolist()} recomputed {dbg[m, 2:].tolist()} "
                          f"buffer {p0.st1[l][m].tolist()} found in {hits or 'no stats buffer'}")
        d = [digest(t) for t in outs]
        if ref is None:
            ref = d
            keep = [t.clone() for t in outs]
        elif d != ref:
            bad += 1
            if bad <= 3:
                for k, (a, b) in enumerate(zip(keep, outs)):
                    diff = (a - b).abs().reshape(a.shape[0], -1)
                    rows = torch.nonzero(diff.amax(1) > 0).flatten()
                    if len(rows) and k == 0 and victim.startswith("qkv"):
                        m = int(rows[0])
                        x = p0.H[l][m].double()
                        st = p0.st1[l][m].double()
                        xhat = (x - st[0]) * st[1]
                        dd = (b[m] - a[m]).double()
                        Xm = torch.stack([torch.ones_like(xhat), xhat], 1)
                        coef = torch.linalg.lstsq(Xm.cpu(), dd.cpu().unsqueeze(1)).solution.flatten()
                        resid = (dd.cpu() - Xm.cpu() @ coef).abs().max().item()
                        nzf = torch.nonzero(dd.abs() > 0).flatten().tolist()
                        print(f"  row {m}: {len(nzf)} features differ {nzf[:12]}; affine fit a={coef[0]:.3e} "
                              f"b={coef[1]:.3e} resid {resid:.3e} (max |d| {dd.abs().max().item():.3e})")
                    if len(rows):
                        print(f"  rep {r} out{k}: {len(rows)} rows differ (first {rows[:6].tolist()}), "
                              f"max |d| {diff.max().item():.3e}, |ref| max {a.abs().max().item():.3e}, "
                              f"nan {torch.isnan(b).sum().item()}")
    print(f"victim {victim} aggressor {aggr}: {bad}/{reps - 1} repetitions differ"
          + (f"; loaded statistics != the buffer's in {n_dbg}/{reps} repetitions" if victim.startswith("qkv_dbg")
             else ""))
    if os.environ.get("GHM_PROBE_STATS") == "1" and victim == "qkv_bwd":
        # debug build GHM_QKV_DBG=13: dH[m][0:2] holds the (mean, rstd) the kernel read
        got = outH[:, :2]
        true = p0.st1[l]
        bad_rows = torch.nonzero((got != true).any(1)).flatten()
        print(f"stats read wrong for {len(bad_rows)} tokens: {bad_rows[:20].tolist()}")
        for m in bad_rows[:4].tolist():
            v = got[m]
            # where else does this value live?
            hits = []
            for name, t in (("p0.st1", p0.st1), ("p0.st2", p0.st2), ("p1.st1", p1.st1), ("p1.st2", p1.st2)):
                flat = t.reshape(-1, 2)
                idx = torch.nonzero((flat == v).all(1)).flatten()
                if len(idx):
                    hits.append(f"{name}[{idx[:3].tolist()}]")
            print(f"  token {m}: read {v.tolist()} true {true[m].tolist()} found in {hits}")


if __name__ == "__main__":
    main()
