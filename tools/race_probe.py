"""Cross-stream interference probe: one kernel (victim) runs repeatedly on fixed
inputs on stream A while another kernel (aggressor) runs on stream B; the
victim's outputs must be bit-identical across repetitions.

    python tools/race_probe.py [victim] [aggressor] [reps]
    victim: qkv_bwd | qkv_load | qkv_dev | qkv_sc1 | qkv_dbg | qkv_dbgu | qkv_xcc | mlp_bwd | wgrad | attn_bwd
    aggressor: mlp_bwd | wgrad | wgrad0 | wgrad_nb | attn_bwd | fwd_mlp | mm | copy | none

qkv_xcc (probe mode 6): the plain statistics load, used, with no per-token debug
store; each workgroup records its XCC_ID / HW_ID.  The reference output is the
same kernel run alone (checked deterministic).  Rows that differ beside the
aggressor come in 16-token groups = one 128-byte line of the [M][2] statistics
buffer; for each wrong group the line it used is searched among every 16-pair
line of every statistics buffer of both towers, as this step's forward left
them and as the previous step's did (snapshot): a float64 restatement of the LN
backward (ghm_ln.h ln_bwd_acc) scores each line, and the best line is confirmed
by rerunning the kernel alone with that line substituted (bit-exact rows = the
line it read).  A stale cross-XCD L2 line is the previous step's line at the
same index.
"""
import ctypes
import hashlib
import os
import sys

import numpy as np
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


QKV_MODES = {"qkv_load": 1, "qkv_dev": 2, "qkv_sc1": 3, "qkv_dbg": 4, "qkv_dbgu": 5, "qkv_xcc": 6}


def stats_candidates(plans, prev):
    """(label, [L*M, 2] f32 pairs) for every statistics buffer, current and previous step."""
    out = []
    for i, pl in enumerate(plans):
        for name in ("st1", "st2"):
            out.append((f"p{i}.{name}", getattr(pl, name).reshape(-1, 2)))
            out.append((f"p{i}.{name}@prev", prev[f"p{i}.{name}"].reshape(-1, 2)))
    return out


def ln_bwd64(X, G, R, mu, rs):
    """float64 LN backward of 16 rows for candidate lines: X, G (= dx * gamma), R
    (residual) [16, 128]; mu, rs [K, 16] -> dH [K, 16, 128] (ln_bwd_acc)."""
    xh = (X[None] - mu[..., None]) * rs[..., None]
    gm = G.mean(-1)[None, :, None]
    c2 = (G[None] * xh).mean(-1, keepdim=True)
    return R[None] + rs[..., None] * (G[None] - gm - xh * c2)


def search_line(X, G, R, W, cands):
    """The 16-pair line of the candidate buffers whose pairs best reproduce the
    16 wrong rows W: (worst-row error, label, first flat index, pairs)."""
    best = (float("inf"), None, None, None)
    for label, c in cands:
        lines = c.double().view(-1, 16, 2)
        for k0 in range(0, lines.shape[0], 1024):
            blk = lines[k0:k0 + 1024]
            err = (ln_bwd64(X, G, R, blk[..., 0], blk[..., 1]) - W[None]).abs().amax(-1).amax(-1)
            v, k = torch.min(err, 0)
            if v.item() < best[0]:
                best = (v.item(), label, 16 * (k0 + int(k)), c.view(-1, 16, 2)[k0 + int(k)].clone())
    return best


def main():
    victim = sys.argv[1] if len(sys.argv) > 1 else "qkv_bwd"
    aggr = sys.argv[2] if len(sys.argv) > 2 else "mlp_bwd"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    sampler, tr = bench.build(0, 128, 5, 0.2, 3000, "x3")
    ring = bench.make_ring(sampler, 128, 2)
    tr.set_tokens(ring[0, 0], ring[0, 1])
    tr.step()
    torch.cuda.synchronize()
    p0, p1 = tr.plans
    # the statistics as the previous step left them, then a step on another batch
    prev = {f"p{i}.{n}": getattr(pl, n).clone() for i, pl in enumerate((p0, p1)) for n in ("st1", "st2")}
    tr.set_tokens(ring[1, 0], ring[1, 1])
    tr.step()
    torch.cuda.synchronize()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    c = _native.call
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    A = ctypes.c_void_p(sa.cuda_stream)
    B = ctypes.c_void_p(sb.cuda_stream)
    l = 2
    w0, w1 = tr.views[0][0], tr.views[1][0]
    M = p0.M
    # victim inputs: plan 0 buffers as left by the step; outputs into fresh tensors
    dHmid = torch.randn(M, 128, device="cuda") * 1e-3
    dqkv = torch.randn(M, 384, device="cuda") * 1e-3
    outH = torch.empty(M, 128, device="cuda")
    outH2 = torch.empty(M, 128, device="cuda")  # the probe's reference reruns (qkv_xcc)
    outP = torch.empty_like(p0.part_ln2)
    outP2 = torch.empty_like(p0.part_ln2)
    outG, outU = torch.empty(M, 512, device="cuda"), torch.randn(M, 512, device="cuda") * 1e-3
    vpart, vpb = torch.empty_like(p0.part_w1), torch.empty_like(p0.part_b1)
    vdS, outQ = torch.zeros_like(p0.dS), torch.empty(M, 384, device="cuda")
    xH, xP = torch.empty(M, 128, device="cuda"), torch.empty_like(p1.part_ln2)
    nblk = int(_native.hip_lib().ghm_token_blocks(M))
    dbg = torch.zeros(M + nblk, 4, device="cuda")  # modes 4 / 5: per token; 4 / 6: per-workgroup placement
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
          M, 128, 512, 0, A)
        return [outG, outU, outH, outP]

    def run_recompute():
        c("ghm_qkv_bwd_x3", P(dqkv), P(p0.H[l]), P(p0.st1[l]), P(w0[f"_lns_1.{l}.weight"]), P(p0.pack[l]),
          P(dHmid), P(outH2), P(outP2), M, 128, p0.eps, A)
        torch.cuda.synchronize()
        return outH2.clone()

    def run_with_stats(st):  # mode 6 alone on a given statistics buffer
        c("ghm_qkv_bwd_x3_probe", P(dqkv), P(p0.H[l]), P(st), P(w0[f"_lns_1.{l}.weight"]),
          P(p0.pack[l]), P(dHmid), P(outH2), P(outP2), P(dbg), M, 128, p0.eps, 6, A)
        torch.cuda.synchronize()
        return outH2.clone()

    def run_aggr():
        if aggr == "mlp_bwd":
            c("ghm_mlp_bwd_rc_x3", P(p1.H[l + 1]), P(p1.Hmid[l]), P(p1.st2[l]), P(w1[f"_lns_2.{l}.weight"]),
              P(w1[f"_lns_2.{l}.bias"]), P(p1.pack[l]), P(w1[f"_mlps.{l}.0.bias"]), P(p1.G), P(p1.dU), P(xH), P(xP),
              M, 128, 512, 0, B)
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

    if victim == "qkv_xcc":  # the reference output: the same kernel alone, twice (deterministic)
        alone = []
        for _ in range(2):
            run_victim()
            torch.cuda.synchronize()
            alone.append(outH.clone())
        truthH = alone[0]
        print(f"mode 6 alone: repeat bit-identical {torch.equal(alone[0], alone[1])}; vs the product kernel: "
              f"max |d| {(truthH - run_recompute()).abs().max().item():.2e}")
        Wqkv = torch.cat([w0[f"_queries.{l}.weight"], w0[f"_keys.{l}.weight"], w0[f"_values.{l}.weight"]], 0).double()
        gam64 = w0[f"_lns_1.{l}.weight"].double()
        cands = stats_candidates((p0, p1), prev)
        float_tensors = [(f"p{i}.{k}", v) for i, pl in enumerate((p0, p1)) for k, v in vars(pl).items()
                         if isinstance(v, torch.Tensor) and v.is_cuda and v.dtype == torch.float32]
        float_tensors += [(k, v) for k, v in prev.items()] + [("pflat", tr.pflat), ("gflat", tr.gflat)]
        n_xcc, wrong_xcc, found, n_checked = 0, {}, {}, 0
        all_xcc = None
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
        if victim == "qkv_xcc":
            xcc = dbg[:nblk, 0].contiguous().view(torch.int32).cpu()
            if all_xcc is None:
                all_xcc = torch.bincount(xcc & 15, minlength=8).tolist()
            got = outH.clone()
            rows = torch.nonzero((got != truthH).any(1)).flatten().cpu()
            if len(rows):
                n_xcc += 1
                groups = sorted(set((rows // 16 * 16).tolist()))
                wgs = sorted(set(g // 128 for g in groups))
                for wg in wgs:
                    k = int(xcc[wg]) & 15
                    wrong_xcc[k] = wrong_xcc.get(k, 0) + 1
                print(f"  rep {r}: {len(rows)} wrong rows in 16-token groups {groups[:8]} (max |d| "
                      f"{(got - truthH).abs().max().item():.2e}); workgroups {wgs[:8]} on XCC "
                      f"{[int(xcc[w]) & 15 for w in wgs[:8]]}")
                for m0 in groups:
                    if n_checked >= 8:
                        break
                    n_checked += 1
                    sl = slice(m0, m0 + 16)
                    X, R = p0.H[l][sl].double(), dHmid[sl].double()
                    G = (dqkv[sl].double() @ Wqkv) * gam64[None]
                    W = got[sl].double()
                    true_err = (ln_bwd64(X, G, R, p0.st1[l][sl, 0].double()[None], p0.st1[l][sl, 1].double()[None])
                                - W[None]).abs().max().item()
                    err, label, idx, pairs = search_line(X, G, R, W, cands)
                    st = p0.st1[l].clone()
                    st[sl] = pairs
                    exact = int((run_with_stats(st)[sl] == got[sl]).all(1).sum())
                    lay, tok = idx // M, idx % M
                    same = label == "p0.st1@prev" and lay == l and tok == m0
                    key = f"{label}{' same index' if same else ''}{' (exact)' if exact == 16 else ''}"
                    found[key] = found.get(key, 0) + 1
                    print(f"    group {m0} (XCC {int(xcc[m0 // 128]) & 15}): best line {label}[layer {lay}, tokens "
                          f"{tok}..{tok + 15}] fit {err:.2e} (its own line {true_err:.2e}); rerun with that line "
                          f"substituted: {exact}/16 rows bit-identical to the wrong rows")
                    # does ANY (mean, rstd) explain a wrong row?  continuous fit per row vs the
                    # model's own noise (the reference rows fitted with their true pair)
                    from scipy.optimize import least_squares
                    Tr = truthH[sl].double()
                    for rr in range(2):
                        xs, gs, rs_, ws = (v[rr].cpu().numpy() for v in (X, G, R, W))
                        tp = p0.st1[l][m0 + rr].double().cpu().numpy()

                        def res(q, xs=xs, gs=gs, rs_=rs_, ws=ws):
                            xh = (xs - q[0]) * q[1]
                            return rs_ + q[1] * (gs - gs.mean() - xh * (gs * xh).mean()) - ws
                        fit = least_squares(res, tp, x_scale=[1e-2, 1e-2], xtol=1e-15, ftol=1e-15, gtol=1e-15)
                        noise = np.abs(res(tp, ws=Tr[rr].cpu().numpy())).max()
                        print(f"      row {m0 + rr}: best-fit pair {fit.x.tolist()} (true {tp.tolist()}) leaves "
                              f"{np.abs(fit.fun).max():.2e}; the true pair leaves {np.abs(res(tp)).max():.2e} on the "
                              f"wrong row and {noise:.2e} on the correct row (model noise)")
                        if np.abs(fit.fun).max() < 3 * noise:  # a (mean, rstd) pair explains the row: find it
                            tgt = torch.tensor(fit.x, dtype=torch.float32, device="cuda")
                            best = (float("inf"), None)
                            for name, t in float_tensors:
                                flat = t.reshape(-1)
                                for off in (0, 1):
                                    n2 = (flat.numel() - off) // 2
                                    if n2 < 1:
                                        continue
                                    pr = flat[off:off + 2 * n2].view(n2, 2)
                                    d = ((pr - tgt).abs() / tgt.abs().clamp_min(1e-12)).amax(1)
                                    v, k = torch.min(d, 0)
                                    if v.item() < best[0]:
                                        best = (v.item(), f"{name}[float {off + 2 * int(k)}]")
                            print(f"        nearest float pair anywhere: {best[1]} (relative {best[0]:.1e})")
        if victim in ("qkv_dbg", "qkv_dbgu"):  # loaded (and used) vs the buffer's statistics, per token
            if victim == "qkv_dbg" and r == 0:
                xq = dbg[M:M + nblk, 0].contiguous().view(torch.int32).cpu() & 15
                print(f"  workgroups per XCC (mode 4 placement record): {torch.bincount(xq, minlength=8).tolist()}")
            bad_rows = torch.nonzero((dbg[:M, :2] != p0.st1[l]).any(1)).flatten()
            if len(bad_rows):
                n_dbg += 1
                rows = bad_rows.tolist()
                print(f"  rep {r}: loaded stats differ from the buffer's for {len(rows)} tokens "
                      f"(first {rows[:4]}, last {rows[-1]}; 16-aligned groups "
                      f"{sorted(set(x // 16 * 16 for x in rows))[:8]}; their workgroups' XCC "
                      f"{sorted(set(int(dbg[M + x // 128, 0].view(torch.int32)) & 15 for x in rows))})")
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
    if victim == "qkv_xcc":
        print(f"workgroups per XCC (all {nblk}): {all_xcc}; repetitions with wrong rows {n_xcc}/{reps}; "
              f"wrong workgroups per XCC {dict(sorted(wrong_xcc.items()))}; lines the wrong groups read: {found}")
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
