"""Per-kernel timing of the default CLIP config with HIP events (one process).

    python tools/kbench.py [--reps 20] [--only name,name]

Builds the default-config trainer, runs two real steps to populate every
activation, then re-launches each kernel of encoder 0 / layer 0 `reps` times
on the current stream between two events.  Prints us/launch and the MFMA
fraction for the GEMM-shaped kernels (f32 peak; x3 kernels: bf16 peak / 3).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-ghm_amd"))
sys.path.insert(0, ROOT)

PEAK = 157.3e12       # f32 MFMA, dense
BF16_PEAK = 2.5e15    # bf16 MFMA, dense (x3 issues 3 bf16 products per f32 product)


def _with_env(key, val, fn):
    """Run fn() with os.environ[key] = val (the library reads some switches per call)."""
    old = os.environ.get(key)
    os.environ[key] = val
    try:
        return fn()
    finally:
        if old is None:
            del os.environ[key]
        else:
            os.environ[key] = old


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--precision", default="x3", choices=["f32", "x3"],
                    help="trainer precision; x3 also enables the *_x3 kernel entries")
    a = ap.parse_args()
    import bench
    from ghmclip import _native
    sampler, tr = bench.build(0, 128, 5, 0.2, 3000, a.precision)
    ring = bench.make_ring(sampler, 128, 2)
    for k in range(2):
        tr.set_tokens(ring[k, 0], ring[k, 1])
        tr.step()
    torch.cuda.synchronize()
    plan, p = tr.plans[0], tr.views[0][0]
    g = tr.views[0][1]
    M, N, T = plan.M, plan.N, plan.T
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    c = _native.call
    l = 0
    tps_w2, ns_w2 = plan.wg["w2"]
    tps_w1, ns_w1 = plan.wg["w1"]
    tps_q, ns_q = plan.wg["qkv"]
    gf = lambda flop: flop / 1e9  # noqa: E731
    kernels = {}
    if plan.pack is None:  # exact-f32 kernels
        kernels.update({
            "ln_qkv_fwd": (lambda: c("ghm_ln_qkv_fwd", P(plan.H[l]), P(p["_lns_1.0.weight"]), P(p["_lns_1.0.bias"]),
                                     P(p["_queries.0.weight"]), P(p["_keys.0.weight"]), P(p["_values.0.weight"]),
                                     P(plan.qkv[l]), P(plan.st1[l]), M, 128, plan.eps, sp), gf(2 * M * 128 * 384)),
            "attn_fwd": (lambda: c("ghm_attn_fwd", P(plan.qkv[l]), P(plan.H[l]), P(plan.Hmid[l]), P(plan.P[l]), N, T,
                                   128, plan.scale_div, sp), gf(4 * N * T * T * 128)),
            "ln_mlp_fwd": (lambda: c("ghm_ln_mlp_fwd", P(plan.Hmid[l]), P(p["_lns_2.0.weight"]),
                                     P(p["_lns_2.0.bias"]), P(p["_mlps.0.0.weight"]), P(p["_mlps.0.0.bias"]),
                                     P(p["_mlps.0.2.weight"]), P(p["_mlps.0.2.bias"]), P(plan.H[l + 1]), P(plan.G[l]),
                                     P(plan.Dg[l]), P(plan.st2[l]), M, 128, 512, plan.eps, sp), gf(4 * M * 128 * 512)),
            # the same with nothing saved for the backward (precision "f32fwd")
            "ln_mlp_fwd_nosave": (lambda: c("ghm_ln_mlp_fwd", P(plan.Hmid[l]), P(p["_lns_2.0.weight"]),
                                            P(p["_lns_2.0.bias"]), P(p["_mlps.0.0.weight"]), P(p["_mlps.0.0.bias"]),
                                            P(p["_mlps.0.2.weight"]), P(p["_mlps.0.2.bias"]), P(plan.H[l + 1]), None,
                                            None, P(plan.st2[l]), M, 128, 512, plan.eps, sp), gf(4 * M * 128 * 512)),
            "mlp_bwd": (lambda: c("ghm_mlp_bwd", P(plan.H[l + 1]), P(plan.Hmid[l]), P(plan.st2[l]),
                                  P(p["_lns_2.0.weight"]), P(p["_mlps.0.0.weight"]), P(p["_mlps.0.2.weight"]),
                                  P(plan.Dg[l]), P(plan.dU), P(plan.dH[1]), P(plan.part_ln), M, 128, 512, sp),
                        gf(4 * M * 128 * 512)),
        })
    else:  # the split-bf16 kernels the x3 step launches (+ the superseded MLP pair)
        pk = P(plan.pack[l])
        xo = {"H": torch.empty_like(plan.H[l + 1]), "st": torch.empty_like(plan.st2[l]),
              "G": torch.empty(M, 512, device=plan.H.device), "Dg": torch.empty(M, 512, device=plan.H.device),
              "dHm": torch.empty_like(plan.H[l + 1]),
              "pack3": torch.empty(_native.GHM_SPLIT3_PACK_ELEMS, dtype=torch.bfloat16, device=plan.H.device)}
        # the pre-split LN planes (the plan's own when GHM_LN_PRESPLIT=1)
        xs = plan.xs[l] if plan.xs is not None else torch.zeros(2, 2, M, 128, dtype=torch.bfloat16,
                                                                 device=plan.H.device)
        j3 = _native.SplitJob()
        j3.Wq, j3.Wk, j3.Wv = (p[f"_{k}.0.weight"].data_ptr() for k in ("queries", "keys", "values"))
        j3.W1, j3.W2, j3.pack = p["_mlps.0.0.weight"].data_ptr(), p["_mlps.0.2.weight"].data_ptr(), xo["pack3"].data_ptr()
        c("ghm_split3_weights", (_native.SplitJob * 1)(j3), 1, sp)
        kernels.update({
            "ln_qkv_fwd_x3": (lambda: c("ghm_ln_qkv_fwd_x3", P(plan.H[l]), P(p["_lns_1.0.weight"]),
                                        P(p["_lns_1.0.bias"]), pk, P(plan.qkv[l]), P(plan.st1[l]), M, 128, plan.eps,
                                        sp), gf(2 * M * 128 * 384)),
            "attn_fwd_x3": (lambda: c("ghm_attn_fwd_x3", P(plan.qkv[l]), P(plan.H[l]), P(plan.Hmid[l]), P(plan.P[l]),
                                      N, T, 128, plan.scale_div, sp), gf(4 * N * T * T * 128)),
            # three-way split operands (precision f32fwd's mlp6 stage): pack3 of layer 0
            "ln_mlp_fwd_x6": (lambda: c("ghm_ln_mlp_fwd_x6", P(plan.Hmid[l]), P(p["_lns_2.0.weight"]),
                                        P(p["_lns_2.0.bias"]), pk, P(xo["pack3"]), P(p["_mlps.0.0.bias"]),
                                        P(p["_mlps.0.2.bias"]), P(xo["H"]), P(xo["st"]), None, None, M, 128, 512,
                                        plan.eps, sp),
                              gf(4 * M * 128 * 512)),
            "ln_qkv_fwd_x6": (lambda: c("ghm_ln_qkv_fwd_x6", P(plan.H[l]), P(p["_lns_1.0.weight"]),
                                        P(p["_lns_1.0.bias"]), pk, P(xo["pack3"]), P(plan.qkv[l]), P(plan.st1[l]), M,
                                        128, plan.eps, sp), gf(2 * M * 128 * 384)),
            "ln_mlp_fwd_x3b": (lambda: c("ghm_ln_mlp_fwd_x3b", P(plan.Hmid[l]), P(p["_lns_2.0.weight"]),
                                         P(p["_lns_2.0.bias"]), pk, P(p["_mlps.0.0.bias"]), P(p["_mlps.0.2.bias"]),
                                         P(xo["H"]), P(xo["st"]), M, 128, 512, plan.eps, sp),
                               gf(4 * M * 128 * 512)),
            "ln_mlp_fwd_x3w": (lambda: _with_env("GHM_MLP_FWD_WS", "1", lambda: c(
                "ghm_ln_mlp_fwd_x3b", P(plan.Hmid[l]), P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]), pk,
                P(p["_mlps.0.0.bias"]), P(p["_mlps.0.2.bias"]), P(xo["H"]), P(xo["st"]), M, 128, 512, plan.eps, sp)),
                               gf(4 * M * 128 * 512)),
            "ln_mlp_fwd_x3w16": (lambda: _with_env("GHM_MLP_FWD_WS", "2", lambda: c(
                "ghm_ln_mlp_fwd_x3b", P(plan.Hmid[l]), P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]), pk,
                P(p["_mlps.0.0.bias"]), P(p["_mlps.0.2.bias"]), P(xo["H"]), P(xo["st"]), M, 128, 512, plan.eps, sp)),
                               gf(4 * M * 128 * 512)),
            "ln_mlp_fwd_x3w82": (lambda: _with_env("GHM_MLP_FWD_WS", "3", lambda: c(
                "ghm_ln_mlp_fwd_x3b", P(plan.Hmid[l]), P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]), pk,
                P(p["_mlps.0.0.bias"]), P(p["_mlps.0.2.bias"]), P(xo["H"]), P(xo["st"]), M, 128, 512, plan.eps, sp)),
                               gf(4 * M * 128 * 512)),
            "ln_mlp_fwd_x3b16": (lambda: _with_env("GHM_MLP_FWD_WS", "4", lambda: c(
                "ghm_ln_mlp_fwd_x3b", P(plan.Hmid[l]), P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]), pk,
                P(p["_mlps.0.0.bias"]), P(p["_mlps.0.2.bias"]), P(xo["H"]), P(xo["st"]), M, 128, 512, plan.eps, sp)),
                               gf(4 * M * 128 * 512)),
            "mlp_bwd_rc_x3": (lambda: c("ghm_mlp_bwd_rc_x3", P(plan.H[l + 1]), P(plan.Hmid[l]), P(plan.st2[l]),
                                        P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]), pk, P(p["_mlps.0.0.bias"]),
                                        P(plan.G), P(plan.dU), P(xo["dHm"]), P(plan.part_ln2), M, 128, 512,
                                        int(plan.wgrad_ring), sp),
                              gf(6 * M * 128 * 512)),
            "qkv_bwd_x3": (lambda: c("ghm_qkv_bwd_x3", P(plan.dqkv), P(plan.H[l]), P(plan.st1[l]), P(p["_lns_1.0.weight"]), pk,
                                     P(plan.dH[1]), P(plan.dH[0]), P(plan.part_ln), M, 128, plan.eps, sp),
                           gf(2 * M * 128 * 384)),
            "attn_bwd_x3": (lambda: c("ghm_attn_bwd_x3", P(plan.qkv[l]), P(plan.P[l]), P(plan.dH[1]), P(plan.dS),
                                      P(plan.dqkv), N, T, 128, plan.scale_div, sp), gf(8 * N * T * T * 128)),
            "wgrad_w2_x3": (lambda: c("ghm_wgrad_x3", P(plan.H[l + 1]), 128, 128, P(plan.G), 512, 512, 0, None,
                                      None, None, P(plan.part_w2), P(plan.part_b2), M, tps_w2, sp),
                            gf(2 * M * 128 * 512)),
            "wgrad_w1_x3": (lambda: c("ghm_wgrad_x3", P(plan.dU), 512, 512, P(plan.Hmid[l]), 128, 128, 2,
                                      P(plan.st2[l]), P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]),
                                      P(plan.part_w1), P(plan.part_b1), M, tps_w1, sp), gf(2 * M * 128 * 512)),
            "wgrad_qkv_x3": (lambda: c("ghm_wgrad_x3", P(plan.dqkv), 384, 384, P(plan.H[l]), 128, 128, 2,
                                       P(plan.st1[l]), P(p["_lns_1.0.weight"]), P(p["_lns_1.0.bias"]),
                                       P(plan.part_wq), None, M, tps_q, sp), gf(2 * M * 128 * 384)),
            # round 6: the weight gradients on the forward's pre-split LN outputs (ghm_wgrad_x3p),
            # and the forward kernels that write them
            "wgrad_w1_x3p": (lambda: c("ghm_wgrad_x3p", P(plan.dU), 512, 512, P(xs[1]), 128, 128, M * 128,
                                       P(plan.part_w1), P(plan.part_b1), M, tps_w1, sp), gf(2 * M * 128 * 512)),
            "wgrad_qkv_x3p": (lambda: c("ghm_wgrad_x3p", P(plan.dqkv), 384, 384, P(xs[0]), 128, 128, M * 128,
                                        P(plan.part_wq), None, M, tps_q, sp), gf(2 * M * 128 * 384)),
            "mlp_bwd_rc_x3g": (lambda: c("ghm_mlp_bwd_rc_x3", P(plan.H[l + 1]), P(plan.Hmid[l]), P(plan.st2[l]),
                                         P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]), pk, P(p["_mlps.0.0.bias"]),
                                         P(plan.G), P(plan.dU), P(xo["dHm"]), P(plan.part_ln2), M, 128, 512, 2, sp),
                               gf(6 * M * 128 * 512)),
            "wgrad_w2_x3p": (lambda: c("ghm_wgrad_x3p", P(plan.H[l + 1]), 128, 128, P(plan.G), 512, 512, M * 512,
                                       P(plan.part_w2), P(plan.part_b2), M, tps_w2, sp), gf(2 * M * 128 * 512)),
            "ln_qkv_fwd_x3s": (lambda: c("ghm_ln_qkv_fwd_x3s", P(plan.H[l]), P(p["_lns_1.0.weight"]),
                                         P(p["_lns_1.0.bias"]), pk, P(plan.qkv[l]), P(plan.st1[l]), P(xs[0]),
                                         M, 128, plan.eps, sp), gf(2 * M * 128 * 384)),
            "ln_mlp_fwd_x3bs": (lambda: c("ghm_ln_mlp_fwd_x3bs", P(plan.Hmid[l]), P(p["_lns_2.0.weight"]),
                                          P(p["_lns_2.0.bias"]), pk, P(p["_mlps.0.0.bias"]), P(p["_mlps.0.2.bias"]),
                                          P(xo["H"]), P(xo["st"]), P(xs[1]), M, 128, 512, plan.eps, sp),
                                gf(4 * M * 128 * 512)),
            # the ring weight gradients (ghm_wgrad_ring_x3) on the MLP backward's split G / dU planes
            "wgrad_ring_w2": (lambda: c("ghm_wgrad_ring_x3", P(plan.H[l + 1]), 128, 128, 0, 0, P(plan.G), 512, 512,
                                        2, M * 512, None, None, None, P(plan.part_w2), P(plan.part_b2), M, tps_w2,
                                        sp), gf(2 * M * 128 * 512)),
            "wgrad_ring_w1": (lambda: c("ghm_wgrad_ring_x3", P(plan.dU), 512, 512, 2, M * 512, P(plan.Hmid[l]), 128,
                                        128, 1, 0, P(plan.st2[l]), P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]),
                                        P(plan.part_w1), P(plan.part_b1), M, tps_w1, sp), gf(2 * M * 128 * 512)),
            "wgrad_ring_qkv": (lambda: c("ghm_wgrad_ring_x3", P(plan.dqkv), 384, 384, 0, 0, P(plan.H[l]), 128, 128,
                                         1, 0, P(plan.st1[l]), P(p["_lns_1.0.weight"]), P(p["_lns_1.0.bias"]),
                                         P(plan.part_wq), None, M, tps_q, sp), gf(2 * M * 128 * 384)),
        })
    lib = _native.hip_lib()
    if plan.pack is not None and hasattr(lib, "ghm_mlp_bwd_fused_proto"):
        # review item 2 timing prototype (ablation build only: tools/build_variant.sh ...
        # -DGHM_ABLATION_BUILD -DGHM_FUSED_DW_PROTO): MLP backward with dW2 / dW1 fused
        # at 64 tokens per workgroup, and the fixed-order reduction of its partials
        nb = (M + 63) // 64
        pw = torch.empty(nb, 16 * 4 * 64 * 32, device=plan.H.device)
        red_out = torch.empty(16 * 4 * 64 * 32, device=plan.H.device)
        pln = torch.empty(nb, 2, 128, device=plan.H.device)
        fp = lib.ghm_mlp_bwd_fused_proto
        fp.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_int64, ctypes.c_void_p]
        job = _native.ReduceJob()
        job.part, job.n_split, job.n_seg, job.n = pw.data_ptr(), nb, 1, pw.shape[1]
        job.dst[0] = red_out.data_ptr()
        job.off[0], job.off[1] = 0, pw.shape[1]
        jobs = (_native.ReduceJob * 1)(job)
        kernels.update({
            "mlp_bwd_fused_proto": (lambda: _native.check(fp(
                P(plan.H[l + 1]), P(plan.Hmid[l]), P(plan.st2[l]), P(p["_lns_2.0.weight"]), P(p["_lns_2.0.bias"]),
                pk, P(p["_mlps.0.0.bias"]), P(pw), P(xo["dHm"]), P(pln), M, sp), "proto"), gf(10 * M * 128 * 512)),
            "fused_proto_reduce": (lambda: c("ghm_reduce_batch", jobs, 1, sp), None),
        })
    kernels.update({
        "reduce_w2": (lambda: plan._reduce(plan.part_w2, ns_w2, 128 * 512, [g["_mlps.0.2.weight"]], sp), None),
        "reduce_ln": (lambda: plan._reduce(plan.part_ln, plan.nblk, 256, [g["_lns_1.0.weight"], g["_lns_1.0.bias"]],
                                           sp), None),
        "readout_bwd": (lambda: c("ghm_readout_bwd", P(plan.H[5]), P(p["_read_out.weight"]), P(p["_read_out.bias"]),
                                  P(p["_out.weight"]), P(plan.d_emb), P(plan.dH[0]), P(plan.part_ro),
                                  P(plan.part_bro), P(plan.part_wout), P(plan.part_bout), N, T, 128, 10, sp), None),
        "embed_bwd_tok": (lambda: c("ghm_wcolsum", None, P(plan.tokens), 10, P(plan.dH[0]), M, M, 0, M, 128,
                                    P(g["token_embeddings.weight"]), None, P(plan.part_emb), sp), None),
        "embed_bwd_pos": (lambda: c("ghm_colsum", P(plan.dH[0]), N, T * 128, P(g["position_embeddings.weight"]),
                                    P(plan.part_emb), sp), None),
    })
    only = set(a.only.split(",")) if a.only else None
    res = {}
    for name, (fn, gflop) in kernels.items():
        if only and name not in only:
            continue
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            fn()
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        peak = PEAK if plan.pack is None else BF16_PEAK / 3  # x3: 3 bf16 products per f32 product
        frac = (gflop * 1e9 / (us * 1e-6)) / peak if gflop else None
        res[name] = {"us": round(us, 2), "gflop": gflop, "mfma_frac": round(frac, 4) if frac else None}
        print(f"{name:20s} {us:9.2f} us" + (f"   {gflop:7.3f} GF  {frac*100:5.1f}% of MFMA peak" if gflop else ""),
              flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
