"""The reference's actual CLIP workload on one MI355X: exp_clip_{standard,guided,
shallow}TF.sh, 20 p_flip values each (scripts/experiments/exp_clip_*.sh:6-41),
total_iters = 3000, through the drop-in CLI code path (train_CLIP.run).  Each
run's final CLIP risk = mean(loss_history[-100:]) (figures/eval-clip-risk.py:29)
is compared with the published figures/data/ghm-data/clip-risk.json
(tests/golden/clip_risk_published.json).

    python tools/clip_risk_sweep.py --arch "Standard TF" --out profiles/r2_clip_risk_standard.json

Writes a JSON shaped like clip-risk.json (p_flip in percent, one list per
architecture, "Bayes") plus per-run timing, and the loss histories (.npz next
to it).  Runs are sequential on one GPU (the reference ran 20 concurrent
processes per GPU).
"""
import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-ghm_amd"))


def main():
    from ghmclip.training.clip_runs import ARCHS, P_FLIPS, run_clip
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="Standard TF", choices=list(ARCHS))
    ap.add_argument("--out", required=True)
    ap.add_argument("--total-iters", type=int, default=3000)
    ap.add_argument("--p", type=float, nargs="*", default=None)
    a = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "clip_risk_published.json")) as f:
        pub = json.load(f)
    ps = a.p if a.p else P_FLIPS
    res = {"p_flip": [], a.arch: [], "Bayes": [], "seconds": [], "published": [], "published_bayes": []}
    hists = {}
    t_all = time.time()
    for p in ps:
        with contextlib.redirect_stdout(sys.stderr):
            r = run_clip(a.arch, p, total_iters=a.total_iters)
        pct = int(round(p * 100))
        k = pub["p_flip"].index(pct)
        res["p_flip"].append(pct)
        res[a.arch].append(r["final_risk"])
        res["Bayes"].append(float(r["bayes"]))
        res["seconds"].append(round(r["loop_seconds"], 2))
        res["published"].append(pub[a.arch][k])
        res["published_bayes"].append(pub["Bayes"][k])
        hists[f"p{pct}"] = r["loss_history"]
        print(f"{a.arch} p={p:.2f}: risk {r['final_risk']:.4f} (published {pub[a.arch][k]:.4f}), "
              f"Bayes {r['bayes']:.4f} (published {pub['Bayes'][k]:.4f}), loop {r['loop_seconds']:.1f}s, "
              f"{time.time() - t_all:.0f}s total", flush=True)
    d = np.array(res[a.arch]) - np.array(res["published"])
    res["deviation"] = {"mean": float(d.mean()), "mean_abs": float(np.abs(d).mean()), "max_abs": float(np.abs(d).max()),
                        "excess_over_bayes_ours": float(np.mean(np.array(res[a.arch]) - np.array(res["Bayes"]))),
                        "excess_over_bayes_published": float(np.mean(np.array(res["published"]) -
                                                                     np.array(res["published_bayes"]))),
                        "bayes_max_abs_diff": float(np.abs(np.array(res["Bayes"]) -
                                                           np.array(res["published_bayes"])).max())}
    res["definition"] = "final risk = mean(loss_history[-100:]) after total_iters+1 steps (figures/eval-clip-risk.py:29)"
    res["total_iters"] = a.total_iters
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    np.savez_compressed(os.path.splitext(a.out)[0] + "_hist.npz", **hists)
    print(json.dumps(res["deviation"]), flush=True)


if __name__ == "__main__":
    main()
