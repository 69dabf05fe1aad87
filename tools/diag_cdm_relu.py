"""Joint CDM relu attention: per-gradient error of each HIP mode and of the f32
oracle, all against the oracle in float64 (the test_gpu_cdm_joint.py module case
B=5, relu).  Prints the max-abs error relative to the tensor's max-abs; the *_vs_kmask
columns compare with the float64 oracle taken with the kernels' own relu masks
(conftest.masked_relu_oracle: relu's derivative on the kernels' side of zero), and
counts the mask entries that differ from the float64 scores' signs.
usage: python tools/diag_cdm_relu.py [B]"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multimodal-ghm_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import kernel_relu_masks, masked_relu_oracle  # noqa: E402
from oracle import cdm_oracle as CO  # noqa: E402


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-300)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from ghmclip import ConditionalDenoiseEncoderTransformer
    torch.manual_seed(11)
    ref = CO.OracleCdm(162, 81, 10, 128, 2, 512, sequential=False, activation="relu")
    g = torch.Generator().manual_seed(B)
    with torch.no_grad():
        for k, v in ref.named_parameters():
            if "_lns_" in k or k.endswith("bias"):
                v.add_(0.1 * torch.randn(v.shape, generator=g))
    xt = torch.randint(0, 10, (B, 81), generator=g)
    z = torch.randint(0, 10, (B, 81), generator=g).float() + torch.randn(B, 81, generator=g)
    R = torch.randn(B, 81, generator=g)

    ref32 = copy.deepcopy(ref)
    (ref32(xt, z) * R).sum().backward()
    torch.set_default_dtype(torch.float64)
    ref64 = copy.deepcopy(ref).double()
    scores, orig = [], torch.einsum
    torch.einsum = lambda eq, *a: scores.append(orig(eq, *a)) or scores[-1] if eq == "bid,bjd->bij" else orig(eq, *a)
    p64 = ref64(xt, z.double())
    torch.einsum = orig
    scores = [s.detach() for s in scores]
    (p64 * R.double()).sum().backward()
    truth = {k: v.grad.clone() for k, v in ref64.named_parameters() if v.grad is not None}
    # the problem's own sensitivity: the float64 oracle under a 2^-17 relative
    # perturbation of the q / k weights (the split-bf16 rounding scale)
    pg = torch.Generator().manual_seed(1)
    for trial in range(3):
        m = copy.deepcopy(ref).double()
        with torch.no_grad():
            for k, v in m.named_parameters():
                if "_queries" in k or "_keys" in k:
                    v.mul_(1 + 2 ** -17 * (2 * torch.rand(v.shape, generator=pg, dtype=torch.float64) - 1))
        (m(xt, z.double()) * R.double()).sum().backward()
        ch = {k: rel(v.grad, truth[k]) for k, v in m.named_parameters() if v.grad is not None}
        w = max(ch, key=ch.get)
        print(f"float64 oracle, q/k weights x (1 + 2^-17 u), trial {trial}: worst gradient change {ch[w]:.3e} ({w})")
    torch.set_default_dtype(torch.float32)

    rows = {"oracle_f32": {k: rel(v.grad, truth[k]) for k, v in ref32.named_parameters() if v.grad is not None}}
    for mode in ("x3", "f32"):
        torch.manual_seed(11)
        prod = ConditionalDenoiseEncoderTransformer(162, 81, 10, 128, 2, [4, 4], 4, 512, sequential=False,
                                                    activation="relu")
        with torch.no_grad():
            for (k, vp), (_, vr) in zip(prod.named_parameters(), ref.named_parameters()):
                vp.copy_(vr)
        prod.precision = "x3" if mode == "x3" else "f32"
        prod = prod.cuda()
        pred, _ = prod(xt.cuda(), z.cuda())
        (pred * R.cuda()).sum().backward()
        torch.cuda.synchronize()
        rows[mode] = {k: rel(v.grad, truth[k]) for k, v in prod.named_parameters() if v.grad is not None}
        # the float64 oracle taken with the kernels' own relu masks (their saved P > 0)
        km = masked_relu_oracle(ref, kernel_relu_masks(prod), lambda m: (m(xt, z.double()) * R.double()).sum())
        truth_k = {k: v.grad for k, v in km.named_parameters() if v.grad is not None}
        rows[mode + "_vs_kmask"] = {k: rel(v.grad, truth_k[k]) for k, v in prod.named_parameters()
                                    if v.grad is not None}
        nflip = sum(int((m != (s > 0)).sum()) for m, s in zip(kernel_relu_masks(prod), scores))
        print(f"{mode}: {nflip} relu mask entries differ from the float64 scores' signs")
    keys = list(rows["oracle_f32"])
    print(f"B={B}  max-abs error / max-abs of the float64 oracle gradient")
    print(f"{'param':34s} " + " ".join(f"{m[:14]:>14s}" for m in rows))
    for k in keys:
        print(f"{k[:34]:34s} " + " ".join(f"{rows[m].get(k, float('nan')):14.3e}" for m in rows))
    for m in rows:
        w = max(rows[m].values())
        print(f"worst {m:15s} {w:.3e} ({max(rows[m], key=rows[m].get)})")


if __name__ == "__main__":
    main()
