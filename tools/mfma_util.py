"""MFMA utilisation table from tools/gpu_pmc.sh passes.

    python tools/mfma_util.py <pmc_dir_prefix, e.g. gpurun_out/r2_p3> [out.txt]

MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): GRBM_GUI_ACTIVE
sums the 8 XCDs, the busy cycles sum every SIMD.
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def kname(raw):
    m = re.match(r"_Z(\d+)(\w+)", raw)
    if m:
        return m.group(2)[:int(m.group(1))]
    name = raw.replace("(anonymous namespace)::", "").split("(")[0]
    return name[5:] if name.startswith("void ") else name


def main():
    base = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{base}/pmc*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = [f"MFMA utilisation per kernel from rocprofv3 --pmc passes ({base}; tools/gpu_pmc.sh over tools/kbench.py,",
           "isolated launches, one tower-layer per launch).  util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE/8).",
           "k_wgrad_x3<2> averages dW1 and dWqkv (same instantiation).", "",
           f"{'kernel':28s} {'GRBM/8':>8s} {'MFMA insts':>11s} {'MFMA util':>9s} {'VALU insts':>11s} "
           f"{'LDS insts':>10s} {'LDS confl':>10s} {'waves':>6s}"]
    for k in sorted(acc):
        if not k.startswith("k_"):
            continue
        cs = acc[k]
        g = lambda c: sum(cs[c]) / len(cs[c]) if cs.get(c) else float("nan")  # noqa: E731
        grbm = g("GRBM_GUI_ACTIVE") / 8
        util = g("SQ_VALU_MFMA_BUSY_CYCLES") / (1024 * grbm)
        out.append(f"{k:28s} {grbm:8.0f} {g('SQ_INSTS_MFMA'):11.0f} {100 * util:8.1f}% {g('SQ_INSTS_VALU'):11.0f} "
                   f"{g('SQ_INSTS_LDS'):10.0f} {g('SQ_LDS_BANK_CONFLICT'):10.0f} {g('SQ_WAVES'):6.0f}")
    text = "\n".join(out) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
