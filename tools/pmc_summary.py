"""Summarise rocprofv3 --pmc passes: mean counter value per kernel (all dispatches).

    python tools/pmc_summary.py <dir> [<dir> ...] [--kernels substr,substr]
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
    name = raw.split("(")[0]
    return name[5:] if name.startswith("void ") else name


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = None
    if "--kernels" in sys.argv:
        filt = sys.argv[sys.argv.index("--kernels") + 1].split(",")
        args = [a for a in args if a != sys.argv[sys.argv.index("--kernels") + 1]]
    acc = defaultdict(lambda: defaultdict(list))
    for d in args:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = kname(r["Kernel_Name"])
                if filt and not any(s in k for s in filt):
                    continue
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()
