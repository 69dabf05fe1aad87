"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/traffic.py <fetch_dir> <write_dir> [--json out.json] [--over "what ran"]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced read (MI355X_MICROARCH.md, HBM section), so
it is doubled here; WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def kname(raw):
    """Plain kernel name: 'void k_x<3>(...)' -> 'k_x<3>', '_Z15k_ln_mlp_fwd_x3PKf...' -> 'k_ln_mlp_fwd_x3'."""
    m = re.match(r"_Z(\d+)(\w+)", raw)
    if m:
        return m.group(2)[:int(m.group(1))]
    name = raw.replace("(anonymous namespace)::", "").split("(")[0]
    return name[5:] if name.startswith("void ") else name


def load(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    acc = defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == counter:
            acc[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        rd = 2.0 * fetch.get(k, 0.0)
        wr = write.get(k, 0.0)
        out[k] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr}
        print(f"{k[:40]:40s} read {rd/1e6:9.2f} MB  write {wr/1e6:9.2f} MB  total {(rd+wr)/1e6:9.2f} MB")
    if "--json" in sys.argv:
        over = sys.argv[sys.argv.index("--over") + 1] if "--over" in sys.argv else "tools/kbench.py"
        doc = {"source": f"rocprofv3 --pmc FETCH_SIZE ({sys.argv[1]}) and --pmc WRITE_SIZE ({sys.argv[2]}) "
                         f"over {over}; bytes per dispatch, FETCH_SIZE doubled (gfx950 correction)",
               "kernels": out}
        json.dump(doc, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
