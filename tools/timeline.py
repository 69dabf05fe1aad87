"""One training step's kernel timeline from a rocprofv3 kernel trace.

    python tools/timeline.py <run_kernel_trace.csv> [step_delimiter=k_adamw] [which=-5]

Steps are delimited by the optimizer kernel (one dispatch per step); `which`
picks the step (negative: from the end, skipping bench.py's trailing isolated
launches).  Prints every dispatch of that step (start offset, duration, queue),
the union of busy time (at least one kernel running), the time with two or
more kernels resident, and the idle gaps: where a captured step waits on
latency chains rather than bandwidth.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    delim = sys.argv[2] if len(sys.argv) > 2 else "k_adamw"
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -5
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    ends = [r["e"] for r in rows if delim in r["Kernel_Name"]]
    if len(ends) < 3:
        sys.exit("not enough steps in trace")
    t0, t1 = ends[which - 1], ends[which]
    step = [r for r in rows if t0 < r["s"] <= t1 or (r["s"] <= t0 < r["e"])]
    q = sorted({r.get("Queue_Id", r.get("Stream_Id", "?")) for r in step})
    print(f"step window {(t1 - t0) / 1e3:.1f} us, {len(step)} dispatches, queues {q}")
    ev = []
    for r in step:
        ev.append((max(r["s"], t0), 1))
        ev.append((min(r["e"], t1), -1))
    ev.sort()
    busy = multi = 0
    cur, last = 0, t0
    gaps = []
    for t, d in ev:
        if cur >= 1:
            busy += t - last
        if cur >= 2:
            multi += t - last
        if cur == 0 and t - last > 2000:
            gaps.append((last - t0, t - last))
        cur += d
        last = t
    print(f"busy {busy / 1e3:.1f} us ({100 * busy / (t1 - t0):.0f}%), >=2 kernels {multi / 1e3:.1f} us, "
          f"idle gaps >2us: {[(round(a / 1e3, 1), round(b / 1e3, 1)) for a, b in gaps]}")
    agg = {}
    for r in step:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:48]
        a = agg.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += (r["e"] - r["s"]) / 1e3
    for k, (n, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {k:48s} n={n:3d} sum={d:8.1f} us  avg={d / n:7.1f}")
    if "-v" in sys.argv:
        for r in step:
            print(f"{(r['s'] - t0) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f} q{r.get('Queue_Id', '?')} "
                  f"{r['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main()
