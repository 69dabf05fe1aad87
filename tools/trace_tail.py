"""Mean duration of the last N dispatches of a kernel in a rocprofv3 kernel trace.

    python tools/trace_tail.py <run_kernel_trace.csv> <kernel-substring> [N]

bench.py times its dominant kernel with HIP events over 20 back-to-back launches
(plus one warm-up) after the timed steps; those are the last 21 dispatches of the
kernel in the trace of `rocprofv3 --kernel-trace -- python bench.py ...`, so this
mean is the profiler's view of the same number (roofline.kernel_ms).
"""
import csv
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = [r for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = rows[-n:]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tail]
    print(f"{key}: {len(rows)} dispatches in trace; last {len(tail)}: mean {sum(d) / len(d):.2f} us, "
          f"min {min(d):.2f}, max {max(d):.2f}")


if __name__ == "__main__":
    main()
