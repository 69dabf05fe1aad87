"""Cross-queue wait latency on one MI355X: the gap a stream pays for a
hipStreamWaitEvent on another stream's event, when the event has long
completed ("satisfied") and when it completes just in time ("jit"), against
the same kernel pair with no wait ("none"); event kinds: torch's default
event and the native device-scope ones (ghm_event_create 1 / 2).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python tools/xq_latency.py
    python tools/xq_latency.py --report OUT/run_kernel_trace.csv

Kernels: torch.cuda._sleep (spin) and a one-element fill; each case is marked
by the fill's value (a distinct tensor per case), so the trace tells them apart
by kernel order.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-ghm_amd")]

CASES = ["none", "satisfied", "jit", "satisfied_dev1", "jit_dev1", "satisfied_dev2", "jit_dev2"]
REPS = 20


def run():
    import torch
    from ghmclip import _native
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.zeros(16, device="cuda")
    lib = _native.hip_lib()
    evs = {1: ctypes.c_void_p(lib.ghm_event_create(1)), 2: ctypes.c_void_p(lib.ghm_event_create(2))}
    cyc = 200_000  # ~ 100 us of spin
    torch.cuda.synchronize()
    for case in CASES:
        for _ in range(REPS):
            kind = int(case[-1]) if case[-1].isdigit() else 0

            def wait():
                if kind:
                    _native.call("ghm_event_record", evs[kind], ctypes.c_void_p(s1.cuda_stream))
                    _native.call("ghm_stream_wait", ctypes.c_void_p(s2.cuda_stream), evs[kind])
                else:
                    s2.wait_stream(s1)
            if case == "none":  # dispatches: sleep(s2), fill(s2)
                with torch.cuda.stream(s2):
                    torch.cuda._sleep(cyc)
                    x.fill_(1.0)
            elif case.startswith("satisfied"):  # sleep(s2), sleep/10(s1), fill(s1), fill(s2)
                with torch.cuda.stream(s2):
                    torch.cuda._sleep(cyc)
                with torch.cuda.stream(s1):
                    torch.cuda._sleep(cyc // 10)
                    x.fill_(2.0)
                wait()
                with torch.cuda.stream(s2):
                    x.fill_(3.0)
            else:  # jit: sleep(s1), fill(s2) -- s2 idles until s1's spin ends
                with torch.cuda.stream(s1):
                    torch.cuda._sleep(cyc)
                wait()
                with torch.cuda.stream(s2):
                    x.fill_(4.0)
            torch.cuda.synchronize()
    print("done")


def report(path):
    import csv
    rows = [r for r in csv.DictReader(open(path)) if r["Kind"] == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    ks = ks[1:]  # the zeros() fill
    i = 0
    for case in CASES:
        gaps = []
        for _ in range(REPS):
            if case == "none" or case.startswith("jit"):
                a, b = ks[i], ks[i + 1]
                i += 2
            else:
                a, b = ks[i], ks[i + 3]  # the s2 sleep -> the s2 fill after the (long satisfied) wait
                i += 4
            gaps.append((b[1] - a[2]) / 1000.0)
        gaps.sort()
        print(f"{case:16s} gap (us): median {gaps[len(gaps) // 2]:7.2f}  min {gaps[0]:7.2f}  max {gaps[-1]:7.2f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
