"""Instruction mix and waits of the main loop(s) of a kernel in a hipcc --save-temps .s file.

    python tools/isa_loop.py <file.s> <mangled-name-substring> [-v]
"""
import collections
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    key = sys.argv[2]
    names = [m.group(1) for m in re.finditer(r"^(\S+):\s*(?:;.*)?$", s, re.M) if key in m.group(1) and not m.group(1).startswith(".")]
    for name in names:
        a = s.index(name + ":")
        b = s.index(".Lfunc_end", a)
        body = s[a:b].splitlines()
        heads = {}
        for i, l in enumerate(body):
            if l.startswith(".LBB"):
                heads[l.split(":")[0]] = i
        for i, l in enumerate(body):
            m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)", l)
            if m and m.group(1) in heads and heads[m.group(1)] < i:  # backedge
                lo, hi = heads[m.group(1)], i
                c = collections.Counter()
                waits = []
                for x in body[lo:hi + 1]:
                    t = x.strip().split()
                    if not t or t[0].startswith((";", ".")):
                        continue
                    op = t[0]
                    k = ("mfma" if op.startswith("v_mfma") else "ds_read" if op.startswith("ds_read") else
                         "ds_write" if op.startswith("ds_write") else "lds_dma" if op.startswith("global_load_lds")
                         else "vmem" if op.startswith(("global_", "buffer_")) else "wait" if op == "s_waitcnt"
                         else "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else op)
                    c[k] += 1
                    if op == "s_waitcnt" or op == "s_barrier":
                        waits.append(" ".join(t[1:]) if op == "s_waitcnt" else "BARRIER")
                print(f"{name[:60]} loop lines {lo}-{hi}: {dict(c)}")
                print("   waits:", waits)
                if "-v" in sys.argv:
                    print("\n".join(body[lo:hi + 1]))


if __name__ == "__main__":
    main()
