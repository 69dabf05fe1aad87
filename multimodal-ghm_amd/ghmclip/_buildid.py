"""Source hash baked into the native libraries (ghm_build_id / ghm_sampler_build_id).

sha256 over the sorted relative paths and bytes of every file the libraries are
built from (multimodal-ghm_amd/csrc/*, include/*.h, Makefile).  The Makefile
bakes it in at build time (tools/build_id.py); smoke() and bench.py recompute
it from the tree they run in and require the loaded library to carry the same
value, so a run names the sources of the binary it exercised.  No imports
beyond the standard library: the build script loads this file by path.
"""
import hashlib
import os

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def source_files(root=REPO):
    csrc = os.path.join("multimodal-ghm_amd", "csrc")
    files = [os.path.join(csrc, f) for f in os.listdir(os.path.join(root, csrc))]
    files += [os.path.join("include", f) for f in os.listdir(os.path.join(root, "include")) if f.endswith(".h")]
    files.append("Makefile")
    return sorted(f for f in files if os.path.isfile(os.path.join(root, f)))


def source_build_id(root=REPO):
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.replace(os.sep, "/").encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
