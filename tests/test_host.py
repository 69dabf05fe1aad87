"""CPU tests of the host side: the C-ABI library loads and exports every
declared symbol (no compute calls without a GPU), the native sampler is
bit-exact against the reference fixtures, and the module API mirrors the
reference (parameter order, init, schedule)."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ghm_[a-z0-9_]+)\s*\(", src)))


def test_hip_library_exports_every_declared_symbol():
    import ctypes
    from ghmclip import _native
    lib = ctypes.CDLL(_native.HIP_LIB)
    names = _declared("ghm_hip.h")
    assert len(names) >= 18
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_native.HIP_SIGNATURES), "ctypes table out of sync with ghm_hip.h"


def _prototypes(header):
    """name -> list of parameter types (ctypes) of every declaration in the header."""
    import ctypes
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//.*", "", src)
    scalar = {"int": ctypes.c_int, "int64_t": ctypes.c_int64, "float": ctypes.c_float,
              "double": ctypes.c_double, "uint32_t": ctypes.c_uint32, "int32_t": ctypes.c_int32}
    out = {}
    for m in re.finditer(r"\b(ghm_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src):
        params = [p.strip() for p in m.group(2).split(",") if p.strip() and p.strip() != "void"]
        types = []
        for p in params:
            p = re.sub(r"\b(const|struct)\b", "", p).strip()
            types.append(ctypes.c_void_p if "*" in p else scalar[p.split()[0]])
        out[m.group(1)] = types
    return out


@pytest.mark.parametrize("header,table", [("ghm_hip.h", "HIP_SIGNATURES"), ("ghm_sampler.h", "HOST_SIGNATURES")])
def test_ctypes_table_matches_header_prototypes(header, table):
    """Every ctypes argtypes list has the header's arity and parameter types
    (pointer -> c_void_p, int64_t -> c_int64, ...), so no caller can shift an
    argument into the wrong slot."""
    from ghmclip import _native
    protos = _prototypes(header)
    sigs = getattr(_native, table)
    assert set(protos) == set(sigs)
    for name, want in protos.items():
        got = sigs[name]
        assert len(got) == len(want) and all(a is b for a, b in zip(got, want)), name


def test_integration_doc_bindings_match_header():
    """The reference-side bindings shown in INTEGRATION.md (`_lib.<fn>.argtypes = ...`
    and the calls `_lib.<fn>(...)` / `_h.<fn>(...)`) have the header's arity and
    types: the doc fails this test as soon as it drifts from include/*.h."""
    import ast
    import ctypes
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", doc, flags=re.S)
    assert blocks
    protos = {**_prototypes("ghm_hip.h"), **_prototypes("ghm_sampler.h")}
    n_argtypes = n_calls = 0
    for code in blocks:
        tree = ast.parse(code)
        for node in ast.walk(tree):
            if (isinstance(node, ast.Assign) and isinstance(node.targets[0], ast.Attribute)
                    and node.targets[0].attr == "argtypes"):
                name = node.targets[0].value.attr
                got = eval(compile(ast.Expression(node.value), "doc", "eval"), {"ctypes": ctypes})
                want = protos[name]
                assert len(got) == len(want) and all(a is b for a, b in zip(got, want)), name
                n_argtypes += 1
            if (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)
                    and isinstance(node.func.value, ast.Name) and node.func.value.id in ("_lib", "_h")
                    and node.func.attr.startswith("ghm_")):
                name = node.func.attr
                nargs = 0
                for a in node.args:  # *x[i:j] with constant bounds counts j - i arguments
                    if isinstance(a, ast.Starred):
                        sl = a.value.slice
                        nargs += sl.upper.value - sl.lower.value
                    else:
                        nargs += 1
                if name in protos:
                    assert nargs == len(protos[name]), f"{name}: {nargs} args"
                    n_calls += 1
    assert n_argtypes >= 1 and n_calls >= 4


def test_libraries_carry_the_source_build_id():
    """Both libraries were built from the sources of this tree (the hash the
    Makefile baked in == the hash recomputed here); smoke() and bench.py make the
    same check on the GPU box."""
    from ghmclip import _native
    from ghmclip._buildid import source_build_id, source_files
    files = source_files()
    assert "Makefile" in files and any(f.endswith("ghm_x3.hip") for f in files)
    assert any(f.endswith("ghm_hip.h") for f in files)
    assert _native.check_build_id() == source_build_id()


def test_host_library_exports_every_declared_symbol():
    import ctypes
    from ghmclip import _native
    lib = ctypes.CDLL(_native.HOST_LIB)
    names = _declared("ghm_sampler.h")
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_native.HOST_SIGNATURES)


@pytest.mark.parametrize("name", ["sampler_p20.npz", "sampler_p40_b16.npz"])
def test_native_sampler_bit_exact(name):
    from ghmclip import ClipSampler, seed_everything
    g = np.load(os.path.join(GOLDEN, name))
    p, B = float(g["p"]), int(g["B"])
    p_y = np.ones(10) / 10
    s = ClipSampler([4, 4], [3, 3], [p_y, p_y], [p, p], K=4, seedtree=42)
    np.testing.assert_array_equal(s.t_templ, g["t_transition"])
    np.testing.assert_array_equal(s.i_templ, g["i_transition"])
    seed_everything(224)
    for b in range(g["t_leaves"].shape[0]):
        t, i = s.get_batch("cpu", B)
        np.testing.assert_array_equal(t[0].numpy(), g["t_leaves"][b])
        np.testing.assert_array_equal(i[0].numpy(), g["i_leaves"][b])
        np.testing.assert_array_equal(t[1].numpy(), g["t_root"][b])
        np.testing.assert_array_equal(i[1].numpy(), g["i_root"][b])


def test_native_rng_matches_numpy_stream():
    from ghmclip import ClipSampler
    p_y = np.ones(10) / 10
    s = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
    import ctypes
    from ghmclip import _native
    lib = _native.host_lib()
    for seed in (0, 1, 224, 2**32 - 1):
        s.native.seed(seed)
        out = np.zeros(3000)
        assert lib.ghm_sampler_random_sample(s.native._h, out.ctypes.data, 3000) == 0
        rs = np.random.RandomState(seed)
        np.testing.assert_array_equal(out, rs.random_sample(3000))
        ch = np.zeros(500, np.int64)
        assert lib.ghm_sampler_choice(s.native._h, 10, 500, ch.ctypes.data) == 0
        np.testing.assert_array_equal(ch, rs.choice(10, size=500))


def test_numpy_state_round_trip():
    """get_batch advances numpy's global RNG exactly like the reference would."""
    from ghmclip import ClipSampler, seed_everything
    from oracle import ghm_oracle as O
    p_y = np.ones(10) / 10
    s = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.3, 0.3], K=3, seedtree=42)
    o = O.ClipSamplerOracle([4, 4], [3, 3], [0.3, 0.3], K=3, seedtree=42)
    seed_everything(5)
    s.get_batch("cpu", 7)
    after_native = np.random.random_sample(5)
    seed_everything(5)
    o.get_batch(7)
    after_oracle = np.random.random_sample(5)
    np.testing.assert_array_equal(after_native, after_oracle)


def test_param_order_and_init_match_oracle():
    from ghmclip import EncoderTransformer
    from ghmclip.models.hip_encoder import param_names
    from oracle import ghm_oracle as O
    torch.manual_seed(224)
    a = EncoderTransformer(81, 10, 128, 3)
    torch.manual_seed(224)
    b = O.OracleEncoder(81, 10, 128, 3)
    assert list(a.state_dict()) == list(b.state_dict()) == param_names(3)
    assert [n for n, _ in a.named_parameters()] == param_names(3)
    for (ka, va), (_, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(va, vb), ka


def test_product_rejects_cpu_tensors():
    from ghmclip import EncoderTransformer
    m = EncoderTransformer(81, 10, 128, 1)
    with pytest.raises(RuntimeError, match="HIP device"):
        m(torch.zeros(2, 81, dtype=torch.long))


def test_lr_schedule_matches_oracle():
    from ghmclip import get_lr_cosine_schedule
    from oracle import ghm_oracle as O
    for t in (0, 1, 5, 1500, 2999, 3000, 3001):
        for w in (0, 10):
            assert get_lr_cosine_schedule(t, 3e-4, 3e-7, w, 3000) == O.lr_cosine(t, 3e-4, 3e-7, w, 3000)


def test_bayes_product_matches_published():
    import json
    from ghmclip import ClipSampler
    with open(os.path.join(GOLDEN, "bayes.json")) as f:
        d = json.load(f)
    p_y = np.ones(10) / 10
    s = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
    bayes, _ = s.get_Bayes(10000)
    np.testing.assert_allclose(bayes, d["Bayes"][9], rtol=1e-12)


def test_guided_targets_host_match_reference():
    """ClipSampler.get_batch(guide=True)'s host BP targets == the reference's
    guided_info on its own draws (tests/golden/guide_bp.npz)."""
    import numpy as np
    from ghmclip.data.data_random_GHM import bp_cls_posterior, guided_targets
    g = np.load(os.path.join(GOLDEN, "guide_bp.npz"))
    for pref in ("t", "i"):
        leaves = g[f"{pref}_leaves"]
        tg = guided_targets(g[f"{pref}_transition"], leaves, "cpu")
        assert len(tg) == 4
        for k, t in enumerate(tg):
            want = g[f"{pref}_msg{k}"]
            ext = 81 // want.shape[1]
            np.testing.assert_allclose(t.numpy(), np.repeat(want, ext, axis=1), rtol=1e-6, atol=1e-6)
        pp = bp_cls_posterior(g[f"{pref}_transition"], leaves, np.ones(10) / 10)
        np.testing.assert_allclose(pp, g[f"{pref}_pp"], rtol=1e-10, atol=1e-12)


def test_sampler_shard_equals_row_slice():
    """ghm_sampler_next_shard (the data-parallel producer) returns exactly
    shard_rows of the full draw and leaves the stream where the full draw does."""
    from ghmclip import ClipSampler
    from ghmclip.training.pipeline import shard_rows
    p_y = np.ones(10) / 10
    full = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
    part = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
    full.native.seed(11)
    part.native.seed(11)
    B, world = 16, 4
    t = np.empty((5 * B, 81), np.uint8)
    i = np.empty((5 * B, 81), np.uint8)
    tr = np.empty(5 * B, np.uint8)
    ir = np.empty(5 * B, np.uint8)
    for step in range(3):
        rank = step % world
        n = B // world
        ts = np.empty((5 * n, 81), np.uint8)
        is_ = np.empty((5 * n, 81), np.uint8)
        trs = np.empty(5 * n, np.uint8)
        irs = np.empty(5 * n, np.uint8)
        full.native.next_into(B, t, i, tr, ir)
        part.native.next_shard_into(B, rank * n, n, ts, is_, trs, irs)
        idx = shard_rows(B, 5, rank, world)
        np.testing.assert_array_equal(ts, t[idx])
        np.testing.assert_array_equal(is_, i[idx])
        np.testing.assert_array_equal(trs, tr[idx])
        np.testing.assert_array_equal(irs, ir[idx])
    k1, p1 = full.native.get_state()
    k2, p2 = part.native.get_state()
    assert p1 == p2 and (k1 == k2).all()


@pytest.mark.parametrize("world", [2, 4])
def test_batch_pipeline_producer_shards(world):
    """BatchPipeline(row_slice=(B, rank, world)) — the producer train_CLIP runs
    on every rank — fills its slots with exactly shard_rows of the global draws,
    in order, for every rank."""
    from ghmclip import ClipSampler
    from ghmclip.training.pipeline import BatchPipeline, shard_rows
    p_y = np.ones(10) / 10
    B = 16
    full = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
    full.native.seed(5)
    t = np.empty((5 * B, 81), np.uint8)
    i = np.empty((5 * B, 81), np.uint8)
    draws = []
    for _ in range(2):
        full.native.next_into(B, t, i)
        draws.append((t.copy(), i.copy()))
    for rank in range(world):
        s = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
        s.native.seed(5)
        pipe = BatchPipeline(s.native, B, n_slots=2, row_slice=(B, rank, world))
        try:
            idx = shard_rows(B, 5, rank, world)
            for k in range(2):
                assert pipe.ready[k].wait(timeout=30)
                ts, is_ = pipe.slots[k]
                assert ts.shape == (5 * B // world, 81)
                np.testing.assert_array_equal(ts.numpy(), draws[k][0][idx])
                np.testing.assert_array_equal(is_.numpy(), draws[k][1][idx])
        finally:
            pipe.close()


def test_sampler_usable_after_fork():
    """A handle created before fork() draws in the child (serially: the parent's
    worker threads do not exist there) the same batch the parent draws from
    the same state — no deadlock (ghm_sampler.h, fork note)."""
    import os
    from ghmclip import ClipSampler
    p_y = np.ones(10) / 10
    s = ClipSampler([4, 4], [3, 3], [p_y, p_y], [0.2, 0.2], K=4, seedtree=42)
    s.native.seed(3)
    B = 32
    t = np.empty((5 * B, 81), np.uint8)
    i = np.empty((5 * B, 81), np.uint8)
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:  # child: draw, send, exit without running the parent's atexit handlers
        try:
            s.native.next_into(B, t, i)
            os.write(w, t.tobytes() + i.tobytes())
        finally:
            os._exit(0)
    os.close(w)
    buf = b""
    while True:
        chunk = os.read(r, 1 << 16)
        if not chunk:
            break
        buf += chunk
    os.close(r)
    os.waitpid(pid, 0)
    s.native.next_into(B, t, i)
    assert buf == t.tobytes() + i.tobytes()


def test_bench_finds_the_dominant_kernels_stamped_twin():
    """bench.py's roofline line reads the dominant kernel and its serialized-measurement
    twin (STAMP 1 of the same instantiation) from the newest committed kernel
    statistics; a template argument added to the kernel must not lose the twin
    (round 5: profile_avg_ms was null until the lookup parsed the arguments)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b._rc_twin("k_mlp_bwd_rc_x3<8, 0, false>", 1) == "k_mlp_bwd_rc_x3<8, 1, false>"
    assert b._rc_twin("k_mlp_bwd_rc_x3<8, 0, 0>", 1) == "k_mlp_bwd_rc_x3<8, 1, 0>"  # (SPLITOUT an int since round 6)
    assert b._rc_twin("k_mlp_bwd_rc_x3<8, 0>", 2) == "k_mlp_bwd_rc_x3<8, 2>"
    assert b._rc_twin("k_wgrad_x3<0, 4, 128, 512>", 1) is None
    path, prof = b.profiled_kernels()
    assert path is not None
    rc = [k for k in prof if k.startswith("k_mlp_bwd_rc_x3<") and b._rc_twin(k, 0) == k]
    assert rc and all(b._rc_twin(k, 1) in prof for k in rc), (path, sorted(prof))
    assert b.pmc_traffic("k_mlp_bwd_rc_x3") is not None
    # the VLM line's roofline kernel (the instantiation its step launches: the pre-split
    # weight images, V = 5, the default since round 6) in the VLM traffic passes
    assert b.pmc_traffic("k_gemm_x3<false, true, 1, 2, false, 5, 128>", "traffic_vlm.json") > 0
