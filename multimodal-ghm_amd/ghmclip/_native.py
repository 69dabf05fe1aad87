"""ctypes bindings of the in-tree native libraries.

libghm_hip.so  — HIP (gfx950) kernels behind the C ABI in include/ghm_hip.h
libghm_host.so — host GHM sampler behind include/ghm_sampler.h

There is no fallback: if a library is missing or a call fails, a RuntimeError
is raised.  Build them with ``make`` (or ``__graft_entry__.build()``).
"""
import ctypes
import os

_LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
HIP_LIB = os.environ.get("GHM_HIP_LIB") or os.path.join(_LIBDIR, "libghm_hip.so")
HOST_LIB = os.path.join(_LIBDIR, "libghm_host.so")

_p = ctypes.c_void_p


class ReduceJob(ctypes.Structure):
    """ghm_reduce_job (include/ghm_hip.h)."""
    _fields_ = [("part", ctypes.c_void_p), ("n_split", ctypes.c_int32), ("n_seg", ctypes.c_int32),
                ("n", ctypes.c_int64), ("dst", ctypes.c_void_p * 4), ("off", ctypes.c_int64 * 5)]


class SplitJob(ctypes.Structure):
    """ghm_split_job (include/ghm_hip.h)."""
    _fields_ = [("Wq", ctypes.c_void_p), ("Wk", ctypes.c_void_p), ("Wv", ctypes.c_void_p),
                ("W1", ctypes.c_void_p), ("W2", ctypes.c_void_p), ("pack", ctypes.c_void_p)]


GHM_SPLIT_PACK_ELEMS = 983040  # include/ghm_hip.h
GHM_SPLIT3_PACK_ELEMS = 180224  # include/ghm_hip.h

_i = ctypes.c_int
_i64 = ctypes.c_int64
_f = ctypes.c_float
_u32 = ctypes.c_uint32

# name -> argtypes (restype int unless listed in _RESTYPE)
HIP_SIGNATURES = {
    "ghm_last_error_string": [],
    "ghm_device_ok": [],
    "ghm_build_id": [],
    "ghm_token_blocks": [_i64],
    "ghm_mlp_bwd_rc_x3_blocks": [_i64],
    "ghm_embed_fwd": [_p, _p, _p, _p, _i64, _i, _i, _i, _p],
    "ghm_ln_qkv_fwd": [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _f, _p],
    "ghm_attn_fwd": [_p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_ln_mlp_fwd": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_readout_fwd": [_p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _p],
    "ghm_clip_loss": [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p],
    "ghm_readout_bwd": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _p],
    "ghm_readout_bwd_clip": [_p, _p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _p],
    "ghm_embed_bwd_splits": [],
    "ghm_embed_bwd_part_elems": [_i, _i],
    "ghm_embed_bwd_part": [_p, _p, _i64, _i, _i, _i, _p, _p],
    "ghm_mlp_bwd": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _p],
    "ghm_attn_bwd": [_p, _p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_qkv_bwd": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _p],
    "ghm_wgrad": [_p, _i, _i, _p, _i, _i, _i, _p, _p, _p, _p, _p, _i64, _i, _p],
    "ghm_reduce_partials": [_p, _i, _i64, _i, _p, _p, _p],
    "ghm_reduce_batch": [_p, _i, _p],
    "ghm_clip_prepare": [_p, _i64, _f, _p, _i, _p, _p, _p, _p],
    "ghm_split_weights": [_p, _i, _p],
    "ghm_cdm_embed_fwd": [_p, _p, _i, _p, _p, _i64, _i, _i, _i, _i, _p],
    "ghm_cdm_embed_joint_fwd": [_p, _p, _p, _p, _p, _i64, _i, _i, _i, _i, _p],
    "ghm_bp_dns": [_p, _p, _p, _p, ctypes.c_double, _p, _p, _i64, _i, _i, _i, _i, _i, _i, _p],
    "ghm_bp_dns_msgs": [_p, _p, _p, _p, ctypes.c_double, _p, _p, _p, _i64, _i, _i, _i, _i, _i, _i, _p],
    "ghm_guide_blk_fwd": [_p, _i, _i, _i, _i, _p, _i64, _i64, _i, _i, _p, _i64, _p],
    "ghm_guide_blk_bwd": [_p, _i, _i, _i, _i, _p, _i64, _i64, _i, _i, _p, _f, _i64, _p],
    "ghm_guide_blks_fwd": [_p, _p, _p, _p, _i, _p, _i64, _p],
    "ghm_guide_blks_bwd": [_p, _p, _p, _p, _i, _p, _f, _i64, _p],
    "ghm_guide_blks_fwd_d": [_p, _p, _p, _p, _i, _i, _p, _i64, _p],
    "ghm_guide_blks_bwd_d": [_p, _p, _p, _p, _i, _i, _p, _f, _i64, _p],
    "ghm_guide_max_blocks": [],
    "ghm_cdm_readout_fwd": [_p, _p, _p, _p, _i64, _i, _i, _i, _p],
    "ghm_ls_loss": [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _p],
    "ghm_cdm_readout_bwd": [_p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _p],
    "ghm_vlm_embed_fwd": [_p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _i, _p],
    "ghm_vlm_embed_joint_fwd": [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _i, _p],
    "ghm_ln_rows_fwd": [_p, _p, _p, _p, _p, _i64, _i, _f, _p],
    "ghm_ln_rows_blocks": [_i64],
    "ghm_ln_rows_bwd": [_p, _p, _p, _p, _p, _p, _p, _i64, _i, _p],
    "ghm_vlm_attn_fwd": [_p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _f, _p],
    "ghm_vlm_attn_bwd": [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_gelu_fwd": [_p, _p, _p, _i64, _p],
    "ghm_gemm_slab_elems": [_i64, _i64, _i],
    "ghm_vlm_attn_fwd_x3": [_p, _p, _p, _p, _i64, _i, _i, _i, _f, _p],
    "ghm_vlm_attn_bwd_x3": [_p, _p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_attn_ext_fwd_x3": [_p, _p, _p, _p, _i64, _i, _i, _i, _f, _f, _p],
    "ghm_attn_ext_bwd_x3": [_p, _p, _p, _p, _p, _i64, _i, _i, _i, _f, _f, _p],
    "ghm_attn_ext_fwd_x3_act": [_p, _p, _p, _p, _p, _i64, _i, _i, _i, _f, _f, _i, _p],
    "ghm_attn_ext_bwd_x3_act": [_p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _f, _f, _i, _p],
    "ghm_gemm_x3": [_i, _i, _i, _p, _i64, _p, _p, _p, _i64, _i64, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64,
                    _i, _p],
    "ghm_event_create": [_i],
    "ghm_event_destroy": [_p],
    "ghm_event_record": [_p, _p],
    "ghm_stream_wait": [_p, _p],
    "ghm_gemm_f32": [_i, _i, _i, _p, _i64, _p, _p, _p, _i64, _i64, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64,
                     _i, _p],
    "ghm_gemm_x3p": [_i, _p, _i64, _p, _i64, _i64, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _i, _p],
    "ghm_split_pack": [_p, _i, _i, _p],
    "ghm_gemm_reduce": [_p, _i, _i64, _i64, _p, _p, _p, _i64, _p],
    "ghm_gemm_reduce_bias": [_p, _i, _i64, _i64, _p, _p, _p, _i64, _p, _p, _p],
    "ghm_colsum_part_elems": [_i64, _i64],
    "ghm_colsum": [_p, _i64, _i64, _p, _p, _p],
    "ghm_wcolsum_part_elems": [_i64, _i64, _i],
    "ghm_wcolsum": [_p, _p, _i, _p, _i64, _i64, _i64, _i64, _i64, _p, _p, _p, _p],
    "ghm_rows_linear": [_p, _p, _p, _p, _i64, _i, _i, _p],
    "ghm_rows_linear_t": [_p, _p, _p, _i64, _i, _i, _p],
    "ghm_tok_embed_fwd": [_p, _p, _p, _p, _i64, _i, _i, _i, _p],
    "ghm_tok_readout_fwd": [_p, _p, _p, _p, _i64, _i, _i, _p],
    "ghm_tok_readout_bwd": [_p, _p, _p, _p, _p, _p, _i64, _i, _i, _p],
    "ghm_mul": [_p, _p, _p, _i64, _p],
    "ghm_add": [_p, _p, _p, _i64, _p],
    "ghm_ce_kl": [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _p],
    "ghm_ce_kl_out_elems": [_i64, _i, _i],
    "ghm_ln_qkv_fwd_x3": [_p, _p, _p, _p, _p, _p, _i64, _i, _f, _p],
    "ghm_ln_mlp_fwd_x3b": [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_ln_qkv_fwd_x3s": [_p, _p, _p, _p, _p, _p, _p, _i64, _i, _f, _p],
    "ghm_ln_mlp_fwd_x3bs": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_split3_weights": [_p, _i, _p],
    "ghm_ln_qkv_fwd_x6": [_p, _p, _p, _p, _p, _p, _p, _i64, _i, _f, _p],
    "ghm_ln_mlp_fwd_x6": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_wgrad_x3p": [_p, _i, _i, _p, _i, _i, _i64, _p, _p, _i64, _i, _p],
    "ghm_mlp_bwd_rc_x3": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _p],
    "ghm_mlp_bwd_rc_x3_stamped": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _p, _i, _p],
    "ghm_qkv_bwd_x3": [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _f, _p],
    "ghm_qkv_bwd_x3_probe": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _f, _i, _p],
    "ghm_wgrad_x3": [_p, _i, _i, _p, _i, _i, _i, _p, _p, _p, _p, _p, _i64, _i, _p],
    "ghm_wgrad_ring_x3": [_p, _i, _i, _i, _i64, _p, _i, _i, _i, _i64, _p, _p, _p, _p, _p, _i64, _i, _p],
    "ghm_attn_fwd_x3": [_p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_attn_bwd_x3": [_p, _p, _p, _p, _p, _i64, _i, _i, _f, _p],
    "ghm_attn_fwd_act": [_p, _p, _p, _p, _p, _i64, _i, _i, _f, _i, _p],
    "ghm_attn_bwd_act": [_p, _p, _p, _p, _p, _p, _i64, _i, _i, _f, _i, _p],
    "ghm_attn_fwd_x3_act": [_p, _p, _p, _p, _p, _i64, _i, _i, _f, _i, _p],
    "ghm_attn_bwd_x3_act": [_p, _p, _p, _p, _p, _i64, _i, _i, _f, _i, _p],
    "ghm_bp_cls": [_p, _p, _p, _i64, _i, _i, _i, _i, _p],
    "ghm_guide_fwd": [_p, _p, _p, _i64, _i, _i, _i, _i, _p],
    "ghm_guide_bwd": [_p, _p, _p, _i64, _i, _i, _i, _i, _f, _p],
    "ghm_guide_total": [_p, _i, _i64, _f, _p, _p, _p, _p],
    "ghm_sqdiff_rows": [_p, _p, _p, _i64, _i64, _p],
    "ghm_scaled_diff": [_p, _p, _p, _f, _p, _i64, _p],
    "ghm_add_cols": [_p, _p, _i64, _i, _p],
    "ghm_adamw": [_p, _p, _p, _p, _i64, _p, _f, _f, _f, _f, _f, _p],
    "ghm_zsc_logits": [_p, _i64, _p, _i, _p, _i, _i, _p, _i, _p, _p],
}
_RESTYPE = {"ghm_last_error_string": ctypes.c_char_p, "ghm_build_id": ctypes.c_char_p, "ghm_event_create": ctypes.c_void_p, "ghm_embed_bwd_part_elems": _i64, "ghm_embed_bwd_splits": _i, "ghm_guide_max_blocks": _i, "ghm_token_blocks": _i64,
            "ghm_mlp_bwd_rc_x3_blocks": _i64,
            "ghm_ln_rows_blocks": _i64, "ghm_gemm_slab_elems": _i64, "ghm_colsum_part_elems": _i64,
            "ghm_wcolsum_part_elems": _i64,
            "ghm_ce_kl_out_elems": _i64}

HOST_SIGNATURES = {
    "ghm_sampler_create": [_p, _p, _i, _i, _i, _i],
    "ghm_sampler_create_edges": [_p, _i, _i, _p, _i, _i, _i, _i],
    "ghm_sampler_destroy": [_p],
    "ghm_sampler_build_id": [],
    "ghm_sampler_seed": [_p, _u32],
    "ghm_sampler_set_state": [_p, _p, _i],
    "ghm_sampler_get_state": [_p, _p, _p],
    "ghm_sampler_next": [_p, _i, _p, _p, _p, _p],
    "ghm_sampler_next_shard": [_p, _i, _i, _i, _p, _p, _p, _p],
    "ghm_sampler_random_sample": [_p, _p, _i64],
    "ghm_sampler_choice": [_p, _i, _i64, _p],
    "ghm_sampler_next_cdm": [_p, _i, ctypes.c_double, _p, _p, _p, _p],
    "ghm_sampler_set_gauss": [_p, _i, ctypes.c_double],
    "ghm_sampler_get_gauss": [_p, _p, _p],
    "ghm_sampler_randn": [_p, _p, _i64],
}
_HOST_RESTYPE = {"ghm_sampler_create": ctypes.c_void_p, "ghm_sampler_create_edges": ctypes.c_void_p,
                 "ghm_sampler_destroy": None, "ghm_sampler_build_id": ctypes.c_char_p}

_hip = None
_host = None


def _load(path, sigs, restypes):
    if not os.path.exists(path):
        raise RuntimeError(f"native library missing: {path} (run `make` in the repo root)")
    lib = ctypes.CDLL(path)
    for name, args in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = restypes.get(name, ctypes.c_int)
    return lib


def hip_lib():
    """The HIP kernel library (loaded once)."""
    global _hip
    if _hip is None:
        _hip = _load(HIP_LIB, HIP_SIGNATURES, _RESTYPE)
    return _hip


def host_lib():
    """The host sampler library (loaded once)."""
    global _host
    if _host is None:
        _host = _load(HOST_LIB, HOST_SIGNATURES, _HOST_RESTYPE)
    return _host


def check_build_id():
    """The source hash both loaded libraries were built from, checked against the
    tree this process runs in (ghmclip/_buildid.py); raises on a mismatch (a
    stale or foreign binary).  Returns the id."""
    from ._buildid import source_build_id
    want = source_build_id()
    got = hip_lib().ghm_build_id().decode()
    if os.environ.get("GHM_HIP_LIB") and got.startswith("variant-"):
        return got  # an explicit A/B variant library (tools/build_variant.sh): reported, not the tree's
    got_host = host_lib().ghm_sampler_build_id().decode()
    if got != want or got_host != want:
        raise RuntimeError(f"native libraries were built from other sources: libghm_hip {got}, "
                           f"libghm_host {got_host}, tree {want} (run `make`)")
    return got


def check(rc, what):
    if rc != 0:
        msg = hip_lib().ghm_last_error_string()
        raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def call(name, *args):
    """Call a libghm_hip entry point and raise on a non-zero status."""
    check(getattr(hip_lib(), name)(*args), name)
