"""Host logic of the matrix-product modes (no GPU): which forward stages an
encoder plan keeps at f32 accuracy (hip_encoder.forward_stages, $GHM_F32FWD) and
which mode the CDM resolves to by default (cdm.cdm_precision).  The modes'
numerics are the GPU tests' (test_gpu_parity.py MODES, test_gpu_cdm_joint.py,
test_gpu_cdm_guided.py); DESIGN.md section 4b."""
import pytest

from ghmclip.models.cdm import cdm_precision
from ghmclip.models.hip_encoder import ENCODER_PRECISIONS, PRECISIONS, default_precision, forward_stages


def test_forward_stages_per_precision():
    assert forward_stages("x3") == frozenset()
    assert forward_stages("f32") == {"qkv", "attn", "mlp"}
    assert forward_stages("f32x6") == {"qkv6", "attn", "mlp6"}
    assert forward_stages("f32fwd", env={}) == {"qkv6", "mlp6"}  # the guided CLIP default
    assert forward_stages("f32fwd", env={"GHM_F32FWD": "qkv,mlp"}) == {"qkv", "mlp"}
    assert forward_stages("f32fwd", env={"GHM_F32FWD": "qkv,attn,mlp6"}) == {"qkv", "attn", "mlp6"}
    with pytest.raises(ValueError):
        forward_stages("bf16")


@pytest.mark.parametrize("bad", ["mlp,mlp6", "qkv,qkv6", "qkv,gelu"])
def test_forward_stages_reject_conflicting_sets(bad):
    with pytest.raises(ValueError):
        forward_stages("f32fwd", env={"GHM_F32FWD": bad})


def test_mode_lists():
    assert set(PRECISIONS) == {"f32", "x3"}
    assert set(ENCODER_PRECISIONS) == {"f32", "x3", "f32fwd", "f32x6"}


def test_default_precision_env(monkeypatch):
    monkeypatch.setenv("GHM_PRECISION", "f32fwd")
    assert default_precision(allowed=ENCODER_PRECISIONS) == "f32fwd"
    with pytest.raises(ValueError):  # the VLM / GEMM plans take f32 / x3 only
        default_precision()


def test_cdm_precision_defaults(monkeypatch):
    monkeypatch.delenv("GHM_PRECISION", raising=False)
    # (precision, joint, guide, layernorm) -> resolved
    assert cdm_precision(None, True, False, True) == "f32fwd"
    assert cdm_precision(None, True, True, True) == "f32x6"
    assert cdm_precision(None, False, False, True) is None  # sequential: CdmPlan's own default
    assert cdm_precision(None, True, False, False) is None  # no LayerNorm: the GEMM layer stack
    assert cdm_precision("x3", True, True, True) == "x3"    # explicit wins
    monkeypatch.setenv("GHM_PRECISION", "f32")
    assert cdm_precision(None, True, True, True) is None    # the environment wins through CdmPlan
