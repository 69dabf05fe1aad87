"""Fixtures of the CLIP encoders with a non-softmax attention activation
(train_CLIP.py --clip_activation=relu|gelu -> EncoderTransformer(activation=...),
models/model.py:121-130 get_activation, applied at :781).

Run ONLY in the build container (imports the reference from /root/reference/src
through make_golden.py; only the .npz data is committed):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_act.py

clip_d128_relu.npz / clip_d128_gelu.npz: the d=128, L=2, B=8 config of
clip_d128.npz for 2 steps (embeddings, loss, gradient and post-step weight
checksums), same seeds and draws.
"""
import make_golden as G

if __name__ == "__main__":
    for act in ("relu", "gelu"):
        G.step_fixture(f"clip_d128_{act}.npz", L=2, d=128, B=8, nsteps=2, checksum_only=True, activation=act)
