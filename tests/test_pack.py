"""MLP weight packing: the fused kernel's fragment layout, run through a numpy
emulation of its MFMA dataflow, reproduces the oracle MLP (CPU only)."""
import numpy as np
import pytest

from nerfhip.pack import SLICES, SLICE_FLOATS, HEAD_FLOATS, col_act, emulate, pack_mlp
from nerfhip.synthetic import make_params
from oracle import nerf_oracle as O


@pytest.mark.parametrize("seed,gain,prefix", [(0, 2.0, "model"), (1, 3.0, "model_fine")])
def test_packed_network_matches_oracle(seed, gain, prefix):
    p = make_params(seed, gain, 1.0)
    sl, hd = pack_mlp(p, prefix)
    assert sl.shape == (SLICES * SLICE_FLOATS,) and hd.shape == (HEAD_FLOATS,)
    rng = np.random.default_rng(seed)
    pts = rng.uniform(-2, 2, (33, 3)).astype(np.float32)
    d = rng.normal(size=(33, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    x = np.concatenate([O.embed(pts, 10), O.embed(d, 4)], -1)
    ref = O.nerf_mlp(x, p, prefix)
    em = emulate(sl, hd, pts, d)
    scale = np.maximum(1.0, np.abs(ref).max(0))
    assert (np.abs(em - ref) / scale).max() < 2e-5


def test_act_permutation_is_a_bijection():
    for h in (0, 1):
        pass
    cols = np.concatenate([col_act(np.arange(64), g) for g in range(4)])
    assert sorted(cols.tolist()) == list(range(256))


def test_padding_slices_are_zero():
    sl, _ = pack_mlp(make_params(0), "model")
    used = (2 + 8 * 4 + 10 + 8 * 2 + 8) * 32 + 144     # blocks actually consumed
    assert not sl.reshape(-1, 256)[used:].any()
