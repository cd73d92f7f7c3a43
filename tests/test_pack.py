"""MLP weight packing: the fused kernel's fragment layout, run through a numpy
emulation of its MFMA dataflow, reproduces the oracle MLP (CPU only)."""
import numpy as np
import pytest

from nerfhip.pack import (H_SCALES, HEAD_FLOATS, SLICE_FLOATS, SLICES, X3_SLICES, col_act, emulate,
                          emulate_x3, pack_mlp, pack_mlp_x3, x3_cols_act, x3_cols_dir,
                          x3_cols_enc)
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
    cols = np.concatenate([col_act(np.arange(64), g) for g in range(4)])
    assert sorted(cols.tolist()) == list(range(256))


def test_padding_slices_are_zero():
    sl, _ = pack_mlp(make_params(0), "model")
    used = (2 + 8 * 4 + 10 + 8 * 2 + 8) * 32 + 144     # blocks actually consumed
    assert not sl.reshape(-1, 256)[used:].any()


# ---------------------------------------------------------------- FP16 x3 layout
@pytest.mark.parametrize("seed,gain,prefix", [(0, 2.0, "model"), (1, 3.0, "model_fine"),
                                              (2, 0.05, "model")])
def test_x3_packed_network_matches_oracle(seed, gain, prefix):
    """3-term FP16 split (exact products): within 1e-5 of the FP32 oracle, at
    normal and at tiny weight scales (the power-of-two scaling keeps the splits
    in FP16's normal range)."""
    p = make_params(seed, gain, 1.0)
    sl, hd = pack_mlp_x3(p, prefix)
    assert sl.shape == (X3_SLICES * SLICE_FLOATS,) and hd.shape == (HEAD_FLOATS,)
    assert np.all(hd[H_SCALES:H_SCALES + 10] >= 0)
    rng = np.random.default_rng(seed)
    pts = rng.uniform(-2, 2, (65, 3)).astype(np.float32)
    d = rng.normal(size=(65, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    x = np.concatenate([O.embed(pts, 10), O.embed(d, 4)], -1)
    ref = O.nerf_mlp(x, p, prefix)
    em = emulate_x3(sl, hd, pts, d)
    scale = np.maximum(np.abs(ref).max(0), 1e-30)
    assert (np.abs(em - ref) / scale).max() < 1e-5


def test_x3_k_maps_cover_inputs_once():
    enc = x3_cols_enc().reshape(-1)
    assert sorted(enc[enc >= 0].tolist()) == list(range(63))
    dr = x3_cols_dir().reshape(-1)
    assert sorted(dr[dr >= 0].tolist()) == list(range(27))
    assert sorted(x3_cols_act().reshape(-1).tolist()) == list(range(256))
