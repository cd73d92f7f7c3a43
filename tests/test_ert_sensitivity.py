"""The reference's own ERT-cut spread on the ESS + ERT whole frames
(tests/golden/rs_r2_c4_frame16.npz, rs_r3_c4_yaml_frame24.npz, made by
make_ert_sensitivity.py: whole 2048-ray chunks re-rendered by the reference on
16 exact reparametrisations of its network). test_gpu_frames.py exempts a ray
from the on-reference-depths gate only when its cut sits at the threshold by
the oracle AND moves under one of these variants; here the fixtures are
checked for consistency with the reference's own frame records (zh_*.npz)."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FRAMES = ["r2_c4_frame16", "r3_c4_yaml_frame24"]


@pytest.mark.parametrize("name", FRAMES)
def test_ert_spread_fixture_consistent(name):
    p = os.path.join(GOLDEN, f"rs_{name}.npz")
    if not os.path.exists(p):
        pytest.skip(f"{p} not captured")
    fs = np.load(p)
    zh = np.load(os.path.join(GOLDEN, f"zh_{name}.npz"))
    pix, chunks = fs["pixels"].astype(np.int64), fs["chunks"].astype(np.int64)
    assert np.array_equal(pix, np.concatenate([np.arange(c * 2048, (c + 1) * 2048) for c in chunks]))
    K = int(fs["k_variants"])
    assert fs["cut_var"].shape == (K, len(pix)) and fs["cut_ref"].shape == (len(pix),)
    assert fs["chunk_any_var"].shape == (K, len(chunks))
    # the unpermuted network's chunk decisions are the stored frame's (VR:1116)
    assert np.array_equal(fs["chunk_any_ref"], zh["chunk_any"][2 * chunks + 1])
    per_chunk = (fs["cut_ref"].reshape(len(chunks), 2048) >= 0).any(1)
    assert np.array_equal(per_chunk, fs["chunk_any_ref"])
    # every candidate (the oracle's T within the band of thr) lies in a captured chunk,
    # and the reference itself moves the cut of some of them
    cand = fs["cand_pixels"].astype(np.int64)
    assert np.isin(cand, pix).all() and (fs["cand_rel"] < float(fs["band"])).all()
    pos = np.searchsorted(pix, cand)
    moved = (fs["cut_var"][:, pos] != fs["cut_ref"][pos][None]).any(0)
    assert moved.any()
    # the variants are the reference's rounding spread, not a different render
    assert min(fs["variant_frac_ok"]) > 0.99
