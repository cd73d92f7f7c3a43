"""Helpers shared by the golden-fixture tests (CPU oracle and GPU parity)."""
from __future__ import annotations

import os

import numpy as np

from nerfhip.synthetic import make_occupancy_grid, make_params, params_digest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

MAP_KEYS = ("rgb_map_0", "disp_map_0", "acc_map_0", "depth_map_0",
            "rgb_map", "disp_map", "acc_map", "depth_map")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def params_of(z):
    p = make_params(int(z["w_seed"]), float(z["w_gain"]), float(z["w_alpha_bias"]))
    assert params_digest(p) == str(z["w_digest"]), "weight generator drifted from fixture"
    return p


def grid_of(z):
    if "grid_seed" not in z:
        return None
    return make_occupancy_grid(int(z["grid_seed"]), 128, float(z["grid_radius"]),
                               float(z["grid_noise"]))


def oracle_cfg(z, **kw):
    from oracle.nerf_oracle import RenderConfig
    return RenderConfig(N_samples=int(z["N_samples"]), N_importance=int(z["N_importance"]),
                        near=float(z["near"]), far=float(z["far"]), lindisp=bool(z["lindisp"]),
                        perturb=float(z["perturb"]), enable_ess=bool(z["enable_ess"]),
                        enable_ert=bool(z["enable_ert"]), ert_threshold=float(z["ert_threshold"]),
                        white_bkgd=bool(z["white_bkgd"]), **kw)


def max_err(a, b, nan_aware=True):
    """max |a-b| over entries where the reference is finite; NaN positions must agree."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if nan_aware:
        if not np.array_equal(np.isnan(a), np.isnan(b)):
            return np.inf
        m = ~np.isnan(b)
        return float(np.abs(a[m] - b[m]).max()) if m.any() else 0.0
    return float(np.abs(a - b).max())


def rel_err(a, b, floor=1.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if not np.array_equal(np.isnan(a), np.isnan(b)):
        return np.inf
    m = ~np.isnan(b)
    if not m.any():
        return 0.0
    return float((np.abs(a[m] - b[m]) / np.maximum(floor, np.abs(b[m]))).max())


def psnr(a, b):
    mse = float(np.mean((np.clip(a, 0, 1).astype(np.float64) - np.clip(b, 0, 1)) ** 2))
    return float("inf") if mse == 0 else -10.0 * np.log10(mse)
