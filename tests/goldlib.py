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
    if "w_seed" not in z:   # stored weights (another topology, the reference's own init)
        return {k[3:]: z[k] for k in z if k.startswith("wt_")}
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


# --------------------------------------------------------------------------
# End-to-end fine-map gate against the reference's own float32 noise floor.
#
# tests/golden/s_<fixture>.npz (make_sensitivity.py) holds, per ray, the largest
# deviation of the reference from its own golden render over 16 exact
# reparametrisations of the network (hidden units permuted: same function,
# another GEMM summation order; half of them also with a +-1-ulp libm). The
# reference itself keeps only 46-85 % of rays within 1e-5 on the fine maps of
# the C2-type synthetic fixtures (VR:239-268 is
# ill-conditioned in the coarse weights' rounding), so a fixed 1e-5 on every
# ray is not a property any float32 implementation has. The gate instead holds
# an implementation to that floor ray by ray:
#   (1) >= 99 % of rays: |err| <= 4 x max(tol, reference spread) on every map
#   (2) fraction of rays within tol >= the worst reparametrised reference - 0.02
#   (3) fine rgb PSNR vs golden >= min(80 dB, median reparametrised PSNR - 6 dB)
# where tol = 1e-5 abs (rgb, acc), 1e-5 x max(1, |depth|) (depth) and
# 1e-4 x max(1e-3, |disp|) (disp); a NaN-pattern change is an infinite error
# unless the reference itself flipped NaN on that ray.
# --------------------------------------------------------------------------
FINE_KEYS = ("rgb_map", "acc_map", "depth_map", "disp_map")
GATE_RATIO = 4.0
GATE_FRAC = 0.99


def _tol(key, ref):
    if key.startswith("depth"):
        return 1e-5 * np.maximum(1.0, np.abs(ref))
    if key.startswith("disp"):
        return 1e-4 * np.maximum(1e-3, np.abs(np.nan_to_num(ref)))
    return np.full(ref.shape, 1e-5)


def ray_errors(res, z, n, keys=FINE_KEYS):
    """key -> (per-ray max abs error, per-ray tolerance) against the golden maps."""
    out = {}
    for k in keys:
        a = np.asarray(res[k], np.float64).reshape(n, -1)
        b = np.asarray(z["out_" + k], np.float64).reshape(n, -1)
        e = np.nan_to_num(np.abs(a - b), nan=0.0).max(-1)
        e[(np.isnan(a) != np.isnan(b)).any(-1)] = np.inf
        tol = _tol(k, np.nan_to_num(b, nan=0.0)).max(-1)
        out[k] = (e, tol)
    return out


def load_zall(name):
    """z_<fixture>.npz (make_golden.py --zall): the reference's fine depths of every
    ray and its per-call chunk termination decisions, or None."""
    p = os.path.join(GOLDEN, "z_" + name + ".npz")
    return dict(np.load(p)) if os.path.exists(p) else None


REF_CHUNK = 2048


def row_hash(rows):
    """32-bit FNV-1a-style hash of each row's float32 bit patterns ([n, k] -> uint32 [n]).
    Equal rows give equal hashes; the whole-frame fixtures store the reference's
    fine depths this way (make_ref_frames.py --zall)."""
    w = np.ascontiguousarray(np.asarray(rows, np.float32)).view(np.uint32).astype(np.uint64)
    h = np.full(w.shape[0], 0xCBF29CE484222325, np.uint64)
    p = np.uint64(0x100000001B3)
    with np.errstate(over="ignore"):
        for j in range(w.shape[1]):
            h = (h ^ w[:, j]) * p
    return ((h >> np.uint64(32)) ^ (h & np.uint64(0xFFFFFFFF))).astype(np.uint32)


def attribute_tail(ratio, z, zref, zall_hip):
    """(4) Every ray outside GATE_RATIO x the reference's spread must be explained
    by sampling, not by the MLP or the composite: its fine depths differ from the
    reference's (VR:239-268 searchsorted / denom-clamp flips move a fine sample), or
    - with ERT, whose termination rule is chunk-wide (VR:1115-1123) - some ray of
    its 2048-ray chunk has different fine depths. Given identical depths the fine
    pass is held to 1e-5 separately (test_fine_pass_given_reference_depths), so a
    tail ray with identical depths across its chunk would be a kernel defect.
    Returns (tail rays, unexplained rays, rays with different depths)."""
    n = ratio.shape[0]
    zr = zref["zall"].reshape(n, -1)
    zh = np.asarray(zall_hip).reshape(n, -1)
    ddiff = (zr != zh).any(-1)
    expl = ddiff.copy()
    if bool(z["enable_ert"]):
        ch = np.arange(n) // REF_CHUNK
        cd = np.zeros(ch.max() + 1, bool)
        np.logical_or.at(cd, ch, ddiff)
        expl |= cd[ch]
    tail = ratio > GATE_RATIO
    return tail, tail & ~expl, ddiff


def fine_gate(res, z, s, zref=None, zall_hip=None):
    """Evaluate the three criteria above (and, given the reference's fine depths
    of every ray `zref` and the implementation's `zall_hip`, the tail attribution
    of attribute_tail as a fourth); returns (ok, report dict)."""
    n = int(z["H"]) * int(z["W"])
    errs = ray_errors(res, z, n)
    ratio = np.zeros(n)
    within = np.ones(n, bool)
    for k, (e, tol) in errs.items():
        sp = s["spread_" + k].astype(np.float64)
        r = np.where(np.isinf(sp), 0.0, e / np.maximum(sp, tol))
        ratio = np.maximum(ratio, r)
        if k != "disp_map":
            within &= e <= tol
    p = psnr(np.reshape(res["rgb_map"], (n, 3)), np.reshape(z["out_rgb_map"], (n, 3)))
    vp = np.asarray(s["variant_psnr"], np.float64)
    rep = {"frac_ratio_ok": float(np.mean(ratio <= GATE_RATIO)),
           "frac_within_tol": float(within.mean()),
           "ref_self_frac_within_tol_min": float(np.min(s["variant_frac_ok"])),
           "psnr": p, "ref_self_psnr_median": float(np.median(vp)),
           "worst_ratio": float(ratio.max()), "n": n}
    ok = (rep["frac_ratio_ok"] >= GATE_FRAC
          and rep["frac_within_tol"] >= rep["ref_self_frac_within_tol_min"] - 0.02
          and p >= min(80.0, rep["ref_self_psnr_median"] - 6.0))
    if zref is not None and zall_hip is not None:
        tail, unexpl, ddiff = attribute_tail(ratio, z, zref, zall_hip)
        rep.update(tail_rays=int(tail.sum()), tail_unexplained=int(unexpl.sum()),
                   rays_with_other_fine_depths=int(ddiff.sum()),
                   tail_unexplained_worst_ratio=float(ratio[unexpl].max()) if unexpl.any() else 0.0)
        ok = ok and not unexpl.any()
    return ok, rep
