"""Capture the reference renderer's own float32 noise floor per ray (survey container).

The fine maps of the reference (``volume_renderer.py:145-216``) are an
ill-conditioned function of the coarse MLP's float32 rounding: fine depths come
from a searchsorted over the coarse weights (VR:239-268), the `denom < 1e-5`
clamp (VR:263-264) and the ERT cut (VR:1115-1123) are discontinuities, and the
encoding's ``sin(2^9 x)`` (freq.py:19) turns a 1-ulp depth shift into ~1e-4 of
feature change. Any two float32 implementations therefore disagree on some rays
by far more than 1e-5 -- including the reference against itself.

This script measures exactly that. It renders every golden fixture again with
the reference's own ``Renderer`` on K exact reparametrisations of the same
network: the hidden units of every layer are permuted (rows of the producing
Linear, columns of every consumer, including the skip concat at layer 5 and the
feature/views concat), which leaves the function unchanged in real arithmetic
and changes only the summation order inside the reference's CPU GEMMs. Half of
the variants also model another (faithfully rounded) libm: every ``torch.sin``,
``torch.cos`` (the encoder's periodic functions, freq.py:24-26), ``torch.exp``
and ``torch.sigmoid`` result (VR:288, 301) is moved by +-1 ulp at random. The
per ray maximum |variant - golden| over the variants is the reference's own
rounding sensitivity; tests hold the HIP renderer to it ray by ray
(``goldlib.fine_gate``).

Outputs ``tests/golden/s_<fixture>.npz``: ``spread_<map>`` (float32 per ray,
NaN-aware: a NaN pattern change counts as +inf), ``variant_frac_ok`` (fraction
of rays within the 1e-5 gate, per variant) and ``variant_psnr`` (fine rgb PSNR
of each variant vs the golden render). Only numbers are stored.

    python tests/golden/make_sensitivity.py            # all fixtures, K=16
    python tests/golden/make_sensitivity.py f1 f3      # selected
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402

K_VARIANTS = 16          # 0..7: permuted GEMMs; 8..15: + a +-1-ulp libm
MAPS = ("rgb_map_0", "disp_map_0", "acc_map_0", "depth_map_0",
        "rgb_map", "disp_map", "acc_map", "depth_map")


def permute_params(params, seed, prefixes=("model", "model_fine")):
    """Function-preserving permutation of every hidden layer's units."""
    rng = np.random.default_rng(seed)
    out = dict(params)
    for pre in prefixes:
        P = {i: rng.permutation(256) for i in range(8)}
        Pf, Pv = rng.permutation(256), rng.permutation(128)

        def rows(name, perm):
            out[f"{pre}.{name}.weight"] = out[f"{pre}.{name}.weight"][perm].copy()
            out[f"{pre}.{name}.bias"] = out[f"{pre}.{name}.bias"][perm].copy()

        def cols(name, perm, off=0):
            w = out[f"{pre}.{name}.weight"].copy()
            w[:, off:off + len(perm)] = w[:, off:off + len(perm)][:, perm]
            out[f"{pre}.{name}.weight"] = w

        for i in range(8):
            rows(f"pts_linears.{i}", P[i])
            if i < 7:   # layer 5 reads cat(input_pts[63], h4) (network.py:57-58)
                cols(f"pts_linears.{i + 1}", P[i], off=63 if i == 4 else 0)
        cols("alpha_linear", P[7])
        cols("feature_linear", P[7])
        rows("feature_linear", Pf)
        cols("views_linears.0", Pf)          # cat(feature, input_views) (network.py:64)
        rows("views_linears.0", Pv)
        cols("rgb_linear", Pv)
    return out


def _ulp_libm(torch, seed):
    """Wrap sin/cos/exp/sigmoid: each result moves one ulp up or down at random."""
    gen = torch.Generator().manual_seed(seed)
    orig = {k: getattr(torch, k) for k in ("sin", "cos", "exp", "sigmoid")}

    def wrap(fn):
        def f(x, *a, **kw):
            y = fn(x, *a, **kw)
            d = torch.randint(0, 3, y.shape, generator=gen) - 1        # -1, 0, +1
            to = torch.where(d > 0, torch.full_like(y, float("inf")),
                             torch.full_like(y, float("-inf")))
            return torch.where(d == 0, y, torch.nextafter(y, to))
        return f
    for k, fn in orig.items():
        setattr(torch, k, wrap(fn))
    return orig


def render(spec, cfg, Network, vr, frames, angle, params, ulp_seed=None):
    """The same call sequence as make_golden.capture (same seeds, same draws)."""
    import torch
    from nerfhip.synthetic import make_occupancy_grid, load_into_network
    orig = _ulp_libm(torch, ulp_seed) if ulp_seed is not None else None
    try:
        return _render(torch, make_occupancy_grid, load_into_network, spec, cfg, Network, vr,
                       frames, angle, params)
    finally:
        for k, fn in (orig or {}).items():
            setattr(torch, k, fn)


def _render(torch, make_occupancy_grid, load_into_network, spec, cfg, Network, vr, frames,
            angle, params):
    for k in ("N_importance", "perturb", "lindisp"):
        if k in spec["cfg"]:
            cfg.task_arg[k] = spec["cfg"][k]
    cfg.task_arg.lindisp = spec["cfg"].get("lindisp", False)
    cfg.task_arg.raw_noise_std = spec["cfg"].get("raw_noise_std", 0.0)
    for k in ("enable_ess", "enable_ert", "ert_threshold"):
        if k in spec["cfg"]:
            cfg[k] = spec["cfg"][k]
    net = Network()
    load_into_network(net, params)
    net.eval()
    torch.manual_seed(1234)
    rend = vr.Renderer(net)
    rend.use_cuda_kernels = False
    if "grid" in spec:
        g = spec["grid"]
        rend.occupancy_grid = torch.from_numpy(
            make_occupancy_grid(g["seed"], 128, g["radius"], g["noise"]).copy())
        rend.grid_update_counter = spec.get("counter", 0)
    pose, K = MG._camera(spec, frames, angle)
    batch = {"H": spec["H"], "W": spec["W"], "pose": torch.from_numpy(pose)[None],
             "intrinsics": torch.from_numpy(K)[None]}
    with torch.no_grad():
        out = rend.render(batch)
    return {k: v.numpy() for k, v in out.items()}


def per_ray_dev(a, b, n):
    a = np.asarray(a, np.float64).reshape(n, -1)
    b = np.asarray(b, np.float64).reshape(n, -1)
    nan_flip = (np.isnan(a) != np.isnan(b)).any(-1)
    d = np.nan_to_num(np.abs(a - b), nan=0.0).max(-1)
    d[nan_flip] = np.inf
    return d


def main(argv):
    from nerfhip.synthetic import make_params
    cfg, Network, vr = MG._import_reference()
    meta = json.load(open(os.path.join(MG.REF, "data/nerf_synthetic/lego/transforms_test.json")))
    frames, angle = meta["frames"], meta["camera_angle_x"]
    names = [k for k in MG.FIXTURES if not argv or any(k == a or k.startswith(a + "_") for a in argv)]
    for name in names:
        spec = MG.FIXTURES[name]
        gold = dict(np.load(os.path.join(MG.OUT, name + ".npz")))
        params = make_params(*spec["w"])
        n = spec["H"] * spec["W"]
        spread = {}
        frac_ok, vpsnr = [], []
        for v in range(K_VARIANTS):
            out = render(spec, cfg, Network, vr, frames, angle, permute_params(params, 100 + v),
                         ulp_seed=(200 + v) if v >= K_VARIANTS // 2 else None)
            ok = np.ones(n, bool)
            for k in MAPS:
                if k not in out:
                    continue
                d = per_ray_dev(out[k], gold["out_" + k], n)
                spread[k] = d if k not in spread else np.maximum(spread[k], d)
                if k.endswith("_map") and not k.startswith("disp"):
                    ok &= d <= (1e-5 * np.maximum(1.0, np.abs(gold["out_" + k]).reshape(n))
                                if k.startswith("depth") else 1e-5)
            frac_ok.append(float(ok.mean()))
            if "rgb_map" in out:
                mse = np.mean((np.clip(out["rgb_map"], 0, 1).astype(np.float64)
                               - np.clip(gold["out_rgb_map"], 0, 1)) ** 2)
                vpsnr.append(float("inf") if mse == 0 else float(-10 * np.log10(mse)))
        rec = {"spread_" + k: v.astype(np.float32) for k, v in spread.items()}
        rec.update(variant_frac_ok=np.array(frac_ok), variant_psnr=np.array(vpsnr),
                   k_variants=K_VARIANTS)
        np.savez_compressed(os.path.join(MG.OUT, "s_" + name + ".npz"), **rec)
        print(f"{name}: fine frac within 1e-5 per variant {np.round(frac_ok, 4).tolist()}, "
              f"psnr {np.round(vpsnr, 1).tolist()}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
