"""The reference renderer's own float32 noise floor on the whole-frame fixtures
(survey container; the companion of make_sensitivity.py for the crops).

tests/test_gpu_frames.py holds every pixel of the r0 / r1 frames to 1e-5 or
attributes it. Pixels whose fine depths match the reference's bit for bit can
still move: on a partially transparent ray (acc well inside (0, 1)) a
1-ulp-level change of the MLP's density moves acc by a few 1e-6 and the depth
(about acc x the ray's z) by several 1e-5. Whether that is the reference's own
rounding sensitivity is measured here, as make_sensitivity.py does for the
crops: the reference's ``Renderer`` re-renders the frame's partially
transparent pixels (fine acc of the stored frame in (1e-6, 0.9999)) on K exact
reparametrisations of the same network (hidden units permuted: the same
function, another GEMM summation order; half of them also a +-1-ulp libm), and
the per-pixel maximum |variant - stored frame| is stored.

With ESS / ERT off (r0, r1) every ray is independent of the others
(VR:154-204: no chunk-wide rule, no grid), so the subset is rendered in
2048-ray chunks of its own through the reference's own per-chunk methods
(``_sample_coarse``, ``_query_network``, ``_raw2outputs``, ``_sample_fine``,
VR:158-201) on the reference's rays (VR:115-143, computed for the whole frame
and indexed); perturb draws (r1) are the frame's own rows, regenerated from
its seed in the reference's chunk order (VR:233-234). The unpermuted network
reproduces the stored maps of these pixels bit for bit (asserted), which pins
the subset rendering.

Outputs ``tests/golden/rs_<frame>.npz``: ``pixels`` (int32), ``spread_<map>``
(float32 per pixel, NaN-aware), ``variant_frac_ok``. Only numbers are stored.

    python tests/golden/make_frame_sensitivity.py [r0_c2_frame0 r1_c2_frame8_pert]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_ref_frames as MRF  # noqa: E402
import make_sensitivity as MS  # noqa: E402

K_VARIANTS = 8            # 0..3: permuted GEMMs; 4..7: + a +-1-ulp libm
FRAMES = ("r0_c2_frame0", "r1_c2_frame8_pert")
MAPS = ("rgb_map", "acc_map", "depth_map", "disp_map")
CHUNK = 2048


def reference_rays(torch, H, W, pose, K):
    """VR:115-143 for the whole frame (the reference's op sequence)."""
    i, j = torch.meshgrid(torch.linspace(0, W - 1, W), torch.linspace(0, H - 1, H),
                          indexing="ij")
    i, j = i.t(), j.t()
    dirs = torch.stack([(i - K[0, 2]) / K[0, 0], -(j - K[1, 2]) / K[1, 1],
                        -torch.ones_like(i)], -1)
    rays_d = torch.sum(dirs[..., np.newaxis, :] * pose[:3, :3], -1)
    rays_o = pose[:3, 3].expand(rays_d.shape)
    rays_o, rays_d = rays_o.reshape(-1, 3), rays_d.reshape(-1, 3)
    return rays_o, rays_d / torch.norm(rays_d, dim=-1, keepdim=True)


def render_subset(torch, rend, rays_o, rays_d, t_rand):
    """VR:154-201 (ESS / ERT off) over rays of independent chunks; t_rand [n, 64]
    rows (perturb) served to _sample_coarse's torch.rand in order."""
    out = {k: [] for k in ("rgb_map", "disp_map", "acc_map", "depth_map")}
    orig = torch.rand
    for c in range(0, rays_o.shape[0], CHUNK):
        ro, rd = rays_o[c:c + CHUNK], rays_d[c:c + CHUNK]
        if t_rand is not None:
            rows = t_rand[c:c + CHUNK]
            torch.rand = lambda *a, **kw: rows.clone()
        try:
            t_vals = rend._sample_coarse(ro.shape[0])
        finally:
            torch.rand = orig
        pts = ro[..., None, :] + rd[..., None, :] * t_vals[..., :, None]
        raw = rend._query_network(pts, rd, rend.coarse_model)
        _, _, _, weights, _ = rend._raw2outputs(raw, t_vals, rd)
        t_mid = .5 * (t_vals[..., 1:] + t_vals[..., :-1])
        t_fine = rend._sample_fine(t_mid, weights[..., 1:-1])
        t_vals, _ = torch.sort(torch.cat([t_vals, t_fine], -1), -1)
        pts = ro[..., None, :] + rd[..., None, :] * t_vals[..., :, None]
        raw = rend._query_network(pts, rd, rend.fine_model)
        rgb, disp, acc, _, depth = rend._raw2outputs(raw, t_vals, rd)
        for k, v in (("rgb_map", rgb), ("disp_map", disp), ("acc_map", acc),
                     ("depth_map", depth)):
            out[k].append(v.numpy())
    return {k: np.concatenate(v, 0) for k, v in out.items()}


def main(argv):
    import torch
    cfg, Network, vr = MRF._import_reference()
    meta = json.load(open(os.path.join(MRF.REF, "data/nerf_synthetic/lego/transforms_test.json")))
    sd = torch.load(MRF.CKPT, map_location="cpu", weights_only=True)["net"]
    base = {k: v.numpy() for k, v in sd.items()}
    for name in argv or FRAMES:
        spec = MRF.FRAMES[name]
        z = dict(np.load(os.path.join(MRF.OUT, name + ".npz")))
        zh = dict(np.load(os.path.join(MRF.OUT, "zh_" + name + ".npz")))
        H, W = int(z["H"]), int(z["W"])
        n = H * W
        acc = z["out_acc_map"].reshape(n)
        pix = np.flatnonzero((acc > 1e-6) & (acc < 0.9999)).astype(np.int32)
        if os.environ.get("NERF_FS_LIMIT"):   # a quick check of the subset rendering only
            pix = pix[::max(1, len(pix) // int(os.environ["NERF_FS_LIMIT"]))]
        cfg.task_arg.N_importance = 128
        cfg.task_arg.perturb = spec["perturb"]
        cfg.task_arg.lindisp = False
        cfg.enable_ess = False
        cfg.enable_ert = False
        rays_o, rays_d = reference_rays(torch, H, W, torch.from_numpy(z["pose"]),
                                        torch.from_numpy(z["K"]))
        idx = torch.from_numpy(pix.astype(np.int64))
        ro, rd = rays_o[idx].contiguous(), rays_d[idx].contiguous()
        t_rand = None
        if spec["perturb"]:
            torch.manual_seed(int(z["seed"]))          # the capture's draws, in chunk order
            t_rand = torch.cat([torch.rand([min(CHUNK, n - c), 64]) for c in range(0, n, CHUNK)])
            t_rand = t_rand[idx].contiguous()
        ref = {"rgb_map": z["out_rgb_map"].reshape(n, 3)[pix],
               "acc_map": z["out_acc_map"].reshape(n)[pix],
               "depth_map": z["out_depth_map"].reshape(n)[pix],
               "disp_map": zh["disp_map"].reshape(n)[pix]}
        spread, frac_ok = {}, []
        for v in range(-1, 0 if os.environ.get("NERF_FS_LIMIT") else K_VARIANTS):
            params = {k: torch.from_numpy(np.ascontiguousarray(a)) for k, a in
                      (base.items() if v < 0 else MS.permute_params(base, 100 + v).items())}
            net = Network()
            net.load_state_dict(params)
            net.eval()
            rend = vr.Renderer(net)
            rend.use_cuda_kernels = False
            orig = MS._ulp_libm(torch, 200 + v) if v >= K_VARIANTS // 2 else None
            t0 = time.time()
            try:
                with torch.no_grad():
                    out = render_subset(torch, rend, ro, rd, t_rand)
            finally:
                for k, fn in (orig or {}).items():
                    setattr(torch, k, fn)
            if v < 0:   # the unpermuted network: the stored frame's pixels, bit for bit
                for k in MAPS:
                    assert np.array_equal(out[k], ref[k], equal_nan=True), (name, k)
                print(f"{name}: {len(pix)} pixels reproduced ({time.time() - t0:.0f} s)",
                      flush=True)
                continue
            m = len(pix)
            ok = np.ones(m, bool)
            for k in MAPS:
                d = MS.per_ray_dev(out[k], ref[k], m)
                spread[k] = d if k not in spread else np.maximum(spread[k], d)
                if k != "disp_map":
                    tol = (1e-5 * np.maximum(1.0, np.abs(ref[k]).reshape(m))
                           if k == "depth_map" else 1e-5)
                    ok &= d <= tol
            frac_ok.append(float(ok.mean()))
            print(f"{name} variant {v}: {time.time() - t0:.0f} s, within 1e-5 {ok.mean():.4f}",
                  flush=True)
        np.savez_compressed(os.path.join(MRF.OUT, "rs_" + name + ".npz"), pixels=pix,
                            variant_frac_ok=np.array(frac_ok), k_variants=K_VARIANTS,
                            ckpt_sha256=MRF.ckpt_sha(),
                            **{"spread_" + k: v.astype(np.float32) for k, v in spread.items()})


if __name__ == "__main__":
    main(sys.argv[1:])
