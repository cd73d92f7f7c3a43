"""The reference's own spread on the ESS + ERT whole frames r2 / r3, chunk by
chunk (survey container; the ERT companion of make_frame_sensitivity.py).

The ERT rule is chunk-wide (VR:1108-1123): the reference cuts each ray at its
first sample with transmittance T < thr, and when any ray of the 2048-ray chunk
terminates, every non-terminating ray of that chunk is cut at sample 0. A ray
whose T at its own cut sits within float32 rounding of thr therefore moves the
cut -- and acc / depth by up to its last weights -- under ANY change of
summation order, the reference's own included. test_gpu_frames.py exempts at
most 5 such rays per frame from the on-reference-depths gate; this script
measures whether the reference itself moves them.

Rays: every captured tail pixel of the frame (tests/golden/zt_<frame>.npz)
whose T at its own cut, or the T before it, lies within BAND (relative) of the
threshold by the oracle's fine pass on the reference's own depths
(oracle/nerf_oracle.py on the zt rows; the test's exemption uses 1e-4). Their
2048-ray chunks are rendered again by the reference's own per-chunk methods
(VR:154-204 with ESS: ``_sample_coarse_with_ess``, ``_query_network``,
``_raw2outputs_with_ert``, ``_sample_fine``) on K exact reparametrisations of
its network (make_sensitivity.permute_params; half of them also with a
+-1-ulp libm, make_sensitivity._ulp_libm). The sequential state of the frame is
rebuilt for each variant: the grid as the frame started (r2: the synthetic
grid spec, r3: the Renderer's own draw, ``grid_init_bits``), the grid-updating
chunks before a target (the calls whose counter is 0 mod 500, VR:1147-1155:
chunks 0 and 250) rendered first at their own counter, each target chunk at
its counter (2 calls per chunk, VR:1157), and with perturb (r3) each chunk's
rows of the frame's draws (torch.manual_seed(seed): the grid's draw, then one
[m, 64] per chunk in order, VR:861, :1080-1085). The unpermuted network
reproduces the stored maps of every target chunk bit for bit (asserted).

Outputs ``tests/golden/rs_<frame>.npz``: ``pixels`` (every pixel of the target
chunks, int32), ``spread_<map>`` (per pixel, max |variant - stored| over the
variants, NaN-aware), ``variant_frac_ok``, ``cut_ref`` (the fine call's cut,
argmax of T < thr, per pixel; -1 where the ray never drops below thr),
``cut_var`` [K, pixels], ``chunks``, ``chunk_any_ref`` / ``chunk_any_var`` (the
fine call's chunk-wide decision), ``cand_pixels`` / ``cand_rel`` (the oracle
candidates). Only numbers are stored.

    python tests/golden/make_ert_sensitivity.py [r2_c4_frame16 r3_c4_yaml_frame24]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
import make_ref_frames as MRF  # noqa: E402
import make_sensitivity as MS  # noqa: E402
from make_frame_sensitivity import reference_rays  # noqa: E402

FRAMES = ("r2_c4_frame16", "r3_c4_yaml_frame24")
K_VARIANTS = 16           # 0..7: permuted GEMMs; 8..15: + a +-1-ulp libm
BAND = 1e-3               # candidate rays: T at the cut within 1e-3 (relative) of thr
CHUNK = 2048
GRID_INTERVAL = 500       # VR:63-64 grid_update_interval
MAPS = ("rgb_map", "acc_map", "depth_map", "disp_map")


def candidates(name, z):
    """zt pixels whose oracle T at the cut (or just before it) is within BAND of thr."""
    import torch
    from oracle import nerf_oracle as O
    zt = np.load(os.path.join(MRF.OUT, f"zt_{name}.npz"))
    sd = torch.load(MRF.CKPT, map_location="cpu", weights_only=True)["net"]
    params = {k: v.numpy() for k, v in sd.items()}
    P = zt["pixels"].astype(np.int64)
    zc, wc = zt["z_coarse"], zt["w_coarse"]
    mids = (np.float32(0.5) * (zc[:, 1:] + zc[:, :-1])).astype(np.float32)
    zf = O.sample_fine(mids, wc[:, 1:-1], O.linspace_f32(0.0, 1.0, 128))
    zall = np.ascontiguousarray(np.sort(np.concatenate([zc, zf], -1), -1), np.float32)
    ro, rd = O.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"])
    ro, rd = ro[P], rd[P]
    pts = (ro[:, None, :] + rd[:, None, :] * zall[:, :, None]).astype(np.float32)
    raw = O.query_network(pts, rd, params, "model_fine")
    d = O._dists(zall, rd)
    alpha = (np.float32(1.0) - np.exp(-(np.maximum(raw[..., 3], np.float32(0.0)) * d)
                                      .astype(np.float32)).astype(np.float32)).astype(np.float32)
    sh = np.concatenate([np.zeros((alpha.shape[0], 1), np.float32), alpha[:, :-1]], 1)
    Tr = np.cumprod((np.float32(1.0) - sh).astype(np.float64), 1)
    thr = float(z["thr"])
    rel = np.empty(len(P))
    for i in range(len(P)):
        below = np.flatnonzero(Tr[i] < thr)
        if len(below) == 0:
            rel[i] = abs(Tr[i, -1] / thr - 1.0)
            continue
        k = below[0]
        rel[i] = abs(Tr[i, k] / thr - 1.0)
        if k > 0:
            rel[i] = min(rel[i], abs(Tr[i, k - 1] / thr - 1.0))
    keep = rel < BAND
    return P[keep], rel[keep]


class _CutRecorder:
    """Wraps _raw2outputs_with_ert: per call, each ray's cut (argmax of T < thr,
    VR:1108-1118, -1 where none) and the chunk-wide decision, recomputed with
    the reference's op sequence on the call's own raw."""

    def __init__(self, rend):
        import torch
        self.calls = []
        orig = rend._raw2outputs_with_ert

        def rec(raw, z, rays_d):
            r = orig(raw, z, rays_d)
            d = torch.cat([z[..., 1:] - z[..., :-1], torch.full_like(z[..., :1], 1e10)], -1)
            d = d * torch.norm(rays_d[..., None, :], dim=-1)
            a = 1. - torch.exp(-torch.relu(raw[..., 3]) * d)
            sh = torch.cat([torch.zeros_like(a[:, :1]), a[:, :-1]], 1)
            low = torch.cumprod(1.0 - sh, 1) < rend.ert_threshold
            cut = torch.where(low.any(1), low.float().argmax(1), torch.full_like(low[:, 0], -1,
                                                                                  dtype=torch.long))
            self.calls.append((cut.numpy().astype(np.int16), bool(low.any())))
            return r
        rend._raw2outputs_with_ert = rec


def render_chunk(torch, rend, ro, rd, t_rows):
    """VR:154-204 for one chunk with ESS + ERT on; t_rows: the chunk's perturb draw."""
    orig = torch.rand
    if t_rows is not None:
        torch.rand = lambda *a, **kw: t_rows.clone()
    try:
        t_vals = rend._sample_coarse_with_ess(ro, rd)
    finally:
        torch.rand = orig
    pts = ro[..., None, :] + rd[..., None, :] * t_vals[..., :, None]
    raw = rend._query_network(pts, rd, rend.coarse_model)
    rgb0, disp0, acc0, weights, depth0 = rend._raw2outputs_with_ert(raw, t_vals, rd)
    t_mid = .5 * (t_vals[..., 1:] + t_vals[..., :-1])
    t_fine = rend._sample_fine(t_mid, weights[..., 1:-1])
    t_vals, _ = torch.sort(torch.cat([t_vals, t_fine], -1), -1)
    pts = ro[..., None, :] + rd[..., None, :] * t_vals[..., :, None]
    raw = rend._query_network(pts, rd, rend.fine_model)
    rgb, disp, acc, _, depth = rend._raw2outputs_with_ert(raw, t_vals, rd)
    return {"rgb_map": rgb.numpy(), "disp_map": disp.numpy(), "acc_map": acc.numpy(),
            "depth_map": depth.numpy(), "rgb_map_0": rgb0.numpy(), "acc_map_0": acc0.numpy()}


def main(argv):
    import torch
    cfg, Network, vr = MRF._import_reference()
    sd = torch.load(MRF.CKPT, map_location="cpu", weights_only=True)["net"]
    base = {k: v.numpy() for k, v in sd.items()}
    for name in argv or FRAMES:
        spec = MRF.FRAMES[name]
        z = dict(np.load(os.path.join(MRF.OUT, name + ".npz")))
        zh = dict(np.load(os.path.join(MRF.OUT, "zh_" + name + ".npz")))
        H, W = int(z["H"]), int(z["W"])
        n = H * W
        cand, rel = candidates(name, z)
        targets = sorted(set((cand // CHUNK).tolist()))
        updates = [c for c in range(0, max(targets) + 1)
                   if (int(z["counter0"]) + 2 * c) % GRID_INTERVAL == 0]
        order = sorted(set(targets) | set(updates))
        print(f"{name}: {len(cand)} candidate rays in chunks {targets}; updates {updates}",
              flush=True)
        cfg.task_arg.N_importance = 128
        cfg.task_arg.perturb = spec["perturb"]
        cfg.task_arg.lindisp = False
        cfg.enable_ess = True
        cfg.enable_ert = True
        cfg.ert_threshold = float(z["thr"])
        rays_o, rays_d = reference_rays(torch, H, W, torch.from_numpy(z["pose"]),
                                        torch.from_numpy(z["K"]))
        if spec.get("grid") == "own":
            bits = np.unpackbits(z["grid_init_bits"])[:128 ** 3].astype(bool)
            grid0 = torch.from_numpy(bits.reshape(128, 128, 128))
        else:
            gs = z["grid_spec"]
            grid0 = torch.from_numpy(MRF.make_occupancy_grid(int(gs[0]), int(gs[1]), float(gs[2]),
                                                             float(gs[3])).copy())
        t_rand = None
        if spec["perturb"]:   # the frame's draws: the grid's first (own grid), then per chunk
            torch.manual_seed(int(z["seed"]))
            if spec.get("grid") == "own":
                torch.rand((128, 128, 128))
            t_rand = torch.cat([torch.rand([min(CHUNK, n - c), 64]) for c in range(0, n, CHUNK)])
        pix = np.concatenate([np.arange(c * CHUNK, min(n, (c + 1) * CHUNK)) for c in targets])
        m = len(pix)
        ref = {"rgb_map": z["out_rgb_map"].reshape(n, 3)[pix],
               "acc_map": z["out_acc_map"].reshape(n)[pix],
               "depth_map": z["out_depth_map"].reshape(n)[pix],
               "disp_map": zh["disp_map"].reshape(n)[pix]}
        spread, frac_ok, cut_var, any_var = {}, [], [], []
        cut_ref = any_ref = None
        for v in range(-1, K_VARIANTS):
            params = {k: torch.from_numpy(np.ascontiguousarray(a)) for k, a in
                      (base.items() if v < 0 else MS.permute_params(base, 300 + v).items())}
            net = Network()
            net.load_state_dict(params)
            net.eval()
            rend = vr.Renderer(net)
            rend.use_cuda_kernels = False
            rend.occupancy_grid = grid0.clone()
            rec = _CutRecorder(rend)
            orig = MS._ulp_libm(torch, 400 + v) if v >= K_VARIANTS // 2 else None
            t0 = time.time()
            outs, cuts, anys = [], [], []
            try:
                with torch.no_grad():
                    for c in order:
                        rend.grid_update_counter = int(z["counter0"]) + 2 * c
                        a, b = c * CHUNK, min(n, (c + 1) * CHUNK)
                        tr = None if t_rand is None else t_rand[a:b].contiguous()
                        o = render_chunk(torch, rend, rays_o[a:b].contiguous(),
                                         rays_d[a:b].contiguous(), tr)
                        if c in targets:
                            outs.append(o)
                            cuts.append(rec.calls[-1][0])     # the fine call
                            anys.append(rec.calls[-1][1])
            finally:
                for k, fn in (orig or {}).items():
                    setattr(torch, k, fn)
            out = {k: np.concatenate([o[k] for o in outs], 0) for k in MAPS}
            cut, anyc = np.concatenate(cuts), np.array(anys, bool)
            if v < 0:   # the unpermuted network: the stored frame's chunks, bit for bit
                for k in MAPS:
                    assert np.array_equal(out[k].reshape(-1), ref[k].reshape(-1),
                                          equal_nan=True), (name, k)
                assert np.array_equal(anyc, zh["chunk_any"][2 * np.array(targets) + 1]), name
                cut_ref, any_ref = cut, anyc
                print(f"{name}: {len(targets)} chunks reproduced ({time.time() - t0:.0f} s)",
                      flush=True)
                continue
            ok = np.ones(m, bool)
            for k in MAPS:
                d = MS.per_ray_dev(out[k], ref[k], m)
                spread[k] = d if k not in spread else np.maximum(spread[k], d)
                if k != "disp_map":
                    tol = (1e-5 * np.maximum(1.0, np.abs(ref[k]).reshape(m))
                           if k == "depth_map" else 1e-5)
                    ok &= d <= tol
            frac_ok.append(float(ok.mean()))
            cut_var.append(cut)
            any_var.append(anyc)
            pos = np.searchsorted(pix, cand)
            moved = int((np.asarray(cut)[pos] != cut_ref[pos]).sum())
            print(f"{name} variant {v}: {time.time() - t0:.0f} s, within 1e-5 {ok.mean():.4f}, "
                  f"candidate cuts moved {moved}/{len(cand)}", flush=True)
        np.savez_compressed(os.path.join(MRF.OUT, "rs_" + name + ".npz"), pixels=pix.astype(np.int32),
                            variant_frac_ok=np.array(frac_ok), k_variants=K_VARIANTS,
                            ckpt_sha256=MRF.ckpt_sha(), chunks=np.array(targets, np.int32),
                            cut_ref=cut_ref, cut_var=np.stack(cut_var),
                            chunk_any_ref=any_ref, chunk_any_var=np.stack(any_var),
                            cand_pixels=cand.astype(np.int32), cand_rel=rel, band=BAND,
                            **{"spread_" + k: v.astype(np.float32) for k, v in spread.items()})
        moved = (np.stack(cut_var)[:, np.searchsorted(pix, cand)] != cut_ref[np.searchsorted(pix, cand)])
        print(json.dumps({"frame": name, "candidates": len(cand),
                          "candidates_moved_by_some_variant": int(moved.any(0).sum()),
                          "variant_frac_ok_min": min(frac_ok)}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
