"""Element-wise gradient fixtures of the reference training step (survey container).

The train goldens (make_train_golden.py) keep each gradient's norm, sum and
first 64 values. This script re-runs the reference training step of each of
them (asserting the same norms bit for bit) and stores every gradient tensor,
plus the reference's own element-wise noise floor: the step is re-run on
K = 16 exact reparametrisations of the network (hidden units permuted, half
with a +-1-ulp libm; make_train_sensitivity.py), each variant's gradients are
compared with the golden's gradients permuted the same way (a permutation of
the units permutes the gradient exactly in real arithmetic), and per tensor
the largest relative L2 distance ||g_variant - P g_gold|| / ||g_gold|| is kept:

  tests/golden/tg_<fixture>.npz: g__<param> float32 (full loss),
      gc__<param> float32 (coarse loss), gdist__<param> / gcdist__<param>
      (float64: the reference's largest relative L2 distance from itself),
      k_variants

Only numbers are stored.

    python tests/golden/make_train_fullgrad.py        # t1, t2
    python tests/golden/make_train_fullgrad.py t3     # t3_c3_scatter (+ tg_), see T3 below
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402
import make_sensitivity as MS  # noqa: E402
import make_train_golden as MT  # noqa: E402
from make_train_sensitivity import K_VARIANTS, _ulp_libm_ad  # noqa: E402


def _rel(a, b):
    nb = float(np.linalg.norm(b))
    return float(np.linalg.norm(a - b)) / max(nb, 1e-30)


# ---------------------------------------------------------------------------
# t3: the bench's own C3 shape (BASELINE configs[2]; bench.py bench_train):
# 1024 pixels scattered over the lego test views, ESS / ERT off, perturb 1,
# training-mode u, the trained lego checkpoint, MSE coarse + fine against a
# uniform random target. The reference trains on whole images through
# Renderer.render(batch) (trainers/nerf.py:20-37); a batch of rays from many
# cameras has no render(batch) form, so the step runs the reference's own
# per-chunk methods on one 1024-ray chunk in _render_pytorch's order
# (VR:154-193: _sample_coarse, _query_network, _raw2outputs, _sample_fine,
# sort, _query_network, _raw2outputs) on the reference's rays of each view
# (VR:115-143, whole frames computed and indexed), and the loss of
# trainers/nerf.py:39-76.
T3 = "t3_c3_scatter"
T3_RAYS = 1024
T3_SEED = 20261018


_T3_CACHE = {}


def _t3_batch(torch, meta):
    """(view, pixel) pairs, the reference's rays for them and the target."""
    if "b" in _T3_CACHE:
        return _T3_CACHE["b"]
    from make_frame_sensitivity import reference_rays
    rng = np.random.default_rng(T3_SEED)
    frames, angle = meta["frames"], float(meta["camera_angle_x"])
    view = rng.integers(0, len(frames), T3_RAYS)
    pix = rng.integers(0, 800 * 800, T3_RAYS)
    target = rng.random((T3_RAYS, 3)).astype(np.float32)
    focal = 0.5 * 800 / np.tan(0.5 * angle)                 # blender.py:41-42
    K = np.array([[focal, 0, 400.0], [0, focal, 400.0], [0, 0, 1]], np.float32)
    ro = np.empty((T3_RAYS, 3), np.float32)
    rd = np.empty((T3_RAYS, 3), np.float32)
    for v in np.unique(view):
        pose = np.array(frames[v]["transform_matrix"], np.float32)
        o, d = reference_rays(torch, 800, 800, torch.from_numpy(pose), torch.from_numpy(K))
        sel = view == v
        ro[sel] = o[torch.from_numpy(pix[sel])].numpy()
        rd[sel] = d[torch.from_numpy(pix[sel])].numpy()
    _T3_CACHE["b"] = (view, pix, K, ro, rd, target)
    return _T3_CACHE["b"]


def capture_t3(cfg, Network, vr, meta, params, draws=None):
    """One reference training step on the t3 batch. draws = (t_rand, u) replays
    recorded torch.rand draws (the reparametrised variants use the golden's);
    returns the record with every gradient (full loss and coarse loss)."""
    import torch
    cfg.task_arg.N_importance = 128
    cfg.task_arg.perturb = 1
    cfg.task_arg.lindisp = False
    cfg.enable_ess = False
    cfg.enable_ert = False
    net = Network()
    net.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()})
    net.train()
    rend = vr.Renderer(net)
    rend.use_cuda_kernels = False
    view, pix, K, ro_np, rd_np, target_np = _t3_batch(torch, meta)
    ro, rd = torch.from_numpy(ro_np), torch.from_numpy(rd_np)
    rec_draws = []
    orig = torch.rand
    it = iter(draws) if draws is not None else None

    def rand(*a, **kw):
        t = torch.from_numpy(next(it).copy()) if it is not None else orig(*a, **kw)
        rec_draws.append(t.detach().clone().numpy())
        return t
    if draws is None:
        torch.manual_seed(T3_SEED)
    torch.rand = rand
    try:
        t_vals = rend._sample_coarse(T3_RAYS)                              # VR:158-161
        pts = ro[..., None, :] + rd[..., None, :] * t_vals[..., :, None]   # VR:163
        raw = rend._query_network(pts, rd, rend.coarse_model)             # VR:166
        rgb0, disp0, acc0, weights, depth0 = rend._raw2outputs(raw, t_vals, rd)
        t_mid = .5 * (t_vals[..., 1:] + t_vals[..., :-1])                  # VR:180
        t_fine = rend._sample_fine(t_mid, weights[..., 1:-1])
        t_all, _ = torch.sort(torch.cat([t_vals, t_fine], -1), -1)         # VR:182
        pts_f = ro[..., None, :] + rd[..., None, :] * t_all[..., :, None]
        raw_f = rend._query_network(pts_f, rd, rend.fine_model)           # VR:186
        rgb, disp, acc, _, depth = rend._raw2outputs(raw_f, t_all, rd)
    finally:
        torch.rand = orig
    target = torch.from_numpy(target_np)
    loss_c = torch.nn.functional.mse_loss(rgb0, target)                    # trainers/nerf.py:54-55
    loss_f = torch.nn.functional.mse_loss(rgb, target)                     # :64-66
    loss = loss_c + loss_f
    net.zero_grad()
    loss_c.backward(retain_graph=True)
    gc = {k: p.grad.detach().double().numpy().copy() for k, p in net.named_parameters()
          if p.grad is not None}
    net.zero_grad()
    loss.backward()
    g = {k: p.grad.detach().double().numpy().copy() for k, p in net.named_parameters()}
    assert [d.shape for d in rec_draws] == [(T3_RAYS, 64), (T3_RAYS, 128)]
    return dict(view=view, pix=pix, K=K, rays_o=ro_np, rays_d=rd_np, target=target_np,
                t_rand=rec_draws[0], u=rec_draws[1], loss=np.float64(loss.item()),
                loss_coarse=np.float64(loss_c.item()), loss_fine=np.float64(loss_f.item()),
                rgb_map_0=rgb0.detach().numpy(), rgb_map=rgb.detach().numpy(),
                acc_map_0=acc0.detach().numpy(), acc_map=acc.detach().numpy(),
                depth_map_0=depth0.detach().numpy(), depth_map=depth.detach().numpy(),
                zall=t_all.detach().numpy()), g, gc


def main_t3():
    import torch
    cfg, Network, vr = MG._import_reference()
    with open(os.path.join(MG.REF, "data", "nerf_synthetic", "lego", "transforms_test.json")) as f:
        meta = json.load(f)
    import make_ref_frames as MRF
    sd = torch.load(MRF.CKPT, map_location="cpu", weights_only=True)["net"]
    params = {k: v.numpy() for k, v in sd.items()}
    rec, g, gc = capture_t3(cfg, Network, vr, meta, params)
    dist = {k: 0.0 for k in g}
    cdist = {k: 0.0 for k in gc}
    for v in range(K_VARIANTS):
        orig = _ulp_libm_ad(torch, 300 + v) if v >= K_VARIANTS // 2 else None
        try:
            _, gv, gcv = capture_t3(cfg, Network, vr, meta, MS.permute_params(params, 100 + v),
                                    draws=(rec["t_rand"], rec["u"]))
        finally:
            for k, fn in (orig or {}).items():
                setattr(torch, k, fn)
        pg = MS.permute_params(g, 100 + v)
        pgc = MS.permute_params({**g, **gc}, 100 + v)
        for k in g:
            dist[k] = max(dist[k], _rel(gv[k], pg[k]))
        for k in gc:
            cdist[k] = max(cdist[k], _rel(gcv[k], pgc[k]))
        print(f"t3 variant {v} done", flush=True)
    zall = rec.pop("zall")
    sys.path.insert(0, os.path.join(os.path.dirname(HERE)))
    from goldlib import row_hash
    rec["zall_hash"] = row_hash(zall)
    rec["param_names"] = np.array(list(g))
    rec["ckpt_sha256"] = MRF.ckpt_sha()
    np.savez_compressed(os.path.join(HERE, T3 + ".npz"), **rec)
    out = {"g__" + k: v.astype(np.float32) for k, v in g.items()}
    out.update({"gc__" + k: v.astype(np.float32) for k, v in gc.items()})
    out.update({"gdist__" + k: np.float64(v) for k, v in dist.items()})
    out.update({"gcdist__" + k: np.float64(v) for k, v in cdist.items()})
    out["k_variants"] = K_VARIANTS
    path = os.path.join(HERE, "tg_" + T3 + ".npz")
    np.savez_compressed(path, **out)
    worst = sorted(dist.items(), key=lambda kv: -kv[1])[:4]
    print(path, f"{os.path.getsize(path) / 2**20:.1f} MiB; loss {rec['loss']:.6f}; worst "
          "full-loss self-distances", [(k, round(v, 5)) for k, v in worst], flush=True)


def main():
    import torch
    if sys.argv[1:] == ["t3"]:
        return main_t3()
    cfg, Network, vr = MG._import_reference()
    with open(os.path.join(MG.REF, "data", "nerf_synthetic", "lego", "transforms_test.json")) as f:
        meta = json.load(f)
    for name, spec in MT.SPECS.items():
        gold = dict(np.load(os.path.join(HERE, name + ".npz")))
        params = MG.make_params(*spec["w"])
        rec = MT.capture(name, spec, cfg, Network, vr, meta, params=params, write=False, full=True)
        names = [str(k) for k in gold["param_names"]]
        for k in names:
            assert float(rec["gnorm__" + k]) == float(gold["gnorm__" + k]), k
        g = {k: rec["gfull__" + k] for k in names}
        gc = {k: rec["gcfull__" + k] for k in names if "gcfull__" + k in rec}
        dist = {k: 0.0 for k in g}
        cdist = {k: 0.0 for k in gc}
        for v in range(K_VARIANTS):
            orig = _ulp_libm_ad(torch, 300 + v) if v >= K_VARIANTS // 2 else None
            try:
                rv = MT.capture(name, spec, cfg, Network, vr, meta,
                                params=MS.permute_params(params, 100 + v), write=False, full=True)
            finally:
                for k, fn in (orig or {}).items():
                    setattr(torch, k, fn)
            pg = MS.permute_params(g, 100 + v)       # the golden's gradients, permuted alike
            pgc = MS.permute_params({**g, **gc}, 100 + v)
            for k in g:
                dist[k] = max(dist[k], _rel(rv["gfull__" + k], pg[k]))
            for k in gc:
                cdist[k] = max(cdist[k], _rel(rv["gcfull__" + k], pgc[k]))
        out = {"g__" + k: v.astype(np.float32) for k, v in g.items()}
        out.update({"gc__" + k: v.astype(np.float32) for k, v in gc.items()})
        out.update({"gdist__" + k: np.float64(v) for k, v in dist.items()})
        out.update({"gcdist__" + k: np.float64(v) for k, v in cdist.items()})
        out["k_variants"] = K_VARIANTS
        path = os.path.join(HERE, "tg_" + name + ".npz")
        np.savez_compressed(path, **out)
        worst = sorted(dist.items(), key=lambda kv: -kv[1])[:4]
        print(path, f"{os.path.getsize(path) / 2**20:.1f} MiB; worst full-loss distances",
              [(k, round(v, 5)) for k, v in worst], flush=True)


if __name__ == "__main__":
    main()
