"""Capture a train-step golden from the reference renderer (run in the survey container).

C3 semantics: the reference's training-mode render (perturb = 1,
fine-sampling u ~ U[0,1), gradients through _sample_fine, volume_renderer.py:
145-268) on a small ray batch, loss = MSE(rgb_map_0, gt) + MSE(rgb_map, gt)
(trainers/nerf.py:39-76), then backward. Stores the inputs (every torch.rand
draw), the losses and, per parameter, the gradient's float64 norm and sum plus
its first 64 values. Nothing from the reference's source is stored.

    python tests/golden/make_train_golden.py          # t1 and t2

t1: ESS/ERT off, 8x16 crop. t2: ESS + ERT on (lego.yaml:96-99) over a 48x48 crop
(2304 rays = one full 2048-ray chunk + 256), a deterministic occupancy grid and
call counter 0 (the grid self-updates from chunk 0's coarse call), dense weights
so that some rays terminate and the chunk-wide argmax rule (VR:1115-1123) fires;
it also stores all 8 maps, the updated grid and the counter.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

SPECS = {
    "t1_train_step": dict(H=8, W=16, res=800, x0=392, y0=396, frame=0, w=(5, 2.0, 0.5)),
    "t2_train_ess_ert": dict(H=48, W=48, res=800, x0=376, y0=376, frame=0, w=(0, 3.0, 1.0),
                             ess_ert=True, grid=dict(seed=4, radius=0.5, noise=0.01), counter=0),
}


def synthetic_gt(H, W):
    """Deterministic target image in [0, 1] (no dataset offline)."""
    y, x = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    g = np.stack([(x + 0.5) / W, (y + 0.5) / H, 0.5 + 0.25 * np.sin(x * 0.7 + y * 1.3)], -1)
    return g.astype(np.float32)


def main():
    cfg, Network, vr = mg._import_reference()
    with open(os.path.join(mg.REF, "data", "nerf_synthetic", "lego", "transforms_test.json")) as f:
        meta = json.load(f)
    for name, spec in SPECS.items():
        capture(name, spec, cfg, Network, vr, meta)


def capture(name, SPEC, cfg, Network, vr, meta, params=None, write=True, full=False):
    """One reference training step; writes tests/golden/<name>.npz (write=True)
    and returns the record. params overrides the spec's generated weights
    (make_train_sensitivity.py: exact reparametrisations). full: the record
    also holds every gradient tensor, ``gfull__<param>`` (full loss) and
    ``gcfull__<param>`` (coarse loss), float64 (make_train_fullgrad.py)."""
    import torch
    frames, angle = meta["frames"], float(meta["camera_angle_x"])
    cfg.task_arg.N_importance = 128
    cfg.task_arg.perturb = 1
    cfg.task_arg.lindisp = False
    cfg.enable_ess = bool(SPEC.get("ess_ert", False))
    cfg.enable_ert = bool(SPEC.get("ess_ert", False))
    cfg.ert_threshold = 0.01
    seed, gain, ab = SPEC["w"]
    if params is None:
        params = mg.make_params(seed, gain, ab)
    net = Network()
    mg.load_into_network(net, params)
    net.train()
    rend = vr.Renderer(net)
    rend.use_cuda_kernels = False
    if "grid" in SPEC:
        g = SPEC["grid"]
        rend.occupancy_grid = torch.from_numpy(
            mg.make_occupancy_grid(g["seed"], 128, g["radius"], g["noise"]).copy())
        rend.grid_update_counter = SPEC.get("counter", 0)
    pose, K = mg._camera(SPEC, frames, angle)
    H, W = SPEC["H"], SPEC["W"]
    gt = synthetic_gt(H, W)

    draws = []
    orig_rand = torch.rand

    def rec_rand(*a, **kw):
        t = orig_rand(*a, **kw)
        draws.append(t.detach().clone().numpy())
        return t

    batch = {"H": H, "W": W, "pose": torch.from_numpy(pose)[None],
             "intrinsics": torch.from_numpy(K)[None]}
    torch.manual_seed(99)
    torch.rand = rec_rand
    try:
        out = rend.render(batch)
    finally:
        torch.rand = orig_rand
    target = torch.from_numpy(gt).view(-1, 3)
    loss_c = torch.nn.functional.mse_loss(out["rgb_map_0"].view(-1, 3), target)
    loss_f = torch.nn.functional.mse_loss(out["rgb_map"].view(-1, 3), target)
    loss = loss_c + loss_f
    # gradients of the coarse loss alone (no path through the fine samples)
    net.zero_grad()
    loss_c.backward(retain_graph=True)
    coarse_only = {k: p.grad.detach().double().clone() for k, p in net.named_parameters()
                   if p.grad is not None}
    net.zero_grad()
    loss.backward()

    n = H * W
    t_rand = [d for d in draws if d.ndim == 2 and d.shape[1] == cfg.task_arg.N_samples]
    u = [d for d in draws if d.ndim == 2 and d.shape[1] == cfg.task_arg.N_importance]
    rec = dict(H=H, W=W, pose=pose, K=K, gt=gt, w_seed=seed, w_gain=gain, w_alpha_bias=ab,
               w_digest=mg.params_digest(params), t_rand=np.concatenate(t_rand, 0)[:n],
               u=np.concatenate(u, 0)[:n], loss=np.float64(loss.item()),
               loss_coarse=np.float64(loss_c.item()), loss_fine=np.float64(loss_f.item()),
               rgb_map_0=out["rgb_map_0"].detach().numpy().reshape(n, 3),
               rgb_map=out["rgb_map"].detach().numpy().reshape(n, 3),
               enable_ess=cfg.enable_ess, enable_ert=cfg.enable_ert,
               ert_threshold=np.float64(cfg.ert_threshold))
    for k, v in out.items():
        rec["out_" + k] = v.detach().numpy()
    if "grid" in SPEC:
        g = SPEC["grid"]
        rec.update(grid_seed=g["seed"], grid_radius=g["radius"], grid_noise=g["noise"],
                   grid_counter_in=SPEC.get("counter", 0),
                   grid_counter_out=rend.grid_update_counter,
                   grid_out_packed=np.packbits(rend.occupancy_grid.numpy().reshape(-1)))
    names = []
    for k, p in net.named_parameters():
        g = p.grad.detach().double()
        names.append(k)
        rec["gnorm__" + k] = np.float64(g.norm().item())
        rec["gsum__" + k] = np.float64(g.sum().item())
        rec["ghead__" + k] = p.grad.detach().numpy().reshape(-1)[:64].copy()
        if k in coarse_only:
            rec["gcnorm__" + k] = np.float64(coarse_only[k].norm().item())
            rec["gchead__" + k] = coarse_only[k].numpy().reshape(-1)[:64].copy()
        if full:
            rec["gfull__" + k] = g.numpy().copy()
            if k in coarse_only:
                rec["gcfull__" + k] = coarse_only[k].numpy().copy()
    rec["param_names"] = np.array(names)
    if not write:
        return rec
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    print("wrote", path, "loss", loss.item(), "params", len(names))
    return rec


if __name__ == "__main__":
    main()
