"""torch-CPU restatement of the reference render path — TEST INFRASTRUCTURE ONLY.

The same op sequence as the reference's ``_render_pytorch`` (``VR`` =
``src/models/nerf/renderer/volume_renderer.py``) with ESS/ERT off, evaluated by
torch's own CPU kernels (MKL GEMMs, vectorised sin/cos/exp), so it runs at the
speed of the reference's CPU path on the same host. ``bench.py`` times it as the
CPU baseline (``cpu_baseline.kind = "port"``); ``oracle/nerf_oracle.py`` stays
the parity oracle. Checked against the golden renders in
``tests/test_oracle_golden.py::test_torch_cpu_restatement_matches_golden``.
Builder-written; none of the reference's source is used.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def camera_rays(H, W, pose, K):
    """VR:115-143: pixel grid (integer centres), camera directions, rotation by
    the pose (sum over the last axis), origins = translation, unit directions."""
    pose = torch.as_tensor(pose, dtype=torch.float32)
    K = torch.as_tensor(K, dtype=torch.float32)
    i, j = torch.meshgrid(torch.linspace(0, W - 1, W), torch.linspace(0, H - 1, H), indexing="ij")
    i, j = i.t(), j.t()
    dirs = torch.stack([(i - K[0, 2]) / K[0, 0], -(j - K[1, 2]) / K[1, 1], -torch.ones_like(i)], -1)
    rays_d = torch.sum(dirs[..., None, :] * pose[:3, :3], -1).reshape(-1, 3)
    rays_o = pose[:3, 3].expand(H * W, 3)
    rays_d = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
    return rays_o, rays_d


def embed(x, n_freq):
    """FREQ:7-32: cat([x] + [sin(2^k x), cos(2^k x)])."""
    out = [x]
    for f in 2.0 ** torch.linspace(0.0, n_freq - 1, n_freq):
        out += [torch.sin(x * f), torch.cos(x * f)]
    return torch.cat(out, -1)


def nerf_mlp(x, p, prefix):
    """NET:49-74 with use_viewdirs: 8 ReLU layers with the skip cat after layer 4,
    alpha head, feature (no activation), views layer (ReLU), rgb head."""
    lin = lambda h, n: F.linear(h, p[f"{prefix}.{n}.weight"], p[f"{prefix}.{n}.bias"])  # noqa: E731
    pts, views = x[:, :63], x[:, 63:90]
    h = pts
    for i in range(8):
        h = F.relu(lin(h, f"pts_linears.{i}"))
        if i == 4:
            h = torch.cat([pts, h], -1)
    alpha = lin(h, "alpha_linear")
    h = F.relu(lin(torch.cat([lin(h, "feature_linear"), views], -1), "views_linears.0"))
    return torch.cat([lin(h, "rgb_linear"), alpha], -1)


def query(pts, rays_d, p, prefix, chunk=4096):
    """VR:270-284: encode points and per-sample view directions, MLP in 4096-point chunks."""
    n, s, _ = pts.shape
    x = torch.cat([embed(pts.reshape(-1, 3), 10),
                   embed(rays_d[:, None, :].expand(n, s, 3).reshape(-1, 3), 4)], -1)
    return torch.cat([nerf_mlp(x[i:i + chunk], p, prefix)
                      for i in range(0, x.shape[0], chunk)], 0).reshape(n, s, 4)


def raw2outputs(raw, z, rays_d, white_bkgd=True):
    """VR:286-357 (raw_noise_std = 0)."""
    dists = torch.cat([z[..., 1:] - z[..., :-1], torch.full_like(z[..., :1], 1e10)], -1)
    dists = dists * torch.norm(rays_d[..., None, :], dim=-1)
    rgb = torch.sigmoid(raw[..., :3])
    alpha = 1.0 - torch.exp(-F.relu(raw[..., 3]) * dists)
    w = alpha * torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1.0 - alpha + 1e-10], -1),
                              -1)[:, :-1]
    rgb_map = torch.sum(w[..., None] * rgb, -2)
    depth = torch.sum(w * z, -1)
    acc = torch.sum(w, -1)
    disp = 1.0 / torch.max(1e-10 * torch.ones_like(depth), depth / acc)
    if white_bkgd:
        rgb_map = rgb_map + (1.0 - acc[..., None])
    return rgb_map, disp, acc, w, depth


def sample_fine(mids, weights, n_importance):
    """VR:239-268, eval mode (u = linspace)."""
    weights = weights + 1e-5
    pdf = weights / torch.sum(weights, -1, keepdim=True)
    cdf = torch.cat([torch.zeros_like(pdf[..., :1]), torch.cumsum(pdf, -1)], -1)
    u = torch.linspace(0.0, 1.0, n_importance).expand(cdf.shape[0], n_importance).contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    below = torch.clamp(inds - 1, min=0)
    above = torch.clamp(inds, max=cdf.shape[-1] - 1)
    c0, c1 = torch.gather(cdf, -1, below), torch.gather(cdf, -1, above)
    b0, b1 = torch.gather(mids, -1, below), torch.gather(mids, -1, above)
    denom = c1 - c0
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    t = (u - c0) / denom
    return b0 + t * (b1 - b0)


@torch.no_grad()
def render_rays(rays_o, rays_d, params, N_samples=64, N_importance=128, near=2.0, far=6.0,
                white_bkgd=True, ray_chunk=2048):
    """VR:145-216 over 2048-ray chunks, perturb 0, eval. Returns flat maps."""
    p = {k: torch.as_tensor(v, dtype=torch.float32) for k, v in params.items()}
    t = torch.linspace(0.0, 1.0, N_samples)
    zrow = near * (1.0 - t) + far * t
    outs = {}
    for c0 in range(0, rays_o.shape[0], ray_chunk):
        ro, rd = rays_o[c0:c0 + ray_chunk], rays_d[c0:c0 + ray_chunk]
        z = zrow.expand(ro.shape[0], N_samples)
        raw = query(ro[..., None, :] + rd[..., None, :] * z[..., :, None], rd, p, "model")
        rgb0, disp0, acc0, w, depth0 = raw2outputs(raw, z, rd, white_bkgd)
        ret = {"rgb_map_0": rgb0, "disp_map_0": disp0, "acc_map_0": acc0, "depth_map_0": depth0}
        if N_importance > 0:
            zf = sample_fine(0.5 * (z[..., 1:] + z[..., :-1]), w[..., 1:-1], N_importance)
            z2, _ = torch.sort(torch.cat([z, zf], -1), -1)
            raw2 = query(ro[..., None, :] + rd[..., None, :] * z2[..., :, None], rd, p,
                         "model_fine")
            rgb, disp, acc, _, depth = raw2outputs(raw2, z2, rd, white_bkgd)
            ret.update(rgb_map=rgb, disp_map=disp, acc_map=acc, depth_map=depth)
        for k, v in ret.items():
            outs.setdefault(k, []).append(v)
    return {k: torch.cat(v, 0).numpy() for k, v in outs.items()}
