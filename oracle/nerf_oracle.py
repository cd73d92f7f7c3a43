"""numpy restatement of the reference NeRF render path (test oracle only).

Every function names the reference lines it restates; citations are relative
to the reference repository root (``src/models/nerf/renderer/volume_renderer.py``
is abbreviated ``VR``, ``src/models/nerf/network.py`` is ``NET``,
``src/models/encoding/freq.py`` is ``FREQ``).

Numerics: elementwise work is float32 with one rounding per torch op (no fused
multiply-adds), matching the op sequence of the reference. ``torch.cumsum`` /
``torch.cumprod`` on CPU accumulate float32 inputs in double and round each
output, so the scans here do the same. Reductions (``torch.sum``) and GEMMs
use a different summation order than torch's CPU kernels; they agree to a few
float32 ulps. RNG draws (``torch.rand``) are explicit inputs.

Constant tables that the reference builds with ``torch.linspace`` on the CPU
(coarse depths, eval-mode fine ``u``) are built with ``torch.linspace`` here
too, so the exact float32 values match.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


# ----------------------------------------------------------------------------
# constant tables (VR:218-226, VR:247-251)
# ----------------------------------------------------------------------------
def linspace_f32(start, end, steps) -> np.ndarray:
    """torch.linspace on the CPU in float32 (the values the reference sees)."""
    import torch
    return torch.linspace(float(start), float(end), steps=int(steps),
                          dtype=torch.float32).numpy()


def coarse_depths(near: float, far: float, n_samples: int, lindisp: bool) -> np.ndarray:
    """VR:220-224: z = near*(1-t) + far*t (or the lindisp form), float32."""
    t = linspace_f32(0.0, 1.0, n_samples)
    near32, far32 = F32(near), F32(far)
    if not lindisp:
        return (near32 * (F32(1.0) - t) + far32 * t).astype(F32)
    inv = (F32(1.0) / near32) * (F32(1.0) - t) + (F32(1.0) / far32) * t
    return (F32(1.0) / inv).astype(F32)


# ----------------------------------------------------------------------------
# rays (VR:115-143)
# ----------------------------------------------------------------------------
def camera_rays(H: int, W: int, pose: np.ndarray, K: np.ndarray):
    """VR:119-140. Integer pixel centres, R·d, t as origin, then normalise.

    Returns rays_o [H*W,3], rays_d [H*W,3] (unit length) in float32.
    """
    pose = np.asarray(pose, F32)
    K = np.asarray(K, F32)
    xs = linspace_f32(0, W - 1, W)
    ys = linspace_f32(0, H - 1, H)
    i = np.broadcast_to(xs[None, :], (H, W))        # VR:120-123 (i.t())
    j = np.broadcast_to(ys[:, None], (H, W))
    dx = (i - K[0, 2]) / K[0, 0]
    dy = (-(j - K[1, 2])) / K[1, 1]
    dz = -np.ones_like(dx)
    dirs = np.stack([dx, dy, dz], -1).astype(F32)   # VR:126-128
    R = pose[:3, :3]
    prod = dirs[..., None, :] * R                   # [H,W,3,3], VR:132
    rays_d = ((prod[..., 0] + prod[..., 1]) + prod[..., 2]).astype(F32)
    rays_o = np.broadcast_to(pose[:3, 3], rays_d.shape).astype(F32)
    rays_o = rays_o.reshape(-1, 3)
    rays_d = rays_d.reshape(-1, 3)
    rays_d = (rays_d / ray_norm(rays_d)[:, None]).astype(F32)    # VR:140
    return rays_o, rays_d


def fma32(a, b, c):
    """float32 fused multiply-add (via exact float64 product; double rounding is
    possible only at exact float32 midpoints)."""
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64)
            + np.asarray(c, np.float64)).astype(F32)


def ray_norm(rays_d: np.ndarray) -> np.ndarray:
    """torch.norm(rays_d, dim=-1) on the CPU in float32 (VR:140, VR:292, VR:1095).

    torch's vectorised 2-norm reduction accumulates with fused multiply-adds:
    sqrt(fma(z, z, fma(y, y, x*x))) — checked bit-exact on 200k random rows.
    """
    d = rays_d.astype(F32)
    x2 = (d[:, 0] * d[:, 0]).astype(F32)
    return np.sqrt(fma32(d[:, 2], d[:, 2], fma32(d[:, 1], d[:, 1], x2))).astype(F32)


# ----------------------------------------------------------------------------
# torch CPU float32 reduction orders (used by VR:331-334, VR:255)
# ----------------------------------------------------------------------------
# ATen's cascade sum (SumKernel.cpp; float32, x86 build in this image) reduces
# a contiguous row with 8-wide vectors, 4 independent vector accumulators fed
# through a 4-level cascade, a scalar tail, then the 8 lanes in order; a strided
# reduction (dim -2 of [N,S,3]) uses the same 4-accumulator cascade on scalars.
# Reproduced bit-exactly here (tests/test_oracle_golden.py::test_torch_sum_order).

def _cascade(rows, size, nrows):
    """ATen multi_row_sum: ``rows(i)`` -> list of ``nrows`` float32 arrays."""
    num_levels = 4
    clog2 = 0 if size <= 1 else int(np.ceil(np.log2(size)))
    level_power = max(4, clog2 // num_levels)
    step = 1 << level_power
    lmask = step - 1
    acc = [[None] * nrows for _ in range(num_levels)]

    def add(a, b):
        return b.astype(F32) if a is None else (a + b).astype(F32)

    i = 0
    while i + step <= size:
        for j in range(step):
            r = rows(i + j)
            for k in range(nrows):
                acc[0][k] = add(acc[0][k], r[k])
        i += step
        for j in range(1, num_levels):
            for k in range(nrows):
                if acc[j - 1][k] is not None:
                    acc[j][k] = add(acc[j][k], acc[j - 1][k])
                acc[j - 1][k] = None
            if i & (lmask << (j * level_power)):
                break
    for ii in range(i, size):
        r = rows(ii)
        for k in range(nrows):
            acc[0][k] = add(acc[0][k], r[k])
    for j in range(1, num_levels):
        for k in range(nrows):
            if acc[j][k] is not None:
                acc[0][k] = add(acc[0][k], acc[j][k])
    return acc[0]


def _row_sum(load, size, zero):
    """ATen row_sum: 4-way ILP over ``load(i)`` then a serial tail."""
    ilp = 4
    n_ilp = size // ilp
    ps = _cascade(lambda i: [load(i * ilp + k) for k in range(ilp)], n_ilp, ilp)
    for i in range(n_ilp * ilp, size):
        ps[0] = load(i).astype(F32) if ps[0] is None else (ps[0] + load(i)).astype(F32)
    out = ps[0]
    for k in range(1, ilp):
        if ps[k] is not None:
            out = ps[k] if out is None else (out + ps[k]).astype(F32)
    return zero if out is None else out


def tsum_last(x: np.ndarray) -> np.ndarray:
    """torch.sum(x, -1) for contiguous float32 rows, bit-exact."""
    x = np.ascontiguousarray(x, F32)
    n = x.shape[-1]
    lead = x.shape[:-1]
    x2 = x.reshape(-1, n)
    zero = np.zeros(x2.shape[0], F32)
    V = 8
    if n < V:
        return _row_sum(lambda i: x2[:, i], n, zero).reshape(lead)
    nv = n // V
    vec = _row_sum(lambda i: x2[:, i * V:(i + 1) * V], nv, np.zeros((x2.shape[0], V), F32))
    fin = zero.copy()
    for k in range(nv * V, n):
        fin = (fin + x2[:, k]).astype(F32)
    for lane in range(V):
        fin = (fin + vec[:, lane]).astype(F32)
    return fin.reshape(lead)


def tsum_dim2(x: np.ndarray) -> np.ndarray:
    """torch.sum(x, -2) for x [N, S, C] float32 (strided reduction), bit-exact."""
    x = np.asarray(x, F32)
    zero = np.zeros(x.shape[0], F32)
    return np.stack([_row_sum(lambda i, c=c: x[:, i, c], x.shape[1], zero)
                     for c in range(x.shape[2])], -1)


# ----------------------------------------------------------------------------
# sampling (VR:218-268, VR:1009-1087)
# ----------------------------------------------------------------------------
def stratify(z: np.ndarray, t_rand: np.ndarray) -> np.ndarray:
    """VR:228-235 / VR:1080-1085: jitter inside [lower, upper]."""
    mids = (F32(0.5) * (z[..., 1:] + z[..., :-1])).astype(F32)
    upper = np.concatenate([mids, z[..., -1:]], -1)
    lower = np.concatenate([z[..., :1], mids], -1)
    return (lower + (upper - lower) * t_rand.astype(F32)).astype(F32)


def sample_coarse(n_rays: int, near, far, n_samples, lindisp, perturb, t_rand=None):
    """VR:218-237."""
    z = np.broadcast_to(coarse_depths(near, far, n_samples, lindisp), (n_rays, n_samples))
    if perturb > 0.0:
        if t_rand is None:
            raise ValueError("perturb>0 needs explicit t_rand [N, n_samples]")
        return stratify(z, t_rand)
    return np.ascontiguousarray(z)


GRID_BBOX_MIN = np.array([-2.0, -2.0, -2.0], F32)   # VR:842
GRID_BBOX_MAX = np.array([2.0, 2.0, 2.0], F32)      # VR:843


def grid_coords(pts: np.ndarray, res: int) -> np.ndarray:
    """VR:998-1002 / VR:970-974: voxel = long(clamp((p-min)/(max-min),0,1)*(res-1))."""
    nrm = ((pts.astype(F32) - GRID_BBOX_MIN) / (GRID_BBOX_MAX - GRID_BBOX_MIN)).astype(F32)
    nrm = np.clip(nrm, F32(0.0), F32(1.0))
    c = (nrm * F32(res - 1)).astype(F32).astype(np.int64)   # truncation
    return np.clip(c, 0, res - 1)


def is_empty_space(pts: np.ndarray, grid: np.ndarray) -> np.ndarray:
    """VR:992-1007."""
    c = grid_coords(pts, grid.shape[0])
    return ~grid[c[:, 0], c[:, 1], c[:, 2]]


def sample_coarse_ess(rays_o, rays_d, grid, near, far, n_samples, lindisp, perturb,
                      t_rand=None, skip_threshold=0.5):
    """VR:1009-1087 including the shared-row quirk.

    ``z_vals`` is an ``expand``-ed view in the reference (VR:1020), so every
    ``z_vals[i] = ...`` (VR:1077) overwrites the one shared 64-vector and later
    rays read the mutated row (VR:1042). That sequential fold is kept here.
    """
    import torch
    n = rays_o.shape[0]
    row = coarse_depths(near, far, n_samples, lindisp).copy()   # the shared storage
    z0 = np.broadcast_to(row, (n, n_samples))
    pts = (rays_o[:, None, :] + rays_d[:, None, :] * z0[:, :, None]).astype(F32)
    empty = is_empty_space(pts.reshape(-1, 3), grid).reshape(n, n_samples)
    ratios = (empty.sum(1).astype(F32) / F32(n_samples)).astype(F32)
    highly = ratios > F32(skip_threshold)
    for i in np.nonzero(highly)[0]:
        occ = row[~empty[i]]
        if occ.size == 0:
            continue
        mn, mx = occ.min(), occ.max()
        n_add = max(0, n_samples - occ.size)
        if n_add > 0:
            add = torch.linspace(torch.tensor(mn), torch.tensor(mx), n_add,
                                 dtype=torch.float32).numpy()
            comb = np.concatenate([occ, add])
        else:
            comb = occ.copy()
        row[:] = np.sort(comb)
    z = np.broadcast_to(row, (n, n_samples))
    if perturb > 0.0:
        if t_rand is None:
            raise ValueError("perturb>0 needs explicit t_rand")
        return stratify(z, t_rand)
    return np.ascontiguousarray(z)


def sample_fine(z_mids: np.ndarray, weights_inner: np.ndarray, u: np.ndarray) -> np.ndarray:
    """VR:239-268: inverse-CDF sampling. ``u`` is [N_importance] (eval) or [N, N_importance]."""
    w = (weights_inner.astype(F32) + F32(1e-5)).astype(F32)
    s = tsum_last(w)
    pdf = (w / s[:, None]).astype(F32)
    cdf = np.cumsum(pdf.astype(np.float64), -1).astype(F32)
    cdf = np.concatenate([np.zeros_like(cdf[:, :1]), cdf], -1)       # [N, nb]
    n, nb = cdf.shape
    if u.ndim == 1:
        u = np.broadcast_to(u.astype(F32), (n, u.shape[0]))
    u = u.astype(F32)
    inds = np.empty(u.shape, np.int64)
    for r in range(n):                                               # searchsorted right=True
        inds[r] = np.searchsorted(cdf[r], u[r], side="right")
    below = np.maximum(0, inds - 1)
    above = np.minimum(nb - 1, inds)
    c0 = np.take_along_axis(cdf, below, 1)
    c1 = np.take_along_axis(cdf, above, 1)
    b0 = np.take_along_axis(z_mids, below, 1)
    b1 = np.take_along_axis(z_mids, above, 1)
    denom = (c1 - c0).astype(F32)
    denom = np.where(denom < F32(1e-5), F32(1.0), denom).astype(F32)
    t = ((u - c0) / denom).astype(F32)
    return (b0 + t * (b1 - b0)).astype(F32)


# ----------------------------------------------------------------------------
# encoder + MLP (FREQ:7-32, NET:49-74, VR:270-284)
# ----------------------------------------------------------------------------
def embed(x: np.ndarray, n_freq: int) -> np.ndarray:
    """FREQ:7-32 with include_input, log_sampling, [sin, cos] per band."""
    bands = (2.0 ** np.arange(n_freq)).astype(F32)   # exact powers of two (FREQ:19)
    out = [x.astype(F32)]
    for f in bands:
        xf = (x * f).astype(F32)
        out.append(np.sin(xf).astype(F32))
        out.append(np.cos(xf).astype(F32))
    return np.concatenate(out, -1)


def _lin(x, p, name, relu):
    y = x @ p[name + ".weight"].T
    y = (y + p[name + ".bias"]).astype(F32)
    return np.maximum(y, F32(0.0)) if relu else y


def topology(p, prefix):
    """(D, W, skips, L_xyz, L_dir) of a NeRF state dict (NET:9-43): D from the
    pts_linears present, skips from the layers whose input is [encoding | h]."""
    D = 0
    while f"{prefix}.pts_linears.{D}.weight" in p:
        D += 1
    W, in_x = p[f"{prefix}.pts_linears.0.weight"].shape
    skips = tuple(i for i in range(D - 1)
                  if p[f"{prefix}.pts_linears.{i + 1}.weight"].shape[1] == W + in_x)
    in_v = p[f"{prefix}.views_linears.0.weight"].shape[1] - W
    return D, W, skips, (in_x - 3) // 6, (in_v - 3) // 6


def nerf_mlp(x: np.ndarray, p, prefix: str, skips=None, D=None) -> np.ndarray:
    """NET:49-74 (use_viewdirs=True): returns raw [P,4] = (rgb logits, sigma raw).
    The topology (D, skips, encoding widths) from the state dict (lego: 8, (4,))."""
    D0, _, skips0, lx, _ = topology(p, prefix)
    D = D0 if D is None else D
    skips = skips0 if skips is None else skips
    pts, views = x[:, :3 + 6 * lx], x[:, 3 + 6 * lx:]
    h = pts
    for i in range(D):
        h = _lin(h, p, f"{prefix}.pts_linears.{i}", True)
        if i in skips:
            h = np.concatenate([pts, h], -1)
    alpha = _lin(h, p, f"{prefix}.alpha_linear", False)
    feat = _lin(h, p, f"{prefix}.feature_linear", False)
    h = _lin(np.concatenate([feat, views], -1), p, f"{prefix}.views_linears.0", True)
    rgb = _lin(h, p, f"{prefix}.rgb_linear", False)
    return np.concatenate([rgb, alpha], -1).astype(F32)


def query_network(pts, viewdirs, p, prefix, chunk=4096):
    """VR:270-284: embed xyz (lego: L=10) and dirs (L=4), 4096-point MLP chunks."""
    n, s, _ = pts.shape
    _, _, _, lx, ld = topology(p, prefix)
    flat = pts.reshape(-1, 3)
    e = embed(flat, lx)
    d = np.broadcast_to(viewdirs[:, None, :], pts.shape).reshape(-1, 3)
    e = np.concatenate([e, embed(d, ld)], -1)
    out = np.concatenate([nerf_mlp(e[i:i + chunk], p, prefix)
                          for i in range(0, e.shape[0], chunk)], 0)
    return out.reshape(n, s, 4)


# ----------------------------------------------------------------------------
# compositing (VR:286-357, VR:1089-1157)
# ----------------------------------------------------------------------------
def _dists(z, rays_d):
    d = (z[:, 1:] - z[:, :-1]).astype(F32)
    d = np.concatenate([d, np.full((z.shape[0], 1), F32(1e10))], -1)
    return (d * ray_norm(rays_d)[:, None]).astype(F32)


def _sigmoid(x):
    return (F32(1.0) / (F32(1.0) + np.exp(-x).astype(F32))).astype(F32)


def _maps(w, rgb, z, white_bkgd):
    """VR:331-334 (VR:1126-1129): the reductions in torch's CPU order."""
    rgb_map = tsum_dim2((w[..., None] * rgb).astype(F32))
    depth = tsum_last((w * z).astype(F32))
    acc = tsum_last(w)
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = (depth / acc).astype(F32)
        disp = (F32(1.0) / np.maximum(F32(1e-10), ratio)).astype(F32)   # NaN propagates
    if white_bkgd:
        rgb_map = (rgb_map + (F32(1.0) - acc[:, None])).astype(F32)
    return rgb_map, disp, acc, depth


def raw2outputs(raw, z, rays_d, white_bkgd=True):
    """VR:286-357 (raw_noise_std = 0). Returns rgb, disp, acc, weights, depth."""
    dists = _dists(z, rays_d)
    rgb = _sigmoid(raw[..., :3])
    sig = np.maximum(raw[..., 3], F32(0.0))
    alpha = (F32(1.0) - np.exp(-(sig * dists).astype(F32)).astype(F32)).astype(F32)
    tr = ((F32(1.0) - alpha) + F32(1e-10)).astype(F32)
    cp = np.cumprod(np.concatenate([np.ones((alpha.shape[0], 1), F32), tr], -1)
                    .astype(np.float64), -1).astype(F32)[:, :-1]     # VR:329
    w = (alpha * cp).astype(F32)
    rgb_map, disp, acc, depth = _maps(w, rgb, z, white_bkgd)
    return rgb_map, disp, acc, w, depth


def raw2outputs_ert(raw, z, rays_d, thr, white_bkgd=True, chunk_any=None):
    """VR:1089-1133 (no +1e-10 in the transmittance; chunk-level argmax quirk).

    ``chunk_any`` overrides the chunk-wide ``low_transmittance.any()`` decision
    (VR:1116) when only a slice of a 2048-ray chunk is being recomputed.
    """
    dists = _dists(z, rays_d)
    rgb = _sigmoid(raw[..., :3])
    sig = np.maximum(raw[..., 3], F32(0.0))
    alpha = (F32(1.0) - np.exp(-(sig * dists).astype(F32)).astype(F32)).astype(F32)
    shifted = np.concatenate([np.zeros((alpha.shape[0], 1), F32), alpha[:, :-1]], 1)
    T = np.cumprod((F32(1.0) - shifted).astype(F32).astype(np.float64), 1).astype(F32)
    w = (alpha * T).astype(F32)
    low = T < F32(thr)
    any_low = low.any() if chunk_any is None else bool(chunk_any)
    if any_low:                                     # VR:1115-1123
        first = np.argmax(low, axis=1)              # 0 for rays with no low T
        mask = np.arange(w.shape[1])[None, :] >= first[:, None]
        w = (w * (~mask).astype(F32)).astype(F32)
    rgb_map, disp, acc, depth = _maps(w, rgb, z, white_bkgd)
    return rgb_map, disp, acc, w, depth


def update_grid(grid, rays_d, z, raw, w):
    """VR:1147-1155 + VR:963-990: the reference's grid self-update (uses d*z, no origin)."""
    eff = w > F32(1e-4)
    if not eff.any():
        return
    pts = (rays_d[:, None, :] * z[:, :, None]).astype(F32)[eff]
    dens = np.maximum(raw[..., 3], F32(0.0))[eff]
    occ = dens > F32(0.01)
    if occ.any():
        c = grid_coords(pts[occ], grid.shape[0])
        grid[c[:, 0], c[:, 1], c[:, 2]] = True


# ----------------------------------------------------------------------------
# full render (VR:109-216)
# ----------------------------------------------------------------------------
class RenderConfig:
    def __init__(self, N_samples=64, N_importance=128, near=2.0, far=6.0, lindisp=False,
                 perturb=0.0, white_bkgd=True, enable_ess=False, enable_ert=False,
                 ert_threshold=0.01, chunk_size=4096, ray_chunk=2048, training=False,
                 grid_update_interval=500):
        self.__dict__.update(locals())
        del self.__dict__["self"]


def add_sigma_noise(raw, noise):
    """VR:310-314 / :1098-1103: ``raw[..., 3] + noise`` (one float32 add; noise =
    the reference's torch.randn(...) * raw_noise_std); rgb logits unchanged."""
    out = raw.astype(F32, copy=True)
    out[..., 3] = (out[..., 3] + noise.astype(F32)).astype(F32)
    return out


def render(H, W, pose, K, params, cfg: RenderConfig, t_rand=None, u_fine=None,
           grid=None, grid_counter=0, rays=None, return_zall=False, noise=None):
    """VR:109-216 on the CPU. Returns (dict of maps, final grid_counter).

    ``t_rand`` [H*W, N_samples] supplies the stratification draws when
    ``perturb>0``; ``u_fine`` [H*W, N_importance] the training-mode ``u``; ``grid``
    is the ESS occupancy grid (mutated in place by the reference's update rule).
    ``rays`` = (rays_o, rays_d) overrides the camera (used by sharded tests).
    ``return_zall`` adds ``res["zall"]`` [n, S+NI]: the merged fine depths (VR:183).
    ``noise`` = (coarse [H*W, S], fine [H*W, S+NI]): raw_noise_std > 0's density
    noise, added before each composite (VR:310-314); the grid update reads raw
    without it (VR:1150-1153).
    """
    if rays is None:
        rays_o, rays_d = camera_rays(H, W, pose, K)
    else:
        rays_o, rays_d = rays
    n = rays_o.shape[0]
    u_eval = linspace_f32(0.0, 1.0, cfg.N_importance) if cfg.N_importance > 0 else None
    out = {}
    zalls = []
    counter = grid_counter
    for c0 in range(0, n, cfg.ray_chunk):
        sl = slice(c0, min(n, c0 + cfg.ray_chunk))
        ro, rd = rays_o[sl], rays_d[sl]
        tr = None if t_rand is None else t_rand[sl]
        if cfg.enable_ess:
            z = sample_coarse_ess(ro, rd, grid, cfg.near, cfg.far, cfg.N_samples,
                                  cfg.lindisp, cfg.perturb, tr)
        else:
            z = sample_coarse(ro.shape[0], cfg.near, cfg.far, cfg.N_samples,
                              cfg.lindisp, cfg.perturb, tr)
        pts = (ro[:, None, :] + rd[:, None, :] * z[:, :, None]).astype(F32)
        raw = query_network(pts, rd, params, "model", cfg.chunk_size)

        def comp(raw_, z_, k):
            nonlocal counter
            rn = raw_ if noise is None else add_sigma_noise(raw_, noise[k][sl])
            if cfg.enable_ert:
                r = raw2outputs_ert(rn, z_, rd, cfg.ert_threshold, cfg.white_bkgd)
                if cfg.enable_ess and counter % cfg.grid_update_interval == 0:
                    update_grid(grid, rd, z_, raw_, r[3])
                counter += 1
                return r
            return raw2outputs(rn, z_, rd, cfg.white_bkgd)

        rgb0, disp0, acc0, w0, depth0 = comp(raw, z, 0)
        ret = {"rgb_map_0": rgb0, "disp_map_0": disp0, "acc_map_0": acc0, "depth_map_0": depth0}
        if cfg.N_importance > 0:
            mids = (F32(0.5) * (z[:, 1:] + z[:, :-1])).astype(F32)
            if cfg.training:
                u = u_fine[sl]
            else:
                u = u_eval
            zf = sample_fine(mids, w0[:, 1:-1], u)
            zall = np.sort(np.concatenate([z, zf], -1), -1)
            zalls.append(zall)
            pts_f = (ro[:, None, :] + rd[:, None, :] * zall[:, :, None]).astype(F32)
            raw_f = query_network(pts_f, rd, params, "model_fine", cfg.chunk_size)
            rgb, disp, acc, _, depth = comp(raw_f, zall, 1)
            ret.update({"rgb_map": rgb, "disp_map": disp, "acc_map": acc, "depth_map": depth})
        for k, v in ret.items():
            out.setdefault(k, []).append(v)
    res = {}
    for k, v in out.items():
        a = np.concatenate(v, 0)
        res[k] = a.reshape(H, W, 3) if k.startswith("rgb") else a.reshape(H, W)
    if return_zall and zalls:
        res["zall"] = np.concatenate(zalls, 0)
    return res, counter


# ----------------------------------------------------------------------------
# density-driven occupancy grid (VR:875-961)
# ----------------------------------------------------------------------------
def grid_points(res, bbox_min=(-2.0, -2.0, -2.0), bbox_max=(2.0, 2.0, 2.0)):
    """VR:885-922: the 27 sub-points of every cell, [res^3, 27, 3] float32, in
    the method's flat cell order (f: x = f % res, y = (f % res^2) // res,
    z = f // res^2, VR:903-906) and sub-point order (dz, dy, dx, VR:913-915);
    point = (min + (x, y, z) * cell) + ((dx, dy, dz) / 2) * cell, one float32
    rounding per torch op (VR:908, :918-919)."""
    bmin = np.asarray(bbox_min, F32)
    cell = ((np.asarray(bbox_max, F32) - bmin) / F32(res)).astype(F32)      # VR:889-890
    f = np.arange(res ** 3)
    xyz = np.stack([f % res, (f % (res * res)) // res, f // (res * res)], -1).astype(F32)
    cmin = (bmin + (xyz * cell).astype(F32)).astype(F32)
    d = np.arange(27)
    off = (np.stack([d % 3, (d // 3) % 3, d // 9], -1).astype(F32) / F32(2.0)).astype(F32)
    return (cmin[:, None, :] + (off[None] * cell).astype(F32)).astype(F32)


def reference_cell_order(res, batch=512):
    """VR:950-953: the 512-cell batch's k-th decision lands on the k-th cell of
    list(set(batch_indices)) (each (x, y, z) listed 27 times, VR:922); returns
    the [x][y][z] index per flat cell (int64)."""
    out = np.empty(res ** 3, np.int64)
    rr = res * res
    for b in range(0, res ** 3, batch):
        idx = []
        for f in range(b, min(b + batch, res ** 3)):
            idx += [(f % res, (f % rr) // res, f // rr)] * 27
        order = list(set(idx))
        out[b:b + len(order)] = [(x * res + y) * res + z for x, y, z in order]
    return out


def populate_grid_kilonerf(params, res, threshold=0.01, reference_order=True, prefix="model"):
    """VR:875-961 with the coarse network (sigma does not depend on the view
    input, NET:59-61, so any direction serves; the reference itself cannot run
    the method as written, see tests/golden/make_kilonerf_grid.py): the largest
    relu(sigma) of each cell's 27 points, > threshold, written through the
    reference's cell order. Returns (grid bool [res, res, res], cell max
    density float32 [res^3])."""
    pts = grid_points(res)
    dirs = np.tile(np.array([[0.0, 0.0, 1.0]], F32), (pts.shape[0], 1))
    raw = query_network(pts, dirs, params, prefix)
    dens = np.maximum(raw[..., 3], F32(0.0)).max(1)
    grid = np.zeros(res ** 3, bool)
    dest = reference_cell_order(res) if reference_order else \
        (np.arange(res ** 3) % res * res + (np.arange(res ** 3) % (res * res)) // res) * res \
        + np.arange(res ** 3) // (res * res)
    grid[dest[dens > F32(threshold)]] = True
    return grid.reshape(res, res, res), dens
