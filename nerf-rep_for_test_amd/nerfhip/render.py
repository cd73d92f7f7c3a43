"""Device pipeline of the NeRF render path: the reference ``_render_pytorch``
(``src/models/nerf/renderer/volume_renderer.py:109-216``, "VR") as a chain of
gfx950 kernels behind the C ABI.

Per pass over a block of rays (no 2048-ray Python loop; the reference's chunk
boundaries only matter for ERT/ESS and are kept there):

  nerf_rays -> [nerf_sample_coarse | nerf_sample_coarse_ess] -> nerf_mlp_forward
  -> nerf_composite[_ert] -> nerf_sample_fine -> nerf_mlp_forward -> composite

Constant tables the reference builds with ``torch.linspace`` (coarse depths,
eval-mode fine ``u``) are computed by the same torch CPU ops and uploaded, so
the kernels see the reference's exact float32 values.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import call, ptr
from .pack import pack_mlp, pack_mlp_x3

REF_CHUNK = 2048            # VR:147 ray chunk (ERT/ESS semantics)
GRID_BBOX = (-2.0, 2.0)     # VR:842-843


def coarse_depth_table(near, far, n_samples, lindisp):
    """VR:220-224 with torch on the CPU (float32), exactly the reference's values."""
    t_vals = torch.linspace(0., 1., steps=n_samples)
    if not lindisp:
        return near * (1. - t_vals) + far * t_vals
    return 1. / (1. / near * (1. - t_vals) + 1. / far * t_vals)


MLP_KERNELS = {"fp32": ("nerf_mlp_forward", pack_mlp),
               "f16x3": ("nerf_mlp_forward_x3", pack_mlp_x3)}


class NerfPipeline:
    """Packed weights + constant tables resident on one GPU; renders rays/frames."""

    def __init__(self, device, N_samples=64, N_importance=128, near=2.0, far=6.0,
                 lindisp=False, white_bkgd=True, enable_ess=False, enable_ert=False,
                 ert_threshold=0.05, ess_skip_threshold=0.5, grid_update_interval=500,
                 max_rays_per_pass=1 << 20, mlp_precision="f16x3", ert_compaction=True,
                 ert_segment=8):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _lib.NerfHipError("NerfPipeline needs a ROCm GPU device (no CPU fallback)")
        _lib.lib()
        self.N_samples = int(N_samples)
        self.N_importance = int(N_importance)
        self.near, self.far, self.lindisp = float(near), float(far), bool(lindisp)
        self.white_bkgd = bool(white_bkgd)
        self.enable_ess, self.enable_ert = bool(enable_ess), bool(enable_ert)
        self.ert_threshold = float(ert_threshold)
        self.ess_skip_threshold = float(ess_skip_threshold)
        self.grid_update_interval = int(grid_update_interval)
        self.grid_update_counter = 0
        self.max_rays_per_pass = int(max_rays_per_pass)
        # "fp32": FP32 MFMA (mlp_fused.hip); "f16x3": 3-term FP16 split of the FP32
        # operands on FP16 MFMA (mlp_x3.hip), ~2^-22 relative per product
        if mlp_precision not in MLP_KERNELS:
            raise ValueError(f"mlp_precision must be one of {sorted(MLP_KERNELS)}")
        self.mlp_precision = mlp_precision
        # ERT passes: the MLP runs depth segment by depth segment and skips the
        # samples after each ray's termination (x3 kernel only; results identical).
        # Segments of 8 evaluate 78.6 % of a lego frame's samples (32: 83.3 %);
        # C4 1.94 vs 1.86 Mrays/s measured (bench.py --ert-segment)
        self.ert_compaction = bool(ert_compaction)
        self.ert_segment = int(ert_segment)
        self.ert_stats = []       # (evaluated-sample counts [segments] device, rays, S) per pass
        self.z_base = coarse_depth_table(self.near, self.far, self.N_samples,
                                         self.lindisp).to(self.device)
        self.u_eval = (torch.linspace(0., 1., steps=self.N_importance).to(self.device)
                       if self.N_importance > 0 else None)
        self.grid = None          # uint8 [res^3] device, ESS occupancy (VR:830-873)
        self.grid_res = 0
        self.coarse = None
        self.fine = None
        self.timer = None         # list -> (start event, end event, samples, bytes) per MLP launch
        self.stage_timer = None   # list -> (kernel, start event, end event, algorithmic bytes)

    # ------------------------------------------------------------------ weights
    def set_weights(self, params, coarse_prefix="model", fine_prefix="model_fine"):
        """params: name -> tensor/array (reference state_dict names)."""
        def up(prefix):
            sl, hd = MLP_KERNELS[self.mlp_precision][1](params, prefix)
            return (torch.from_numpy(sl).to(self.device), torch.from_numpy(hd).to(self.device))
        self.coarse = up(coarse_prefix)
        self.fine = up(fine_prefix) if self.N_importance > 0 else None

    def load_checkpoint(self, model_dir, epoch=-1):
        """Weights from a checkpoint in the reference's format (nerfhip.checkpoint)."""
        from .checkpoint import network_params
        self.set_weights(network_params(model_dir, epoch))

    def set_grid(self, grid):
        g = torch.as_tensor(grid)
        self.grid_res = int(g.shape[0])
        self.grid = g.to(device=self.device, dtype=torch.uint8).contiguous().view(-1)

    # ------------------------------------------------------------------ stages
    # algorithmic MACs of one NeRF MLP evaluation (NET:49-74): 63*256 + 4*256^2
    # + 319*256 + 2*256^2 + 256 (alpha) + 256^2 (feature) + 283*128 + 128*3
    MLP_FLOP_PER_SAMPLE = 2 * 593408
    MLP_WEIGHT_BYTES = 4 * (_lib.MLP_SLICES * _lib.MLP_SLICE_FLOATS + _lib.MLP_HEAD_FLOATS)

    @classmethod
    def mlp_bytes(cls, n, S, z_stride):
        """Algorithmic HBM bytes of one MLP launch: raw out (16 B/sample), rays o/d
        (24 B/ray), z (4 B/sample, or one shared row when z_stride == 0), weights once."""
        return n * S * 16 + n * 24 + (n * S if z_stride else S) * 4 + cls.MLP_WEIGHT_BYTES

    def mlp(self, packed, rays_o, rays_d, z, z_stride, n, S):
        raw = torch.empty((n * S, 4), device=self.device, dtype=torch.float32)
        t = self.timer
        if t is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
        call(MLP_KERNELS[self.mlp_precision][0], ptr(packed[0]), ptr(packed[1]), ptr(rays_o), ptr(rays_d),
             ptr(z), z_stride, n, S, ptr(raw), _lib.stream_of(self.device))
        if t is not None:
            e1.record()
            t.append((e0, e1, n * S, self.mlp_bytes(n, S, z_stride)))
        return raw

    def mlp_ert(self, packed, rays_o, rays_d, z, z_stride, n, S):
        """The MLP of an ERT pass over depth segments of ert_segment samples
        (nerf_ert_segment + nerf_mlp_forward_x3_list, no host round trip): a ray
        stops being evaluated once its transmittance falls below the threshold,
        after which _raw2outputs_with_ert zeroes every weight it has
        (VR:1115-1123); its remaining raw stay 0. The composite then sees exactly
        the values it reads from a full evaluation."""
        dev = self.device
        st = _lib.stream_of(dev)
        raw = torch.zeros((n * S, 4), device=dev, dtype=torch.float32)
        T = torch.ones((n,), device=dev, dtype=torch.float64)
        active = torch.ones((n,), device=dev, dtype=torch.uint8)
        b = list(range(0, S, self.ert_segment)) + [S]
        nseg = len(b) - 1
        counts = torch.zeros((nseg,), device=dev, dtype=torch.int32)
        lst = torch.empty((n * min(S, self.ert_segment),), device=dev, dtype=torch.int32)
        t = self.timer
        for k in range(nseg):
            s0, s1 = (b[k - 1], b[k]) if k else (0, 0)
            cnt = counts[k:k + 1]
            call("nerf_ert_segment", ptr(raw), ptr(z), z_stride, ptr(rays_d), n, S, s0, s1,
                 b[k + 1], self.ert_threshold, ptr(T), ptr(active), ptr(lst), ptr(cnt), st)
            if t is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
            call("nerf_mlp_forward_x3_list", ptr(packed[0]), ptr(packed[1]), ptr(rays_o),
                 ptr(rays_d), ptr(z), z_stride, S, ptr(lst), ptr(cnt), n * (b[k + 1] - b[k]),
                 ptr(raw), st)
            if t is not None:
                e1.record()
                t.append((e0, e1, cnt, None))
        self.ert_stats.append((counts, n, S))
        return raw

    def _timed(self, name, nbytes, fn):
        """Run fn(); with stage_timer set, bracket it by HIP events on the launch
        stream and record (name, events, algorithmic bytes)."""
        t = self.stage_timer
        if t is None:
            return fn()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn()
        e1.record()
        t.append((name, e0, e1, nbytes))
        return r

    def composite(self, raw, z, z_stride, rays_d, n, S, out, off, need_weights=True):
        """Writes rgb/disp/acc/depth rows [off, off+n) of `out`; returns the weights
        [n, S] (or None when not needed: the kernel then skips writing them)."""
        w = (torch.empty((n, S), device=self.device, dtype=torch.float32)
             if need_weights else None)
        rgb, disp, acc, depth = out
        args = (ptr(raw), ptr(z), z_stride, ptr(rays_d), n, S, int(self.white_bkgd))
        tail = (ptr(rgb[off:]), ptr(disp[off:]), ptr(acc[off:]), ptr(depth[off:]), ptr(w),
                _lib.stream_of(self.device))
        if self.enable_ert:
            call("nerf_composite_ert", *args, self.ert_threshold, REF_CHUNK, *tail)
        else:   # raw 16 B/sample, z, rays_d 12 B/ray, maps 24 B/ray, weights 4 B/sample
            nb = n * S * 16 + (n * S if z_stride else S) * 4 + n * 36 + (n * S * 4 if w is not None else 0)
            self._timed("composite", nb, lambda: call("nerf_composite", *args, *tail))
        return w

    # ------------------------------------------------------------------ rays
    def render_rays(self, rays_o, rays_d, t_rand=None, u=None, outputs=None, off=0):
        """Render n rays (rows of rays_o/rays_d, [n,3] float32 on the device).

        With ERT/ESS the rays must start on a 2048-ray chunk boundary of the
        reference's chunking (VR:147). Returns the per-ray output buffers.
        """
        n = rays_o.shape[0]
        S, NI = self.N_samples, self.N_importance
        dev = self.device
        if outputs is None:
            outputs = self.alloc_outputs(n)
        if self.coarse is None:
            raise _lib.NerfHipError("set_weights() first")
        st = _lib.stream_of(dev)
        step = self.max_rays_per_pass
        if self.enable_ess or self.enable_ert:
            step = max(REF_CHUNK, (step // REF_CHUNK) * REF_CHUNK)
        p = 0
        while p < n:
            m = min(step, n - p)
            if self.enable_ess and self.enable_ert:
                m = self._ess_phase_len(m)
            counter0 = self.grid_update_counter
            ro, rd = rays_o[p:p + m], rays_d[p:p + m]
            tr = None if t_rand is None else t_rand[p:p + m]
            if self.enable_ess:
                if self.grid is None:
                    raise _lib.NerfHipError("ESS enabled but no occupancy grid set")
                z = torch.empty((m, S), device=dev, dtype=torch.float32)
                call("nerf_sample_coarse_ess", ptr(ro), ptr(rd), ptr(self.grid), self.grid_res,
                     ptr(self.z_base), ptr(tr), m, S, REF_CHUNK, self.ess_skip_threshold,
                     ptr(z), st)
                zs = S
            elif tr is not None:
                z = torch.empty((m, S), device=dev, dtype=torch.float32)
                call("nerf_sample_coarse", ptr(self.z_base), ptr(tr), m, S, ptr(z), st)
                zs = S
            else:
                z, zs = self.z_base, 0                     # one shared row (expand)
            raw = self._pass_mlp(self.coarse, ro, rd, z, zs, m, S)
            w = self.composite(raw, z, zs, rd, m, S, outputs["coarse"], off + p)
            self._grid_updates(0, counter0, rd, z, zs, raw, w, m, S)
            if NI > 0:
                zall = torch.empty((m, S + NI), device=dev, dtype=torch.float32)
                if u is None:
                    uu, us = self.u_eval, 0
                else:
                    uu, us = u[p:p + m], NI
                nb = m * S * 4 + (m * S if zs else S) * 4 + (m * NI if us else NI) * 4 \
                    + m * (S + NI) * 4   # weights, z, u in; merged depths out
                self._timed("sample_fine", nb, lambda: call(
                    "nerf_sample_fine", ptr(z), zs, ptr(w), ptr(uu), us, m, S, NI, ptr(zall), st))
                del raw, w
                raw_f = self._pass_mlp(self.fine, ro, rd, zall, S + NI, m, S + NI)
                w_f = self.composite(raw_f, zall, S + NI, rd, m, S + NI, outputs["fine"], off + p,
                                     need_weights=self.enable_ert and self.enable_ess)
                self._grid_updates(1, counter0, rd, zall, S + NI, raw_f, w_f, m, S + NI)
                del raw_f, w_f, zall
            if self.enable_ert:       # _raw2outputs_with_ert counts its calls (VR:1157)
                self.grid_update_counter = counter0 + self._calls_per_chunk() * -(-m // REF_CHUNK)
            p += m
        return outputs

    def _pass_mlp(self, packed, ro, rd, z, zs, m, S):
        if self.enable_ert and self.ert_compaction and self.mlp_precision == "f16x3":
            return self.mlp_ert(packed, ro, rd, z, zs, m, S)
        return self.mlp(packed, ro, rd, z, zs, m, S)

    def evaluated_samples(self, reset=True):
        """(MLP samples evaluated, samples of a full evaluation) over the ERT
        passes since the last reset (one host sync)."""
        ev = sum(int(c.sum()) for c, _, _ in self.ert_stats)
        full = sum(n * S for _, n, S in self.ert_stats)
        if reset:
            self.ert_stats = []
        return ev, full

    def _calls_per_chunk(self):
        return 2 if self.N_importance > 0 else 1

    def _grid_updates(self, kind, counter0, rd, z, zs, raw, w, m, S):
        """VR:1147-1155: the ERT composite call whose counter is a multiple of the
        interval updates the ESS grid from that chunk's samples (kind 0 = coarse
        call, 1 = fine call of each chunk)."""
        if not (self.enable_ert and self.enable_ess):
            return
        per = self._calls_per_chunk()
        for c in range(-(-m // REF_CHUNK)):
            if (counter0 + per * c + kind) % self.grid_update_interval == 0:
                a, b = c * REF_CHUNK, min(m, (c + 1) * REF_CHUNK)
                call("nerf_grid_update", ptr(rd[a:b]), ptr(z[a:] if zs else z), zs,
                     ptr(raw[a * S:]), ptr(w[a:b]), b - a, S, ptr(self.grid), self.grid_res,
                     _lib.stream_of(self.device))

    def _ess_phase_len(self, m):
        """Cut a pass after the first chunk that updates the grid, so later
        chunks' ESS sees the updated grid as in the reference's sequential loop."""
        per = self._calls_per_chunk()
        c0 = self.grid_update_counter
        for c in range(-(-m // REF_CHUNK)):
            if any((c0 + per * c + k) % self.grid_update_interval == 0 for k in range(per)):
                return min(m, (c + 1) * REF_CHUNK)
        return m

    def alloc_outputs(self, n):
        def grp():
            return (torch.empty((n, 3), device=self.device, dtype=torch.float32),
                    torch.empty((n,), device=self.device, dtype=torch.float32),
                    torch.empty((n,), device=self.device, dtype=torch.float32),
                    torch.empty((n,), device=self.device, dtype=torch.float32))
        out = {"coarse": grp()}
        if self.N_importance > 0:
            out["fine"] = grp()
        return out

    # ------------------------------------------------------------------ frames
    def camera_rays(self, H, W, pose, K, p0=0, n=None):
        n = H * W - p0 if n is None else n
        cam = torch.cat([torch.as_tensor(pose, dtype=torch.float32).reshape(-1)[:16],
                         torch.as_tensor(K, dtype=torch.float32).reshape(-1)[:9]]).to(self.device)
        rays_o = torch.empty((n, 3), device=self.device, dtype=torch.float32)
        rays_d = torch.empty((n, 3), device=self.device, dtype=torch.float32)
        call("nerf_rays", ptr(cam), int(H), int(W), int(p0), int(n), ptr(rays_o), ptr(rays_d),
             _lib.stream_of(self.device))
        return rays_o, rays_d

    def render_band(self, H, W, pose, K, p0, n):
        """Pixels [p0, p0+n) of a frame whose other pixels other ranks render
        concurrently, with the results of the reference's sequential chunk loop
        (VR:147-205). Without ESS+ERT that is render_image. With both, the ESS
        grid self-updates at the chunks whose ERT call counter hits a multiple of
        grid_update_interval (VR:1147-1157) and later chunks sample against the
        updated grid (VR:1009-1087), so a band must see every earlier update:
        this rank replays each updating chunk before its band (in chunk order,
        each replay at that chunk's counter), renders its band at the counter of
        its first chunk, then replays the updating chunks after its band, so
        that every rank leaves the frame with the grid and counter the
        sequential loop ends with. Bands start on 2048-ray chunk boundaries.
        Cost: one extra chunk per update outside the band (2 per 500 calls).
        Returns the map dict ({} for an empty band)."""
        per = self._calls_per_chunk()
        cf = self.grid_update_counter
        total = -(-H * W // REF_CHUNK)
        if not (self.enable_ess and self.enable_ert):
            res = self.render_image(H, W, pose, K, p0=p0, n=n) if n > 0 else {}
            if self.enable_ert:       # the counter only drives ESS grid updates
                self.grid_update_counter = cf + per * total
            return res
        if n > 0 and p0 % REF_CHUNK:
            raise ValueError("with ESS + ERT a band must start on a 2048-ray chunk boundary")
        # an empty band (a rank past the last pixel, p0 = H*W) lies after every chunk
        c0 = p0 // REF_CHUNK if n > 0 else total
        c1 = -(-(p0 + n) // REF_CHUNK) if n > 0 else total
        upd = [c for c in range(total)
               if any((cf + per * c + k) % self.grid_update_interval == 0 for k in range(per))]

        def replay(c):
            self.grid_update_counter = cf + per * c
            a = c * REF_CHUNK
            self.render_image(H, W, pose, K, p0=a, n=min(REF_CHUNK, H * W - a))

        for c in upd:
            if c < c0:
                replay(c)
        self.grid_update_counter = cf + per * c0
        res = self.render_image(H, W, pose, K, p0=p0, n=n) if n > 0 else {}
        for c in upd:
            if c >= c1:
                replay(c)
        self.grid_update_counter = cf + per * total
        return res

    def render_image(self, H, W, pose, K, t_rand=None, u=None, p0=0, n=None):
        """Render pixels [p0, p0+n) of an H x W image; returns the reference's map dict
        (``rgb_map_0, disp_map_0, acc_map_0, depth_map_0`` + fine maps), flat per pixel."""
        n = H * W - p0 if n is None else n
        rays_o, rays_d = self.camera_rays(H, W, pose, K, p0, n)
        out = self.render_rays(rays_o, rays_d, t_rand=t_rand, u=u)
        return maps_dict(out)


def maps_dict(out):
    rgb0, disp0, acc0, depth0 = out["coarse"]
    res = {"rgb_map_0": rgb0, "disp_map_0": disp0, "acc_map_0": acc0, "depth_map_0": depth0}
    if "fine" in out:
        rgb, disp, acc, depth = out["fine"]
        res.update({"rgb_map": rgb, "disp_map": disp, "acc_map": acc, "depth_map": depth})
    return res
