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

import ctypes

import numpy as np
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


def reference_draws(n, S, NI, perturb, draw_u, device):
    """The torch.rand draws the reference's ``_render_pytorch`` makes for n rays, in
    its order: per 2048-ray chunk (VR:154) the stratification jitter t_rand [m, S]
    when ``perturb > 0`` (``_sample_coarse`` VR:233-234, or the ESS variant
    :1080-1085) and then, when ``draw_u`` (``self.net.training``, VR:247-249), the
    fine-sampling u [m, NI]. Returns (t_rand [n, S] | None, u [n, NI] | None), so
    a whole-frame pass consumes the same random stream as the chunk loop."""
    return reference_draws_noise(n, S, NI, perturb, draw_u, device, 0.0)[:2]


_CELL_ORDER = {}


def reference_cell_order(res, device=None, batch=512):
    """VR:896-953's assignment of a batch's decisions to cells: the batch of
    cells [b, b + 512) (flat order f: x = f % res, y = (f % res^2) // res,
    z = f // res^2; each listed 27 times, once per sub-point, VR:903-922) gives
    its k-th decision to the k-th element of ``list(set(batch_indices))``.
    Returns int32 [res^3]: the [x][y][z] grid index that cell f's decision
    lands on (cached per resolution). CPython's iteration order of a set of
    small-int tuples is deterministic (tuple hashes of ints are not salted);
    building the set from the unique tuples in first-occurrence order gives the
    same table as with the 27 repeats (asserted by tests/test_kilonerf_grid.py)."""
    key = (res, batch)
    if key not in _CELL_ORDER:
        out = np.empty(res ** 3, np.int32)
        rr = res * res
        for b in range(0, res ** 3, batch):
            cells = [(f % res, (f % rr) // res, f // rr) for f in range(b, min(b + batch, res ** 3))]
            order = list(set(cells))
            out[b:b + len(order)] = [(x * res + y) * res + z for x, y, z in order]
        _CELL_ORDER[key] = out
    t = torch.from_numpy(_CELL_ORDER[key])
    return t.to(device) if device is not None else t


def reference_draws_noise(n, S, NI, perturb, draw_u, device, noise_std):
    """reference_draws plus, when ``noise_std > 0``, the density noise of the two
    composites of every chunk (``torch.randn(raw[..., 3].shape) * raw_noise_std``,
    VR:310-314 / :1098-1103), in the chunk's order: t_rand, the coarse noise
    [m, S], u, the fine noise [m, S + NI]. Returns (t_rand, u, noise_c [n, S],
    noise_f [n, S + NI]), each None when not drawn."""
    tr, uu, nc, nf = [], [], [], []
    for c0 in range(0, n, REF_CHUNK):
        m = min(REF_CHUNK, n - c0)
        if perturb > 0:
            tr.append(torch.rand((m, S), device=device))
        if noise_std > 0:
            nc.append(torch.randn((m, S), device=device) * noise_std)
        if draw_u and NI > 0:
            uu.append(torch.rand((m, NI), device=device))
        if noise_std > 0 and NI > 0:
            nf.append(torch.randn((m, S + NI), device=device) * noise_std)

    def cat(x):
        return torch.cat(x).contiguous() if x else None
    return cat(tr), cat(uu), cat(nc), cat(nf)


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
        self.capture_zall = None  # list -> the merged fine depths [m, S+NI] of every pass (tests)
        self.capture_coarse = None   # list -> (coarse depths [m, S], coarse weights [m, S])
                                     # of every pass: what the fine sampling read (tests)
        self._replaying = False   # replays of foreign update chunks: not in ert_stats
        self.replayed_chunks = 0  # foreign update chunks replayed (multi-GPU C4 overhead)
        self._updates_on = True   # render_chunks switches the grid self-update off for blocks
                                  # of non-consecutive chunks that hold no updating chunk

    # ------------------------------------------------------------------ weights
    def set_weights(self, params, coarse_prefix="model", fine_prefix="model_fine"):
        """params: name -> tensor/array (reference state_dict names). Lego's
        topology (8 x 256, skip 4, L = 10 / 4) is packed for the fused MLP kernels;
        any other runs layer by layer (nerfhip.generic_mlp, FP32)."""
        from .generic_mlp import LEGO, GenericMLP, topology

        def up(prefix):
            if topology(params, prefix) != LEGO:
                return GenericMLP(params, prefix, self.device)
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

    def populate_grid_kilonerf(self, res=None, bbox_min=(-2.0, -2.0, -2.0),
                               bbox_max=(2.0, 2.0, 2.0), threshold=0.01, reference_order=True,
                               cells_per_pass=1 << 18):
        """The reference's density-driven occupancy grid (VR:875-961,
        ``_populate_occupancy_grid_kilonerf_method``) on the HIP path: the 27
        sub-points of every cell (nerf_grid_points), the coarse network's density
        there (the fused MLP of this pipeline's precision: points as rays with a
        zero depth; sigma does not depend on the view input, network.py:59-61),
        and a cell marked where the largest relu(sigma) exceeds ``threshold``
        (nerf_grid_decide). ``reference_order``: each 512-cell batch's decisions
        land on the cells in CPython's iteration order of the batch's
        ``set`` of (x, y, z) tuples, as the reference writes them (VR:950-953,
        reference_cell_order); False: every cell's own decision at its own
        place. Replaces the pipeline's grid and returns it ([res^3] uint8)."""
        res = int(res or self.grid_res or 128)
        bmin = np.asarray(bbox_min, np.float32)
        cell = (np.asarray(bbox_max, np.float32) - bmin) / np.float32(res)   # VR:889-890
        dev = self.device
        st = _lib.stream_of(dev)
        grid = torch.zeros(res ** 3, device=dev, dtype=torch.uint8)       # VR:894
        cell_of = reference_cell_order(res, dev) if reference_order else None
        cf = (ctypes.c_float * 3)
        bm, cs = cf(*bmin.tolist()), cf(*cell.tolist())
        z0 = torch.zeros(1, device=dev, dtype=torch.float32)
        dirs = None
        total = res ** 3
        for c0 in range(0, total, cells_per_pass):
            nc = min(cells_per_pass, total - c0)
            m = nc * 27
            pts = torch.empty((m, 3), device=dev, dtype=torch.float32)
            call("nerf_grid_points", c0, nc, res, bm, cs, ptr(pts), st)
            if dirs is None or dirs.shape[0] < m:
                dirs = torch.tensor([0.0, 0.0, 1.0], device=dev).expand(m, 3).contiguous()
            raw = self.mlp(self.coarse, pts, dirs[:m], z0, 0, m, 1)
            call("nerf_grid_decide", ptr(raw), c0, nc, res, float(threshold), ptr(cell_of),
                 ptr(grid), st)
            del pts, raw
        self.set_grid(grid.view(res, res, res))
        return self.grid

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
        if not isinstance(packed, tuple):   # another topology: the layer-by-layer MLP
            return packed.forward(rays_o, rays_d, z, z_stride, n, S)
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
        if not self._replaying:
            self.ert_stats.append((counts, n, S, active))
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

    def composite(self, raw, z, z_stride, rays_d, n, S, out, off, need_weights=True, noise=None):
        """Writes rgb/disp/acc/depth rows [off, off+n) of `out`; returns the weights
        [n, S] (or None when not needed: the kernel then skips writing them).
        noise [n, S]: added to the density logits first (raw_noise_std > 0,
        VR:310-314 / :1098-1103; `raw` itself is left as it is)."""
        w = (torch.empty((n, S), device=self.device, dtype=torch.float32)
             if need_weights else None)
        if noise is not None:
            noisy = torch.empty_like(raw)
            call("nerf_add_sigma_noise", ptr(raw), ptr(noise), n * S, ptr(noisy),
                 _lib.stream_of(self.device))
            raw = noisy
        rgb, disp, acc, depth = out
        args = (ptr(raw), ptr(z), z_stride, ptr(rays_d), n, S, int(self.white_bkgd))
        tail = (ptr(rgb[off:]), ptr(disp[off:]), ptr(acc[off:]), ptr(depth[off:]), ptr(w),
                _lib.stream_of(self.device))
        if self.enable_ert:   # + the two-pass kernel's workspace (cut maps, chunk flags)
            nb = int(_lib.lib().nerf_composite_ert_workspace(n, REF_CHUNK))
            ws = torch.empty((nb,), device=self.device, dtype=torch.uint8)
            nb = n * S * 16 + (n * S if z_stride else S) * 4 + n * 36 + (n * S * 4 if w is not None else 0)
            self._timed("composite_ert", nb, lambda: call(
                "nerf_composite_ert", *args, self.ert_threshold, REF_CHUNK, *tail[:-1], ptr(ws),
                tail[-1]))
        else:   # raw 16 B/sample, z, rays_d 12 B/ray, maps 24 B/ray, weights 4 B/sample
            nb = n * S * 16 + (n * S if z_stride else S) * 4 + n * 36 + (n * S * 4 if w is not None else 0)
            self._timed("composite", nb, lambda: call("nerf_composite", *args, *tail))
        return w

    # ------------------------------------------------------------------ rays
    def render_rays(self, rays_o, rays_d, t_rand=None, u=None, outputs=None, off=0, noise=None):
        """Render n rays (rows of rays_o/rays_d, [n,3] float32 on the device).

        With ERT/ESS the rays must start on a 2048-ray chunk boundary of the
        reference's chunking (VR:147). noise = (coarse [n, S], fine [n, S+NI]):
        the density noise of raw_noise_std > 0 (reference_draws_noise); the ERT
        sample compaction is off then (its termination test reads raw without
        noise). Returns the per-ray output buffers.
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
            nz_c, nz_f = (None, None) if noise is None else tuple(
                None if x is None else x[p:p + m] for x in noise)
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
            raw = self._pass_mlp(self.coarse, ro, rd, z, zs, m, S, compact=noise is None)
            w = self.composite(raw, z, zs, rd, m, S, outputs["coarse"], off + p, noise=nz_c)
            if self.capture_coarse is not None:
                self.capture_coarse.append(((z if zs else z.expand(m, S)).clone(),
                                            w.reshape(m, S).clone()))
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
                if self.capture_zall is not None:
                    self.capture_zall.append(zall.clone())
                raw_f = self._pass_mlp(self.fine, ro, rd, zall, S + NI, m, S + NI,
                                       compact=noise is None)
                w_f = self.composite(raw_f, zall, S + NI, rd, m, S + NI, outputs["fine"], off + p,
                                     need_weights=self.enable_ert and self.enable_ess, noise=nz_f)
                self._grid_updates(1, counter0, rd, zall, S + NI, raw_f, w_f, m, S + NI)
                del raw_f, w_f, zall
            if self.enable_ert:       # _raw2outputs_with_ert counts its calls (VR:1157)
                self.grid_update_counter = counter0 + self._calls_per_chunk() * -(-m // REF_CHUNK)
            p += m
        return outputs

    def _pass_mlp(self, packed, ro, rd, z, zs, m, S, compact=True):
        if (compact and self.enable_ert and self.ert_compaction and self.mlp_precision == "f16x3"
                and isinstance(packed, tuple)):
            return self.mlp_ert(packed, ro, rd, z, zs, m, S)
        return self.mlp(packed, ro, rd, z, zs, m, S)

    def evaluated_samples(self, reset=True):
        """(MLP samples evaluated, samples of a full evaluation) over the ERT
        passes since the last reset (one host sync)."""
        ev = sum(int(c.sum()) for c, _, _, _ in self.ert_stats)
        full = sum(n * S for _, n, S, _ in self.ert_stats)
        if reset:
            self.ert_stats = []
        return ev, full

    def ert_termination(self):
        """Per ERT pass kind (samples per ray S: coarse / fine), over the passes
        since the last reset: rays retired by the sample compaction (transmittance
        below the threshold before the last depth segment: the reference zeroes
        their later weights, VR:1115-1123) and reference chunks holding at least
        one such ray (where the chunk-wide argmax rule applies)."""
        out = {}
        for _, n, S, active in self.ert_stats:
            d = out.setdefault(S, [0, 0, 0, 0])
            ret = active == 0
            nch = -(-n // REF_CHUNK)
            pad = torch.zeros((nch * REF_CHUNK,), device=ret.device, dtype=torch.bool)
            pad[:n] = ret
            d[0] += n
            d[1] += int(ret.sum())
            d[2] += nch
            d[3] += int(pad.view(nch, REF_CHUNK).any(1).sum())
        return out

    def _calls_per_chunk(self):
        return 2 if self.N_importance > 0 else 1

    def _grid_updates(self, kind, counter0, rd, z, zs, raw, w, m, S):
        """VR:1147-1155: the ERT composite call whose counter is a multiple of the
        interval updates the ESS grid from that chunk's samples (kind 0 = coarse
        call, 1 = fine call of each chunk)."""
        if not (self.enable_ert and self.enable_ess and self._updates_on):
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
        if not self._updates_on:
            return m
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
            self._replay(lambda: self.render_image(H, W, pose, K, p0=a,
                                                   n=min(REF_CHUNK, H * W - a)))

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

    def _replay(self, fn):
        """Run a replay of a foreign chunk (its grid update only; its samples are
        not this rank's and stay out of ert_stats)."""
        self._replaying = True
        self.replayed_chunks += 1
        try:
            return fn()
        finally:
            self._replaying = False

    def _update_chunks(self, total):
        """Chunks of a frame whose ERT calls update the ESS grid (VR:1147-1157),
        given the counter at the frame's first chunk."""
        per, cf = self._calls_per_chunk(), self.grid_update_counter
        return [c for c in range(total)
                if any((cf + per * c + k) % self.grid_update_interval == 0 for k in range(per))]

    def render_chunks(self, H, W, pose, K, chunks, t_rand=None, noise=None):
        """The reference chunks `chunks` (ascending ids of 2048 consecutive
        pixels, VR:147) of a frame whose other chunks other ranks render
        concurrently (dist.render_frame_interleaved: chunk c on rank c mod P),
        with the results of the reference's sequential chunk loop. Returns the
        flat maps of the chunks' pixels, concatenated in the given order
        ({} for an empty list).

        Without ESS + ERT the chunks render as one block (ERT's chunk rule holds
        within it: every chunk is whole and keeps its 2048-ray alignment). With
        both, the ESS grid changes at the chunks whose ERT call counter hits a
        multiple of grid_update_interval, so the owned chunks are rendered in
        blocks between those update chunks (grid updates off inside a block,
        which holds none), each update chunk is rendered -- or, when another
        rank owns it, replayed and discarded -- at its own counter in chunk
        order, and the updates after the last owned chunk are replayed too,
        so every rank leaves the frame with the sequential loop's grid and
        counter. Cost: one extra chunk per foreign update chunk (2 per 500
        ERT calls). t_rand: the frame's perturb draws [H * W, N_samples] (every
        rank holds the same; a chunk reads its own rows); noise: the frame's
        density noise (coarse [H * W, S], fine [H * W, S + NI], raw_noise_std > 0,
        reference_draws_noise), read by rows the same way."""
        total = -(-H * W // REF_CHUNK)
        chunks = [int(c) for c in chunks]
        if chunks != sorted(set(chunks)) or (chunks and not 0 <= chunks[0] <= chunks[-1] < total):
            raise ValueError("chunks must be ascending, distinct ids of the frame's chunks")
        per, cf = self._calls_per_chunk(), self.grid_update_counter
        rays_o, rays_d = self.camera_rays(H, W, pose, K)
        lens = [min(REF_CHUNK, H * W - c * REF_CHUNK) for c in chunks]
        offs = [0]
        for ln in lens:
            offs.append(offs[-1] + ln)
        outputs = self.alloc_outputs(offs[-1]) if chunks else None

        def rows(cs):
            idx = torch.cat([torch.arange(c * REF_CHUNK, c * REF_CHUNK + min(
                REF_CHUNK, H * W - c * REF_CHUNK), device=self.device) for c in cs])
            tr = None if t_rand is None else t_rand.index_select(0, idx)
            nz = None if noise is None else tuple(
                None if x is None else x.index_select(0, idx) for x in noise)
            return rays_o.index_select(0, idx), rays_d.index_select(0, idx), tr, nz

        def block(i0, i1):           # own chunks chunks[i0:i1] as one block, no updates inside
            if i1 <= i0:
                return
            ro, rd, tr, nz = rows(chunks[i0:i1])
            self._updates_on = False
            try:
                self.render_rays(ro, rd, t_rand=tr, outputs=outputs, off=offs[i0], noise=nz)
            finally:
                self._updates_on = True

        if not (self.enable_ess and self.enable_ert):
            block(0, len(chunks))
            if self.enable_ert:
                self.grid_update_counter = cf + per * total
            return maps_dict(outputs) if chunks else {}
        i = 0
        for u in self._update_chunks(total):
            j = i
            while j < len(chunks) and chunks[j] < u:
                j += 1
            block(i, j)
            i = j
            self.grid_update_counter = cf + per * u
            ro, rd, tr, nz = rows([u])
            if i < len(chunks) and chunks[i] == u:
                self.render_rays(ro, rd, t_rand=tr, outputs=outputs, off=offs[i], noise=nz)
                i += 1
            else:
                self._replay(lambda: self.render_rays(ro, rd, t_rand=tr, noise=nz))
        block(i, len(chunks))
        self.grid_update_counter = cf + per * total
        return maps_dict(outputs) if chunks else {}

    def render_image(self, H, W, pose, K, t_rand=None, u=None, p0=0, n=None, noise=None):
        """Render pixels [p0, p0+n) of an H x W image; returns the reference's map dict
        (``rgb_map_0, disp_map_0, acc_map_0, depth_map_0`` + fine maps), flat per pixel.
        noise: (coarse, fine) density noise of these pixels (render_rays)."""
        n = H * W - p0 if n is None else n
        rays_o, rays_d = self.camera_rays(H, W, pose, K, p0, n)
        out = self.render_rays(rays_o, rays_d, t_rand=t_rand, u=u, noise=noise)
        return maps_dict(out)


def maps_dict(out):
    rgb0, disp0, acc0, depth0 = out["coarse"]
    res = {"rgb_map_0": rgb0, "disp_map_0": disp0, "acc_map_0": acc0, "depth_map_0": depth0}
    if "fine" in out:
        rgb, disp, acc, depth = out["fine"]
        res.update({"rgb_map": rgb, "disp_map": disp, "acc_map": acc, "depth_map": depth})
    return res
