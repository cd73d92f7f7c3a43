"""NeRF volume renderer plugin backed by gfx950 HIP kernels.

Drop-in for the reference's ``src/models/nerf/renderer/volume_renderer.py``:
``make_renderer`` loads this file by path (``make_renderer.py:4-7``) and calls
``Renderer(network)``; callers then use ``render(batch) -> dict`` with
``batch = {'H', 'W', 'pose' [1,4,4], 'intrinsics' [1,3,3], ...}`` and get the
reference's maps (``rgb_map_0, disp_map_0, acc_map_0, depth_map_0`` and, with
``N_importance > 0``, ``rgb_map, disp_map, acc_map, depth_map``) shaped [H,W,3] /
[H,W] on ``net.device``.

Semantics follow ``_render_pytorch`` (reference ``volume_renderer.py:109-216``)
including ESS/ERT (``:1009-1157``) and their chunk-level behaviour. There is no
PyTorch fallback: without the built HIP library or a ROCm device, construction
raises ``NerfHipError``.
"""
import numpy as np
import torch

from src.config import cfg
from nerfhip import _lib
from nerfhip.paths import spiral_poses
from nerfhip.render import NerfPipeline, reference_draws_noise


class Renderer:
    def __init__(self, net):
        ta = cfg.task_arg
        self.net = net
        self.N_samples = ta.N_samples
        self.N_importance = ta.N_importance
        self.chunk_size = ta.chunk_size
        self.white_bkgd = bool(ta.white_bkgd)
        self.use_viewdirs = ta.use_viewdirs
        self.lindisp = ta.lindisp
        self.perturb = ta.perturb
        self.raw_noise_std = ta.raw_noise_std
        self.embed_fn = net.embed_fn
        self.embeddirs_fn = net.embeddirs_fn
        self.coarse_model = net.model
        self.fine_model = net.model_fine
        self.device = net.device
        self.near = getattr(cfg, "near", 2.0)
        self.far = getattr(cfg, "far", 6.0)
        self.enable_ess = getattr(cfg, "enable_ess", True)
        self.enable_ert = getattr(cfg, "enable_ert", True)
        self.ert_threshold = getattr(cfg, "ert_threshold", 0.05)
        self.occupancy_grid_resolution = getattr(cfg, "occupancy_grid_resolution", 128)
        self.use_cuda_kernels = True     # the only path here
        self.cuda_blocks = getattr(cfg, "cuda_blocks", 128)
        self.cuda_threads = getattr(cfg, "cuda_threads", 256)
        if not self.use_viewdirs:
            # the reference cannot render it either: its _query_network (VR:270-284)
            # hands NeRF.forward the 63 xyz-encoding columns alone, which splits them
            # as 63 + 27 (network.py:49-51) and raises a RuntimeError
            raise NotImplementedError("use_viewdirs=False: the reference's own NeRF.forward "
                                      "cannot run it (network.py:49-51 splits 63 + 27 columns "
                                      "off a 63-column input)")
        self._check_topology()
        self.pipeline = NerfPipeline(
            self.device, N_samples=self.N_samples, N_importance=self.N_importance,
            near=self.near, far=self.far, lindisp=self.lindisp, white_bkgd=self.white_bkgd,
            enable_ess=self.enable_ess, enable_ert=self.enable_ert,
            ert_threshold=self.ert_threshold,
            # not a reference key: "f16x3" (default, FP32 operands as 3-term FP16
            # splits on FP16 MFMA) or "fp32" (FP32 MFMA); both meet the same parity
            mlp_precision=getattr(cfg, "mlp_precision", "f16x3"))
        self._weights_key = None
        self.scene_bbox_min = torch.tensor([-2.0, -2.0, -2.0], device=self.device)
        self.scene_bbox_max = torch.tensor([2.0, 2.0, 2.0], device=self.device)
        self.grid_update_interval = 1000
        if self.enable_ess:
            self._initialize_occupancy_grid()

    def _check_topology(self):
        """Both networks must be NeRF modules of the reference's kind (network.py:9-43,
        use_viewdirs=True) with the same topology. Lego's (8 x 256, skip after
        layer 4, L = 10 / 4 encodings, lego.yaml:29-44) runs on the fused MLP
        kernels; any other D / W / skips / encoding widths on the layer-by-layer
        FP32 path (nerfhip.generic_mlp), and training then uses the torch MLP back end."""
        from nerfhip.generic_mlp import LEGO, topology
        tops = []
        for prefix, mod in (("model", self.coarse_model), ("model_fine", self.fine_model)):
            sd = {f"{prefix}.{k}": v for k, v in mod.state_dict().items()}
            tops.append(topology(sd, prefix))
        if self.N_importance > 0 and tops[0] != tops[1]:
            raise NotImplementedError(f"coarse {tops[0]} and fine {tops[1]} topologies differ")
        self.lego_topology = tops[0] == LEGO

    # ------------------------------------------------------------- ESS state
    def _initialize_occupancy_grid(self):
        """Reference VR:830-873: sphere (|c| <= 1.2 in [-1,1]^3) OR rand < 0.1. Only
        with ESS on: the reference's version returns at once otherwise (:832-833),
        so its torch.rand draw happens exactly when it does here."""
        res = self.occupancy_grid_resolution
        ax = torch.arange(res, device=self.device, dtype=torch.float32) / (res - 1) * 2.0 - 1.0
        coords = torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1)
        sphere = torch.norm(coords, dim=-1) <= 1.2
        noise = torch.rand((res, res, res), device=self.device) < 0.1
        self.occupancy_grid = sphere | noise
        self.ess_skip_threshold = 0.5
        self.grid_update_interval = 500
        self.pipeline.ess_skip_threshold = self.ess_skip_threshold
        self.pipeline.grid_update_interval = self.grid_update_interval

    def _populate_occupancy_grid_kilonerf_method(self):
        """Reference VR:875-961: the Renderer's grid rebuilt from the coarse
        network's density -- the largest relu(sigma) of 3 x 3 x 3 sub-points per
        cell above 0.01 -- at its resolution over the scene box, on the HIP path
        (NerfPipeline.populate_grid_kilonerf: the sub-points and the decision as
        two small kernels around one fused MLP launch per pass). Each 512-cell
        batch's decisions land on the cells in the order the reference writes
        them (VR:950-953, list(set(...))). Unlike the reference, which hands the
        network its xyz encoding alone and so raises in NeRF.forward
        (network.py:49-51), it runs: the density does not depend on the view
        input. Only with ESS on (VR:880-881)."""
        if not self.enable_ess or self.coarse_model is None:
            return
        self._sync_weights()
        self.pipeline.populate_grid_kilonerf(
            self.occupancy_grid_resolution, self.scene_bbox_min.tolist(),
            self.scene_bbox_max.tolist(), threshold=0.01)

    @property
    def occupancy_grid(self):
        g = self.pipeline.grid
        if g is None:
            return None
        r = self.pipeline.grid_res
        return g.view(r, r, r).bool()

    @occupancy_grid.setter
    def occupancy_grid(self, grid):
        if grid is None:
            self.pipeline.grid = None
        else:
            self.pipeline.set_grid(grid)

    @property
    def grid_update_counter(self):
        return self.pipeline.grid_update_counter

    @grid_update_counter.setter
    def grid_update_counter(self, v):
        self.pipeline.grid_update_counter = int(v)

    # ------------------------------------------------------------- weights
    def _sync_weights(self):
        """Repack when the MLP parameters changed (in-place updates bump _version)."""
        params = list(self.coarse_model.parameters()) + list(self.fine_model.parameters())
        key = tuple((p.data_ptr(), p._version) for p in params)
        if key != self._weights_key:
            sd = {}
            for prefix, mod in (("model", self.coarse_model), ("model_fine", self.fine_model)):
                for k, v in mod.state_dict().items():
                    sd[f"{prefix}.{k}"] = v.detach().float().cpu()
            self.pipeline.set_weights(sd)
            self._weights_key = key

    # ------------------------------------------------------------- render
    def render(self, batch):
        """Reference VR:89-107 -> _render_pytorch contract (HIP path only). With
        the network in training mode and autograd on (trainers/nerf.py:20-37),
        the maps carry gradients into net.model / net.model_fine."""
        if torch.is_grad_enabled() and self.net.training:
            return self._render_train(batch)
        H, W = int(batch["H"]), int(batch["W"])
        pose = torch.as_tensor(batch["pose"]).reshape(-1, 4, 4)[0].float()
        K = torch.as_tensor(batch["intrinsics"]).reshape(-1, 3, 3)[0].float()
        self._sync_weights()
        # the reference's draws in its order: per 2048-ray chunk t_rand (perturb > 0,
        # also at eval: lego.yaml:22), the coarse composite's density noise
        # (raw_noise_std > 0, VR:310-314), u when the net is in training mode, the
        # fine composite's noise
        std = float(self.raw_noise_std or 0.0)
        t_rand, u, nc, nf = reference_draws_noise(H * W, self.N_samples, self.N_importance,
                                                  float(self.perturb), self.net.training,
                                                  self.device, std)
        noise = (nc, nf if nf is not None else nc) if std > 0 else None
        with torch.no_grad():
            res = self.pipeline.render_image(H, W, pose, K, t_rand=t_rand, u=u, noise=noise)
        out = {}
        for k, v in res.items():
            out[k] = v.view(H, W, 3) if k.startswith("rgb") else v.view(H, W)
        return out

    def _render_train(self, batch):
        """Training-mode render (VR:109-268 with self.net.training): rays and
        coarse depths from the HIP kernels, both MLPs forward + backward on the
        x3 MFMA training kernels (cfg ``train_mlp``: "x3", default, or "torch"),
        compositing and importance sampling on the HIP training ops
        (nerfhip/train_ops.py; with ERT the chunk-rule composite of
        nerfhip.train.composite_ert); the reference's
        RNG order per 2048-ray chunk (perturb draw, then fine u) and its ESS/ERT
        chunk semantics (nerfhip.train.render_rays_train)."""
        from nerfhip.train import query, render_rays_train
        from nerfhip.train_mlp import query_x3
        H, W = int(batch["H"]), int(batch["W"])
        pose = torch.as_tensor(batch["pose"]).reshape(-1, 4, 4)[0].float()
        K = torch.as_tensor(batch["intrinsics"]).reshape(-1, 3, 3)[0].float()
        rays_o, rays_d = self.pipeline.camera_rays(H, W, pose, K)
        qf = (query if getattr(cfg, "train_mlp", "x3") == "torch" or not self.lego_topology
              else query_x3)
        res = render_rays_train(self.pipeline, self.coarse_model,
                                self.fine_model if self.N_importance > 0 else None,
                                rays_o, rays_d, float(self.perturb), qf,
                                noise_std=float(self.raw_noise_std or 0.0))
        return {k: v.view(H, W, 3) if k.startswith("rgb") else v.view(H, W)
                for k, v in res.items()}

    # ------------------------------------------------------------- paths
    def generate_spiral_poses(self, poses, n_frames=None, n_rots=2, zrate=0.5):
        """VR:359-419: spiral camera path around the given poses ([n_frames, 4, 4])."""
        if n_frames is None:
            n_frames = getattr(cfg, "render_num", 30)
        poses = poses.cpu().numpy() if torch.is_tensor(poses) else np.asarray(poses)
        return spiral_poses(poses, int(n_frames), n_rots, zrate)

    def render_path(self, render_poses, hwf, intrinsics=None, chunk_size=None):
        """VR:421-509: rgb [N,H,W,3] and disp [N,H,W] of every pose through
        render(batch) under no_grad (so perturb / density-noise draws and the ESS
        grid self-update happen as in the reference's loop), clipped like the
        reference (rgb to [0,1], disp to [0, max]). Errors propagate (the reference
        substitutes black frames)."""
        H, W, focal = hwf
        H, W = int(H), int(W)
        if intrinsics is None:
            K = np.array([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], np.float32)
        else:
            K = intrinsics.cpu().numpy() if torch.is_tensor(intrinsics) else np.asarray(intrinsics)
        Kt = torch.as_tensor(np.asarray(K, np.float32))[None]
        rgbs, disps = [], []
        for pose in render_poses:
            pose = pose.cpu().numpy() if torch.is_tensor(pose) else np.asarray(pose, np.float32)
            batch = {"pose": torch.as_tensor(np.asarray(pose, np.float32))[None],
                     "intrinsics": Kt, "H": H, "W": W}
            with torch.no_grad():
                res = self.render(batch)
            key = "rgb_map" if "rgb_map" in res else "rgb_map_0"
            rgb = res[key].cpu().numpy()
            disp = res[key.replace("rgb", "disp")].cpu().numpy()
            mx = np.max(disp)
            rgbs.append(np.clip(rgb, 0, 1))
            disps.append(np.clip(disp, 0, mx if mx > 0 else 1.0))
        return np.array(rgbs), np.array(disps)

    def render_novel_view_sequence(self, poses, hwf, output_dir, exp_name, iteration=0,
                                   intrinsics=None, render_type="spiral"):
        """VR:511-616: render the spiral (cfg.render_num frames) or the given poses
        through render(batch) under no_grad, clip rgb to [0,1] and disp to
        [0, max], convert to 8 bit like the reference, and write
        ``<output_dir>/novel_views/view%04d_{rgb,disp}.png`` (PIL instead of cv2;
        skipped when output_dir is None). The 8-bit frames are also kept in
        ``self.last_sequence`` = (rgb [N,H,W,3] uint8, disp [N,H,W] uint8).
        Video encoding is out of scope: the returned video path is None. Errors
        propagate (the reference prints them and goes on)."""
        import os
        if render_type == "spiral":
            render_poses = self.generate_spiral_poses(poses, n_frames=getattr(cfg, "render_num",
                                                                              120))
        else:
            render_poses = poses.cpu().numpy() if torch.is_tensor(poses) else np.asarray(poses)
        H, W, focal = hwf
        if intrinsics is None:
            Kt = torch.tensor([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]],
                              dtype=torch.float32, device=self.device)
        else:
            Kt = torch.as_tensor(intrinsics).to(self.device)
        images_dir = None
        if output_dir is not None:
            images_dir = os.path.join(output_dir, "novel_views")
            os.makedirs(images_dir, exist_ok=True)
        rgb8s, disp8s = [], []
        with torch.no_grad():
            for i, pose in enumerate(render_poses):
                batch = {"pose": torch.as_tensor(np.asarray(pose), dtype=torch.float32)
                         .to(self.device)[None], "intrinsics": Kt[None], "H": H, "W": W}
                ret = self.render(batch)
                key = "rgb_map" if "rgb_map" in ret else "rgb_map_0"
                rgb = np.clip(ret[key].cpu().numpy(), 0, 1)
                disp = ret[key.replace("rgb", "disp")].cpu().numpy()
                mx = np.max(disp)
                disp = np.clip(disp, 0, mx if mx > 0 else 1.0)
                mx = np.max(disp)
                rgb8 = (255 * rgb).astype(np.uint8)
                with np.errstate(invalid="ignore"):   # NaN disp (acc = 0) casts as the reference's
                    disp8 = (255 * disp / mx if mx > 0 else disp).astype(np.uint8)
                rgb8s.append(rgb8)
                disp8s.append(disp8)
                if images_dir is not None:
                    from PIL import Image
                    Image.fromarray(rgb8).save(os.path.join(images_dir, f"view{i:04d}_rgb.png"))
                    Image.fromarray(disp8).save(os.path.join(images_dir, f"view{i:04d}_disp.png"))
        self.last_sequence = (np.stack(rgb8s), np.stack(disp8s))
        return images_dir, None

    def create_video_from_result_images(self, *a, **kw):
        raise NotImplementedError("video encoding is outside the render hot path")
