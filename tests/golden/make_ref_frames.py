"""Full 800x800 lego frames rendered by the reference itself (run in this container).

Imports the reference's own ``Network`` and ``Renderer`` from ``/root/reference``
(read-only; the two I/O-only imports ``imageio``/``cv2`` of
``volume_renderer.py:4,7`` get empty stand-ins), loads the trained lego
checkpoint ``checkpoints/lego/latest.pth`` (written by this repository's trainer
in the reference's ``{'net': state_dict}`` format; read with
``weights_only=True``) and renders whole test frames on the CPU through
``Renderer.render(batch)`` (``volume_renderer.py:89-216``) exactly as
``run.py --type evaluate`` would (``run.py:66-78``), under ``torch.no_grad()``.

Frames (BASELINE configs[1] = C2 and configs[3] = C4):
  r0_c2_frame0      test view 0, 64c+128f, ESS/ERT off, perturb 0
  r1_c2_frame8_pert test view 8, 64c+128f, ESS/ERT off, perturb 1 with
                    torch.manual_seed(RSEED) just before render: the per-chunk
                    ``torch.rand([m, 64])`` draws of ``_sample_coarse``
                    (VR:233-234) come from torch's CPU generator, which the
                    test replays with the same seed and chunk order
  r2_c4_frame16     test view 16, ESS + ERT (threshold 0.01), the synthetic
                    occupancy grid ``make_occupancy_grid(0, 128, 1.2, 0.1)``,
                    grid_update_counter 0 (so the reference's call-0 and
                    call-500 grid self-updates, VR:1147-1155, fall inside the
                    frame), perturb 0

Stored per frame (``tests/golden/<name>.npz``, float32 maps, compressed):
rgb_map/depth_map/acc_map and the coarse rgb_map_0/depth_map_0/acc_map_0
(disp is ``1/max(1e-10, depth/acc)`` of these, VR:333); the reference's own
PSNR against the ground truth (evaluators/nerf.py:465-473 formula, GT
white-composited as blender.py:69-71) and that test view's PNG file (``gt_png``,
the dataset's bytes, so the GPU test scores against the same pixels); the
checkpoint's sha256; the render's wall time; for C4 the
final occupancy grid (bit-packed) and call counter. Nothing of the
reference's source is stored - only numbers it produced.

    python tests/golden/make_ref_frames.py            # all frames (~20 min, 8 threads)
    python tests/golden/make_ref_frames.py r0_c2_frame0
    python tests/golden/make_ref_frames.py --add-gt   # store the GT PNG in older files
    python tests/golden/make_ref_frames.py --zall     # zh_<name>.npz, see below

``--zall`` renders each frame again (asserting every map equals the stored
one) and writes ``tests/golden/zh_<name>.npz``: the reference's disp maps
(``disp_map``, ``disp_map_0``, VR:333, NaN where acc = 0), the fine depths
the fine composite received for EVERY ray as a 32-bit row hash
(``zall_hash``, ``goldlib.row_hash`` of the float32 bits of the [S+NI]
sorted row, VR:183: 2.5 MB per frame instead of 491 MB of depths) and, with
ERT, each chunk's ``low_transmittance.any()`` decision per composite call
(VR:1108-1116). A hash collision can only make two different rows look equal,
which the tail attribution then counts as unexplained (a test failure), never
the other way round.
"""
from __future__ import annotations

import json
import os
import sys
import time
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
CKPT = os.path.join(REPO, "checkpoints", "lego", "latest.pth")
RSEED = 20261017

sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))
from nerfhip.synthetic import make_occupancy_grid  # noqa: E402

FRAMES = {
    "r0_c2_frame0": dict(frame=0, perturb=0, ess=False, ert=False),
    "r1_c2_frame8_pert": dict(frame=8, perturb=1, ess=False, ert=False, seed=RSEED),
    "r2_c4_frame16": dict(frame=16, perturb=0, ess=True, ert=True, thr=0.01,
                          grid=(0, 128, 1.2, 0.1), counter=0),
}


def _import_reference():
    sys.argv = ["make_ref_frames", "--cfg_file", "configs/nerf/lego.yaml"]
    os.chdir(REF)
    sys.path.insert(0, REF)
    for m in ("imageio", "cv2"):
        sys.modules.setdefault(m, types.ModuleType(m))
    from src.config import cfg
    from src.models.nerf.network import Network
    import src.models.nerf.renderer.volume_renderer as vr
    return cfg, Network, vr


def ckpt_sha():
    import hashlib
    with open(CKPT, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def gt_png(frame):
    """The test view's PNG file, byte for byte (the dataset's own data)."""
    return np.fromfile(os.path.join(REF, "data/nerf_synthetic/lego/test", f"r_{frame}.png"),
                       np.uint8)


def gt_image(frame):
    """blender.py:53-71: RGBA png / 255, rgb*a + (1-a) (white background), 800x800."""
    import io
    from PIL import Image
    img = np.asarray(Image.open(io.BytesIO(gt_png(frame).tobytes())), np.float32) / 255.0
    return img[..., :3] * img[..., 3:] + (1.0 - img[..., 3:])


def psnr(pred, gt):
    """evaluators/nerf.py:465-473: clip both to [0,1], mse in float32, -10 log10(mse)."""
    pred = np.clip(pred, 0, 1)
    gt = np.clip(gt, 0, 1)
    mse = np.mean((pred - gt) ** 2)
    return float(-10.0 * np.log10(mse))


def capture(name, spec, cfg, Network, vr, meta):
    import torch
    cfg.task_arg.N_importance = 128
    cfg.task_arg.perturb = spec["perturb"]
    cfg.task_arg.lindisp = False
    cfg.enable_ess = spec["ess"]
    cfg.enable_ert = spec["ert"]
    if "thr" in spec:
        cfg.ert_threshold = spec["thr"]
    net = Network()
    sd = torch.load(CKPT, map_location="cpu", weights_only=True)["net"]
    net.load_state_dict(sd)
    net.eval()
    rend = vr.Renderer(net)
    rend.use_cuda_kernels = False
    if "grid" in spec:
        rend.occupancy_grid = torch.from_numpy(make_occupancy_grid(*spec["grid"]).copy())
        rend.grid_update_counter = spec["counter"]
    H = W = 800
    angle = float(meta["camera_angle_x"])
    focal = 0.5 * W / np.tan(0.5 * angle)                       # blender.py:41-42
    pose = np.array(meta["frames"][spec["frame"]]["transform_matrix"], np.float32)
    K = np.array([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], np.float32)
    batch = {"H": H, "W": W, "pose": torch.from_numpy(pose)[None],
             "intrinsics": torch.from_numpy(K)[None]}
    if "seed" in spec:
        torch.manual_seed(spec["seed"])
    t0 = time.time()
    with torch.no_grad():
        ret = rend.render(batch)
    dt = time.time() - t0
    out = {k: v.numpy().astype(np.float32) for k, v in ret.items() if not k.startswith("disp")}
    gt = gt_image(spec["frame"])
    extra = {}
    if "grid" in spec:
        extra["grid_final_bits"] = np.packbits(rend.occupancy_grid.numpy().reshape(-1))
        extra["grid_counter_final"] = np.int64(rend.grid_update_counter)
    p = psnr(out["rgb_map"], gt)
    p0 = psnr(out["rgb_map_0"], gt)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), pose=pose, K=K, H=H, W=W,
                        frame=spec["frame"], perturb=spec["perturb"],
                        seed=spec.get("seed", -1), ess=spec["ess"], ert=spec["ert"],
                        thr=spec.get("thr", 0.0), grid_spec=np.array(spec.get("grid", ()),
                                                                      np.float64),
                        counter0=spec.get("counter", -1), psnr_ref=p, psnr_ref_0=p0,
                        cpu_seconds=dt, torch_threads=torch.get_num_threads(),
                        gt_png=gt_png(spec["frame"]), ckpt_sha256=ckpt_sha(),
                        **{f"out_{k}": v for k, v in out.items()}, **extra)
    print(f"{name}: {dt:.0f} s on {torch.get_num_threads()} threads, PSNR fine {p:.4f} dB, "
          f"coarse {p0:.4f} dB", flush=True)


def capture_zall(name, spec, cfg, Network, vr, meta):
    """Re-render `name` with the fine composite's depths hashed per ray."""
    import torch
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from goldlib import row_hash
    cfg.task_arg.N_importance = 128
    cfg.task_arg.perturb = spec["perturb"]
    cfg.task_arg.lindisp = False
    cfg.enable_ess = spec["ess"]
    cfg.enable_ert = spec["ert"]
    if "thr" in spec:
        cfg.ert_threshold = spec["thr"]
    net = Network()
    net.load_state_dict(torch.load(CKPT, map_location="cpu", weights_only=True)["net"])
    net.eval()
    rend = vr.Renderer(net)
    rend.use_cuda_kernels = False
    if "grid" in spec:
        rend.occupancy_grid = torch.from_numpy(make_occupancy_grid(*spec["grid"]).copy())
        rend.grid_update_counter = spec["counter"]
    comp_name = "_raw2outputs_with_ert" if rend.enable_ert else "_raw2outputs"
    orig_c = getattr(rend, comp_name)
    calls = {"n": 0}
    hashes, chunk_any = [], []

    def rec_c(raw, z, rays_d):
        r = orig_c(raw, z, rays_d)
        if rend.enable_ert:          # VR:1104-1116, the chunk-wide decision of this call
            d = torch.cat([z[..., 1:] - z[..., :-1], torch.full_like(z[..., :1], 1e10)], -1)
            d = d * torch.norm(rays_d[..., None, :], dim=-1)
            a = 1. - torch.exp(-torch.relu(raw[..., 3]) * d)
            sh = torch.cat([torch.zeros_like(a[:, :1]), a[:, :-1]], 1)
            chunk_any.append(bool((torch.cumprod(1.0 - sh, 1) < rend.ert_threshold).any()))
        if calls["n"] % 2 == 1:      # fine call of the chunk (VR:190-193)
            hashes.append(row_hash(z.detach().numpy()))
        calls["n"] += 1
        return r

    setattr(rend, comp_name, rec_c)
    H = W = 800
    focal = 0.5 * W / np.tan(0.5 * float(meta["camera_angle_x"]))
    pose = np.array(meta["frames"][spec["frame"]]["transform_matrix"], np.float32)
    K = np.array([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], np.float32)
    batch = {"H": H, "W": W, "pose": torch.from_numpy(pose)[None],
             "intrinsics": torch.from_numpy(K)[None]}
    if "seed" in spec:
        torch.manual_seed(spec["seed"])
    t0 = time.time()
    with torch.no_grad():
        ret = rend.render(batch)
    dt = time.time() - t0
    old = np.load(os.path.join(OUT, f"{name}.npz"))
    for k, v in ret.items():
        if not k.startswith("disp"):
            assert np.array_equal(v.numpy(), old["out_" + k]), (name, k)
    zh = np.concatenate(hashes)
    assert zh.shape == (H * W,), zh.shape
    path = os.path.join(OUT, f"zh_{name}.npz")
    np.savez_compressed(path, zall_hash=zh, chunk_any=np.array(chunk_any, bool),
                        disp_map=ret["disp_map"].numpy().astype(np.float32),
                        disp_map_0=ret["disp_map_0"].numpy().astype(np.float32),
                        ckpt_sha256=ckpt_sha())
    print(f"{path}: {os.path.getsize(path) / 1e6:.1f} MB, {dt:.0f} s", flush=True)


def add_gt(name):
    """Add the ground-truth PNG to a frame file written before it was stored."""
    p = os.path.join(OUT, f"{name}.npz")
    z = dict(np.load(p))
    if "gt_png" not in z or "ckpt_sha256" not in z:
        z["gt_png"] = gt_png(int(z["frame"]))
        z["ckpt_sha256"] = ckpt_sha()
        assert abs(psnr(z["out_rgb_map"], gt_image(int(z["frame"]))) - float(z["psnr_ref"])) < 1e-9
        np.savez_compressed(p, **z)


def main(argv):
    if argv and argv[0] == "--add-gt":
        for n in argv[1:] or list(FRAMES):
            add_gt(n)
        return
    zall = "--zall" in argv
    argv = [a for a in argv if a != "--zall"]
    cfg, Network, vr = _import_reference()
    meta = json.load(open(os.path.join(REF, "data/nerf_synthetic/lego/transforms_test.json")))
    names = argv or list(FRAMES)
    for n in names:
        (capture_zall if zall else capture)(n, FRAMES[n], cfg, Network, vr, meta)


if __name__ == "__main__":
    main(sys.argv[1:])
