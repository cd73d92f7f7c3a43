"""Blender ground truth and PSNR as the reference evaluates them.

* ground truth: RGBA in [0, 1] composited on white, rgb * a + (1 - a)
  (src/datasets/nerf/blender.py:60-75), bilinear resize (align_corners=False)
  when the render size differs (:77-84);
* PSNR: both images clipped to [0, 1], mse = mean((pred - gt)^2),
  psnr = -10 log10(mse) (inf for mse = 0) (src/evaluators/nerf.py:465-473,
  :50-58), averaged over frames (:502-504).
"""
from __future__ import annotations

import numpy as np


def composite_white(rgba):
    rgba = np.asarray(rgba, np.float32)
    if rgba.shape[-1] == 4:
        a = rgba[..., 3:4]
        return rgba[..., :3] * a + (np.float32(1.0) - a)
    return rgba[..., :3]


def resize_bilinear(img, H, W):
    import torch
    if img.shape[:2] == (H, W):
        return img
    t = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1)[None]
    t = torch.nn.functional.interpolate(t, size=(H, W), mode="bilinear", align_corners=False)
    return t[0].permute(1, 2, 0).numpy()


def load_gt(path, H=None, W=None):
    """A Blender test image (PNG, RGBA 8-bit) as the reference's target."""
    from PIL import Image
    img = np.asarray(Image.open(path), np.float32) / np.float32(255.0)
    img = composite_white(img)
    return resize_bilinear(img, H or img.shape[0], W or img.shape[1])


def decode_png(buf):
    """uint8 PNG file bytes -> float32 [H,W,C] in [0, 1] (blender.py:53-56: /255)."""
    import io
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(np.asarray(buf).tobytes())), np.float32) / \
        np.float32(255.0)


def load_packed(path, H=None, W=None, indices=None):
    """Views packed by tools/pack_lego.py as the reference's dataset yields them
    (blender.py:38-84): white-composited RGB [N,H,W,3] float32, poses [N,4,4],
    focal (0.5 W / tan(0.5 camera_angle_x), blender.py:41-42) and the json frame
    indices."""
    z = np.load(path)
    offs = z["png_offsets"]
    idx = range(len(offs) - 1) if indices is None else indices
    imgs = []
    for i in idx:
        img = composite_white(decode_png(z["png_bytes"][offs[i]:offs[i + 1]]))
        imgs.append(resize_bilinear(img, H or img.shape[0], W or img.shape[1]))
    imgs = np.stack(imgs)
    focal = 0.5 * imgs.shape[2] / np.tan(0.5 * float(z["camera_angle_x"]))
    return imgs, z["poses"][list(idx)], float(focal), z["frames"][list(idx)]


def psnr(pred, gt):
    pred = np.clip(np.asarray(pred, np.float64), 0, 1)
    gt = np.clip(np.asarray(gt, np.float64), 0, 1)
    mse = np.mean((pred - gt) ** 2)
    return float("inf") if mse == 0 else float(-10.0 * np.log10(mse))


def evaluate(render, frames):
    """frames: iterable of (pose, K, gt [H,W,3]); render(H, W, pose, K) -> rgb
    [H*W,3] or [H,W,3]. Returns per-frame PSNRs and their mean."""
    vals = []
    for pose, K, gt in frames:
        H, W = gt.shape[:2]
        rgb = np.asarray(render(H, W, pose, K)).reshape(H, W, 3)
        vals.append(psnr(rgb, gt))
    return {"psnr": vals, "psnr_mean": float(np.mean(vals)) if vals else float("nan")}
