"""Blender ground truth and PSNR as the reference evaluates them.

* ground truth: RGBA in [0, 1] composited on white, rgb * a + (1 - a)
  (src/datasets/nerf/blender.py:60-75), bilinear resize (align_corners=False)
  when the render size differs (:77-84);
* PSNR: both images clipped to [0, 1], mse = mean((pred - gt)^2),
  psnr = -10 log10(mse) (inf for mse = 0) (src/evaluators/nerf.py:465-473,
  :50-58), averaged over frames (:502-504);
* SSIM: skimage's structural_similarity as the evaluator calls it (:65-107),
  restated (scikit-image is not in this image).
"""
from __future__ import annotations

import os

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


def load_packed(path, H=None, W=None, indices=None, workers=None):
    """Views packed by tools/pack_lego.py as the reference's dataset yields them
    (blender.py:38-84): white-composited RGB [N,H,W,3] float32, poses [N,4,4],
    focal (0.5 W / tan(0.5 camera_angle_x), blender.py:41-42) and the json frame
    indices. The views are decoded and composited on a thread pool (PIL's
    decoder and numpy release the GIL; ~75 ms of CPU per 800x800 view), each
    into its slot of one preallocated array."""
    from concurrent.futures import ThreadPoolExecutor
    z = np.load(path)
    offs = z["png_offsets"]
    buf = z["png_bytes"]
    idx = list(range(len(offs) - 1) if indices is None else indices)

    def one(i):
        img = composite_white(decode_png(buf[offs[i]:offs[i + 1]]))
        return resize_bilinear(img, H or img.shape[0], W or img.shape[1])

    first = one(idx[0]) if idx else np.zeros((H or 0, W or 0, 3), np.float32)
    imgs = np.empty((len(idx),) + first.shape, np.float32)
    if idx:
        imgs[0] = first

        def put(k):
            imgs[k] = one(idx[k])
        n = workers or min(16, os.cpu_count() or 1, len(idx))
        with ThreadPoolExecutor(max(1, n)) as ex:
            list(ex.map(put, range(1, len(idx))))
    focal = 0.5 * imgs.shape[2] / np.tan(0.5 * float(z["camera_angle_x"]))
    return imgs, z["poses"][list(idx)], float(focal), z["frames"][list(idx)]


def psnr(pred, gt):
    """evaluators/nerf.py:463-473 + psnr_metric (:24-63): both images clipped to
    [0, 1] in their own dtype (float32 renders), mse = np.mean((pred - gt)^2) in
    that dtype, psnr = 20 log10(1) - 10 log10(mse) (inf for mse = 0)."""
    pred = np.clip(np.asarray(pred), 0, 1)
    gt = np.clip(np.asarray(gt), 0, 1)
    mse = np.mean((pred - gt) ** 2)
    if mse == 0:
        return float("inf")
    return float(20 * np.log10(1.0) - 10 * np.log10(mse))


def ssim(pred, gt, win_size=None, data_range=1.0):
    """evaluators/nerf.py:65-107: skimage.metrics.structural_similarity(pred, gt,
    win_size=min(7, H, W), data_range=1.0, channel_axis=2) on the [0, 1]-clipped
    images. scikit-image is absent here and unpinned by the reference
    (requirements.txt), so this restates its published default algorithm (Wang
    et al. 2004 as skimage implements it): uniform win x win window
    (scipy.ndimage.uniform_filter), K1 = 0.01, K2 = 0.03, sample covariance
    (N / (N - 1)), the SSIM map cropped by (win - 1) / 2 on every side and
    averaged, then averaged over the channels; computed in float64. Parity with
    skimage itself is unpinned."""
    from scipy.ndimage import uniform_filter
    X = np.clip(np.asarray(pred, np.float64), 0, 1)
    Y = np.clip(np.asarray(gt, np.float64), 0, 1)
    if X.shape != Y.shape:
        raise ValueError("ssim: images differ in shape")
    if X.ndim == 2:
        X, Y = X[..., None], Y[..., None]
    if win_size is None:
        win_size = min(7, X.shape[0], X.shape[1])
    if win_size % 2 == 0 or win_size > min(X.shape[0], X.shape[1]):
        raise ValueError("ssim: win_size must be odd and fit the image")
    C1, C2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
    cov = win_size ** 2 / (win_size ** 2 - 1.0)
    pad = (win_size - 1) // 2
    vals = []
    for c in range(X.shape[2]):
        x, y = X[..., c], Y[..., c]
        f = lambda a: uniform_filter(a, size=win_size)   # noqa: E731
        ux, uy = f(x), f(y)
        vx = cov * (f(x * x) - ux * ux)
        vy = cov * (f(y * y) - uy * uy)
        vxy = cov * (f(x * y) - ux * uy)
        S = ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux * ux + uy * uy + C1) * (vx + vy + C2))
        vals.append(S[pad:S.shape[0] - pad, pad:S.shape[1] - pad].mean())
    return float(np.mean(vals))


def evaluate(render, frames, with_ssim=True):
    """frames: iterable of (pose, K, gt [H,W,3]); render(H, W, pose, K) -> rgb
    [H*W,3] or [H,W,3]. Per-frame PSNR (and SSIM) and their means
    (evaluators/nerf.py:495-517)."""
    vals, ssims = [], []
    for pose, K, gt in frames:
        H, W = gt.shape[:2]
        rgb = np.asarray(render(H, W, pose, K)).reshape(H, W, 3)
        vals.append(psnr(rgb, gt))
        if with_ssim:
            ssims.append(ssim(rgb, gt))
    res = {"psnr": vals, "psnr_mean": float(np.mean(vals)) if vals else float("nan")}
    if with_ssim:
        res.update(ssim=ssims, ssim_mean=float(np.mean(ssims)) if ssims else float("nan"))
    return res
