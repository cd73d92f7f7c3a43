"""Novel-view spiral path and the PSNR evaluator (CPU)."""
import numpy as np
import pytest

from goldlib import load
from nerfhip import evaluate as E
from nerfhip.paths import spiral_poses


@pytest.mark.parametrize("n,rots,zr", [(30, 2, 0.5), (7, 1, 0.25)])
def test_spiral_matches_reference(n, rots, zr):
    ref = load("p1_spiral_poses")[f"spiral_{n}_{rots}_{zr}"]
    poses = load("lego_test_cameras")["poses"]
    got = spiral_poses(poses, n, rots, zr)
    assert got.shape == (n, 4, 4)
    np.testing.assert_allclose(got, ref, atol=1e-12, rtol=0)
    R = got[:, :3, :3]            # orthonormal camera frames
    np.testing.assert_allclose(np.einsum("nij,nik->njk", R, R), np.tile(np.eye(3), (n, 1, 1)),
                               atol=1e-12)


def test_white_composite_and_resize():
    rgba = np.zeros((4, 6, 4), np.float32)
    rgba[..., 0] = 1.0
    rgba[..., 3] = 0.25
    gt = E.composite_white(rgba)
    np.testing.assert_allclose(gt[..., 0], 1.0)
    np.testing.assert_allclose(gt[..., 1:], 0.75)
    assert E.resize_bilinear(gt, 4, 6) is gt
    small = E.resize_bilinear(gt, 2, 3)
    assert small.shape == (2, 3, 3)
    np.testing.assert_allclose(small, gt[:2, :3], atol=1e-6)      # constant image


def test_psnr_formula_and_average():
    gt = np.full((8, 8, 3), 0.5, np.float32)
    pred = gt + 0.1
    assert abs(E.psnr(pred, gt) - 20.0) < 1e-5                     # mse 0.01
    assert E.psnr(gt, gt) == float("inf")
    assert abs(E.psnr(np.full_like(gt, 2.0), np.ones_like(gt))) == float("inf")   # clipped
    frames = [(None, None, gt), (None, None, gt)]
    res = E.evaluate(lambda H, W, pose, K: pred.reshape(-1, 3), frames)
    assert res["psnr"] == [pytest.approx(20.0, abs=1e-5)] * 2 and abs(res["psnr_mean"] - 20) < 1e-5


def _ssim_bruteforce(x, y, win=7, C1=1e-4, C2=9e-4):
    """Window-by-window SSIM over the interior windows (the ones skimage keeps
    after cropping), sample (N-1) covariance, mean over pixels then channels."""
    H, W, C = x.shape
    p = win // 2
    out = []
    for c in range(C):
        vals = []
        for i in range(p, H - p):
            for j in range(p, W - p):
                a = x[i - p:i + p + 1, j - p:j + p + 1, c].ravel()
                b = y[i - p:i + p + 1, j - p:j + p + 1, c].ravel()
                ma, mb = a.mean(), b.mean()
                va, vb = a.var(ddof=1), b.var(ddof=1)
                cab = ((a - ma) * (b - mb)).sum() / (a.size - 1)
                vals.append(((2 * ma * mb + C1) * (2 * cab + C2)) /
                            ((ma * ma + mb * mb + C1) * (va + vb + C2)))
        out.append(np.mean(vals))
    return float(np.mean(out))


def test_ssim_matches_windowed_definition():
    rng = np.random.default_rng(0)
    gt = rng.random((20, 17, 3)).astype(np.float32)
    pred = np.clip(gt + rng.normal(0, 0.05, gt.shape), 0, 1).astype(np.float32)
    assert abs(E.ssim(pred, gt) - _ssim_bruteforce(pred.astype(np.float64),
                                                   gt.astype(np.float64))) < 1e-12
    assert E.ssim(gt, gt) == pytest.approx(1.0, abs=1e-12)
    assert E.ssim(pred, gt) < 1.0
    assert E.ssim(pred[:5, :5], gt[:5, :5]) == pytest.approx(
        _ssim_bruteforce(pred[:5, :5].astype(np.float64), gt[:5, :5].astype(np.float64), win=5),
        abs=1e-12)
    res = E.evaluate(lambda H, W, pose, K: pred, [(None, None, gt)])
    assert res["ssim_mean"] == pytest.approx(E.ssim(pred, gt))
