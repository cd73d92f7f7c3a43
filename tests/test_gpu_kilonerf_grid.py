"""The density-driven occupancy grid on the HIP path (VR:875-961,
``_populate_occupancy_grid_kilonerf_method``): NerfPipeline.populate_grid_kilonerf
and the plugin's method of the reference's name, against the reference's own
grids (tests/golden/kg_res<R>.npz, make_kilonerf_grid.py) in both MLP
precisions: bit for bit, apart from cells whose reference max density lies
within 1e-4 of the threshold (none at R = 16, 32); the sub-points bit-equal to
the oracle's (float32 op order of VR:908-919); the cells' own-position option
equal to the reference's per-cell decisions."""
import os

import numpy as np
import pytest

from oracle import nerf_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
CKPT = os.path.join(os.path.dirname(HERE), "checkpoints", "lego")
MARGIN = 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _pipe(dev, prec):
    from nerfhip.render import NerfPipeline
    p = NerfPipeline(dev, N_samples=64, N_importance=128, enable_ess=True, enable_ert=True,
                     mlp_precision=prec)
    p.load_checkpoint(CKPT)
    return p


def _own(res, dec):
    f = np.arange(res ** 3)
    g = np.zeros(res ** 3, bool)
    g[((f % res) * res + (f % (res * res)) // res) * res + f // (res * res)] = dec
    return g


def test_grid_points_bit_equal_to_oracle(dev):
    from nerfhip._lib import call, ptr, stream_of
    import ctypes
    for res in (16, 37):
        pts = torch.empty((res ** 3 * 27, 3), device=dev)
        cf = ctypes.c_float * 3
        cell = (np.float32(4.0) / np.float32(res)).item()
        call("nerf_grid_points", 0, res ** 3, res, cf(-2.0, -2.0, -2.0), cf(cell, cell, cell),
             ptr(pts), stream_of(dev))
        torch.cuda.synchronize()
        assert np.array_equal(pts.cpu().numpy().reshape(-1, 27, 3), O.grid_points(res)), res


@pytest.mark.parametrize("res", [16, 32])
@pytest.mark.parametrize("prec", ["f16x3", "fp32"])
def test_populated_grid_equals_reference(dev, res, prec):
    z = np.load(os.path.join(GOLDEN, f"kg_res{res}.npz"))
    thr = float(z["threshold"])
    ref = np.unpackbits(z["grid_bits"])[:res ** 3].astype(bool)
    rd = z["cell_max_density"].astype(np.float64)
    pipe = _pipe(dev, prec)
    g = pipe.populate_grid_kilonerf(res, threshold=thr, cells_per_pass=5000).cpu().numpy()
    assert pipe.grid_res == res and g.dtype == np.uint8
    near = np.abs(rd - thr) < MARGIN
    dest = O.reference_cell_order(res)
    diff = g.astype(bool) != ref
    assert not (diff & ~np.isin(np.arange(res ** 3), dest[near])).any(), (int(diff.sum()),
                                                                          int(near.sum()))
    assert int(diff.sum()) == 0 or near.any()
    # the cells' own positions: the reference's per-cell decisions, unpermuted
    own = pipe.populate_grid_kilonerf(res, threshold=thr, reference_order=False).cpu().numpy()
    assert np.array_equal(own.astype(bool) | _own(res, near), _own(res, rd > thr) | _own(res, near))


def test_plugin_method_populates_the_renderers_grid(dev):
    """The drop-in's Renderer._populate_occupancy_grid_kilonerf_method (the
    reference's name and effect: the Renderer's grid replaced in place, at its
    resolution) on the trained checkpoint, at resolution 16 via cfg."""
    from src.config import cfg, reset
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    z = np.load(os.path.join(GOLDEN, "kg_res16.npz"))
    reset()
    cfg.enable_ess = True
    cfg.occupancy_grid_resolution = 16
    try:
        net = Network().to(dev)
        sd = torch.load(os.path.join(CKPT, "latest.pth"), map_location="cpu",
                        weights_only=True)["net"]
        net.load_state_dict(sd)
        net.eval()
        rend = Renderer(net)
        assert rend.occupancy_grid.shape == (16, 16, 16)
        rend._populate_occupancy_grid_kilonerf_method()
        got = rend.occupancy_grid.cpu().numpy().reshape(-1)
    finally:
        reset()
    assert np.array_equal(np.packbits(got), z["grid_bits"])
