"""Network topologies other than lego's (reference ``network.py:9-74``: any D,
W, skips and encoding widths), CPU side: the oracle against the reference's own
render of the g1 fixture (``tests/golden/make_golden.py g1``: D 6, W 128, skips
[2, 3], L 8 / 3, the reference's own initialisation, 32x32 crop, 64 + 64
samples). The HIP layer-by-layer path is held to the same numbers in
``test_gpu_generic.py``."""
import numpy as np
import pytest

from goldlib import load, load_zall, max_err, oracle_cfg, params_of, rel_err
from oracle import nerf_oracle as O

TOL = 1e-5


def test_topology_of_the_fixture():
    from nerfhip.generic_mlp import LEGO, topology
    p = params_of(load("g1_generic"))
    assert topology(p, "model") == topology(p, "model_fine") == (6, 128, (2, 3), 8, 3)
    assert O.topology(p, "model") == (6, 128, (2, 3), 8, 3)
    from nerfhip.synthetic import make_params
    assert topology(make_params(0, 2.0, 0.0), "model") == LEGO


def test_oracle_render_matches_reference():
    """Coarse maps within 1e-5; fine maps within 1e-4 end to end (fine depths are
    ill-conditioned) and within 1e-5 on the reference's own depths."""
    z = load("g1_generic")
    p = params_of(z)
    n = int(z["H"]) * int(z["W"])
    res, _ = O.render(int(z["H"]), int(z["W"]), z["pose"], z["K"], p, oracle_cfg(z))
    assert max_err(res["rgb_map_0"], z["out_rgb_map_0"]) < TOL
    assert max_err(res["acc_map_0"], z["out_acc_map_0"]) < TOL
    assert rel_err(res["depth_map_0"], z["out_depth_map_0"]) < TOL
    assert max_err(res["rgb_map"], z["out_rgb_map"]) < 1e-4
    zall = load_zall("g1_generic")["zall"]
    ro, rd = O.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"])
    raw = O.query_network((ro[:, None, :] + rd[:, None, :] * zall[:, :, None]).astype(np.float32),
                          rd, p, "model_fine")
    rgb, disp, acc, _, depth = O.raw2outputs(raw, zall, rd, bool(z["white_bkgd"]))
    assert max_err(rgb, z["out_rgb_map"].reshape(n, 3)) < TOL
    assert max_err(acc, z["out_acc_map"].reshape(n)) < TOL
    assert rel_err(depth, z["out_depth_map"].reshape(n)) < TOL
