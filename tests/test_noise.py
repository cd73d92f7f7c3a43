"""Density noise (``raw_noise_std > 0``, reference ``volume_renderer.py:310-314``
and ``:1098-1103``): the draw order and the CPU oracle against the reference's
own renders of the n1 fixtures (``tests/golden/make_golden.py n1 n1b``: 48x48
crops over two 2048-ray chunks, perturb 1, raw_noise_std 0.5; n1b with ESS +
ERT and the call-0 grid self-update). Every torch.rand / torch.randn draw of the
reference's render is stored with its order, so the plugin's draws
(``nerfhip.render.reference_draws_noise``) are pinned to them here, and the GPU
tests (``test_gpu_noise.py``) replay them."""
import numpy as np
import pytest
import torch

from goldlib import fine_gate, grid_of, load, load_zall, max_err, oracle_cfg, params_of, rel_err
from oracle import nerf_oracle as O

NOISE = ["n1_c2_noise", "n1b_ess_ert_noise"]
TOL = 1e-5


def _draws(z):
    """reference_draws_noise on the CPU generator seeded as the capture was
    (torch.manual_seed(1234) before the Renderer is built; with ESS its grid
    draw, VR:857-864, comes first), with the sequence of draws it makes."""
    from nerfhip.render import reference_draws_noise
    n = int(z["H"]) * int(z["W"])
    torch.manual_seed(1234)
    if bool(z["enable_ess"]):
        torch.rand((128, 128, 128))
    order = []
    rand, randn = torch.rand, torch.randn

    def rec(kind, f):
        def g(size, *a, **k):
            t = f(size, *a, **k)
            order.append(f"{kind}:{t.shape[0]}x{t.shape[1]}")
            return t
        return g
    torch.rand, torch.randn = rec("rand", rand), rec("randn", randn)
    try:
        out = reference_draws_noise(n, int(z["N_samples"]), int(z["N_importance"]),
                                    float(z["perturb"]), False, "cpu", float(z["raw_noise_std"]))
    finally:
        torch.rand, torch.randn = rand, randn
    return out, order


@pytest.mark.parametrize("name", NOISE)
def test_draws_replay_the_reference_stream(name):
    """Same generator, same draws: per chunk t_rand [m, 64], the coarse noise
    [m, 64], the fine noise [m, 192] (eval: no u), bit for bit, the noise scaled
    by raw_noise_std as the reference scales it."""
    z = load(name)
    (t_rand, u, nc, nf), order = _draws(z)
    assert order == [str(s) for s in z["draw_order"]]
    assert u is None
    std = float(z["raw_noise_std"])
    assert torch.equal(t_rand, torch.from_numpy(z["t_rand"]))
    assert torch.equal(nc, torch.from_numpy(z["noise_c"]) * std)
    assert torch.equal(nf, torch.from_numpy(z["noise_f"]) * std)


def _noise(z):
    std = np.float32(float(z["raw_noise_std"]))
    return ((z["noise_c"] * std).astype(np.float32), (z["noise_f"] * std).astype(np.float32))


@pytest.mark.parametrize("name", NOISE)
def test_oracle_coarse_maps_with_noise(name):
    """The oracle's chunk loop with the recorded draws: coarse maps within 1e-5,
    the ESS grid and the ERT call counter as the reference left them."""
    z = load(name)
    g = grid_of(z)
    res, counter = O.render(int(z["H"]), int(z["W"]), z["pose"], z["K"], params_of(z),
                            oracle_cfg(z), t_rand=z["t_rand"], grid=g,
                            grid_counter=int(z["grid_counter_in"]), noise=_noise(z))
    assert counter == int(z["grid_counter_out"])
    assert max_err(res["rgb_map_0"], z["out_rgb_map_0"]) < TOL
    assert max_err(res["acc_map_0"], z["out_acc_map_0"]) < TOL
    assert rel_err(res["depth_map_0"], z["out_depth_map_0"]) < TOL
    if g is not None:
        assert np.array_equal(np.packbits(g.reshape(-1)), z["grid_out_packed"])


@pytest.mark.parametrize("name", NOISE)
def test_oracle_fine_pass_with_noise_given_reference_depths(name):
    """Fine MLP + noisy composite on the reference's fine depths of every ray
    (z_<name>.npz; with ERT its recorded chunk decisions): fine maps within 1e-5."""
    z, zz = load(name), load_zall(name)
    zall = zz["zall"]
    n = zall.shape[0]
    ro, rd = O.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"])
    raw = O.query_network((ro[:, None, :] + rd[:, None, :] * zall[:, :, None]).astype(np.float32),
                          rd, params_of(z), "model_fine")
    raw = O.add_sigma_noise(raw, _noise(z)[1])
    outs = []
    for k, c0 in enumerate(range(0, n, 2048)):
        sl = slice(c0, min(n, c0 + 2048))
        if bool(z["enable_ert"]):
            outs.append(O.raw2outputs_ert(raw[sl], zall[sl], rd[sl], float(z["ert_threshold"]),
                                          bool(z["white_bkgd"]),
                                          chunk_any=bool(zz["chunk_any"][2 * k + 1])))
        else:
            outs.append(O.raw2outputs(raw[sl], zall[sl], rd[sl], bool(z["white_bkgd"])))
    rgb, disp, acc, _, depth = (np.concatenate(v, 0) for v in zip(*outs))
    assert max_err(rgb, z["out_rgb_map"].reshape(n, 3)) < TOL
    assert max_err(acc, z["out_acc_map"].reshape(n)) < TOL
    assert rel_err(depth, z["out_depth_map"].reshape(n)) < TOL
    assert rel_err(disp, z["out_disp_map"].reshape(n), floor=1e-3) < 1e-4


@pytest.mark.parametrize("name", NOISE)
def test_oracle_fine_maps_with_noise_gate(name):
    """End-to-end fine maps of the oracle with the recorded draws, ray by ray
    against the reference's own spread (s_<name>.npz), the tail attributed to
    other fine depths (goldlib.fine_gate, the gate the HIP path is held to)."""
    z = load(name)
    res, _ = O.render(int(z["H"]), int(z["W"]), z["pose"], z["K"], params_of(z), oracle_cfg(z),
                      t_rand=z["t_rand"], grid=grid_of(z), grid_counter=int(z["grid_counter_in"]),
                      return_zall=True, noise=_noise(z))
    ok, rep = fine_gate(res, z, load("s_" + name), load_zall(name), res["zall"])
    assert ok and rep["tail_unexplained"] == 0, rep


def test_noise_changes_the_render():
    """Not vacuous: without the noise the oracle's coarse maps move well past 1e-5."""
    z = load("n1_c2_noise")
    res, _ = O.render(int(z["H"]), int(z["W"]), z["pose"], z["K"], params_of(z), oracle_cfg(z),
                      t_rand=z["t_rand"])
    assert max_err(res["rgb_map_0"], z["out_rgb_map_0"]) > 1e-3
