"""GPU parity of the HIP render path against the CPU oracle and the golden vectors.

Stage tests feed the HIP kernel and the oracle identical inputs; end-to-end
tests render the golden fixtures' cameras. Tolerances (north_star): rgb/acc
within 1e-5 abs, depth within 1e-5 relative to its magnitude, disp NaN-aware.
Fine maps end-to-end are held ray by ray to the reference's own float32 noise
floor (goldlib.fine_gate, tests/golden/make_sensitivity.py: the reference itself
keeps only 46-85 % of rays within 1e-5 under an exact reparametrisation of its
network), and exactly-staged by feeding the reference's own depths.
"""
import numpy as np
import pytest

from conftest import golden_names
from goldlib import (MAP_KEYS, fine_gate, grid_of, load, load_zall, max_err, oracle_cfg, params_of,
                     psnr, rel_err)
from oracle import nerf_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-5
ALL = golden_names()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _pipe(dev, z=None, **kw):
    from nerfhip.render import NerfPipeline
    if z is not None:
        kw = dict(N_samples=int(z["N_samples"]), N_importance=int(z["N_importance"]),
                  near=float(z["near"]), far=float(z["far"]), lindisp=bool(z["lindisp"]),
                  white_bkgd=bool(z["white_bkgd"]), enable_ess=bool(z["enable_ess"]),
                  enable_ert=bool(z["enable_ert"]), ert_threshold=float(z["ert_threshold"]), **kw)
    return NerfPipeline(dev, **kw)


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


# ---------------------------------------------------------------- stages
@pytest.mark.parametrize("name", ["f1_c2_crop", "f2b_c2_dense", "f6_ragged_lindisp"])
def test_rays_bit_exact(dev, name):
    z = load(name)
    pipe = _pipe(dev, z)
    ro, rd = pipe.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"])
    oro, ord_ = O.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"])
    assert np.array_equal(ro.cpu().numpy(), oro)
    assert np.array_equal(rd.cpu().numpy(), ord_)


def test_rays_row_band(dev):
    """A row band [p0, p0+n) equals the same rows of the full image (tile sharding)."""
    z = load("f1_c2_crop")
    pipe = _pipe(dev, z)
    H, W = int(z["H"]), int(z["W"])
    full = pipe.camera_rays(H, W, z["pose"], z["K"])[1]
    band = pipe.camera_rays(H, W, z["pose"], z["K"], p0=5 * W, n=7 * W)[1]
    assert torch.equal(band, full[5 * W:12 * W])


@pytest.mark.parametrize("n,S,stride0", [(1, 64, True), (3, 64, False), (37, 192, False),
                                         (130, 64, True), (2, 7, False)])
@pytest.mark.parametrize("prec", ["fp32", "f16x3"])
def test_mlp_matches_oracle(dev, n, S, stride0, prec):
    z = load("f1_c2_crop")
    p = params_of(z)
    rng = np.random.default_rng(n * 1000 + S)
    ro = np.repeat(rng.uniform(-3, 3, (1, 3)), n, 0).astype(np.float32) + \
        rng.normal(0, 0.1, (n, 3)).astype(np.float32)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    if stride0:
        zz = np.sort(rng.uniform(2, 6, S)).astype(np.float32)
        zr = np.broadcast_to(zz, (n, S))
    else:
        zr = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    pipe = _pipe(dev, N_samples=S, N_importance=0, mlp_precision=prec)
    pipe.set_weights(p)
    raw = pipe.mlp(pipe.coarse, _t(ro, dev), _t(rd, dev), _t(zz if stride0 else zr, dev),
                   0 if stride0 else S, n, S).cpu().numpy().reshape(n, S, 4)
    pts = (ro[:, None, :] + rd[:, None, :] * zr[:, :, None]).astype(np.float32)
    ref = O.query_network(pts, rd, p, "model")
    scale = np.maximum(1.0, np.abs(ref.reshape(-1, 4)).max(0))
    assert (np.abs(raw - ref).reshape(-1, 4) / scale).max() < 1e-5


@pytest.mark.parametrize("prec", ["fp32", "f16x3"])
def test_mlp_dense_weights(dev, prec):
    """gain-3 weights (large activations): same channel-relative bound."""
    z = load("f2b_c2_dense")
    p = params_of(z)
    oro, ord_ = O.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"])
    n = 200
    zc = np.broadcast_to(O.coarse_depths(2.0, 6.0, 64, False), (n, 64))
    pipe = _pipe(dev, N_samples=64, N_importance=0, mlp_precision=prec)
    pipe.set_weights(p)
    raw = pipe.mlp(pipe.coarse, _t(oro[:n], dev), _t(ord_[:n], dev), pipe.z_base, 0, n, 64)
    pts = (oro[:n, None, :] + ord_[:n, None, :] * zc[:, :, None]).astype(np.float32)
    ref = O.query_network(pts, ord_[:n], p, "model").reshape(-1, 4)
    scale = np.maximum(1.0, np.abs(ref).max(0))
    assert (np.abs(raw.cpu().numpy() - ref) / scale).max() < 1e-5


@pytest.mark.parametrize("gain", [0.05, 8.0])
@pytest.mark.parametrize("prec", ["f16x3"])
def test_mlp_x3_extreme_weight_scales(dev, gain, prec):
    """3-term FP16 split at tiny and at large activations (power-of-two scaling)."""
    from nerfhip.synthetic import make_params
    p = make_params(5, gain, 0.5)
    rng = np.random.default_rng(5)
    n, S = 64, 64
    ro = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    zr = np.sort(rng.uniform(0.5, 3, (n, S)), 1).astype(np.float32)
    pipe = _pipe(dev, N_samples=S, N_importance=0, mlp_precision=prec)
    pipe.set_weights(p)
    raw = pipe.mlp(pipe.coarse, _t(ro, dev), _t(rd, dev), _t(zr, dev), S, n, S)
    pts = (ro[:, None, :] + rd[:, None, :] * zr[:, :, None]).astype(np.float32)
    ref = O.query_network(pts, rd, p, "model").reshape(-1, 4)
    scale = np.maximum(np.abs(ref).max(0), 1e-30)
    assert (np.abs(raw.cpu().numpy() - ref) / scale).max() < 1e-5


def _rand_raw(rng, n, S, dense):
    raw = rng.normal(0, 2.0, (n, S, 4)).astype(np.float32)
    raw[..., 3] = rng.normal(2.0 if dense else -0.5, 3.0, (n, S)).astype(np.float32)
    return raw


@pytest.mark.parametrize("S,dense,white", [(64, False, True), (192, True, True), (64, True, False),
                                           (5, True, True), (130, False, True)])
def test_composite_given_raw(dev, S, dense, white):
    rng = np.random.default_rng(S)
    n = 777
    raw = _rand_raw(rng, n, S, dense)
    zr = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    pipe = _pipe(dev, N_samples=S, N_importance=0, white_bkgd=white)
    out = pipe.alloc_outputs(n)["coarse"]
    w = pipe.composite(_t(raw, dev), _t(zr, dev), S, _t(rd, dev), n, S, out, 0)
    rgb, disp, acc, wt, depth = O.raw2outputs(raw, zr, rd, white)
    # same op sequence; the map sums are wave reductions (another addition order)
    # and exp may differ by an ulp (SLEEF vs ocml)
    assert max_err(w.cpu().numpy(), wt) < 1e-6
    assert max_err(out[0].cpu().numpy(), rgb) < 1e-6
    assert max_err(out[2].cpu().numpy(), acc) < 1e-6
    assert rel_err(out[3].cpu().numpy(), depth) < 1e-6
    assert rel_err(out[1].cpu().numpy(), disp, floor=1e-3) < 1e-5


@pytest.mark.parametrize("ert", [False, True])
def test_composite_without_weights_output(dev, ert):
    """weights=NULL (fine pass without ESS): identical maps, nothing else written."""
    rng = np.random.default_rng(11)
    n, S = 3000, 192
    raw = _t(_rand_raw(rng, n, S, True), dev)
    zr = _t(np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32), dev)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd = _t(rd / np.linalg.norm(rd, axis=1, keepdims=True), dev)
    pipe = _pipe(dev, N_samples=S, N_importance=0, enable_ert=ert, ert_threshold=0.01)
    a, b = pipe.alloc_outputs(n)["coarse"], pipe.alloc_outputs(n)["coarse"]
    w = pipe.composite(raw, zr, S, rd, n, S, a, 0)
    assert pipe.composite(raw, zr, S, rd, n, S, b, 0, need_weights=False) is None
    assert w is not None
    for x, y in zip(a, b):
        assert torch.equal(torch.nan_to_num(x, 7.0), torch.nan_to_num(y, 7.0))


def test_composite_ert_chunks(dev):
    """ERT with the chunk-wide argmax rule over 3 chunks (2048, 2048, 500 rays)."""
    rng = np.random.default_rng(7)
    n, S = 2048 * 2 + 500, 64
    raw = _rand_raw(rng, n, S, True)
    raw[2048:4096, :, 3] = -5.0          # chunk 1: nothing terminates -> weights kept
    raw[2048 + 17, :, 3] = 50.0          # ... except one ray -> whole chunk cut
    raw[4096:, :, 3] = -5.0              # chunk 2: nothing terminates at all
    zr = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    pipe = _pipe(dev, N_samples=S, N_importance=0, enable_ert=True, ert_threshold=0.01)
    out = pipe.alloc_outputs(n)["coarse"]
    w = pipe.composite(_t(raw, dev), _t(zr, dev), S, _t(rd, dev), n, S, out, 0).cpu().numpy()
    for c0 in range(0, n, 2048):
        sl = slice(c0, min(n, c0 + 2048))
        rgb, disp, acc, wt, depth = O.raw2outputs_ert(raw[sl], zr[sl], rd[sl], 0.01)
        assert max_err(w[sl], wt) < 1e-6
        assert max_err(out[0].cpu().numpy()[sl], rgb) < 1e-6
        assert max_err(out[2].cpu().numpy()[sl], acc) < 1e-6
        assert np.array_equal(np.isnan(out[1].cpu().numpy()[sl]), np.isnan(disp))


@pytest.mark.parametrize("name", ["f1_c2_crop", "f2_c2_perturb", "f2b_c2_dense", "f3_ert"])
def test_sample_fine_given_reference_weights(dev, name):
    z = load(name)
    zc, wc = z["int_zc"], z["int_wc"]
    n, S = zc.shape
    NI = int(z["N_importance"])
    pipe = _pipe(dev, z)
    zall = torch.empty((n, S + NI), device=dev)
    from nerfhip._lib import call, ptr, stream_of
    zc_d, wc_d = _t(zc, dev), _t(wc, dev)          # keep the inputs alive across the call
    call("nerf_sample_fine", ptr(zc_d), S, ptr(wc_d), ptr(pipe.u_eval), 0, n, S, NI,
         ptr(zall), stream_of(dev))
    mids = (np.float32(0.5) * (zc[:, 1:] + zc[:, :-1])).astype(np.float32)
    ref = np.sort(np.concatenate([zc, O.sample_fine(mids, wc[:, 1:-1],
                                                   O.linspace_f32(0, 1, NI))], -1), -1)
    got = zall.cpu().numpy()
    assert np.array_equal(got, ref)                   # identical inputs: bit-exact
    err = np.abs(got - z["int_zall"]).max(-1)         # vs the reference's own depths
    assert np.mean(err < 1e-5) >= 0.97


@pytest.mark.parametrize("S,NI,ties", [(64, 128, False), (3, 1, False), (5, 7, False),
                                        (33, 64, False), (100, 200, False), (130, 256, False),
                                        (64, 128, True), (17, 40, True)])
def test_sample_fine_training_u(dev, S, NI, ties):
    """Training-mode u (unsorted uniform draws, VR:247-249), ragged sizes; ties:
    u on a coarse grid (repeated fine depths) and rays with all-zero weights
    (every bin clamped), so the in-register sort meets equal keys."""
    rng = np.random.default_rng(3 + S + NI + ties)
    n = 300
    zc = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    wc = (rng.random((n, S)) ** 4).astype(np.float32)
    u = rng.random((n, NI)).astype(np.float32)
    if ties:
        u = (np.floor(u * 8) / 8).astype(np.float32)
        wc[::7] = 0.0
    zall = torch.empty((n, S + NI), device=dev)
    from nerfhip._lib import call, ptr, stream_of
    zc_d, wc_d, u_d = _t(zc, dev), _t(wc, dev), _t(u, dev)
    call("nerf_sample_fine", ptr(zc_d), S, ptr(wc_d), ptr(u_d), NI, n, S, NI, ptr(zall),
         stream_of(dev))
    mids = (np.float32(0.5) * (zc[:, 1:] + zc[:, :-1])).astype(np.float32)
    ref = np.sort(np.concatenate([zc, O.sample_fine(mids, wc[:, 1:-1], u)], -1), -1)
    assert np.array_equal(zall.cpu().numpy(), ref)


@pytest.mark.parametrize("name", ["f4_ess_ert", "f4b_ess_ert_update"])
def test_ess_depths_given_grid(dev, name):
    z = load(name)
    grid = grid_of(z)
    H, W = int(z["H"]), int(z["W"])
    oro, ord_ = O.camera_rays(H, W, z["pose"], z["K"])
    n = oro.shape[0]
    tr = z["t_rand"] if "t_rand" in z else None
    pipe = _pipe(dev, z)
    pipe.set_grid(grid)
    zz = torch.empty((n, 64), device=dev)
    from nerfhip._lib import call, ptr, stream_of
    ro_d, rd_d = _t(oro, dev), _t(ord_, dev)
    tr_d = None if tr is None else _t(tr, dev)
    call("nerf_sample_coarse_ess", ptr(ro_d), ptr(rd_d), ptr(pipe.grid), 128, ptr(pipe.z_base),
         ptr(tr_d), n, 64, 2048, 0.5, ptr(zz), stream_of(dev))
    for c0 in range(0, n, 2048):
        sl = slice(c0, min(n, c0 + 2048))
        ref = O.sample_coarse_ess(oro[sl], ord_[sl], grid, 2.0, 6.0, 64, False,
                                  float(z["perturb"]), None if tr is None else tr[sl])
        assert np.array_equal(zz.cpu().numpy()[sl], ref)
    assert np.array_equal(zz.cpu().numpy()[:z["int_zc"].shape[0]], z["int_zc"])


# ---------------------------------------------------------------- end to end
def _render_fixture(dev, z, prec="fp32"):
    pipe = _pipe(dev, z, mlp_precision=prec)
    pipe.set_weights(params_of(z))
    g = grid_of(z)
    if g is not None:
        pipe.set_grid(g)
    pipe.grid_update_counter = int(z["grid_counter_in"])
    pipe.capture_zall = []
    tr = _t(z["t_rand"], dev) if "t_rand" in z else None
    res = pipe.render_image(int(z["H"]), int(z["W"]), z["pose"], z["K"], t_rand=tr)
    res = {k: v.cpu().numpy() for k, v in res.items()}
    if pipe.capture_zall:
        res["zall"] = torch.cat(pipe.capture_zall).cpu().numpy()
    return pipe, res


@pytest.mark.parametrize("name", ALL)
@pytest.mark.parametrize("prec", ["fp32", "f16x3"])
def test_render_coarse_maps_vs_golden(dev, name, prec):
    z = load(name)
    pipe, res = _render_fixture(dev, z, prec)
    n = int(z["H"]) * int(z["W"])
    assert max_err(res["rgb_map_0"], z["out_rgb_map_0"].reshape(n, 3)) < TOL
    assert max_err(res["acc_map_0"], z["out_acc_map_0"].reshape(n)) < TOL
    assert rel_err(res["depth_map_0"], z["out_depth_map_0"].reshape(n)) < TOL
    assert rel_err(res["disp_map_0"], z["out_disp_map_0"].reshape(n), floor=1e-3) < 1e-4
    assert pipe.grid_update_counter == int(z["grid_counter_out"])
    if "grid_out_packed" in z:
        g = pipe.grid.cpu().numpy().astype(bool)
        assert np.array_equal(np.packbits(g), z["grid_out_packed"])


@pytest.mark.parametrize("name", [n for n in ALL if not n.startswith("f5")])
@pytest.mark.parametrize("prec", ["fp32", "f16x3"])
def test_render_fine_maps_per_ray_gate(dev, name, prec):
    """All four fine maps end to end, ray by ray: >= 99 % of rays within 4x the
    reference's own reparametrisation spread (or 1e-5), the fraction within 1e-5
    no worse than the reparametrised reference's, PSNR >= min(80, its median - 6)."""
    z = load(name)
    _, res = _render_fixture(dev, z, prec)
    # (4): every ray beyond 4x the reference's spread is attributed to sampling
    ok, rep = fine_gate(res, z, load("s_" + name), load_zall(name), res["zall"])
    assert ok, rep
    assert rep["tail_unexplained"] == 0, rep


@pytest.mark.parametrize("name", [n for n in ALL if not n.startswith("f5")])
@pytest.mark.parametrize("prec", ["fp32", "f16x3"])
def test_fine_pass_given_reference_depths(dev, name, prec):
    """Fine MLP + composite on the reference's own fine depths of EVERY ray
    (z_<fixture>.npz): all four fine maps within 1e-5. With ERT this is the
    fine MLP (with the ERT sample compaction) plus the chunk-rule composite
    (VR:1089-1157) over the fixture's 2048-ray chunks, so termination and the
    argmax-of-zeros quirk are held to 1e-5 on the reference's own depths."""
    z = load(name)
    zall = load_zall(name)["zall"]
    n, S2 = zall.shape
    assert n == int(z["H"]) * int(z["W"])
    oro, ord_ = O.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"])
    pipe = _pipe(dev, z, mlp_precision=prec)
    pipe.set_weights(params_of(z))
    ro, rd = _t(oro, dev), _t(ord_, dev)
    zt = _t(zall, dev)
    raw = pipe._pass_mlp(pipe.fine, ro, rd, zt, S2, n, S2)
    out = pipe.alloc_outputs(n)["coarse"]
    pipe.composite(raw, zt, S2, rd, n, S2, out, 0)
    ref = {k: z["out_" + k].reshape(n, -1) for k in ("rgb_map", "acc_map", "depth_map", "disp_map")}
    assert max_err(out[0].cpu().numpy(), ref["rgb_map"]) < TOL
    assert max_err(out[2].cpu().numpy(), ref["acc_map"][:, 0]) < TOL
    assert rel_err(out[3].cpu().numpy(), ref["depth_map"][:, 0]) < TOL
    assert rel_err(out[1].cpu().numpy(), ref["disp_map"][:, 0], floor=1e-3) < 1e-4


def test_renderer_plugin_contract(dev):
    """src.models.nerf.renderer.volume_renderer.Renderer(net).render(batch) -> 8 maps."""
    from src.config import cfg, reset
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    from nerfhip.synthetic import load_into_network
    z = load("f1_c2_crop")
    reset()
    cfg.task_arg.perturb = 0
    cfg.enable_ess = False
    cfg.enable_ert = False
    net = Network().to(dev)
    load_into_network(net, params_of(z))
    net.eval()
    rend = Renderer(net)
    batch = {"H": int(z["H"]), "W": int(z["W"]), "pose": torch.from_numpy(z["pose"])[None],
             "intrinsics": torch.from_numpy(z["K"])[None]}
    with torch.no_grad():
        out = rend.render(batch)
    assert set(out) == {"rgb_map_0", "disp_map_0", "acc_map_0", "depth_map_0",
                        "rgb_map", "disp_map", "acc_map", "depth_map"}
    assert out["rgb_map"].shape == (32, 32, 3) and out["acc_map"].shape == (32, 32)
    assert out["rgb_map"].device.type == "cuda"
    got = {k: v.cpu().numpy() for k, v in out.items()}
    assert max_err(got["rgb_map_0"], z["out_rgb_map_0"]) < TOL
    assert max_err(got["acc_map_0"], z["out_acc_map_0"]) < TOL
    assert rel_err(got["depth_map_0"], z["out_depth_map_0"]) < TOL
    assert rel_err(got["disp_map_0"], z["out_disp_map_0"], floor=1e-3) < 1e-4
    ok, rep = fine_gate(got, z, load("s_f1_c2_crop"))
    assert ok, rep
    reset()


def _replaying_rand(draws):
    """torch.rand stand-in that hands out recorded draws in order, checking sizes."""
    it = iter(draws)

    def rand(size, *a, device=None, **kw):
        arr = next(it)
        assert tuple(arr.shape) == tuple(size), (arr.shape, size)
        return torch.from_numpy(np.ascontiguousarray(arr)).to(device)
    return rand, it


@pytest.mark.parametrize("name,train_mode", [("f4b_ess_ert_update", False),
                                             ("t2_train_ess_ert", True)])
def test_renderer_eval_consumes_reference_draws(dev, name, train_mode):
    """Renderer.render(batch) under no_grad (run.py --type evaluate, perturb 1 as
    lego.yaml:22 sets it) draws torch.rand exactly as the reference's chunk loop
    does: per 2048-ray chunk t_rand [m, 64] (VR:154, :1083) and, with the net in
    training mode, u [m, 128] (VR:247-249). The recorded draws of the reference
    are replayed call by call (shape-checked, all consumed) and the coarse maps,
    grid and counter match its golden render."""
    from src.config import cfg, reset
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    from nerfhip.synthetic import load_into_network
    z = load(name)
    reset()
    cfg.task_arg.perturb = 1
    cfg.enable_ess = bool(z["enable_ess"])
    cfg.enable_ert = bool(z["enable_ert"])
    cfg.ert_threshold = float(z["ert_threshold"])
    net = Network().to(dev)
    load_into_network(net, params_of(z))
    net.train(train_mode)
    rend = Renderer(net)
    assert "grid_seed" in z
    rend.occupancy_grid = grid_of(z)
    rend.grid_update_counter = int(z["grid_counter_in"])
    n = int(z["H"]) * int(z["W"])
    draws = []
    for c0 in range(0, n, 2048):
        draws.append(z["t_rand"][c0:c0 + 2048])
        if train_mode:
            draws.append(z["u"][c0:c0 + 2048])
    rand, it = _replaying_rand(draws)
    batch = {"H": int(z["H"]), "W": int(z["W"]), "pose": torch.from_numpy(z["pose"])[None],
             "intrinsics": torch.from_numpy(z["K"])[None]}
    orig = torch.rand
    torch.rand = rand
    try:
        with torch.no_grad():
            out = rend.render(batch)
    finally:
        torch.rand = orig
        reset()
    assert next(it, None) is None, "not every recorded draw was consumed"
    got = {k: v.cpu().numpy() for k, v in out.items()}
    assert max_err(got["rgb_map_0"], z["out_rgb_map_0"]) < TOL
    assert max_err(got["acc_map_0"], z["out_acc_map_0"]) < TOL
    assert rel_err(got["depth_map_0"], z["out_depth_map_0"]) < TOL
    if "grid_counter_out" in z:
        assert rend.grid_update_counter == int(z["grid_counter_out"])
        assert np.array_equal(np.packbits(rend.occupancy_grid.cpu().numpy()), z["grid_out_packed"])


def test_renderer_spiral_render_path(dev):
    """generate_spiral_poses + render_path (VR:359-509) through the plugin: one
    image per pose, equal to render(batch) of the same pose, clipped like the
    reference."""
    from src.config import cfg, reset
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    from nerfhip.synthetic import load_into_network
    z = load("f1_c2_crop")
    reset()
    cfg.task_arg.perturb = 0
    cfg.enable_ess = False
    cfg.enable_ert = False
    net = Network().to(dev)
    load_into_network(net, params_of(z))
    net.eval()
    rend = Renderer(net)
    poses = rend.generate_spiral_poses(load("lego_test_cameras")["poses"], n_frames=3)
    H, W = 12, 20
    focal = 30.0
    rgbs, disps = rend.render_path(poses, (H, W, focal))
    assert rgbs.shape == (3, H, W, 3) and disps.shape == (3, H, W)
    assert rgbs.min() >= 0 and rgbs.max() <= 1
    K = np.array([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], np.float32)
    batch = {"H": H, "W": W, "pose": torch.from_numpy(poses[1].astype(np.float32))[None],
             "intrinsics": torch.from_numpy(K)[None]}
    with torch.no_grad():
        one = rend.render(batch)
    np.testing.assert_array_equal(rgbs[1], np.clip(one["rgb_map"].cpu().numpy(), 0, 1))
    reset()


def _band_frame(dev, H, W, world, counter0, grid, params, prec="f16x3"):
    """render_frame_sharded's band / pack / unpack path with world ranks rendered
    one after another on one device (each rank: its own pipeline, same start
    state); returns the assembled frame and every rank's final grid + counter."""
    from nerfhip import dist as nd
    cams = load("lego_test_cameras")
    f = 0.5 * 800 / np.tan(0.5 * float(cams["camera_angle_x"]))
    K = np.array([[f, 0, 400 - 352], [0, f, 400 - 352], [0, 0, 1]], np.float32)
    pose = cams["poses"][0]
    parts, states = [], []
    n_pad = None
    for r in range(world):
        pipe = _pipe(dev, N_samples=64, N_importance=128, enable_ess=True, enable_ert=True,
                     ert_threshold=0.01, mlp_precision=prec)
        pipe.set_weights(params)
        pipe.set_grid(grid)
        pipe.grid_update_counter = counter0
        p0, n, n_pad = nd.band(H, W, r, world, chunk_aligned=True)
        maps = pipe.render_band(H, W, pose, K, p0, n)
        parts.append(nd.pack_maps(maps, n, n_pad, dev)[:n])
        states.append((pipe.grid.clone(), pipe.grid_update_counter))
    full = torch.cat(parts, 0)
    return nd.unpack_maps(full, H, W, set(nd.MAP_ORDER)), states, (pose, K)


def _interleaved_frame(dev, H, W, world, counter0, grid, params, pose, K, prec="f16x3",
                       t_rand=None):
    """render_frame_interleaved's chunk-set / pack / index_select path with the
    world ranks rendered one after another on one device (same start state);
    t_rand: the frame's perturb draws, every rank reading its chunks' rows."""
    from nerfhip import dist as nd
    tiles, states, evals = [], [], []
    for r in range(world):
        pipe = _pipe(dev, N_samples=64, N_importance=128, enable_ess=True, enable_ert=True,
                     ert_threshold=0.01, mlp_precision=prec)
        pipe.set_weights(params)
        pipe.set_grid(grid)
        pipe.grid_update_counter = counter0
        mine, n, n_pad = nd.chunk_set(H, W, r, world)
        maps = pipe.render_chunks(H, W, pose, K, mine, t_rand=t_rand)
        tiles.append(nd.pack_maps(maps, n, n_pad, dev))
        states.append((pipe.grid.clone(), pipe.grid_update_counter))
        evals.append(pipe.evaluated_samples())
    full = torch.cat(tiles, 0).index_select(0, nd.interleave_index(H, W, world, dev))
    return nd.unpack_maps(full, H, W, set(nd.MAP_ORDER)), states, evals


@pytest.mark.parametrize("counter0", [496, 497])
def test_sharded_c4_bands_equal_one_pass_frame(dev, counter0):
    """C4 (ESS + ERT) split into chunk-aligned bands for 2/4/8 ranks: bit-exactly
    the one-pass frame, whose ESS grid self-updates mid-frame (counter0 496: the
    coarse call of chunk 2; 497: the fine call of chunk 1, VR:1147-1157), and
    every rank ends with the sequential loop's grid and counter."""
    from nerfhip.synthetic import make_occupancy_grid, make_params
    H = W = 96                                  # 9216 rays = 4.5 chunks
    params = make_params(0, 3.0, 1.0)
    grid = make_occupancy_grid(4, 128, 0.5, 0.01)
    ref, st1, (pose, K) = _band_frame(dev, H, W, 1, counter0, grid, params)
    one = _pipe(dev, N_samples=64, N_importance=128, enable_ess=True, enable_ert=True,
                ert_threshold=0.01)
    one.set_weights(params)
    one.set_grid(grid)
    one.grid_update_counter = counter0
    direct = one.render_image(H, W, pose, K)
    assert not torch.equal(one.grid, torch.as_tensor(grid).to(dev).to(torch.uint8).view(-1))
    for k in ref:
        assert torch.equal(torch.nan_to_num(ref[k].reshape(-1), 7.0),
                           torch.nan_to_num(direct[k].reshape(-1), 7.0)), k
    for world in (2, 4, 8):
        got, states, _ = _band_frame(dev, H, W, world, counter0, grid, params)
        for k in ref:
            assert torch.equal(torch.nan_to_num(got[k], 7.0), torch.nan_to_num(ref[k], 7.0)), \
                (world, k)
        for g, c in states:
            assert c == one.grid_update_counter
            assert torch.equal(g, one.grid)
    # interleaved ownership (chunk c -> rank c mod P): same frame, grid, counter
    _, full_ev = _interleaved_frame(dev, H, W, 1, counter0, grid, params, pose, K)[1:]
    for world in (2, 3, 4, 8):
        got, states, evals = _interleaved_frame(dev, H, W, world, counter0, grid, params, pose, K)
        for k in ref:
            assert torch.equal(torch.nan_to_num(got[k], 7.0), torch.nan_to_num(ref[k], 7.0)), \
                ("interleaved", world, k)
        for g, c in states:
            assert c == one.grid_update_counter
            assert torch.equal(g, one.grid)
        # every rank's evaluated samples are its own chunks' only (replays excluded)
        assert sum(e[0] for e in evals) == full_ev[0][0]
        assert sum(e[1] for e in evals) == full_ev[0][1]


@pytest.mark.parametrize("name", ["f3_ert", "f4_ess_ert", "f4b_ess_ert_update", "f3b_ert_noterm"])
def test_ert_compaction_bitwise_equals_full_evaluation(dev, name):
    """ERT passes evaluated in depth segments with terminated rays retired
    (NerfPipeline.mlp_ert) give bitwise the maps, grid and counter of the full
    evaluation, and skip samples where rays terminate."""
    z = load(name)
    outs = {}
    for comp in (False, True):
        pipe = _pipe(dev, z, mlp_precision="f16x3", ert_compaction=comp)
        pipe.set_weights(params_of(z))
        g = grid_of(z)
        if g is not None:
            pipe.set_grid(g)
        pipe.grid_update_counter = int(z["grid_counter_in"])
        tr = _t(z["t_rand"], dev) if "t_rand" in z else None
        res = pipe.render_image(int(z["H"]), int(z["W"]), z["pose"], z["K"], t_rand=tr)
        outs[comp] = ({k: torch.nan_to_num(v, 7.0) for k, v in res.items()},
                      None if pipe.grid is None else pipe.grid.clone(), pipe.grid_update_counter,
                      pipe.evaluated_samples() if comp else None)
    (a, ga, ca, _), (b, gb, cb, (ev, full)) = outs[False], outs[True]
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert ca == cb
    assert (ga is None and gb is None) or torch.equal(ga, gb)
    assert ev <= full
    # where the reference's chunk decision shows a terminating ray, samples were skipped
    if bool(z.get("int_chunk_any_0", False)) or bool(z.get("int_chunk_any_1", False)):
        assert ev < full


def test_ert_compaction_frame_with_grid_update(dev):
    """A 96 x 96 C4 frame (4.5 chunks) whose ESS grid self-updates mid-frame:
    compacted and full evaluation agree bitwise."""
    from nerfhip.synthetic import make_occupancy_grid, make_params
    params = make_params(0, 3.0, 1.0)
    grid = make_occupancy_grid(4, 128, 0.5, 0.01)
    cams = load("lego_test_cameras")
    f = 0.5 * 800 / np.tan(0.5 * float(cams["camera_angle_x"]))
    K = np.array([[f, 0, 400 - 352], [0, f, 400 - 352], [0, 0, 1]], np.float32)
    outs = []
    for comp in (False, True):
        pipe = _pipe(dev, N_samples=64, N_importance=128, enable_ess=True, enable_ert=True,
                     ert_threshold=0.01, ert_compaction=comp)
        pipe.set_weights(params)
        pipe.set_grid(grid)
        pipe.grid_update_counter = 496
        res = pipe.render_image(96, 96, cams["poses"][0], K)
        outs.append(({k: torch.nan_to_num(v, 7.0) for k, v in res.items()}, pipe.grid.clone()))
    for k in outs[0][0]:
        assert torch.equal(outs[0][0][k], outs[1][0][k]), k
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("S,NI,kind", [(64, 128, "lin"), (32, 64, "lin"), (48, 16, "lin"),
                                       (64, 128, "zeros"), (5, 7, "lin"), (64, 128, "perm"),
                                       (130, 256, "lin")])
def test_sample_fine_shared_u(dev, S, NI, kind):
    """One shared u row (u_stride 0, as eval passes linspace): the merge-path
    fast path (ascending u, n_imp and S + n_imp multiples of 16), its fallbacks
    (a shared row that is not ascending; weights with zero bins, where the
    denom clamp can make the inverse CDF non-monotonic and the row is sorted
    first) and ragged sizes that never take it; bit-exact vs the oracle."""
    rng = np.random.default_rng(11 + S + NI)
    n = 257
    zc = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    wc = (rng.random((n, S)) ** 4).astype(np.float32)
    if kind == "zeros":
        wc[rng.random((n, S)) < 0.7] = 0.0
    u = O.linspace_f32(0, 1, NI)
    if kind == "perm":
        u = u[rng.permutation(NI)]
    zall = torch.empty((n, S + NI), device=dev)
    from nerfhip._lib import call, ptr, stream_of
    zc_d, wc_d, u_d = _t(zc, dev), _t(wc, dev), _t(np.ascontiguousarray(u), dev)
    call("nerf_sample_fine", ptr(zc_d), S, ptr(wc_d), ptr(u_d), 0, n, S, NI, ptr(zall),
         stream_of(dev))
    mids = (np.float32(0.5) * (zc[:, 1:] + zc[:, :-1])).astype(np.float32)
    ref = np.sort(np.concatenate([zc, O.sample_fine(mids, wc[:, 1:-1],
                                                   np.broadcast_to(u, (n, NI)))], -1), -1)
    assert np.array_equal(zall.cpu().numpy(), ref)


def test_interleaved_perturbed_ess_ert_equals_one_pass(dev):
    """lego.yaml's eval configuration sharded (ESS + ERT + perturb 1, bench
    lego_yaml_eval): chunks dealt round-robin to 2 / 3 / 8 ranks, each reading its
    chunks' rows of the frame's perturb draws, with a grid self-update inside
    the frame: bit-exactly the one-pass perturbed frame, grid and counter."""
    from nerfhip.synthetic import make_occupancy_grid, make_params
    H = W = 96
    params = make_params(0, 3.0, 1.0)
    # a lego-like grid (sphere 1.2 | 10 % noise, as the Renderer draws it): with a
    # small sphere most chunks' shared ESS row collapses to one depth (quirk 2:
    # the last highly-empty ray keeps one sample, VR:1040-1077) and the jitter
    # of a collapsed row is zero
    grid = make_occupancy_grid(4, 128, 1.2, 0.1)
    cams = load("lego_test_cameras")
    f = 0.5 * 800 / np.tan(0.5 * float(cams["camera_angle_x"]))
    K = np.array([[f, 0, 400 - 352], [0, f, 400 - 352], [0, 0, 1]], np.float32)
    pose = cams["poses"][0]
    tr = torch.rand((H * W, 64), device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    one = _pipe(dev, N_samples=64, N_importance=128, enable_ess=True, enable_ert=True,
                ert_threshold=0.01)
    one.set_weights(params)
    one.set_grid(grid)
    one.grid_update_counter = 496
    direct = one.render_image(H, W, pose, K, t_rand=tr)
    plain = _interleaved_frame(dev, H, W, 1, 496, grid, params, pose, K)[0]
    assert not torch.equal(plain["rgb_map"].reshape(-1), direct["rgb_map"].reshape(-1))
    for world in (1, 2, 3, 8):
        got, states, _ = _interleaved_frame(dev, H, W, world, 496, grid, params, pose, K,
                                            t_rand=tr)
        for k in direct:
            assert torch.equal(torch.nan_to_num(got[k].reshape(-1), 7.0),
                               torch.nan_to_num(direct[k].reshape(-1), 7.0)), (world, k)
        for g, c in states:
            assert c == one.grid_update_counter
            assert torch.equal(g, one.grid)
