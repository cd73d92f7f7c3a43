"""GPU: network topologies other than lego's through the HIP pipeline
(``nerfhip.generic_mlp``: ``nerf_freq_encode_fm`` + ``nerf_linear_fm`` layer by
layer, FP32) against the reference's own render of the g1 fixture (D 6, W 128,
skips [2, 3], L 8 / 3; see test_generic_mlp.py), and the layer kernel against
float64 torch."""
import numpy as np
import pytest

from goldlib import grid_of, load, load_zall, max_err, params_of, rel_err
from oracle import nerf_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("M,K,P,relu", [(128, 51, 1000, 1), (3, 64, 4097, 0), (1, 128, 65, 0),
                                        (64, 179, 130, 1), (200, 16, 64, 1)])
def test_linear_fm_matches_float64(dev, M, K, P, relu):
    """nerf_linear_fm over ragged M / K / P, feature-major and the [P][4] raw
    record strides: within 1e-6 of each output row's scale (FP32, one FMA chain)."""
    from nerfhip._lib import call, ptr, stream_of
    g = torch.Generator(device=dev).manual_seed(M * 7 + K)
    W = torch.randn((M, K), device=dev, generator=g)
    b = torch.randn((M,), device=dev, generator=g)
    X = torch.randn((K, P + 3), device=dev, generator=g)   # ldx > P
    ref = W.double() @ X[:, :P].double() + b.double()[:, None]
    if relu:
        ref = ref.clamp_min(0)
    Y = torch.full((M, P), float("nan"), device=dev)
    call("nerf_linear_fm", ptr(W), K, ptr(b), ptr(X), P + 3, K, P, M, relu, ptr(Y), P, 1,
         stream_of(dev))
    scale = (W.double().abs() @ X[:, :P].double().abs()).max(1).values + 1.0
    assert float(((Y.double() - ref).abs().max(1).values / scale).max()) < 1e-6
    if M <= 4:   # the raw record: Y[m + 4 p]
        R = torch.full((P, 4), float("nan"), device=dev)
        call("nerf_linear_fm", ptr(W), K, ptr(b), ptr(X), P + 3, K, P, M, relu, ptr(R), 1, 4,
             stream_of(dev))
        assert torch.equal(R[:, :M].t().contiguous(), Y)


def _pipe(dev, z, **kw):
    from nerfhip.render import NerfPipeline
    pipe = NerfPipeline(dev, N_samples=int(z["N_samples"]), N_importance=int(z["N_importance"]),
                        near=float(z["near"]), far=float(z["far"]), lindisp=bool(z["lindisp"]),
                        white_bkgd=bool(z["white_bkgd"]), enable_ess=bool(z["enable_ess"]),
                        enable_ert=bool(z["enable_ert"]), ert_threshold=float(z["ert_threshold"]),
                        **kw)
    pipe.set_weights(params_of(z))
    return pipe


@pytest.mark.parametrize("prec", ["fp32", "f16x3"])
def test_generic_render_vs_reference(dev, prec):
    """Coarse maps within 1e-5, fine maps within 1e-4 end to end (the oracle's
    own margin, test_generic_mlp.py) and within 1e-5 on the reference's own fine
    depths. The precision switch names the lego kernels; another topology is
    FP32 either way."""
    from nerfhip.generic_mlp import GenericMLP
    z = load("g1_generic")
    n = int(z["H"]) * int(z["W"])
    pipe = _pipe(dev, z, mlp_precision=prec)
    assert isinstance(pipe.coarse, GenericMLP) and isinstance(pipe.fine, GenericMLP)
    res = {k: v.cpu().numpy() for k, v in
           pipe.render_image(int(z["H"]), int(z["W"]), z["pose"], z["K"]).items()}
    assert max_err(res["rgb_map_0"], z["out_rgb_map_0"].reshape(n, 3)) < TOL
    assert max_err(res["acc_map_0"], z["out_acc_map_0"].reshape(n)) < TOL
    assert rel_err(res["depth_map_0"], z["out_depth_map_0"].reshape(n)) < TOL
    assert max_err(res["rgb_map"], z["out_rgb_map"].reshape(n, 3)) < 1e-4
    zall = load_zall("g1_generic")["zall"]
    ro, rd = (_t(a, dev) for a in O.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"]))
    S2 = zall.shape[1]
    zt = _t(zall, dev)
    raw = pipe._pass_mlp(pipe.fine, ro, rd, zt, S2, n, S2)
    out = pipe.alloc_outputs(n)["coarse"]
    pipe.composite(raw, zt, S2, rd, n, S2, out, 0)
    assert max_err(out[0].cpu().numpy(), z["out_rgb_map"].reshape(n, 3)) < TOL
    assert max_err(out[2].cpu().numpy(), z["out_acc_map"].reshape(n)) < TOL
    assert rel_err(out[3].cpu().numpy(), z["out_depth_map"].reshape(n)) < TOL


def _renderer(dev, z):
    from src.config import cfg, reset
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    reset()
    cfg.task_arg.perturb = 0
    cfg.task_arg.N_importance = int(z["N_importance"])
    cfg.enable_ess = cfg.enable_ert = False
    cfg.network.nerf.D, cfg.network.nerf.W, cfg.network.nerf.skips = 6, 128, [2, 3]
    cfg.network.xyz_encoder.freq, cfg.network.dir_encoder.freq = 8, 3
    net = Network().to(dev)
    p = params_of(z)
    with torch.no_grad():
        for pre, mod in (("model", net.model), ("model_fine", net.model_fine)):
            for k, v in mod.state_dict().items():
                v.copy_(torch.from_numpy(p[f"{pre}.{k}"]))
    return Renderer(net), net, reset


def test_renderer_plugin_generic_topology(dev):
    """The plugin builds the network of cfg.network (D 6 / W 128 / skips [2, 3] /
    L 8 / 3) and renders it: the eight maps, coarse within 1e-5 of the reference."""
    z = load("g1_generic")
    rend, net, reset = _renderer(dev, z)
    try:
        assert not rend.lego_topology
        net.eval()
        batch = {"H": int(z["H"]), "W": int(z["W"]), "pose": torch.from_numpy(z["pose"])[None],
                 "intrinsics": torch.from_numpy(z["K"])[None]}
        with torch.no_grad():
            out = rend.render(batch)
        got = {k: v.cpu().numpy() for k, v in out.items()}
        assert len(got) == 8
        assert max_err(got["rgb_map_0"], z["out_rgb_map_0"]) < TOL
        assert max_err(got["acc_map_0"], z["out_acc_map_0"]) < TOL
        assert max_err(got["rgb_map"], z["out_rgb_map"]) < 1e-4
        # training mode: the torch MLP back end, gradients into both networks
        net.train()
        out = rend.render(batch)
        loss = sum(((out[k] - 0.5) ** 2).mean() for k in ("rgb_map_0", "rgb_map"))
        loss.backward()
        grads = [p.grad for p in net.parameters()]
        assert all(g is not None and torch.isfinite(g).all() for g in grads)
        assert any(float(g.abs().max()) > 0 for g in grads)
    finally:
        reset()
