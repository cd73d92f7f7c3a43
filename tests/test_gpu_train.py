"""C3 training step on the GPU vs the reference's own training-mode forward and
backward (tests/golden/t1_train_step.npz, captured by make_train_golden.py).

Tolerances: the coarse pass is deterministic up to FP32 GEMM order (1e-5 on
rgb); the fine samples are a searchsorted of the coarse weights, so the fine
rgb is compared by PSNR; the gradients of the coarse loss alone to 1e-3, those
of the full loss by relative norm to max(2e-3, 2 x the reference's own spread
for that tensor) (tests/golden/ts_*.npz, make_train_sensitivity.py: the fine
loss reaches the coarse network through the sample positions, where sin(2^9 x)
and 1/(cdf[above] - cdf[below]) amplify float32 rounding; the reference itself
moves the coarse density bias's norm by 7.5 % under an exact reparametrisation
of its network, most other tensors by < 0.1 %).
The same math on the CPU matches the reference to 1e-5 (tests/test_train.py).
Both MLP back ends are held to the same bounds: the x3 MFMA kernels
(train_mlp.py, the default) and torch modules on hipBLASLt FP32 GEMMs."""
import os

import numpy as np
import pytest
import torch

from goldlib import load, max_err, params_of, psnr

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _full_loss_tol(name, k):
    """Per-tensor bound on the full-loss gradient norm: the reference's own spread."""
    ts = load("ts_" + name)
    return max(2e-3, 2.0 * float(ts["gnorm_spread__" + k]))


def _coarse_elem_tol(name, k):
    """Per-element bound (x the tensor's norm) on a coarse-loss gradient: 1e-3,
    or twice the reference's own relative L2 distance from itself under exact
    reparametrisations when that is larger (tg_<name>.npz gcdist: up to 2.3e-3
    on t2's gain-3 weights, where a ReLU unit at its edge flips)."""
    return max(1e-3, 2.0 * float(load("tg_" + name)["gcdist__" + k]))


REL_FLOOR = 1e-6


def _elementwise_grads(name, grads, coarse=False):
    """Every element of every gradient tensor against the reference's
    (tests/golden/tg_<name>.npz, make_train_fullgrad.py): per tensor the relative
    L2 distance ||g - g_ref|| / ||g_ref|| within 2x the largest distance of the
    reference from ITSELF under exact reparametrisations (gdist / gcdist) plus
    REL_FLOOR. A permuted, sign-flipped or shifted tail of a tensor fails this, a
    norm check does not. Every tensor's distance is printed (and written with
    NERF_FRAME_REPORT) next to the reference's own.
    grads: name -> tensor (None entries must have no reference gradient)."""
    tg = load("tg_" + name)
    # the bound is the reference's own distance from itself, tensor by tensor (plus
    # 1e-6 of float32 summation noise for tensors the reparametrisations leave
    # bitwise unchanged); round 3's fixed floors (1e-4 coarse, 2e-3 full) set the
    # bound for most tensors and were retired once the measured distances showed
    # every tensor within 2x the reference's own (gpurun_out report)
    key, dkey, floor = ("gc__", "gcdist__", REL_FLOOR) if coarse else ("g__", "gdist__", REL_FLOOR)
    worst = {}
    for k, g in grads.items():
        if key + k not in tg:
            assert g is None or not bool(torch.any(g != 0)), k
            continue
        ref = tg[key + k].astype(np.float64).reshape(-1)
        got = g.detach().double().cpu().numpy().reshape(-1)
        rel = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)
        worst[k] = (rel, float(tg[dkey + k]))
    _report(name, "coarse" if coarse else "full", worst)
    for k, (rel, d) in worst.items():
        assert rel <= 2.0 * d + floor, (k, rel, 2.0 * d + floor)
    return worst


def _report(name, kind, worst):
    """Print (and with NERF_FRAME_REPORT=<dir> write) every tensor's measured
    relative distance next to the reference's own self-distance."""
    import json
    import os
    rows = {k: {"rel": r, "ref_self": d, "ratio": r / d if d > 0 else None}
            for k, (r, d) in sorted(worst.items())}
    print(json.dumps({"case": name, "loss": kind, "grads": rows}))
    out = os.environ.get("NERF_FRAME_REPORT")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, f"grad_dist_{name}_{kind}_{len(_REPORTS)}.json"), "w") as f:
            json.dump(rows, f, indent=1)
    _REPORTS.append(name)


_REPORTS = []


def _setup(dev, mlp="x3", ops="hip"):
    from nerfhip.render import NerfPipeline
    from nerfhip.train import NerfTrainer
    z = load("t1_train_step")
    params = params_of(z)
    tr = NerfTrainer(dev, params, mlp=mlp, ops=ops)
    pipe = NerfPipeline(dev, N_samples=64, N_importance=128)
    ro, rd = pipe.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
    return z, tr, ro, rd, t(z["t_rand"]), t(z["u"]), t(z["gt"].reshape(-1, 3))


@pytest.mark.parametrize("mlp,ops", [("x3", "hip"), ("torch", "hip"), ("x3", "torch"),
                                     ("torch", "torch")])
def test_forward_loss_and_gradients_match_reference(dev, mlp, ops):
    z, tr, ro, rd, t_rand, u, gt = _setup(dev, mlp, ops)
    out = tr.forward(ro, rd, t_rand, u)
    assert max_err(out["rgb_map_0"].detach().cpu().numpy(), z["rgb_map_0"]) < 1e-5
    assert psnr(out["rgb_map"].detach().cpu().numpy(), z["rgb_map"]) > 60.0
    losses = tr.loss(out, gt)
    assert abs(losses["loss_coarse"].item() - float(z["loss_coarse"])) < 1e-6 * max(1.0, float(z["loss_coarse"]))
    assert abs(losses["loss"].item() - float(z["loss"])) / float(z["loss"]) < 1e-4
    # the coarse loss alone: a deterministic path (no fine samples) -> tight
    tr.opt.zero_grad(set_to_none=True)
    losses["loss_coarse"].backward(retain_graph=True)
    for k, p in tr.named_parameters():
        if "gcnorm__" + k not in z:
            continue
        ref = float(z["gcnorm__" + k])
        g = p.grad.detach().double().cpu()
        assert abs(g.norm().item() - ref) <= 1e-3 * ref + 1e-12, k
        assert np.abs(g.reshape(-1)[:64].numpy() - z["gchead__" + k]).max() <= \
            _coarse_elem_tol("t1_train_step", k) * ref + 1e-12, k
    _elementwise_grads("t1_train_step", {k: p.grad for k, p in tr.named_parameters()},
                       coarse=True)
    # the full loss: the fine loss reaches the coarse net through the sample
    # positions, where sin(2^9 x) amplifies FP32 GEMM-order differences
    tr.opt.zero_grad(set_to_none=True)
    losses["loss"].backward()
    grads = {k: p.grad.detach().double().cpu() for k, p in tr.named_parameters()}
    names = [str(n) for n in z["param_names"]]
    assert sorted(names) == sorted(grads)
    for k in names:
        ref_norm = float(z["gnorm__" + k])
        assert abs(grads[k].norm().item() - ref_norm) <= \
            _full_loss_tol("t1_train_step", k) * ref_norm + 1e-9, k
    _elementwise_grads("t1_train_step", grads)


@pytest.mark.parametrize("mlp", ["x3", "torch"])
def test_steps_reduce_loss(dev, mlp):
    z, tr, ro, rd, t_rand, u, gt = _setup(dev, mlp)
    first = tr.step(ro, rd, gt, t_rand, u)["loss"].item()
    for _ in range(30):
        last = tr.step(ro, rd, gt, t_rand, u)["loss"].item()
    assert last < 0.8 * first
    for p in tr.parameters():                       # clip_grad_value_(40) held
        assert p.grad is None or p.grad.abs().max() <= 40.0


@pytest.mark.parametrize("adam", ["hip", "capturable"])
def test_coarse_only_steps(dev, adam):
    """N_importance = 0 (VR:181: no fine pass): the fine network takes no part,
    gets no gradient and is left untouched; the coarse one trains."""
    from nerfhip.train import NerfTrainer
    z = load("t1_train_step")
    tr = NerfTrainer(dev, params_of(z), N_importance=0, adam=adam)
    _, _, ro, rd, t_rand, _, gt = _setup(dev)
    fine0 = [p.detach().clone() for p in tr.fine.parameters()]
    first = tr.step(ro, rd, gt, t_rand)["loss"].item()
    for _ in range(20):
        last = tr.step(ro, rd, gt, t_rand)["loss"].item()
    assert np.isfinite(first) and last < 0.9 * first
    assert all(p.grad is None for p in tr.fine.parameters())
    assert all(torch.equal(a, b) for a, b in zip(fine0, tr.fine.parameters()))
    assert all(p.grad is not None for p in tr.coarse.parameters())


# ------------------------------------------------------------------ the plugin
def _plugin_train_render(dev, name, mlp):
    """Renderer(net).render(batch) in training mode, as trainers/nerf.py:20-37
    calls it, with the reference's recorded torch.rand draws replayed in its
    order (per 2048-ray chunk: perturb t_rand, then the fine u)."""
    from goldlib import grid_of
    from nerfhip.synthetic import load_into_network
    from src.config import cfg, reset
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    z = load(name)
    reset()
    cfg.task_arg.perturb = 1
    cfg.enable_ess = bool(z["enable_ess"])
    cfg.enable_ert = bool(z["enable_ert"])
    cfg.ert_threshold = float(z["ert_threshold"])
    cfg.train_mlp = mlp
    net = Network().to(dev)
    load_into_network(net, params_of(z))
    net.train()
    rend = Renderer(net)
    if "grid_seed" in z:
        rend.occupancy_grid = grid_of(z)
        rend.grid_update_counter = int(z["grid_counter_in"])
    n = int(z["H"]) * int(z["W"])
    draws = []
    for c0 in range(0, n, 2048):
        draws += [z["t_rand"][c0:c0 + 2048], z["u"][c0:c0 + 2048]]
    it = iter(draws)
    orig = torch.rand

    def replay(size, *a, device=None, **kw):
        arr = next(it)
        assert tuple(arr.shape) == tuple(size), (arr.shape, size)
        return torch.from_numpy(np.ascontiguousarray(arr)).to(device)
    batch = {"H": int(z["H"]), "W": int(z["W"]), "pose": torch.from_numpy(z["pose"])[None],
             "intrinsics": torch.from_numpy(z["K"])[None]}
    torch.rand = replay
    try:
        out = rend.render(batch)
    finally:
        torch.rand = orig
        reset()
    assert next(it, None) is None, "not every recorded draw was consumed"
    return z, net, rend, out


@pytest.mark.parametrize("name", ["t1_train_step", "t2_train_ess_ert"])
@pytest.mark.parametrize("mlp", ["x3", "torch"])
def test_plugin_training_render_matches_reference(dev, name, mlp):
    """North_star drop-in for train.py: the plugin's training-mode render gives the
    reference's coarse maps (1e-5), losses and gradients (coarse loss alone 1e-3
    of each tensor's norm; full loss: norms within the reference's own spread,
    as the trainer test),
    with ERT/ESS (t2) also the grid self-update and call counter exactly."""
    from goldlib import rel_err
    z, net, rend, out = _plugin_train_render(dev, name, mlp)
    H, W = int(z["H"]), int(z["W"])
    n = H * W
    assert out["rgb_map"].shape == (H, W, 3) and out["depth_map"].shape == (H, W)
    assert out["rgb_map_0"].requires_grad and out["rgb_map"].requires_grad
    g = {k: v.detach().cpu().numpy() for k, v in out.items()}
    # x3 kernels: 1e-5; torch modules on hipBLASLt FP32 GEMMs reach 1.06e-5 on t2's
    # gain-3 weights (the reference's own reparametrisation floor on coarse maps
    # is 1.004e-5, tests/golden/s_f4b_ess_ert_update.npz)
    tol0 = 1e-5 if mlp == "x3" else 2e-5
    assert max_err(g["rgb_map_0"].reshape(n, 3), z["rgb_map_0"]) < tol0
    if "out_acc_map_0" in z:
        assert max_err(g["acc_map_0"], z["out_acc_map_0"]) < tol0
        assert rel_err(g["depth_map_0"], z["out_depth_map_0"]) < tol0
        assert np.array_equal(np.isnan(g["disp_map_0"]), np.isnan(z["out_disp_map_0"]))
    if "grid_out_packed" in z:
        assert rend.grid_update_counter == int(z["grid_counter_out"])
        assert np.array_equal(np.packbits(rend.occupancy_grid.cpu().numpy().reshape(-1)),
                              z["grid_out_packed"])
    gt = torch.from_numpy(z["gt"].reshape(-1, 3)).to(dev)
    loss_c = torch.nn.functional.mse_loss(out["rgb_map_0"].reshape(-1, 3), gt)
    loss_f = torch.nn.functional.mse_loss(out["rgb_map"].reshape(-1, 3), gt)
    assert abs(loss_c.item() - float(z["loss_coarse"])) <= 1e-6 * max(1.0, float(z["loss_coarse"]))
    assert abs((loss_c + loss_f).item() - float(z["loss"])) / float(z["loss"]) < 1e-3
    params = dict(net.named_parameters())
    net.zero_grad(set_to_none=True)
    loss_c.backward(retain_graph=True)
    for k, p in params.items():
        if "gcnorm__" + k not in z:
            continue
        ref = float(z["gcnorm__" + k])
        gk = p.grad.detach().double().cpu()
        assert abs(gk.norm().item() - ref) <= 1e-3 * ref + 1e-12, k
        assert np.abs(gk.reshape(-1)[:64].numpy() - z["gchead__" + k]).max() <= \
            _coarse_elem_tol(name, k) * ref + 1e-12, k
    _elementwise_grads(name, {k: p.grad for k, p in params.items()}, coarse=True)
    net.zero_grad(set_to_none=True)
    (loss_c + loss_f).backward()
    for k in [str(s) for s in z["param_names"]]:
        ref_norm = float(z["gnorm__" + k])
        assert abs(params[k].grad.detach().double().norm().item() - ref_norm) <= \
            _full_loss_tol(name, k) * ref_norm + 1e-9, k
    _elementwise_grads(name, {k: p.grad for k, p in params.items()})


def test_plugin_novel_view_sequence(dev, tmp_path):
    """render_novel_view_sequence (VR:511-616): one 8-bit frame per spiral pose,
    equal to render(batch) of that pose; PNGs written; no video (out of scope)."""
    from nerfhip.synthetic import load_into_network
    from src.config import cfg, reset
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    z = load("f1_c2_crop")
    reset()
    cfg.task_arg.perturb = 0
    cfg.enable_ess = False
    cfg.enable_ert = False
    cfg.render_num = 3
    net = Network().to(dev)
    load_into_network(net, params_of(z))
    net.eval()
    rend = Renderer(net)
    poses = load("lego_test_cameras")["poses"]
    H, W, focal = 10, 14, 20.0
    images_dir, video = rend.render_novel_view_sequence(poses, (H, W, focal), str(tmp_path), "t")
    rgb8, disp8 = rend.last_sequence
    assert rgb8.shape == (3, H, W, 3) and disp8.shape == (3, H, W) and video is None
    import os
    assert sorted(os.listdir(images_dir))[:2] == ["view0000_disp.png", "view0000_rgb.png"]
    sp = rend.generate_spiral_poses(poses, n_frames=3)
    K = np.array([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], np.float32)
    with torch.no_grad():
        one = rend.render({"H": H, "W": W, "pose": torch.from_numpy(sp[2].astype(np.float32))[None],
                           "intrinsics": torch.from_numpy(K)[None]})
    ref = (255 * np.clip(one["rgb_map"].cpu().numpy(), 0, 1)).astype(np.uint8)
    np.testing.assert_array_equal(rgb8[2], ref)
    reset()


@pytest.mark.parametrize("mlp", ["x3", "torch"])
def test_graph_step_trains_and_honours_lr(dev, mlp):
    """graph=True: eager warm-up steps, then one captured HIP graph replayed per
    step (static inputs refreshed from each batch); the loss falls like the eager
    trainer's, the device-side learning rate is honoured (lr 0 leaves every
    parameter bitwise unchanged), clip_grad_value_(40) holds."""
    from nerfhip.train import NerfTrainer
    z, _, ro, rd, _, _, gt = _setup(dev, mlp)
    torch.manual_seed(1234)   # the step's own draws (perturb t, fine u)
    tr = NerfTrainer(dev, params_of(z), mlp=mlp, graph=True)
    first = tr.step(ro, rd, gt)["loss"].item()
    losses = [tr.step(ro, rd, gt)["loss"].item() for _ in range(30)]
    assert len(tr._graphs) == 1
    # one batch, lr 5e-4, the reference's un-detached fine samples: the loss falls
    # to ~0.55 of its start with occasional spikes (measured over many draws), so
    # the check is on the best of the last 10 steps
    assert np.all(np.isfinite(losses)) and min(losses[-10:]) < 0.8 * first
    for p in tr.parameters():
        assert p.grad is not None and p.grad.abs().max() <= 40.0
    tr.set_lr(0.0)
    before = [p.detach().clone() for p in tr.parameters()]
    tr.step(torch.flip(ro, [0]), torch.flip(rd, [0]), gt)
    for a, b in zip(before, tr.parameters()):
        assert torch.equal(a, b)


@pytest.mark.parametrize("explicit_draws", [True, False])
def test_graph_step_equals_eager_steps(dev, explicit_draws):
    """The HIP-graph step (draws and batch copied into static inputs, Adam with a
    device lr: HipAdam or torch's capturable) against the eager step with the same Adam, from the
    same weights, batches and draws: 6 steps (2 eager warm-ups, the capture, 3
    replays) give bitwise the same losses and final parameters -- a stale
    static input, a host-side branch frozen at capture or an update lost at
    capture would show. Without explicit draws both consume torch.rand's
    device stream in the same order (t_rand, then u) from the same seed. The
    default eager trainer (fused Adam) agrees to 1e-5 over the first two steps,
    after which the reference's un-detached fine sampling makes the trajectory
    chaotic (an ulp in a weight flips fine samples); so does HipAdam (the default)
    against torch's fused Adam."""
    from nerfhip.train import NerfTrainer
    z, _, ro, rd, _, _, gt = _setup(dev, "x3")
    g = torch.Generator(device=dev).manual_seed(7)
    n = ro.shape[0]
    batches = []
    for i in range(6):
        perm = torch.randperm(n, device=dev, generator=g)
        tr_ = torch.rand((n, 64), device=dev, generator=g) if explicit_draws else None
        u_ = torch.rand((n, 128), device=dev, generator=g) if explicit_draws else None
        batches.append((ro[perm], rd[perm], gt[perm], tr_, u_))
    runs = {}
    for mode, adam in (("eager", "hip"), ("graph", "hip"), ("eager", "capturable"),
                       ("graph", "capturable"), ("eager", "fused")):
        torch.manual_seed(99)
        tr = NerfTrainer(dev, params_of(z), mlp="x3", graph=mode == "graph", adam=adam)
        losses = [float(tr.step(*b)["loss"].item()) for b in batches]
        runs[mode, adam] = (np.array(losses), {k: v.clone() for k, v in tr.state().items()})
        if mode == "graph":
            assert len(tr._graphs) == 1
    for adam in ("hip", "capturable"):
        le, lg = runs["eager", adam][0], runs["graph", adam][0]
        assert np.array_equal(le, lg), (adam, le, lg)
        for k, a in runs["eager", adam][1].items():
            assert torch.equal(a, runs["graph", adam][1][k]), (adam, k)
    lf, lh = runs["eager", "fused"][0], runs["graph", "hip"][0]
    assert np.all(np.abs(lf[:2] - lh[:2]) <= 1e-5 * np.abs(lf[:2])), (lf, lh)


@pytest.mark.parametrize("mode", ["eager", "graph"])
def test_side_stream_weight_grads_equal_inline(dev, mode, monkeypatch):
    """NerfTrainer's backward computes the fused MLPs' weight gradients on a side
    stream (train_mlp.side_wgrad_scope; joined at the end of the pass) while
    the main stream runs on through the fine d z and the coarse backward: 5
    steps give bitwise the losses and parameters of the in-line schedule
    (NERF_TRAIN_SIDE_WGRAD=0), eager and as a HIP graph -- a read of a
    gradient before the join, or a buffer reused while the side stream still
    reads it, would show."""
    from nerfhip import train_mlp
    from nerfhip.train import NerfTrainer
    z, _, ro, rd, _, _, gt = _setup(dev, "x3")
    g = torch.Generator(device=dev).manual_seed(3)
    n = ro.shape[0]
    batches = [(ro[p], rd[p], gt[p], torch.rand((n, 64), device=dev, generator=g),
                torch.rand((n, 128), device=dev, generator=g))
               for p in (torch.randperm(n, device=dev, generator=g) for _ in range(5))]
    runs = {}
    for side in (False, True):
        monkeypatch.setattr(train_mlp, "SIDE_WGRAD", side)
        tr = NerfTrainer(dev, params_of(z), mlp="x3", graph=mode == "graph")
        losses = [float(tr.step(*b)["loss"].item()) for b in batches]
        runs[side] = (np.array(losses), {k: v.clone() for k, v in tr.state().items()})
    assert np.array_equal(runs[False][0], runs[True][0]), runs
    for k, a in runs[False][1].items():
        assert torch.equal(a, runs[True][1][k]), k
    assert not train_mlp._SIDE_SCOPE[0]


@pytest.mark.parametrize("reader", ["tensor_hook", "post_accumulate_hook", "create_graph"])
def test_side_stream_join_waits_for_main_stream_readers(dev, reader, monkeypatch):
    """Inside side_wgrad_scope the main stream may read a side-stream weight
    gradient before the pass ends: a tensor hook and a post-accumulate-grad
    hook run there, and with create_graph AccumulateGrad copies the gradient
    there. The join then waits at once, so what each reader sees equals the
    in-line schedule bit for bit (a read before the side stream finished
    would show as a partial or stale gradient)."""
    from nerfhip import train_mlp
    from nerfhip.train import NerfTrainer
    from nerfhip.train_mlp import prepack, side_wgrad_scope
    z, _, ro, rd, _, _, gt = _setup(dev, "x3")
    g = torch.Generator(device=dev).manual_seed(11)
    n = ro.shape[0]
    t_rand = torch.rand((n, 64), device=dev, generator=g)
    u = torch.rand((n, 128), device=dev, generator=g)
    runs = {}
    for side in (False, True):
        monkeypatch.setattr(train_mlp, "SIDE_WGRAD", side)
        tr = NerfTrainer(dev, params_of(z), mlp="x3")
        fine = dict(tr.fine.named_parameters())
        seen = []
        hooks = []
        if reader == "tensor_hook":   # every fine weight: the hook clones on the main stream
            for k in ("pts_linears.0.weight", "pts_linears.7.weight", "rgb_linear.weight"):
                hooks.append(fine[k].register_hook(lambda gr: seen.append(gr.clone())))
        elif reader == "post_accumulate_hook":
            for k in ("pts_linears.3.weight", "views_linears.0.weight"):
                hooks.append(fine[k].register_post_accumulate_grad_hook(
                    lambda q: seen.append(q.grad.clone())))
        tr.opt.zero_grad(set_to_none=True)
        prepack([tr.coarse, tr.fine])
        loss = tr.loss(tr.forward(ro, rd, t_rand, u), gt)["loss"]
        with side_wgrad_scope([tr.fine]):
            loss.backward(create_graph=reader == "create_graph")
        torch.cuda.synchronize()
        for h in hooks:
            h.remove()
        runs[side] = (seen, {k: q.grad.detach().clone() for k, q in fine.items()})
    assert len(runs[True][0]) == len(runs[False][0])
    for a, b in zip(runs[False][0], runs[True][0]):
        assert torch.equal(a, b)
    for k, a in runs[False][1].items():
        assert torch.equal(a, runs[True][1][k]), k
    assert not train_mlp._SIDE_SCOPE[0]


def test_hip_adam_matches_torch_adam(dev):
    """HipAdam (clip_grad_value_ + Adam in one nerf_adam_step launch) against
    torch.optim.Adam (foreach=False) after torch's clip_grad_value_, 6 steps on
    tensors of the network's sizes with gradients past the clip value: the
    parameters, exp_avg and exp_avg_sq within 1e-5 of each tensor's max (the
    same float32 operation order; torch's device lerp may contract to an fma,
    one ulp that the moving averages carry on), the clamped gradients and the
    step count exact; an lr
    change through the device tensor takes effect; state_dict round trip."""
    from nerfhip.adam import HipAdam
    g = torch.Generator(device=dev).manual_seed(5)
    shapes = [(256, 63), (256,), (256, 256), (1,), (3, 128), (3,), (128, 283), (128,)]
    p0 = [torch.randn(s, device=dev, generator=g) for s in shapes]
    pa = [x.clone().requires_grad_(True) for x in p0]
    pb = [x.clone().requires_grad_(True) for x in p0]
    oa = HipAdam(pa, lr=5e-3, eps=1e-8, clip=40.0)
    ob = torch.optim.Adam(pb, lr=5e-3, eps=1e-8, weight_decay=0.0, foreach=False)
    for step in range(6):
        if step == 4:
            oa.param_groups[0]["lr"].fill_(1e-3)
            ob.param_groups[0]["lr"] = 1e-3
        for a, b in zip(pa, pb):
            gr = torch.randn(a.shape, device=dev, generator=g) * 30.0
            a.grad, b.grad = gr.clone(), gr.clone()
        torch.nn.utils.clip_grad_value_(pb, 40.0)
        oa.step()
        ob.step()
        for a, b in zip(pa, pb):
            assert torch.equal(a.grad, b.grad)
            assert (a - b).abs().max() <= 1e-5 * b.abs().max(), step
            sa, sb = oa.state[a], ob.state[b]
            for k in ("exp_avg", "exp_avg_sq"):
                assert (sa[k] - sb[k]).abs().max() <= 1e-5 * sb[k].abs().max(), (step, k)
            assert float(sa["step"]) == float(sb["step"]) == step + 1
    sd = oa.state_dict()
    oc = HipAdam([x.detach().clone().requires_grad_(True) for x in pa], lr=1e-3, clip=40.0)
    oc.load_state_dict(sd)
    for x in oc.param_groups[0]["params"]:
        x.grad = torch.zeros_like(x)
    oc.step()
    assert float(oc.state[oc.param_groups[0]["params"][0]]["step"]) == 7.0


def test_hip_adam_nonfinite_gradients_as_torch(dev):
    """A NaN / +-Inf gradient goes through HipAdam's clamp as through torch's
    clip_grad_value_ (torch.clamp keeps NaN, maps +-Inf to +-clip) and Adam:
    the same NaN positions in the parameters and both moments, finite entries
    within 1e-5; clip = 0 zeroes every gradient as clip_grad_value_(0) does;
    a parameter without a gradient next to ones with is refused (one shared
    step count)."""
    from nerfhip.adam import HipAdam
    g = torch.Generator(device=dev).manual_seed(7)
    p0 = [torch.randn((256, 63), device=dev, generator=g), torch.randn((128,), device=dev, generator=g)]
    for clip in (40.0, 0.0):
        pa = [x.clone().requires_grad_(True) for x in p0]
        pb = [x.clone().requires_grad_(True) for x in p0]
        oa = HipAdam(pa, lr=5e-3, eps=1e-8, clip=clip)
        ob = torch.optim.Adam(pb, lr=5e-3, eps=1e-8, weight_decay=0.0, foreach=False)
        for step in range(3):
            for a, b in zip(pa, pb):
                gr = torch.randn(a.shape, device=dev, generator=g) * 30.0
                if step == 1:
                    flat = gr.view(-1)
                    flat[::17] = float("nan")
                    flat[5::31] = float("inf")
                    flat[7::29] = -float("inf")
                a.grad, b.grad = gr.clone(), gr.clone()
            torch.nn.utils.clip_grad_value_(pb, clip)
            oa.step()
            ob.step()
            for a, b in zip(pa, pb):
                assert torch.equal(a.grad.isnan(), b.grad.isnan()), (clip, step)
                fin = ~b.grad.isnan()
                assert torch.equal(a.grad[fin], b.grad[fin]), (clip, step)
                for x, y in ((a, b), (oa.state[a]["exp_avg"], ob.state[b]["exp_avg"]),
                             (oa.state[a]["exp_avg_sq"], ob.state[b]["exp_avg_sq"])):
                    assert torch.equal(x.isnan(), y.isnan()), (clip, step)
                    m = ~y.isnan()
                    if m.any():
                        assert (x[m] - y[m]).abs().max() <= 1e-5 * y[m].abs().max().clamp_min(1e-30)
            if step == 1 and clip == 40.0:
                assert any(bool(a.isnan().any()) for a in pa)       # the blow-up is visible
    pa = [x.clone().requires_grad_(True) for x in p0]
    oa = HipAdam(pa, clip=40.0)
    pa[0].grad = torch.zeros_like(pa[0])
    with pytest.raises(ValueError):
        oa.step()
    with pytest.raises(ValueError):
        HipAdam(pa, clip=-1.0)


@pytest.mark.parametrize("mlp", ["x3", "torch"])
def test_bench_shape_step_matches_reference(dev, mlp):
    """The bench's own C3 shape (BASELINE configs[2], bench.py bench_train): 1024
    pixels scattered over the lego test views, perturb 1, training-mode u, the
    trained lego checkpoint, MSE coarse + fine (trainers/nerf.py:39-76) against
    a random target; tests/golden/t3_c3_scatter.npz + tg_t3_c3_scatter.npz
    (make_train_fullgrad.py t3: the reference's per-chunk methods on one
    1024-ray chunk, VR:154-193, and its self-distance under 16 exact
    reparametrisations). The rays the bench builds (camera_rays_at) agree with
    the reference's (VR:115-143); the step runs on the reference's own rays and
    draws; every gradient tensor within 2x the reference's own distance from
    itself (full loss and coarse loss alone)."""
    from nerfhip.train import NerfTrainer, camera_rays_at
    z = load("t3_c3_scatter")
    ck = torch.load(os.path.join(REPO, "checkpoints", "lego", "latest.pth"), map_location="cpu",
                    weights_only=True)["net"]
    tr = NerfTrainer(dev, {k: v.float() for k, v in ck.items()}, mlp=mlp)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
    cams = np.load(os.path.join(REPO, "tests", "golden", "lego_test_cameras.npz"))
    ro_b, rd_b = camera_rays_at(t(cams["poses"].astype(np.float32)), t(z["K"]),
                                t(z["pix"].astype(np.int64)), t(z["view"].astype(np.int64)), 800)
    assert float((ro_b - t(z["rays_o"])).abs().max()) == 0.0
    assert float((rd_b - t(z["rays_d"])).abs().max()) <= 2e-7
    ro, rd = t(z["rays_o"]), t(z["rays_d"])
    out = tr.forward(ro, rd, t(z["t_rand"]), t(z["u"]))
    assert max_err(out["rgb_map_0"].detach().cpu().numpy(), z["rgb_map_0"]) < 1e-5
    assert psnr(out["rgb_map"].detach().cpu().numpy(), z["rgb_map"]) > 60.0
    losses = tr.loss(out, t(z["target"]))
    assert abs(losses["loss_coarse"].item() - float(z["loss_coarse"])) <= 1e-6 * float(z["loss_coarse"])
    assert abs(losses["loss"].item() - float(z["loss"])) <= 1e-4 * float(z["loss"])
    tr.opt.zero_grad(set_to_none=True)
    losses["loss_coarse"].backward(retain_graph=True)
    _elementwise_grads("t3_c3_scatter", {k: p.grad for k, p in tr.named_parameters()},
                       coarse=True)
    tr.opt.zero_grad(set_to_none=True)
    losses["loss"].backward()
    _elementwise_grads("t3_c3_scatter", {k: p.grad for k, p in tr.named_parameters()})
