"""The training step's HIP compositing and importance-sampling ops
(nerfhip/train_ops.py on csrc/train_kernels.hip + nerf_sample_fine) against the
oracle (forward, CPU) and torch autograd of the reference's op sequence in
float64 (backward).

Tolerances: forward maps 1e-6 abs (the oracle restates torch's CPU orders; the
kernel sums in the same orders, accumulating T in double), fine depths
bit-exact (as the inference kernel), gradients 1e-4 relative to each tensor's
largest magnitude (float32 kernel vs float64 reference)."""
import numpy as np
import pytest
import torch

from goldlib import max_err
from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _inputs(n, S, seed, dense=True):
    rng = np.random.default_rng(seed)
    raw = rng.normal(0, 2.0, (n, S, 4)).astype(np.float32)
    raw[..., 3] = rng.normal(1.0 if dense else -1.0, 3.0, (n, S)).astype(np.float32)
    raw[: n // 4, :, 3] = -2.0                        # empty rays: every a = 0
    z = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return raw, z, d


def _rel(a, b):
    b = b.double()
    return float((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("S,white", [(64, True), (192, True), (5, False), (130, True)])
def test_composite_forward_matches_oracle(dev, S, white):
    from nerfhip.train_ops import composite_hip
    raw, z, d = _inputs(300, S, S)
    t = lambda a: torch.from_numpy(a).to(dev)   # noqa: E731
    rgb, disp, acc, w, depth = [x.cpu().numpy() for x in composite_hip(t(raw), t(z), t(d), white)]
    ref = O.raw2outputs(raw, z, d, white)
    assert max_err(w, ref[3]) < 1e-6
    assert max_err(rgb, ref[0]) < 1e-6
    assert max_err(acc, ref[2]) < 1e-6
    assert max_err(depth, ref[4]) < 1e-5
    assert np.array_equal(np.isnan(disp), np.isnan(ref[1]))


@pytest.mark.parametrize("S,white,with_z,empty", [(64, True, False, True), (192, True, True, True),
                                                   (7, False, True, True), (64, True, True, False)])
def test_composite_backward_matches_float64_autograd(dev, S, white, with_z, empty):
    """Upstream gradients on rgb, acc, weights and depth (and on disp when no ray
    is empty: disp = 1/max(1e-10, depth/acc) is NaN where acc = 0, and so is its
    float64 autograd gradient)."""
    from nerfhip.train import composite
    from nerfhip.train_ops import composite_hip
    raw, z, d = _inputs(256, S, 100 + S)
    if not empty:
        raw[..., 3] = np.abs(raw[..., 3]) + 0.1
    g = torch.Generator(device=dev).manual_seed(S)
    n = raw.shape[0]
    ups = [torch.randn(sh, device=dev, generator=g) for sh in ((n, 3), (n,), (n,), (n, S), (n,))]
    ups[1] = ups[1] * 1e-3
    keep = [0, 2, 3, 4] if empty else [0, 1, 2, 3, 4]
    r32 = torch.from_numpy(raw).to(dev).requires_grad_(True)
    z32 = torch.from_numpy(z).to(dev).requires_grad_(with_z)
    d32 = torch.from_numpy(d).to(dev)
    out = composite_hip(r32, z32, d32, white)
    got = torch.autograd.grad([out[k] for k in keep], [r32] + ([z32] if with_z else []),
                              [ups[k] for k in keep])
    r64 = torch.from_numpy(raw).to(dev).double().requires_grad_(True)
    z64 = torch.from_numpy(z).to(dev).double().requires_grad_(with_z)
    ref_out = composite(r64, z64, d32.double(), white)
    ref = torch.autograd.grad([ref_out[k] for k in keep], [r64] + ([z64] if with_z else []),
                              [ups[k].double() for k in keep])
    for a, b in zip(got, ref):
        assert torch.isfinite(a).all()
        assert _rel(a, b) < 1e-4, _rel(a, b)


@pytest.mark.parametrize("S,NI", [(64, 128), (5, 7), (130, 256)])
def test_sample_fine_forward_bit_exact_and_backward(dev, S, NI):
    """z_all = sort(cat(z, sample_pdf)) bit-exact vs the oracle (training u);
    dL/dweights vs float64 autograd of the reference's sample_pdf + sort."""
    from nerfhip.train import sample_pdf
    from nerfhip.train_ops import sample_fine_hip
    rng = np.random.default_rng(S + NI)
    n = 200
    z = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    w = (rng.random((n, S)) ** 3).astype(np.float32)
    u = rng.random((n, NI)).astype(np.float32)
    t = lambda a: torch.from_numpy(a).to(dev)   # noqa: E731
    wt = t(w).requires_grad_(True)
    zall = sample_fine_hip(wt, t(z), t(u))
    mids = (np.float32(0.5) * (z[:, 1:] + z[:, :-1])).astype(np.float32)
    ref = np.sort(np.concatenate([z, O.sample_fine(mids, w[:, 1:-1], u)], -1), -1)
    assert np.array_equal(zall.detach().cpu().numpy(), ref)
    g = torch.randn(zall.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    (got,) = torch.autograd.grad(zall, [wt], g)
    # reference: torch autograd of the reference's op sequence on the CPU in
    # float32, the reference's own arithmetic (CPU cumsum accumulates in double
    # as the kernel does). d z_f / d cdf carries 1/(c1 - c0) >= 1e-5: float64,
    # or torch float32 on the GPU (float cumsum), differ from it on 1-8 % of the
    # rays by up to 2e-3; the kernel agrees with it to 1e-4 on >= 99 % of rays.
    wc = torch.from_numpy(w).requires_grad_(True)
    zc = torch.from_numpy(z)
    zf = sample_pdf(0.5 * (zc[:, 1:] + zc[:, :-1]), wc[:, 1:-1], torch.from_numpy(u))
    z2, _ = torch.sort(torch.cat([zc, zf], -1), -1)
    (exp,) = torch.autograd.grad(z2, [wc], g.cpu())
    got = got.cpu()
    assert torch.isfinite(got).all()
    assert (got[:, 0] == 0).all() and (got[:, -1] == 0).all()
    err = (got.double() - exp.double()).abs().amax(1) / exp.abs().amax().double().clamp_min(1e-30)
    assert float((err < 1e-4).double().mean()) >= 0.99, float(err.max())
    assert float(err.max()) < 1e-2


@pytest.mark.parametrize("P", [1, 1000, 196608, 300001])
def test_raw_absmax_matches_torch(dev, P):
    """nerf_raw_absmax (the rgb / alpha heads' weight-gradient scales): max |rgb|
    and max |sigma| of d_raw, exactly torch's amax (order-free), raising the
    caller's slots (never lowering them)."""
    from nerfhip._lib import call, ptr, stream_of
    g = torch.Generator(device=dev).manual_seed(P)
    raw = torch.randn((P, 4), device=dev, generator=g) * torch.tensor([1.0, 2.0, 3.0, 0.5],
                                                                      device=dev)
    out = torch.zeros(2, device=dev)
    call("nerf_raw_absmax", ptr(raw), P, ptr(out), stream_of(dev))
    assert out[0].item() == raw[:, :3].abs().max().item()
    assert out[1].item() == raw[:, 3].abs().max().item()
    big = torch.full((2,), 1e6, device=dev)
    call("nerf_raw_absmax", ptr(raw), P, ptr(big), stream_of(dev))
    assert torch.equal(big, torch.full((2,), 1e6, device=dev))


def test_x3_clock_twin_computes_the_same(dev):
    """nerf_mlp_forward_x3_clock (bench.py's held-clock probe) gives
    nerf_mlp_forward_x3's raw bit for bit, and one stamp per workgroup whose
    clock (d memtime / d realtime x 100 MHz) is a plausible shader clock."""
    from nerfhip._lib import call, ptr, stream_of
    from nerfhip.pack import pack_mlp_x3
    from nerfhip.synthetic import make_params
    sl, hd = (torch.from_numpy(a).to(dev) for a in pack_mlp_x3(make_params(0, 2.0, 0.1)))
    n, S = 5000, 64
    g = torch.Generator(device=dev).manual_seed(3)
    ro = torch.rand((n, 3), device=dev, generator=g) - 0.5
    rd = torch.nn.functional.normalize(torch.randn((n, 3), device=dev, generator=g), dim=1)
    z = torch.linspace(2.0, 6.0, S, device=dev)
    a = torch.empty((n * S, 4), device=dev)
    b = torch.empty((n * S, 4), device=dev)
    call("nerf_mlp_forward_x3", ptr(sl), ptr(hd), ptr(ro), ptr(rd), ptr(z), 0, n, S, ptr(a),
         stream_of(dev))
    clk = torch.zeros(4 * 4096, device=dev, dtype=torch.int64)
    trace = torch.zeros(512 * 4, device=dev, dtype=torch.int64)
    call("nerf_mlp_forward_x3_clock", ptr(sl), ptr(hd), ptr(ro), ptr(rd), ptr(z), 0, n, S, ptr(b),
         ptr(clk), clk.numel(), ptr(trace), stream_of(dev))
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    c = clk.view(-1, 4).cpu().numpy().astype(np.float64)
    used = c[:, 3] > c[:, 2]
    assert used.sum() == min(-(-n * S // 128), torch.cuda.get_device_properties(dev).multi_processor_count)
    ghz = (c[used, 1] - c[used, 0]) / (c[used, 3] - c[used, 2]) * 0.1
    assert 0.5 < np.median(ghz) < 3.0, np.median(ghz)


@pytest.mark.parametrize("S,NI,ties", [(64, 128, False), (64, 128, True), (17, 40, True),
                                        (130, 256, False)])
def test_sample_pdf_bwd_search_equals_count(dev, S, NI, ties):
    """nerf_sample_pdf_bwd with the forward's z_all (each fine sample's place
    found by one search of the merged row, the rank count only for a repeated
    value) is bit-equal to the count over all fine samples (z_all NULL); ties:
    u on a coarse grid and all-zero weight rows, so values repeat (fine-fine and
    fine-coarse)."""
    from nerfhip._lib import call, ptr, stream_of
    rng = np.random.default_rng(7 + S + NI + ties)
    n = 300
    z = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    w = (rng.random((n, S)) ** 3).astype(np.float32)
    u = rng.random((n, NI)).astype(np.float32)
    if ties:
        u = (np.floor(u * 8) / 8).astype(np.float32)
        w[::5] = 0.0
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
    zt, wt, ut = t(z), t(w), t(u)
    zall = torch.empty((n, S + NI), device=dev)
    call("nerf_sample_fine", ptr(zt), S, ptr(wt), ptr(ut), NI, n, S, NI, ptr(zall), stream_of(dev))
    g = torch.randn(zall.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
    out = []
    for za in (zall, None):
        d = torch.empty_like(wt)
        call("nerf_sample_pdf_bwd", ptr(zt), ptr(wt), ptr(ut), ptr(g), ptr(za), n, S, NI, ptr(d),
             stream_of(dev))
        out.append(d.cpu())
    assert torch.isfinite(out[0]).all()
    assert torch.equal(out[0], out[1])
