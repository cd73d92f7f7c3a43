"""The x3-MFMA training MLP (nerfhip/train_mlp.py: nerf_x3_layer / nerf_x3_wgrad)
against the reference NeRF module (network.py:49-74) under torch FP32
autograd on the same device, on a ragged sample count.

Tolerances (relative to each tensor's max magnitude): forward raw 1e-5;
parameter gradients and d/d pts 1e-4 (FP32-accurate products, different
summation order over up to 3000 samples)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def _model(dev, seed=0, gain=2.0):
    from nerfhip.synthetic import make_params
    from src.models.nerf.network import NeRF
    params = make_params(seed, gain, 0.1)
    m = NeRF().to(dev)
    with torch.no_grad():
        for k, p in m.named_parameters():
            p.copy_(torch.as_tensor(np.asarray(params["model." + k])))
    return m


def _inputs(dev, P, seed=1):
    g = torch.Generator().manual_seed(seed)
    pts = (torch.rand((P, 3), generator=g) * 3.0 - 1.5).to(dev)
    dirs = torch.nn.functional.normalize(torch.randn((P, 3), generator=g), dim=1).to(dev)
    return pts, dirs


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _relu_edge_samples(m, pts, dirs, tol=1e-6):
    """Samples with a ReLU pre-activation within tol x the layer's max |.| of 0
    in the reference module (network.py:49-74): there the ReLU decision is a
    coin flip under any FP32 summation order (one such unit of one sample moves
    that sample's gradients by O(1)), so gradient comparisons zero their d_raw."""
    from nerfhip.train import freq_encode
    with torch.no_grad():
        x = torch.cat([freq_encode(pts, 10), freq_encode(dirs, 4)], -1)
        p_in, v_in = x[:, :63], x[:, 63:]
        h, edge = p_in, torch.zeros(pts.shape[0], dtype=torch.bool, device=pts.device)
        for i, lin in enumerate(m.pts_linears):
            pre = lin(h)
            edge |= (pre.abs() <= tol * pre.abs().max()).any(1)
            h = torch.relu(pre)
            if i in m.skips:
                h = torch.cat([p_in, h], -1)
        pre = m.views_linears[0](torch.cat([m.feature_linear(h), v_in], -1))
        edge |= (pre.abs() <= tol * pre.abs().max()).any(1)
    return edge


@pytest.mark.parametrize("P,fused", [(1000, True), (3000, True), (1000, False), (3000, False)])
def test_x3_train_mlp_forward_backward_match_torch(dev, P, fused, monkeypatch):
    from nerfhip import train_mlp
    from nerfhip.train import freq_encode
    from nerfhip.train_mlp import NerfMLPFn, PARAM_NAMES, mlp_params
    monkeypatch.setattr(train_mlp, "FUSED_FORWARD", fused)
    m = _model(dev)
    pts, dirs = _inputs(dev, P)
    g = torch.Generator(device=dev).manual_seed(2)
    d_raw = torch.randn((P, 4), device=dev, generator=g)
    d_raw[_relu_edge_samples(m, pts, dirs)] = 0.0

    # reference: torch FP32 autograd of the reference module
    x = pts.clone().requires_grad_(True)
    ref = m(torch.cat([freq_encode(x, 10), freq_encode(dirs, 4)], -1))
    ref_grads = torch.autograd.grad(ref, [x] + mlp_params(m), d_raw)

    y = pts.clone().requires_grad_(True)
    out = NerfMLPFn.apply(y, dirs, *mlp_params(m))
    got = torch.autograd.grad(out, [y] + mlp_params(m), d_raw)
    assert _rel(out.detach(), ref.detach()) < 1e-5
    for name, a, b in zip(["pts"] + PARAM_NAMES, got, ref_grads):
        assert a.shape == b.shape, name
        assert _rel(a, b) < 1e-4, (name, _rel(a, b))


@pytest.mark.parametrize("P", [1024, 1000])
def test_tiny_sigma_gradient_keeps_its_split_range(dev, P, monkeypatch):
    """The fused forward + backward read the alpha head's gradient off the
    views layer's weight-gradient tile: its A operand is [d hv; d sigma] (d sigma
    at row 128). With one FP16 split range for both (the max of the two), a
    d sigma far below d hv would split into denormal / flushed halves; row 128
    takes its own range (NerfWgradDesc.a2_row; the unaligned P = 1000 goes
    through the per-block fallback). d sigma scaled by 2^-30: every gradient,
    alpha_linear's included, within 1e-4 of torch FP32 autograd of the
    reference module (network.py:49-74)."""
    from nerfhip import train_mlp
    from nerfhip.train import freq_encode
    from nerfhip.train_mlp import NerfMLPFn, PARAM_NAMES, mlp_params
    monkeypatch.setattr(train_mlp, "FUSED_FORWARD", True)
    monkeypatch.setattr(train_mlp, "FUSED_BACKWARD", True)
    m = _model(dev)
    pts, dirs = _inputs(dev, P)
    d_raw = torch.randn((P, 4), device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    d_raw[:, 3] *= 2.0 ** -30
    d_raw[_relu_edge_samples(m, pts, dirs)] = 0.0
    x = pts.clone().requires_grad_(True)
    ref = m(torch.cat([freq_encode(x, 10), freq_encode(dirs, 4)], -1))
    ref_grads = torch.autograd.grad(ref, [x] + mlp_params(m), d_raw)
    y = pts.clone().requires_grad_(True)
    out = NerfMLPFn.apply(y, dirs, *mlp_params(m))
    got = torch.autograd.grad(out, [y] + mlp_params(m), d_raw)
    errs = {name: _rel(a, b) for name, a, b in zip(["pts"] + PARAM_NAMES, got, ref_grads)}
    assert errs["alpha_linear.weight"] < 1e-4 and errs["alpha_linear.bias"] < 1e-4, errs
    assert max(errs.values()) < 1e-4, errs


@pytest.mark.parametrize("shared", [True, False])
@pytest.mark.parametrize("gain", [2.0 ** -10, 2.0 ** -14])
def test_small_views_output_keeps_rgb_gradient_precision(dev, shared, gain, monkeypatch):
    """The shared views-encoding / rgb weight-gradient tile multiplies
    [d hv; d sigma; d rgb] by [view enc; HV]^T with ONE FP16 split range for B,
    max(max |enc|, max |HV|). The views layer's output HV scaled down by
    `gain` (its weight and bias x gain, the rgb head x 1/gain: the same network
    in real arithmetic) sits far below the encoding's |.| <= 1 there; the split
    keeps about 21 bits while max |HV| >= 2^-16 of the range (the low half stays
    an FP16 normal). Every gradient, rgb_linear's included, within 1e-4 of
    torch FP32 autograd of the reference module (network.py:49-74), with the
    shared tile and with the two tiles of its own (NERF_TRAIN_ENC_RGB_TILE=0).
    (The rows between d sigma and d rgb that the shared tile reads, A rows
    129..143, feed only discarded output rows.)"""
    from nerfhip import train_mlp
    from nerfhip.train import freq_encode
    from nerfhip.train_mlp import NerfMLPFn, PARAM_NAMES, mlp_params
    monkeypatch.setattr(train_mlp, "FUSED_FORWARD", True)
    monkeypatch.setattr(train_mlp, "FUSED_BACKWARD", True)
    monkeypatch.setattr(train_mlp, "ENC_RGB_TILE", shared)
    m = _model(dev)
    with torch.no_grad():
        m.views_linears[0].weight.mul_(gain)
        m.views_linears[0].bias.mul_(gain)
        m.rgb_linear.weight.mul_(1.0 / gain)
    P = 1024
    pts, dirs = _inputs(dev, P)
    d_raw = torch.randn((P, 4), device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    d_raw[_relu_edge_samples(m, pts, dirs)] = 0.0
    x = pts.clone().requires_grad_(True)
    ref = m(torch.cat([freq_encode(x, 10), freq_encode(dirs, 4)], -1))
    ref_grads = torch.autograd.grad(ref, [x] + mlp_params(m), d_raw)
    y = pts.clone().requires_grad_(True)
    out = NerfMLPFn.apply(y, dirs, *mlp_params(m))
    got = torch.autograd.grad(out, [y] + mlp_params(m), d_raw)
    errs = {name: _rel(a, b) for name, a, b in zip(["pts"] + PARAM_NAMES, got, ref_grads)}
    assert errs["rgb_linear.weight"] < 1e-4 and errs["rgb_linear.bias"] < 1e-4, errs
    assert max(errs.values()) < 1e-4, errs


def test_pack_tables_follow_rebuilds(dev):
    """The device tables of a network's packing launch (_launch_packs) are cached;
    every rebuild of a packer allocates new output buffers (streams, scales,
    maxima, the fold's Wc / bc, head), so a table made for an earlier build must
    never serve a later one -- also when the parameter addresses repeat
    (parameters A, then B, then A again). A stale table writes the packing into
    the freed buffers of the old build (an intermittent illegal address when
    that memory is returned) and leaves the live stream unpacked. The streams
    after A -> B -> A equal a fresh packer's of A bit for bit."""
    from nerfhip.train_mlp import PARAM_NAMES, X3NetPacker, mlp_params
    m = _model(dev)
    pa = dict(zip(PARAM_NAMES, mlp_params(m)))
    pb = dict(pa, **{"rgb_linear.weight": pa["rgb_linear.weight"].detach().clone()})
    net = X3NetPacker(dev)
    for p in (pa, pb, pa):
        streams = net.streams(p)
    fresh = X3NetPacker(dev).streams(pa)
    torch.cuda.synchronize()
    assert net.gen == 3
    for a, b in zip(streams, fresh):
        assert torch.equal(a, b)
    assert streams[0].abs().sum() > 0


def test_x3_layer_kernel_matches_matmul(dev):
    """One nerf_x3_layer launch per supported shape: bias + ReLU + mask + rank-1."""
    from nerfhip.train_mlp import _layer, pack_x3_matrix
    g = torch.Generator(device=dev).manual_seed(3)
    P = 777
    for mt, nk in [(16, 8)]:       # the all-terms epilogue instance
        M, K = 16 * mt, 32 * nk
        W = torch.randn((M, K), device=dev, generator=g) * 0.1
        B = torch.randn((K, P), device=dev, generator=g) * torch.logspace(-3, 2, P, device=dev)
        bias = torch.randn(M, device=dev, generator=g)
        mask = torch.randn((M, P), device=dev, generator=g)
        ru = torch.randn(M, device=dev, generator=g)
        rw = torch.randn(P, device=dev, generator=g)
        wp, sw = pack_x3_matrix(W)
        C = torch.empty((M, P), device=dev)
        _layer(wp, sw, mt, nk, B, C, P, bias=bias, relu=True, mask=mask, ru=ru, rw=rw)
        ref = torch.relu(W.double() @ B.double() + bias.double()[:, None]
                         + ru.double()[:, None] * rw.double()[None, :]) * (mask > 0)
        # per sample: the magnitude of every term summed into it
        scale = (W.double().abs() @ B.double().abs() + bias.double().abs()[:, None]
                 + ru.double().abs()[:, None] * rw.double().abs()[None, :]).amax(0)
        err = ((C.double() - ref).abs() / scale.clamp_min(1e-30)).max().item()
        assert err < 1e-6, (mt, nk, err)


# terms: b = bias, R = ReLU, m = mask, 1 = rank-1 addend
@pytest.mark.parametrize("mt,nk,terms", [(16, 2, "bR"), (16, 8, "bR"), (16, 10, "bR"),
                                         (8, 9, "bR"), (16, 8, "b"), (16, 4, ""), (16, 8, "m"),
                                         (16, 8, "m1"), (4, 8, "")])
def test_x3_layer_instances(dev, mt, nk, terms):
    """Every (shape, epilogue) instance the training MLP launches."""
    from nerfhip.train_mlp import _layer, pack_x3_matrix
    g = torch.Generator(device=dev).manual_seed(5)
    P = 300
    M, K = 16 * mt, 32 * nk
    W = torch.randn((M, K), device=dev, generator=g) * 0.1
    B = torch.randn((K, P), device=dev, generator=g)
    bias = torch.randn(M, device=dev, generator=g) if "b" in terms else None
    mask = torch.randn((M, P), device=dev, generator=g) if "m" in terms else None
    ru = torch.randn(M, device=dev, generator=g) if "1" in terms else None
    rw = torch.randn(P, device=dev, generator=g) if "1" in terms else None
    wp, sw = pack_x3_matrix(W)
    C = torch.empty((M, P), device=dev)
    relu = "R" in terms
    _layer(wp, sw, mt, nk, B, C, P, bias=bias, relu=relu, mask=mask, ru=ru, rw=rw)
    ref = W.double() @ B.double()
    if bias is not None:
        ref = ref + bias.double()[:, None]
    if ru is not None:
        ref = ref + ru.double()[:, None] * rw.double()[None, :]
    if relu:
        ref = torch.relu(ref)
    if mask is not None:
        ref = ref * (mask > 0)
    scale = (W.double().abs() @ B.double().abs()).amax(0) + 10.0
    assert ((C.double() - ref).abs() / scale).max().item() < 1e-6


def test_x3_wgrad_matches_matmul(dev):
    from nerfhip.train_mlp import _wgrad
    g = torch.Generator(device=dev).manual_seed(4)
    for M, N, P in [(256, 320, 5000), (128, 288, 4096), (256, 64, 33)]:
        A = torch.randn((M, P), device=dev, generator=g)
        B = torch.relu(torch.randn((N, P), device=dev, generator=g))
        got = _wgrad(A, B).double()
        ref = A.double() @ B.double().t()
        scale = (A.double().abs() @ B.double().abs().t()).max().item()
        assert (got - ref).abs().max().item() / scale < 1e-6, (M, N, P)


@pytest.mark.parametrize("M,N,P,pad", [(256, 320, 4096, 32), (3, 256, 2048, 0), (128, 288, 8192, 32),
                                       (256, 64, 32, 32)])
def test_x3_wgrad_dma_path(dev, M, N, P, pad):
    """The LDS-DMA weight-gradient kernel (P % 32 == 0, aligned rows, padded row
    strides as the training MLP allocates them): dW and the fused bias sums."""
    from nerfhip.train_mlp import _wgrad
    g = torch.Generator(device=dev).manual_seed(6)
    A = torch.randn((M, P + pad), device=dev, generator=g)[:, :P]
    B = torch.relu(torch.randn((N, P + pad), device=dev, generator=g))[:, :P]
    got, gb = _wgrad(A, B, with_bias=True)
    ref = A.double() @ B.double().t()
    scale = (A.double().abs() @ B.double().abs().t()).max().item()
    assert (got.double() - ref).abs().max().item() / scale < 1e-6
    rb = A.double().sum(1)
    assert (gb.double() - rb).abs().max().item() / A.double().abs().sum(1).max().item() < 1e-6


def test_x3_packer_matches_reference_packing(dev):
    """The one-launch packer (nerf_x3_pack) == pack_x3_matrix of each padded matrix."""
    from nerfhip.train_mlp import PARAM_NAMES, X3Packer, mlp_params, pack_x3_matrix
    m = _model(dev)
    p = dict(zip(PARAM_NAMES, mlp_params(m)))
    packer = X3Packer(dev)
    got = packer.pack(p)
    for name, (pname, tr, rmap, cmap) in packer.plan(p).items():
        W = p[pname].detach()
        W = W.t() if tr else W
        Wp = torch.zeros((len(rmap), len(cmap)), device=dev)
        ri = torch.tensor(rmap, device=dev)
        ci = torch.tensor(cmap, device=dev)
        ok = (ri[:, None] >= 0) & (ci[None, :] >= 0)
        Wp[ok] = W[ri.clamp_min(0)][:, ci.clamp_min(0)][ok]
        ref, sw = pack_x3_matrix(Wp)
        out, sw_got, mt, nk = got[name]
        assert (mt, nk) == (len(rmap) // 16, len(cmap) // 32), name
        assert int(sw_got.item()) == int(sw.item()), name
        assert torch.equal(out.view(torch.int32), ref.view(torch.int32)), name


@pytest.mark.parametrize("P,L", [(1000, 10), (4099, 4), (1, 10)])
def test_freq_encode_fm_matches_torch(dev, P, L):
    """nerf_freq_encode_fm (feature-major, row stride P + 32, fused max |.|) and
    its backward against freq.py's torch restatement and its autograd on the same
    device: encoding within 2 ulp of 1 (the same device sin/cos), amax equal to
    the max of the written values, d/dx 1e-5 relative."""
    from nerfhip import _lib
    from nerfhip._lib import call, ptr
    from nerfhip.train import freq_encode
    from nerfhip.train_mlp import _act
    g = torch.Generator().manual_seed(P)
    x = ((torch.rand((P, 3), generator=g) - 0.5) * 8.0).to(dev)
    F = 3 + 6 * L
    out = _act(F, P, dev)
    amax = torch.zeros(1, device=dev)
    call("nerf_freq_encode_fm", ptr(x), 3, P, L, ptr(out), out.stride(0), ptr(amax),
         _lib.stream_of(dev))
    ref = freq_encode(x, L).t()
    assert float((out - ref).abs().max()) <= 2.5e-7
    assert float(amax) == float(out.abs().max())
    d_enc = torch.randn((F, P), generator=g).to(dev)
    dx = torch.empty((P, 3), device=dev)
    call("nerf_freq_encode_fm_backward", ptr(d_enc), d_enc.stride(0), ptr(x), 3, P, L, ptr(dx),
         _lib.stream_of(dev))
    xr = x.clone().requires_grad_(True)
    (gr,) = torch.autograd.grad(freq_encode(xr, L), xr, d_enc.t())
    assert _rel(dx, gr) < 1e-5
    # the training backward's form: two gradient row sets summed in the kernel,
    # sin / cos read from the forward's rows (out, padded to the same stride)
    d_a = _act(F, P, dev)
    d_b = _act(F, P, dev)
    d_a.copy_(d_enc * 0.25)
    d_b.copy_(d_enc * 0.75)
    dx2 = torch.empty((P, 3), device=dev)
    call("nerf_freq_encode_fm_backward_sum", ptr(d_a), ptr(d_b), d_a.stride(0), 0, ptr(out),
         out.stride(0), 0, ptr(x), 3, P, L, ptr(dx2), _lib.stream_of(dev))
    (gr2,) = torch.autograd.grad(freq_encode(xr, L), xr, (d_a + d_b).t())
    assert _rel(dx2, gr2) < 1e-5


def test_x3_train_mlp_denormal_sample_gradients(dev):
    """Samples whose output gradient underflows (rays behind an opaque surface:
    transmittance ~ 0, d raw ~ 1e-40) must not turn the per-sample FP16 split
    scale into inf (0 * inf = NaN in every parameter gradient); they contribute
    nothing, as in FP32."""
    from nerfhip.train import freq_encode
    from nerfhip.train_mlp import NerfMLPFn, PARAM_NAMES, mlp_params
    m = _model(dev)
    P = 2048
    pts, dirs = _inputs(dev, P, seed=4)
    g = torch.Generator(device=dev).manual_seed(5)
    d_raw = torch.randn((P, 4), device=dev, generator=g)
    d_raw[P // 2:] *= 1e-40                       # FP32 denormals
    d_raw[P // 4:P // 2] = 0.0
    x = pts.clone().requires_grad_(True)
    ref = m(torch.cat([freq_encode(x, 10), freq_encode(dirs, 4)], -1))
    ref_grads = torch.autograd.grad(ref, [x] + mlp_params(m), d_raw)
    y = pts.clone().requires_grad_(True)
    out = NerfMLPFn.apply(y, dirs, *mlp_params(m))
    got = torch.autograd.grad(out, [y] + mlp_params(m), d_raw)
    for name, a, b in zip(["pts"] + PARAM_NAMES, got, ref_grads):
        assert torch.isfinite(a).all(), name
        assert _rel(a, b) < 1e-4, (name, _rel(a, b))


@pytest.mark.parametrize("nk", [2, 8, 10])
def test_x3_layer_relu_bits_roundtrip(dev, nk):
    """A forward launch writes its ReLU mask as bits (nerf_x3_layer_bits); a
    masked dgrad launch reading those bits is bitwise equal to the same launch
    masked by the FP32 activations, for ragged P (invalid samples' bits 0)."""
    from nerfhip.train_mlp import _layer, pack_x3_matrix, relu_bits_words
    g = torch.Generator(device=dev).manual_seed(11)
    for P in (1, 300, 1000):
        K = 32 * nk
        W = torch.randn((256, K), device=dev, generator=g) * 0.1
        B = torch.randn((K, P), device=dev, generator=g)
        bias = torch.randn(256, device=dev, generator=g) * 0.05
        wp, sw = pack_x3_matrix(W)
        H = torch.empty((256, P), device=dev)
        H2 = torch.empty((256, P), device=dev)
        bits = torch.full((relu_bits_words(P, 16),), -1, device=dev, dtype=torch.int16)
        _layer(wp, sw, 16, nk, B, H, P, bias=bias, relu=True, bits_out=bits)
        _layer(wp, sw, 16, nk, B, H2, P, bias=bias, relu=True)
        assert torch.equal(H, H2)              # the bits do not change the forward
        # decode: u16 word ((p // 128 * 8 + p % 128 // 16) * 4 + m // 64) * 64
        # + p % 16 + 16 (m % 16 // 4), bit 4 (m % 64 // 16) + m % 4
        p = torch.arange(P, device=dev)[None, :]
        m = torch.arange(256, device=dev)[:, None]
        word = ((p // 128 * 8 + p % 128 // 16) * 4 + m // 64) * 64 + p % 16 + 16 * (m % 16 // 4)
        bit = 4 * (m % 64 // 16) + m % 4
        got = (bits.to(torch.int32)[word] >> bit) & 1
        assert torch.equal(got.bool(), H > 0)
        Wb = torch.randn((256, 256), device=dev, generator=g) * 0.1
        wpb, swb = pack_x3_matrix(Wb)
        D = torch.randn((256, P), device=dev, generator=g)
        Cf = torch.empty((256, P), device=dev)
        Cb = torch.empty((256, P), device=dev)
        _layer(wpb, swb, 16, 8, D, Cf, P, mask=H)
        _layer(wpb, swb, 16, 8, D, Cb, P, mask_bits=bits)
        assert torch.equal(Cf, Cb)
        ru = torch.randn(256, device=dev, generator=g)
        rw = torch.randn(P, device=dev, generator=g)
        _layer(wpb, swb, 16, 8, D, Cf, P, mask=H, ru=ru, rw=rw)
        _layer(wpb, swb, 16, 8, D, Cb, P, mask_bits=bits, ru=ru, rw=rw)
        assert torch.equal(Cf, Cb)


def test_x3_wgrad_batch_matches_matmul(dev):
    """WgradBatch: the weight gradients of a whole backward (shapes of the NeRF
    MLP: 256x64 enc, 256x320 skip, 128x288 views, 3x128 rgb, 1x256 alpha) in
    one nerf_x3_wgrad_batch launch + one fixed-order partial sum, with and
    without bias sums, padded row strides; and the ragged-P fallback (P % 32
    != 0: per-layer nerf_x3_wgrad)."""
    from nerfhip.train_mlp import WgradBatch
    g = torch.Generator(device=dev).manual_seed(8)
    for P, pad in ((4096, 32), (1000, 0)):
        shapes = [(256, 64, True), (256, 320, True), (256, 256, True), (128, 288, True),
                  (3, 128, False), (1, 256, False)]
        wb = WgradBatch(dev)
        ops = []
        for M, N, bias in shapes:
            A = torch.randn((M, P + pad), device=dev, generator=g)[:, :P]
            B = torch.relu(torch.randn((N, P + pad), device=dev, generator=g))[:, :P]
            ops.append((A, B, bias))
            wb.add(A, B, with_bias=bias)
        for (A, B, bias), res in zip(ops, wb.results()):
            got, gb = res if bias else (res, None)
            ref = A.double() @ B.double().t()
            scale = (A.double().abs() @ B.double().abs().t()).max().item()
            assert (got.double() - ref).abs().max().item() / scale < 1e-6, (A.shape, B.shape, P)
            if bias:
                rb = A.double().sum(1)
                assert (gb.double() - rb).abs().max().item() / A.double().abs().sum(1).max().item() < 1e-6


def test_x3_wgrad_batch_t16_operands_bitwise(dev):
    """The batched weight gradients read the T16 layout of the fused training
    kernels (train_mlp.BlockRows: NerfWgradDesc bsa / bsb) with the same
    arithmetic in the same order as feature-major operands: bit-identical
    results, for operands at a row offset inside a larger buffer, M / N that
    are not multiples of 16 (the 132-row [d_hv; d raw] operand, the 63
    encoding rows) and a joined column block."""
    from nerfhip.train_mlp import BlockRows, WgradBatch
    g = torch.Generator(device=dev).manual_seed(11)
    P = 4096
    shapes = [(256, 63, True), (132, 288, True), (256, 256, True), (3, 128, True)]
    fm, t16 = [], []
    for M, N, bias in shapes:
        A = torch.randn((M, P + 32), device=dev, generator=g)[:, :P]
        B = torch.relu(torch.randn((N, P + 32), device=dev, generator=g))[:, :P]
        bigA = BlockRows.alloc(M + 48, P, dev)
        bigB = BlockRows.alloc(N + 32, P, dev)
        bigA.buf.fill_(float("nan"))          # rows outside the operand must not be read
        bigB.buf.fill_(float("nan"))
        a16 = BlockRows.from_dense(A, R=M + 48 - 32)
        bigA.buf[:, 32:32 + a16.buf.shape[1]] = a16.buf
        b16 = BlockRows.from_dense(B)
        bigB.buf[:, 16:16 + b16.buf.shape[1]] = b16.buf
        Ab, Bb = bigA.rows(32, 32 + M), bigB.rows(16, 16 + N)
        assert torch.equal(Ab.dense(), A) and torch.equal(Bb.dense(), B)
        fm.append((A, B, bias))
        t16.append((Ab, Bb, bias))
    amax = [(A.abs().max().reshape(1), B.abs().max().reshape(1)) for A, B, _ in fm]
    out = []
    for ops in (fm, t16):
        wb = WgradBatch(dev)
        for (A, B, bias), (aa, ab) in zip(ops, amax):
            wb.add(A, B, aa, ab, with_bias=bias)
        s = wb.add(ops[2][0], ops[1][1], amax[2][0], amax[1][1], width=288 + 63)
        wb.add(ops[2][0], ops[0][1], amax[2][0], amax[0][1], into=(s, 288))
        out.append(wb.results())
    for a, b in zip(*out):
        if a is None:
            assert b is None
            continue
        a = a if isinstance(a, tuple) else (a,)
        b = b if isinstance(b, tuple) else (b,)
        assert all(torch.equal(x, y) for x, y in zip(a, b))


def test_x3_wgrad_batch_joined_column_blocks(dev):
    """WgradBatch column blocks: add(A, B1, width=W) + add(A, B2, into=(slot, c0))
    give one contiguous [M, W] gradient [A B1^T | A B2^T] (the skip layer's
    [63 encoding rows | h4], each block with its own scale: nerf_x3_wgrad_batch
    descriptors with ldo), next to ordinary requests sharing the same partial
    sum; with P % 32 != 0 the host joins the per-layer results the same way."""
    from nerfhip.train_mlp import WgradBatch
    g = torch.Generator(device=dev).manual_seed(9)
    for P in (4096, 1000):
        A = torch.randn((256, P + 32), device=dev, generator=g)[:, :P]
        B1 = torch.randn((63, P + 32), device=dev, generator=g)[:, :P] * 3.0
        B2 = torch.relu(torch.randn((256, P + 32), device=dev, generator=g))[:, :P] * 0.01
        C = torch.randn((128, P + 32), device=dev, generator=g)[:, :P]
        wb = WgradBatch(dev)
        s0 = wb.add(C, B2, with_bias=True)
        s1 = wb.add(A, B1, with_bias=True, width=319)
        s2 = wb.add(A, B2, into=(s1, 63))
        res = wb.results()
        assert res[s2] is None
        got, gb = res[s1]
        assert got.shape == (256, 319) and got.is_contiguous()
        ref = torch.cat([A.double() @ B1.double().t(), A.double() @ B2.double().t()], 1)
        for c0, c1, B in ((0, 63, B1), (63, 319, B2)):   # each block against its own scale
            scale = (A.double().abs() @ B.double().abs().t()).max().item()
            assert (got[:, c0:c1].double() - ref[:, c0:c1]).abs().max().item() / scale < 1e-6, P
        assert (gb.double() - A.double().sum(1)).abs().max().item() / \
            A.double().abs().sum(1).max().item() < 1e-6
        other, ob = res[s0]
        ref0 = C.double() @ B2.double().t()
        scale0 = (C.double().abs() @ B2.double().abs().t()).max().item()
        assert (other.double() - ref0).abs().max().item() / scale0 < 1e-6
        assert (ob.double() - C.double().sum(1)).abs().max().item() / \
            C.double().abs().sum(1).max().item() < 1e-6


def test_x3_stream_packer_matches_host_packing(dev):
    """X3StreamPacker (nerf_fold_views, then nerf_x3_pack into the 65-slice
    stream + the head gather) == nerfhip.pack.pack_mlp_x3 given the same fold:
    the stream bit for bit, the head value for value (scales included); the
    device fold (FP32) within 1e-6 of the float64 fold of
    fold_feature_into_views, relative to each row's magnitude."""
    import numpy as np
    from nerfhip.pack import pack_mlp_x3
    from nerfhip.train_mlp import PARAM_NAMES, X3StreamPacker, mlp_params
    m = _model(dev, seed=3, gain=2.5)
    p = dict(zip(PARAM_NAMES, mlp_params(m)))
    pk = X3StreamPacker(dev)
    stream, head = pk.pack(p)
    hp = {"model." + k: v.detach().cpu() for k, v in p.items()}
    ref_s, ref_h = pack_mlp_x3(hp, folded=(pk.Wc, pk.bc))
    assert stream.numel() == 65 * 8192
    assert torch.equal(stream.view(torch.int32).cpu(), torch.from_numpy(ref_s).view(torch.int32))
    assert torch.equal(head.cpu(), torch.from_numpy(ref_h))
    g = lambda k: hp["model." + k].numpy().astype(np.float64)   # noqa: E731
    Wf, bf, Wv, bv = (g(k) for k in ("feature_linear.weight", "feature_linear.bias",
                                     "views_linears.0.weight", "views_linears.0.bias"))
    W64 = np.concatenate([Wv[:, :256] @ Wf, Wv[:, 256:]], 1)
    b64 = Wv[:, :256] @ bf + bv
    scale = np.abs(Wv[:, :256]) @ np.abs(Wf)
    assert np.max(np.abs(pk.Wc.cpu().numpy()[:, :256] - W64[:, :256]) / (scale + 1e-30)) < 1e-6
    assert np.array_equal(pk.Wc.cpu().numpy()[:, 256:], Wv[:, 256:].astype(np.float32))
    sb = np.abs(Wv[:, :256]) @ np.abs(bf) + np.abs(bv)
    assert np.max(np.abs(pk.bc.cpu().numpy() - b64) / (sb + 1e-30)) < 1e-6



def test_x3_bwd_stream_packer_matches_host_packing(dev):
    """X3BwdStreamPacker: every transposed matrix's slices == pack_x3_matrix of
    that matrix (rows / K columns through the plan's maps, -1 -> 0) bit for bit,
    at the slice offsets the backward kernel consumes (64 slices; the first
    four: the fold Wc[:, :256]^T, which equals the forward packer's fold bit for
    bit); the head's rgb / alpha weights where the forward head holds them, the
    scales at 3100 + matrix slot (slot 1, the unfolded feature layer's: 0)."""
    import numpy as np
    from nerfhip.pack import H_ALPHA_W, H_RGB_W, SLICE_FLOATS, pack_mlp
    from nerfhip.train_mlp import (PARAM_NAMES, X3BwdStreamPacker, X3StreamPacker, mlp_params,
                                   pack_x3_matrix)
    m = _model(dev, seed=3, gain=2.5)
    p = dict(zip(PARAM_NAMES, mlp_params(m)))
    pk = X3BwdStreamPacker(dev)
    stream, head = pk.pack(p)
    plan, nsl = pk.plan()
    assert nsl == 64 and stream.numel() == nsl * SLICE_FLOATS
    fwd = X3StreamPacker(dev)
    fwd.pack(p)
    assert torch.equal(pk.Wc.view(torch.int32), fwd.Wc.view(torch.int32))
    hd = head.cpu()
    assert int(hd[3101]) == 0
    for name, rmap, cmap, off, j in plan:
        Wt = (pk.Wc if name == "fold" else p[name]).detach().t()
        rm, cm = torch.tensor(rmap, device=dev), torch.tensor(cmap, device=dev)
        T = torch.where((rm >= 0)[:, None] & (cm >= 0)[None, :],
                        Wt[rm.clamp_min(0)][:, cm.clamp_min(0)], 0.0)   # +0.0, as the kernel
        ref, sw = pack_x3_matrix(T.contiguous())
        seg = stream[off * SLICE_FLOATS:off * SLICE_FLOATS + ref.numel()]
        assert torch.equal(seg.view(torch.int32), ref.view(torch.int32)), name
        assert int(hd[3100 + j]) == int(sw.item()), name
    _, fwd_head = pack_mlp({"model." + k: v.detach().cpu() for k, v in p.items()})
    for a, n in ((H_RGB_W, 384), (H_ALPHA_W, 256)):
        assert np.array_equal(hd[a:a + n].numpy(), fwd_head[a:a + n])


@pytest.mark.parametrize("P", [1, 130, 4096, 70001])
def test_fused_train_forward_equals_layer_launches(dev, P, monkeypatch):
    """nerf_mlp_train_forward_x3 (one launch) against the ten x3_layer_kernel
    launches it replaces, on the same inputs: raw, every saved activation row
    (h0..h7, feature, views output) and every max |.| within 1e-6 relative
    (the same x3 arithmetic; the layer-0 and skip K steps run in another order),
    the ReLU bits equal wherever the activation is not within 1e-6 of 0, and
    the backward's gradients within 1e-5."""
    from nerfhip import train_mlp
    from nerfhip.train_mlp import NerfMLPFn, PARAM_NAMES, mlp_params
    m = _model(dev, seed=4, gain=2.0)
    pts, dirs = _inputs(dev, P, seed=5)
    d_raw = torch.randn((P, 4), device=dev, generator=torch.Generator(device=dev).manual_seed(6))
    d_raw[_relu_edge_samples(m, pts, dirs)] = 0.0
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(train_mlp, "FUSED_FORWARD", fused)
        y = pts.clone().requires_grad_(True)
        out = NerfMLPFn.apply(y, dirs, *mlp_params(m))
        node = out.grad_fn
        saved = _saved_rows(node, P)
        grads = torch.autograd.grad(out, [y] + mlp_params(m), d_raw)
        res[fused] = (out.detach().clone(), saved, grads)
    (o0, s0, g0), (o1, s1, g1) = res[False], res[True]
    assert _rel(o1, o0) < 1e-6
    # saved: pts, E, h0..h3, h5..h7, V, HV, amax, bits, bits_v
    # (the fused forward keeps h7 in V's first 256 rows instead of the feature rows,
    # which it does not store: only V's view-encoding rows compare)
    names = ["pts", "E", "h0", "h1", "h2", "h3", "h5", "h6", "h7", "V", "HV", "amax"]
    for name, a, b in zip(names, s1[:12], s0[:12]):
        assert a.shape == b.shape, name
        if name == "V":
            a, b = a[256:], b[256:]
        if name == "amax":   # slot 8 (feature rows): the fused forward folds that layer away
            assert float(a[8]) == 0.0
            a, b = torch.cat([a[:8], a[9:]]), torch.cat([b[:8], b[9:]])
        assert _rel(a, b) < 1e-6, (name, _rel(a, b))
    assert torch.equal(s1[9][:256], s1[8])              # fused: V[:256] is h7
    # ReLU bits (x3_layer_kernel's word layout, what the dgrad launches read):
    # a bit can only differ where the activation sits at the ReLU's edge
    for b0, b1, mt in ((s0[12], s1[12], 16), (s0[13], s1[13], 8)):
        assert b0.shape == b1.shape
        w = torch.arange(b0.shape[-1], device=dev)
        lane, blk = w % 64, w // 64                   # word ((tile*8+wave)*mt/4 + k)*64 + lane
        tw = blk // (mt // 4)
        sample = (tw // 8) * 128 + (tw % 8) * 16 + lane % 16
        valid = sample < P                             # words of samples past P are not written
        assert float((b0 != b1)[..., valid].float().mean()) < 1e-3
    for name, a, b in zip(["pts"] + PARAM_NAMES, g1, g0):
        assert _rel(a, b) < 1e-5, (name, _rel(a, b))


def _saved_rows(node, P):
    """What a NerfMLPFn node saved for its backward, feature-major: pts, E,
    h0..h3, h5..h7, V, HV, amax, bits, bits_v (the fused kernels keep E .. HV in
    one T16 buffer, train_mlp._fwd_rows_t16)."""
    from nerfhip.train_mlp import BlockRows, _fwd_rows_t16
    st = node.saved_tensors
    if st[1].dim() == 3:   # (pts, T16 buffer, amax, bits, bits_v, *params)
        E, H, V, HV = _fwd_rows_t16(st[1], P)
        rows = [E, H[0], H[1], H[2], H[3], H[5], H[6], H[7], V, HV]
        return [st[0].clone()] + [r.dense().clone() for r in rows] + [t.clone() for t in st[2:5]]
    return [t.clone() for t in st[:14]]


def _dense(t):
    from nerfhip.train_mlp import BlockRows
    return t.dense() if isinstance(t, BlockRows) else t


@pytest.mark.parametrize("pts_grad", [True, False])
@pytest.mark.parametrize("P", [1, 130, 4096, 70001])
def test_fused_train_backward_equals_layer_launches(dev, P, pts_grad, monkeypatch):
    """nerf_mlp_train_backward_x3 (one launch) against the layer launches it
    replaces, after the same forward: d hv, D0..D7 and the encoding gradient
    rows within 1e-5 of each tensor's max (d hv: FP32 on the VALU instead of an
    x3 product over the 3 rgb rows; D7 through the fold Wc = W_views,feat
    W_feat in one product instead of two; the rest the same x3 products), every
    max |.| slot within 1e-5 (but DF's: the fused kernel has no d feature), the
    same zeros (the forward's ReLU bits), and the parameter / point gradients
    within 1e-5."""
    from nerfhip import train_mlp
    from nerfhip.train_mlp import NerfMLPFn, PARAM_NAMES, mlp_params
    m = _model(dev, seed=7, gain=2.0)
    pts, dirs = _inputs(dev, P, seed=8)
    d_raw = torch.randn((P, 4), device=dev, generator=torch.Generator(device=dev).manual_seed(9))
    rec = {}

    def recording(key, fn, dmax_arg):
        def w(*a):
            out = fn(*a)
            rows = [out[0], out[1], *out[2]] + (list(out[3]) if out[3] is not None else [])
            rec[key] = ([None if t is None else _dense(t).clone() for t in rows],
                        a[dmax_arg].clone(), out[3] is None)
            return out
        return staticmethod(w)

    monkeypatch.setattr(NerfMLPFn, "_backward_fused",
                        recording(True, NerfMLPFn._backward_fused, 4))
    monkeypatch.setattr(NerfMLPFn, "_backward_layers",
                        recording(False, NerfMLPFn._backward_layers, 5))
    grads = {}
    for fused in (False, True):
        monkeypatch.setattr(train_mlp, "FUSED_BACKWARD", fused)
        y = pts.clone().requires_grad_(pts_grad)
        out = NerfMLPFn.apply(y, dirs, *mlp_params(m))
        wrt = ([y] if pts_grad else []) + mlp_params(m)
        grads[fused] = torch.autograd.grad(out, wrt, d_raw)
    (r0, m0, n0), (r1, m1, n1) = rec[False], rec[True]
    assert n0 == n1 == (not pts_grad) and len(r0) == len(r1) == (12 if pts_grad else 10)
    names = ["d_hv", "DF"] + [f"D{i}" for i in range(8)] + ["d_enc5", "d_enc0"]
    assert r1[1] is None      # after the fused forward DF is not stored (weights via G)
    for name, a, b in zip(names, r1, r0):
        if a is None:
            continue
        assert a.shape == b.shape, name
        assert _rel(a, b) < 1e-5, (name, _rel(a, b))
        if name not in ("DF", "d_enc5", "d_enc0"):   # masked products: the same zeros
            assert float(((a == 0) != (b == 0)).float().mean()) <= 1e-6, name
    assert float(m1[8]) == 0.0 and float(m0[8]) > 0.0          # slot 8: DF's max (layers only)
    keep = [i for i in range(m0.numel()) if i != 8]
    assert torch.allclose(m1[keep], m0[keep], rtol=1e-5, atol=0), (m1, m0)
    for name, a, b in zip((["pts"] if pts_grad else []) + PARAM_NAMES, grads[True], grads[False]):
        assert _rel(a, b) < 1e-5, (name, _rel(a, b))


def test_net_packer_packs_live_parameters(dev):
    """X3NetPacker: a network's two fused streams at each forward are a packing
    of the live parameters (after a fused-Adam step they equal a fresh packing
    of the updated ones); prepack of two networks in one launch set == each
    packed alone, and is used by their next forwards."""
    from nerfhip import train_mlp
    from nerfhip.train_mlp import (PARAM_NAMES, X3BwdStreamPacker, X3StreamPacker, mlp_params,
                                   prepack)
    m = _model(dev, seed=3, gain=2.5)
    m2 = _model(dev, seed=5, gain=2.0)
    fs0 = train_mlp._streams_for(mlp_params(m), dev)[0].clone()
    opt = torch.optim.Adam(m.parameters(), lr=1e-2, fused=True)
    sum((p * p).sum() for p in m.parameters()).backward()
    opt.step()

    def check(mod, got):
        p = dict(zip(PARAM_NAMES, mlp_params(mod)))
        rs, rh = X3StreamPacker(dev).pack(p)
        rbs, rbh = X3BwdStreamPacker(dev).pack(p)
        fs, fh, bs, bh = got
        assert torch.equal(fs.view(torch.int32), rs.view(torch.int32)) and torch.equal(fh, rh)
        assert torch.equal(bs.view(torch.int32), rbs.view(torch.int32)) and torch.equal(bh, rbh)

    check(m, train_mlp._streams_for(mlp_params(m), dev))
    assert not torch.equal(train_mlp._streams_for(mlp_params(m), dev)[0].view(torch.int32),
                           fs0.view(torch.int32))
    with torch.no_grad():
        for q in list(m.parameters()) + list(m2.parameters()):
            q.mul_(0.5)
    prepack([m, m2])
    nets = [train_mlp._net_for(mlp_params(x), dev)[0] for x in (m, m2)]
    assert all(n.pending for n in nets)
    check(m, train_mlp._streams_for(mlp_params(m), dev))     # prepack's packing, not a new one
    check(m2, train_mlp._streams_for(mlp_params(m2), dev))
    assert not any(n.pending for n in nets)


@pytest.mark.parametrize("n,S", [(1, 1), (37, 64), (300, 192)])
def test_ray_form_equals_point_form(dev, n, S):
    """RayMLPFn (the points o + d z built in the forward kernel, VR:165; the
    backward straight to d z) against NerfMLPFn on the torch-built points
    rays_o + rays_d * z with per-sample directions: raw and every parameter
    gradient bitwise equal (the same kernels on the same float32 points), d z
    equal to torch's autograd of o + d z through the point gradient within one
    rounding of its 3-term sum."""
    from nerfhip.train_mlp import NerfMLPFn, RayMLPFn, PARAM_NAMES, mlp_params
    m = _model(dev)
    g = torch.Generator().manual_seed(3)
    ro = (torch.rand((n, 3), generator=g) * 2.0 - 1.0).to(dev)
    rd = torch.nn.functional.normalize(torch.randn((n, 3), generator=g), dim=1).to(dev)
    z0 = (2.0 + 4.0 * torch.rand((n, S), generator=g)).to(dev)
    d_raw = torch.randn((n, S, 4), generator=torch.Generator().manual_seed(4)).to(dev)

    z1 = z0.clone().requires_grad_(True)
    pts = ro[:, None, :] + rd[:, None, :] * z1[..., None]
    dirs = rd[:, None, :].expand(n, S, 3).reshape(-1, 3)
    ref = NerfMLPFn.apply(pts.reshape(-1, 3), dirs, *mlp_params(m)).reshape(n, S, 4)
    ref_g = torch.autograd.grad(ref, [z1] + mlp_params(m), d_raw)

    z2 = z0.clone().requires_grad_(True)
    out = RayMLPFn.apply(ro, rd, z2, *mlp_params(m))
    got_g = torch.autograd.grad(out, [z2] + mlp_params(m), d_raw)
    assert torch.equal(out.detach(), ref.detach())
    for name, a, b in zip(PARAM_NAMES, got_g[1:], ref_g[1:]):
        assert torch.equal(a, b), name
    dz, dz_ref = got_g[0], ref_g[0]
    assert dz.shape == (n, S)
    assert float((dz - dz_ref).abs().max()) <= 1e-6 * float(dz_ref.abs().max().clamp_min(1e-30))


def test_views_feature_grads_kernel_matches_float64(dev):
    """nerf_views_feature_grads (the views / feature / alpha gradients from the
    merged G tile): dW_views = [Gh W_f^T + s b_f^T, G_enc], dW_f = W_vf^T Gh,
    db_f = W_vf^T s, the alpha row and the bias copies, against float64 torch
    within 1e-6 of each output's scale (row stride of GA > 288)."""
    from nerfhip._lib import call, ptr, stream_of
    g = torch.Generator(device=dev).manual_seed(21)
    ld = 300
    GA = torch.randn((129, ld), device=dev, generator=g)
    ba = torch.randn((129,), device=dev, generator=g)
    Wf = torch.randn((256, 256), device=dev, generator=g) * 0.1
    bf = torch.randn((256,), device=dev, generator=g)
    Wv = torch.randn((128, 283), device=dev, generator=g) * 0.1
    out = {k: torch.full(s, float("nan"), device=dev) for k, s in (
        ("dWv", (128, 283)), ("dWf", (256, 256)), ("dbf", (256,)), ("dWa", (1, 256)),
        ("dba", (1,)), ("dbv", (128,)))}
    call("nerf_views_feature_grads", ptr(GA), ld, ptr(ba), ptr(Wf), ptr(bf), ptr(Wv),
         ptr(out["dWv"]), ptr(out["dWf"]), ptr(out["dbf"]), ptr(out["dWa"]), ptr(out["dba"]),
         ptr(out["dbv"]), None, 0, None, None, None, stream_of(dev))
    d = {k: v.double() for k, v in (("GA", GA), ("ba", ba), ("Wf", Wf), ("bf", bf), ("Wv", Wv))}
    Gh, s = d["GA"][:128, :256], d["ba"][:128]
    ref = {"dWv": torch.cat([Gh @ d["Wf"].t() + s[:, None] * d["bf"][None, :],
                             d["GA"][:128, 256:283]], 1),
           "dWf": d["Wv"][:, :256].t() @ Gh, "dbf": d["Wv"][:, :256].t() @ s,
           "dWa": d["GA"][128:129, :256], "dba": d["ba"][128:129], "dbv": s}
    scale = {"dWv": (Gh.abs() @ d["Wf"].abs().t() + (s[:, None] * d["bf"][None, :]).abs()).max(),
             "dWf": (d["Wv"][:, :256].abs().t() @ Gh.abs()).max(),
             "dbf": (d["Wv"][:, :256].abs().t() @ s.abs()).max()}
    for k, r in ref.items():
        e = float((out[k].double() - r).abs().max())
        assert e <= 1e-6 * float(scale.get(k, 1.0)), (k, e)


def test_views_feature_grads_from_the_shared_tile(dev):
    """nerf_views_feature_grads with GE (the training backward's tile shared by
    the views layer's encoding columns and the rgb head, [d_hv; d sigma; pad;
    d rgb] [enc; HV]^T): the encoding columns of dW_views and the rgb head's
    weight / bias gradients are copied out of it exactly; the rest as without."""
    from nerfhip._lib import call, ptr, stream_of
    g = torch.Generator(device=dev).manual_seed(22)
    GA = torch.randn((129, 256), device=dev, generator=g)
    ba = torch.randn((129,), device=dev, generator=g)
    Wf = torch.randn((256, 256), device=dev, generator=g) * 0.1
    bf = torch.randn((256,), device=dev, generator=g)
    Wv = torch.randn((128, 283), device=dev, generator=g) * 0.1
    ER = torch.randn((147, 170), device=dev, generator=g)
    be = torch.randn((147,), device=dev, generator=g)
    GA288 = torch.cat([GA, torch.cat([ER[:129, :27], torch.zeros((129, 5), device=dev)], 1)], 1)

    def run(with_ge):
        o = {k: torch.full(s, float("nan"), device=dev) for k, s in (
            ("dWv", (128, 283)), ("dWf", (256, 256)), ("dbf", (256,)), ("dWa", (1, 256)),
            ("dba", (1,)), ("dbv", (128,)), ("dWr", (3, 128)), ("dbr", (3,)))}
        src = GA if with_ge else GA288.contiguous()
        tail = ((ptr(ER), ER.stride(0), ptr(be), ptr(o["dWr"]), ptr(o["dbr"])) if with_ge
                else (None, 0, None, None, None))
        call("nerf_views_feature_grads", ptr(src), src.stride(0), ptr(ba), ptr(Wf), ptr(bf),
             ptr(Wv), ptr(o["dWv"]), ptr(o["dWf"]), ptr(o["dbf"]), ptr(o["dWa"]), ptr(o["dba"]),
             ptr(o["dbv"]), *tail, stream_of(dev))
        return o
    a, b = run(True), run(False)
    for k in ("dWv", "dWf", "dbf", "dWa", "dba", "dbv"):
        assert torch.equal(a[k], b[k]), k
    assert torch.equal(a["dWv"][:, 256:], ER[:128, :27])
    assert torch.equal(a["dWr"], ER[144:147, 32:160]) and torch.equal(a["dbr"], be[144:147])
