"""GPU tests of the `kilonerf_cuda` op contract (cuda/pybind.cu:13-38) against the
numpy restatements in oracle/kilonerf_ops.py. The reference CUDA extension cannot
be built here (no nvcc/MAGMA), so these restatements of the source text are the
oracle; MAGMA/thrust summation orders are parity-unpinned."""
import numpy as np
import pytest

from oracle import kilonerf_ops as KO

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kn():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import kilonerf_cuda
    return kilonerf_cuda


def cu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_get_rays_d(kn):
    R = np.array([[0.9, -0.1, 0.2], [0.3, 0.8, -0.5], [0.1, 0.4, 0.9]], np.float32)
    out = kn.get_rays_d(17, 23, 11.5, 8.25, 20.0, 19.0, cu(R), 128, 256)
    assert out.shape == (17, 23, 3)
    assert np.array_equal(out.cpu().numpy(), KO.get_rays_d(17, 23, 11.5, 8.25, 20.0, 19.0, R))


@pytest.mark.parametrize("n,L", [(1, 10), (255, 4), (1000, 10), (4097, 3)])
def test_compute_fourier_features(kn, n, L):
    x = np.random.default_rng(n).uniform(-2, 2, n).astype(np.float32)
    f = (2.0 ** np.arange(L)).astype(np.float32)
    out = kn.compute_fourier_features(cu(x), cu(f), 128, 256, "").cpu().numpy()
    ref = KO.compute_fourier_features(x, f)
    assert out.shape == ref.shape
    assert np.abs(out - ref).max() < 2e-6   # accurate sin/cos on both sides (<= 2 ulp)


def test_integrate_two_passes(kn):
    rng = np.random.default_rng(0)
    n, spr = 300, 16
    rs = np.concatenate([rng.random((n * spr, 3)), rng.random((n * spr, 1)) * 30], 1).astype(np.float32)
    dists = rng.uniform(0.01, 0.1, n).astype(np.float32)
    rgb = torch.zeros((n, 3), device="cuda")
    acc = torch.zeros(n, device="cuda")
    T = torch.ones(n, device="cuda")
    mask = torch.ones(n, device="cuda", dtype=torch.bool)
    r_rgb, r_acc = np.zeros((n, 3), np.float32), np.zeros(n, np.float32)
    r_T, r_mask = np.ones(n, np.float32), np.ones(n, bool)
    for initial in (True, False):
        kn.integrate(cu(rs), cu(dists), rgb.data_ptr(), acc, T, mask, n, spr, 0.01, initial, 128, 256, 0)
        KO.integrate(rs, dists, r_rgb, r_acc, r_T, r_mask, n, spr, 0.01, initial)
    assert np.abs(rgb.cpu().numpy() - r_rgb).max() < 1e-6
    assert np.abs(acc.cpu().numpy() - r_acc).max() < 1e-6
    assert np.abs(T.cpu().numpy() - r_T).max() < 1e-6
    assert np.array_equal(mask.cpu().numpy(), r_mask)
    bg = np.array([1.0, 0.5, 0.25], np.float32)
    kn.replace_transparency_by_background_color(rgb.data_ptr(), acc.view(20, 15), cu(bg), 128, 256)
    KO.replace_transparency_by_background_color(r_rgb, r_acc, bg)
    assert np.abs(rgb.cpu().numpy() - r_rgb).max() < 1e-6


def test_replace_transparency_rejects_1d_acc(kn):
    """The reference reads acc.size(1) (integrate.cu:105): a 1-D acc map raises."""
    rgb = torch.zeros((4, 3), device="cuda")
    with pytest.raises(IndexError):
        kn.replace_transparency_by_background_color(rgb.data_ptr(), torch.zeros(4, device="cuda"),
                                                    torch.ones(3, device="cuda"), 1, 1)


def test_gather_scatter(kn):
    rng = np.random.default_rng(1)
    x = rng.integers(-1000, 1000, 5000).astype(np.int32)
    m = rng.integers(0, 5000, 7000).astype(np.int32)
    assert np.array_equal(kn.gather_int32(cu(m), cu(x)).cpu().numpy(), KO.gather_int32(m, x))
    perm = rng.permutation(3001).astype(np.int32)
    v = rng.random((3001, 4)).astype(np.float32)
    out = kn.scatter_int32_float4(cu(perm), cu(v)).cpu().numpy()
    assert np.array_equal(out, KO.scatter_int32_float4(perm, v, np.zeros_like(v)))


@pytest.mark.parametrize("n", [1, 2, 1000, 1024, 70001])
@pytest.mark.parametrize("vbytes", [4, 8])
def test_sort_by_key_int16_stable(kn, n, vbytes):
    rng = np.random.default_rng(n + vbytes)
    keys = rng.integers(-40, 40, n).astype(np.int16)
    keys[: n // 7] = -32768
    vals = np.arange(n, dtype=np.int32 if vbytes == 4 else np.int64)
    k, v = cu(keys), cu(vals)
    (kn.sort_by_key_int16_int32 if vbytes == 4 else kn.sort_by_key_int16_int64)(k, v)
    rk, rv = KO.sort_by_key_int16(keys, vals)
    assert np.array_equal(k.cpu().numpy(), rk)
    assert np.array_equal(v.cpu().numpy(), rv)


def test_global_to_local(kn):
    rng = np.random.default_rng(2)
    bspn = [5, 0, 17, 1, 300]
    nets = len(bspn)
    pts = rng.uniform(-3, 3, (sum(bspn), 3)).astype(np.float32)
    mins = rng.uniform(-3, -1, (nets, 3)).astype(np.float32)
    maxs = rng.uniform(1, 3, (nets, 3)).astype(np.float32)
    p = cu(pts.reshape(-1))
    kn.global_to_local(p, cu(mins), cu(maxs), torch.tensor(bspn), 128, 256)
    assert np.array_equal(p.cpu().numpy(), KO.global_to_local(pts, mins, maxs, bspn))


def _order_bound(terms_abs, n):
    """|any-order float32 sum - the sequential one| <= 2 n u sum|terms| (u = 2^-24)."""
    return 2.0 * n * 2.0 ** -24 * terms_abs + 1e-30


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("out_f,in_f,bspn", [
    (32, 63, [0, 3, 130, 1, 64, 0, 200]),              # MFMA kernel (KiloNeRF first layer)
    (3, 32, [17, 0, 300, 5]),                          # rgb head: one padded column tile
    (64, 120, [65, 1, 129]),                           # largest MFMA shapes, ragged tiles
    (64, 32, [127, 128, 129, 256, 0, 300]),            # output tile wider than the X tile
                                                       # (staged in the X region), 128-row edges
    (20, 130, [40, 0, 7])])                            # beyond the LDS budget: fallback kernel
def test_multimatmul_grouped(kn, mode, out_f, in_f, bspn):
    """multimatmul.cu:244-361 vs the sequential restatement; MAGMA's own
    accumulation order is unknown, so the bound is the summation-order bound."""
    rng = np.random.default_rng(mode + in_f)
    nets = len(bspn)
    X = rng.normal(size=(sum(bspn), in_f)).astype(np.float32)
    W = rng.normal(size=(nets * out_f * in_f,)).astype(np.float32)
    b = rng.normal(size=(nets, out_f)).astype(np.float32)
    h = kn.init_multimatmul_magma_grouped(nets, out_f, in_f, [64, 8])
    fn = [kn.multimatmul_magma_grouped_static, kn.multimatmul_magma_grouped_static_without_bias,
          kn.multimatmul_magma_grouped_static_without_bias_transposed_weights][mode]
    out = fn(cu(b), cu(X), cu(W), out_f, in_f, torch.tensor(bspn), 128, 256, [64, 8], h)
    kn.deinit_multimatmul_magma_grouped(h)
    ref = KO.grouped_gemm(mode, b, X, W, out_f, in_f, bspn)
    scale = KO.grouped_gemm(mode, np.abs(b), np.abs(X), np.abs(W), out_f, in_f, bspn)
    got = out.cpu().numpy()
    assert got.shape == ref.shape and np.isfinite(got).all()
    assert (np.abs(got.astype(np.float64) - ref) <= _order_bound(scale, in_f + 1)).all()
    with pytest.raises(RuntimeError):
        kn.deinit_multimatmul_magma_grouped(h)


@pytest.mark.parametrize("ac,bc,bspn", [(32, 7, [4, 0, 33, 100]), (32, 63, [1, 517, 0, 64]),
                                        (3, 64, [2000, 9]), (64, 64, [31, 257, 1100]),
                                        (65, 7, [30, 3])])
def test_row_sum_and_A_transposed(kn, ac, bc, bspn):
    """multimatmul.cu:560-623 (row sums and A^T B per network) within the
    summation-order bound; (64, 64) is the largest MFMA shape (128 KiB of wave
    partials in LDS); (65, 7) exceeds the MFMA tile budget (fallback)."""
    rng = np.random.default_rng(ac * bc)
    M = rng.normal(size=(sum(bspn), 33)).astype(np.float32)
    out = kn.multi_row_sum_reduction(cu(M), torch.tensor(bspn)).cpu().numpy()
    ref = KO.multi_row_sum_reduction(M, bspn)
    scale = KO.multi_row_sum_reduction(np.abs(M), bspn)
    assert (np.abs(out.astype(np.float64) - ref) <= _order_bound(scale, max(bspn))).all()
    A = rng.normal(size=(sum(bspn), ac)).astype(np.float32)
    B = rng.normal(size=(sum(bspn), bc)).astype(np.float32)
    out = kn.multimatmul_A_transposed(cu(A), cu(B), torch.tensor(bspn)).cpu().numpy()
    ref = KO.multimatmul_A_transposed(A, B, bspn)
    scale = KO.multimatmul_A_transposed(np.abs(A), np.abs(B), bspn)
    assert out.shape == ref.shape
    assert (np.abs(out.astype(np.float64) - ref) <= _order_bound(scale, max(bspn))).all()
    assert (out[np.asarray(bspn) == 0] == 0).all()


def test_query_indices_two_passes(kn):
    rng = np.random.default_rng(5)
    n, res = 200, 16
    grid = np.where(rng.random(res ** 3) < 0.3, rng.integers(0, 50, res ** 3), -1).astype(np.int16)
    origin = np.array([0.1, -0.2, 2.5], np.float32)
    dirs = rng.normal(size=(n, 3)).astype(np.float32)
    dirs[:, 2] = -np.abs(dirs[:, 2]) - 0.5
    vsize = np.full(3, 4.0 / res, np.float32)
    gmin, gmax = np.full(3, -2.0, np.float32), np.full(3, 2.0, np.float32)
    strides = np.array([res * res, res, 1], np.int32)
    act = torch.ones(n, dtype=torch.bool, device="cuda")
    dep = torch.zeros(n, dtype=torch.int16, device="cuda")
    r_act, r_dep = np.ones(n, bool), np.zeros(n, np.int16)
    for initial in (True, False):
        qi, nets = kn.generate_query_indices_on_ray(cu(origin), cu(dirs), cu(grid), act, dep, cu(vsize),
                                                    cu(gmin), cu(gmax), cu(strides), 0.05, 12, 120,
                                                    0.5, initial, 128, 256, 0)
        rq, rn = KO.generate_query_indices_on_ray(origin, dirs, grid, r_act, r_dep, vsize, gmin,
                                                  gmax, strides, 0.05, 12, 120, 0.5, initial)
        nets = nets.cpu().numpy()
        assert np.array_equal(nets, rn)
        m = rn != -1
        assert np.array_equal(qi.cpu().numpy()[m], rq[m])
        assert np.array_equal(act.cpu().numpy(), r_act)
        assert np.array_equal(dep.cpu().numpy()[r_act], r_dep[r_act])


def test_network_eval_query_index(kn):
    rng = np.random.default_rng(6)
    nets, psize = 5, KO.kilonerf_param_size(32)
    params = (rng.normal(size=nets * psize) * 0.2).astype(np.float32)
    mins = rng.uniform(-2, -1, (nets, 3)).astype(np.float32)
    maxs = rng.uniform(1, 2, (nets, 3)).astype(np.float32)
    H, W, maxd = 20, 30, 64
    counts = [7, 0, 100, 1, 33]
    starts = np.cumsum([0] + counts[:-1]).astype(np.int32)
    ends = (starts + np.array(counts)).astype(np.int32)
    q = rng.integers(0, H * W * maxd, int(sum(counts))).astype(np.int32)
    origin = np.array([0.0, 0.2, 3.0], np.float32)
    c2w = np.eye(3, dtype=np.float32)
    out = kn.network_eval_query_index(cu(q), cu(params), cu(mins), cu(maxs), cu(starts), cu(ends),
                                      cu(origin), cu(c2w), nets, 32, H, W, 15.0, 10.0, 25.0, 25.0,
                                      maxd, 0.5, 0.05, nets, 256, 0).cpu().numpy()
    ref = KO.network_eval_query_index(q, params, mins, maxs, starts, ends, origin, c2w, W, 15.0,
                                      10.0, 25.0, 25.0, maxd, 0.5, 0.05)
    assert np.abs(out - ref).max() < 1e-5
    with pytest.raises(RuntimeError):
        kn.network_eval_query_index(cu(q), cu(params), cu(mins), cu(maxs), cu(starts), cu(ends),
                                    cu(origin), cu(c2w), nets, 64, H, W, 15.0, 10.0, 25.0, 25.0,
                                    maxd, 0.5, 0.05, nets, 256, 0)


def test_stream_pool_and_magma_init(kn):
    kn.init_stream_pool(4)
    kn.init_magma()
    kn.destroy_stream_pool()
    with pytest.raises(RuntimeError):
        kn.render_to_screen(None, None, 4, 4)
