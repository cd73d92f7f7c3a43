"""HBM roofline of the byte-moving kernels (GPU): algorithmic bytes / HIP-event time.

    python tools/hbm_bench.py [out.json] [only]   # only: "composite" or "sample_fine"

Each case: inputs resident in HBM, 3 warm-up launches, then the median of 10
launches timed with events on torch's current stream (the stream the kernels
are enqueued on). Bytes are the algorithmic minimum each kernel must move
(documented per case); peak 8 TB/s (MI355X_MICROARCH.md).
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))

import kilonerf_cuda as kc  # noqa: E402
from nerfhip import _lib  # noqa: E402
from nerfhip._lib import call, ptr  # noqa: E402

PEAK = 8.0e12


def timed(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return float(np.median(ts))


def main():
    dev = torch.device("cuda:0")
    st = _lib.stream_of(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    res = []

    def report(name, nbytes, t, note):
        r = {"kernel": name, "bytes": int(nbytes), "ms": t * 1e3, "GB/s": nbytes / t / 1e9,
             "frac_hbm": nbytes / t / PEAK, "bytes_def": note}
        res.append(r)
        print(json.dumps(r), flush=True)

    n = 640000
    rd = torch.nn.functional.normalize(torch.randn(n, 3, device=dev, generator=g), dim=1)
    only = sys.argv[2] if len(sys.argv) > 2 else None
    for S, shared, wts in ((64, True, True), (192, False, False)) if only in (None, "composite") else ():
        raw = torch.randn(n * S, 4, device=dev, generator=g)
        z = (torch.sort(torch.rand(n, S, device=dev, generator=g) * 4 + 2, 1)[0]
             if not shared else torch.linspace(2, 6, S, device=dev))
        outs = [torch.empty(n, 3, device=dev)] + [torch.empty(n, device=dev) for _ in range(3)]
        w = torch.empty(n, S, device=dev) if wts else None

        def comp():
            call("nerf_composite", ptr(raw), ptr(z), 0 if shared else S, ptr(rd), n, S, 1,
                 *[ptr(o) for o in outs], ptr(w), st)
        t = timed(comp)
        nb = n * S * 16 + (0 if shared else n * S * 4) + n * 12 + n * 24 + (n * S * 4 if wts else 0)
        report(f"composite S={S}", nb, t,
               "raw 16 B/sample + z 4 B/sample (per-ray rows) + rays_d 12 B + maps 24 B/ray"
               + (" + weights 4 B/sample" if wts else ""))

    S, NI = 64, 128
    zc = torch.linspace(2, 6, S, device=dev)
    wc = torch.rand(n, S, device=dev, generator=g) ** 4
    u = torch.linspace(0, 1, NI, device=dev)
    zall = torch.empty(n, S + NI, device=dev)
    t = timed(lambda: call("nerf_sample_fine", ptr(zc), 0, ptr(wc), ptr(u), 0, n, S, NI,
                           ptr(zall), st))
    report("sample_fine S=64 NI=128", n * S * 4 + n * (S + NI) * 4, t,
           "coarse weights 4 B/sample in + merged depths 4 B/sample out (shared z row, u)")
    if only is not None:
        for _ in range(20):   # a longer run for PMC passes
            call("nerf_sample_fine", ptr(zc), 0, ptr(wc), ptr(u), 0, n, S, NI, ptr(zall), st)
        torch.cuda.synchronize()
        return

    ro = torch.zeros(n, 3, device=dev)
    cam = torch.eye(4, device=dev).reshape(-1)
    cam = torch.cat([cam, torch.tensor([1111., 0, 400, 0, 1111., 400, 0, 0, 1], device=dev)])
    rdo = torch.empty(n, 3, device=dev)
    t = timed(lambda: call("nerf_rays", ptr(cam), 800, 800, 0, n, ptr(ro), ptr(rdo), st))
    report("rays", n * 24, t, "rays_o + rays_d 24 B/ray out")

    nf = 40_960_000 * 3 // 8                    # 1/8 of a frame's coarse xyz scalars
    x = torch.rand(nf, device=dev, generator=g)
    freqs = 2.0 ** torch.arange(10, device=dev, dtype=torch.float32)
    t = timed(lambda: kc.compute_fourier_features(x, freqs, 0, 0, "v2"))
    report("kn_compute_fourier_features L=10", nf * 4 * (1 + 21), t,
           "4 B in + 21 x 4 B out per scalar (88 B/scalar, SURVEY 8d)")

    spr = 64
    nr = 1 << 20
    rs = torch.rand(nr * spr, 4, device=dev, generator=g)
    dists = torch.full((nr,), 0.01, device=dev)
    rgbm = torch.zeros(nr, 3, device=dev)
    accm = torch.zeros(nr, device=dev)
    T = torch.ones(nr, device=dev)
    mask = torch.ones(nr, device=dev, dtype=torch.bool)

    def integ():
        kc.integrate(rs, dists, rgbm.data_ptr(), accm, T, mask, nr, spr, 0.0, True, 0, 0, 0)
    t = timed(integ)
    report("kn_integrate spr=64", nr * (spr * 16 + 4 + 12 + 4 + 4 + 1), t,
           "rgb_sigma 16 B/sample + dist 4 B + rgb 12 B + acc 4 B + T 4 B + mask 1 B per ray")

    ng = 1 << 24
    mp_ = torch.randperm(ng, device=dev, generator=g).to(torch.int32)
    src = torch.randint(0, 1 << 30, (ng,), device=dev, generator=g, dtype=torch.int32)
    t = timed(lambda: kc.gather_int32(mp_, src))
    report("kn_gather_int32 (random map)", ng * 12, t, "map 4 + in 4 + out 4 B/element")
    src4 = torch.rand(ng, 4, device=dev, generator=g)
    t = timed(lambda: kc.scatter_int32_float4(mp_, src4))
    report("kn_scatter_int32_float4 (random map)", ng * 36, t, "map 4 + in 16 + out 16 B/element")
    del mp_, src, src4

    # KiloNeRF grouped GEMMs (multimatmul.cu): 4096 networks, ragged 0..511 rows
    nets, hd, inf = 4096, 32, 63
    bspn = torch.randint(0, 512, (nets,), generator=torch.Generator().manual_seed(1))
    rows = int(bspn.sum())
    X = torch.randn(rows, inf, device=dev, generator=g)
    Wg = torch.randn(nets * hd * inf, device=dev, generator=g) * 0.1
    bg = torch.randn(nets, hd, device=dev, generator=g)
    h = kc.init_multimatmul_magma_grouped(nets, hd, inf, [])
    t = timed(lambda: kc.multimatmul_magma_grouped_static(bg, X, Wg, hd, inf, bspn, 128, 256, [], h))
    kc.deinit_multimatmul_magma_grouped(h)
    report(f"kn_multimatmul_grouped {nets} nets {inf}->{hd} ({rows} rows)",
           rows * (inf + hd) * 4 + nets * hd * (inf + 1) * 4, t,
           "X 4 B/in + out 4 B/out per row + W and bias once (FP32 MFMA kernel; "
           f"{2 * rows * inf * hd / t / 1e12:.2f} TFLOP/s)")
    Bm = torch.randn(rows, inf, device=dev, generator=g)
    Am = torch.randn(rows, hd, device=dev, generator=g)
    t = timed(lambda: kc.multimatmul_A_transposed(Am, Bm, bspn))
    report(f"kn_multimatmul_A_transposed {nets} nets {hd}x{inf}", rows * (inf + hd) * 4
           + nets * hd * inf * 4, t, "A, B 4 B per element once + out")
    t = timed(lambda: kc.multi_row_sum_reduction(Am, bspn))
    report(f"kn_multi_row_sum_reduction {nets} nets x{hd}", rows * hd * 4 + nets * hd * 4, t,
           "M 4 B per element once + out")

    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump({"peak_Bps": PEAK, "device": torch.cuda.get_device_name(0), "cases": res},
                      f, indent=1)


if __name__ == "__main__":
    main()
