#!/usr/bin/env python3
"""Per-tile timeline of mlp_x3_kernel from its diagnostic twin
(nerf_mlp_forward_x3_clock): the held shader clock, the median tile length in
shader cycles and the share of a tile spent before its first MFMA (sample
inputs + encoding), over workgroups 0-3's first 32 tiles -- on the bench
frame's coarse pass shape (800 x 800 rays x 64 depths, synthetic weights).

    python tools/ab/trace_x3.py [reps]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))


def main(reps=5):
    import torch
    from nerfhip._lib import call, ptr, stream_of
    from nerfhip.pack import pack_mlp_x3
    from nerfhip.synthetic import make_params
    dev = torch.device("cuda:0")
    sl, hd = (torch.from_numpy(a).to(dev) for a in pack_mlp_x3(make_params(0, 2.0, 0.1)))
    n, S = 640000, 64
    g = torch.Generator(device=dev).manual_seed(0)
    ro = (torch.rand((n, 3), device=dev, generator=g) - 0.5) * 0.2 + torch.tensor([0.0, -4.0, 1.0], device=dev)
    rd = torch.nn.functional.normalize(torch.randn((n, 3), device=dev, generator=g), dim=1)
    z = torch.linspace(2.0, 6.0, S, device=dev)
    raw = torch.empty((n * S, 4), device=dev)
    clk = torch.zeros(4 * 4096, device=dev, dtype=torch.int64)
    trace = torch.zeros(512 * 4, device=dev, dtype=torch.int64)
    for r in range(reps):
        clk.zero_()
        trace.zero_()
        call("nerf_mlp_forward_x3_clock", ptr(sl), ptr(hd), ptr(ro), ptr(rd), ptr(z), 0, n, S,
             ptr(raw), ptr(clk), clk.numel(), ptr(trace), stream_of(dev))
        torch.cuda.synchronize()
        c = clk.view(-1, 4).cpu().numpy().astype(np.float64)
        c = c[c[:, 3] > c[:, 2]]
        ghz = float(np.median((c[:, 1] - c[:, 0]) / (c[:, 3] - c[:, 2]) * 0.1))
        t = trace.view(-1, 4).cpu().numpy().astype(np.float64)
        t = t[(t[:, 2] > t[:, 0]) & (t[:, 1] >= t[:, 0])]
        print(f"run {r}: clock {ghz:.3f} GHz, tile {np.median(t[:, 2] - t[:, 0]):.0f} cycles, "
              f"start share {np.median((t[:, 1] - t[:, 0]) / (t[:, 2] - t[:, 0])):.4f} "
              f"(loads {np.median((t[:, 3] - t[:, 0]) / (t[:, 2] - t[:, 0])):.4f}), "
              f"launch {np.median(c[:, 1] - c[:, 0]) / ghz / 1e3:.1f} us (median workgroup)",
              flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
