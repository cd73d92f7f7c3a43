#!/usr/bin/env python3
"""A/B timing of nerf_mlp_forward_x3 from two builds of libnerfhip.so in ONE
process (the box-to-box spread of MI355X clocks is ~4 %, larger than most
schedule changes): the launches alternate A, B, A, B ... on the same inputs
(lego-like samples: 160 000 rays x 64 depths, synthetic weights), HIP events on
the launch stream; outputs compared bitwise.

    python tools/ab/ab_x3.py <libA.so> <libB.so> [--reps 20]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rays", type=int, default=160000)
    ap.add_argument("--S", type=int, default=64)
    args = ap.parse_args()
    import torch
    from nerfhip.pack import pack_mlp_x3
    from nerfhip.synthetic import make_params
    dev = torch.device("cuda:0")
    libs = []
    for path in args.libs:
        h = C.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
        f = h.nerf_mlp_forward_x3
        f.restype = C.c_int
        f.argtypes = [C.c_void_p] * 5 + [C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_void_p]
        libs.append(f)
    sl, hd = pack_mlp_x3(make_params(0, 2.0, 0.0))
    sl, hd = torch.from_numpy(sl).to(dev), torch.from_numpy(hd).to(dev)
    n, S = args.rays, args.S
    g = torch.Generator(device=dev).manual_seed(0)
    ro = (torch.rand((n, 3), device=dev, generator=g) - 0.5) * 0.2 + torch.tensor([0.0, -4.0, 1.0], device=dev)
    rd = torch.nn.functional.normalize(torch.randn((n, 3), device=dev, generator=g), dim=1)
    z = torch.linspace(2.0, 6.0, S, device=dev)
    outs = [torch.empty((n * S, 4), device=dev) for _ in libs]
    st = torch.cuda.current_stream().cuda_stream
    times = [[] for _ in libs]
    for rep in range(args.reps + 2):
        for k, f in enumerate(libs):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = f(sl.data_ptr(), hd.data_ptr(), ro.data_ptr(), rd.data_ptr(), z.data_ptr(), 0,
                   n, S, outs[k].data_ptr(), st)
            e1.record()
            assert rc == 0, rc
            torch.cuda.synchronize()
            if rep >= 2:
                times[k].append(e0.elapsed_time(e1))
    same = torch.equal(outs[0], outs[1])
    for path, t in zip(args.libs, times):
        t = np.array(t)
        print(f"{path}: median {np.median(t):.3f} ms  mean {t.mean():.3f}  min {t.min():.3f}")
    print(f"B/A median: {np.median(times[1]) / np.median(times[0]):.4f}; outputs bitwise equal: {same}")


if __name__ == "__main__":
    main()
