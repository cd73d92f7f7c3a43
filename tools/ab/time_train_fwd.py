#!/usr/bin/env python3
"""Time the fused training forward (nerf_mlp_train_forward_x3, 73-slice stream
+ activation / bit stores) against the inference kernel (nerf_mlp_forward_x3,
65 slices, no stores) on the same P samples, HIP events on the launch stream.
Per-slice cost ratio = (t_train / 73) / (t_inf / 65): 1.0 means the stores are
free.

    python tools/ab/time_train_fwd.py [P] [reps]
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))


def main(P=196608, reps=20):
    import torch
    from nerfhip import _lib
    from nerfhip._lib import call, ptr
    from nerfhip.pack import pack_mlp_x3
    from nerfhip.synthetic import make_params
    from nerfhip.train_mlp import _TrainOut, _act, relu_bits_words
    dev = torch.device("cuda:0")
    params = make_params(0, 2.0, 0.1)
    sl_i, hd_i = (torch.from_numpy(a).to(dev) for a in pack_mlp_x3(params))
    sl_t, hd_t = (torch.from_numpy(a).to(dev) for a in pack_mlp_x3(params, fold=False))
    g = torch.Generator(device=dev).manual_seed(0)
    pts = (torch.rand((P, 3), device=dev, generator=g) * 3.0 - 1.5).contiguous()
    dirs = torch.nn.functional.normalize(torch.randn((P, 3), device=dev, generator=g), dim=1)
    zero = torch.zeros(1, device=dev)
    raw = torch.empty((P, 4), device=dev)
    H = [_act(256, P, dev) for _ in range(9)]
    HV = _act(128, P, dev)
    bits = torch.empty((8, relu_bits_words(P, 16)), device=dev, dtype=torch.int16)
    bits_v = torch.empty((relu_bits_words(P, 8),), device=dev, dtype=torch.int16)
    amax = torch.zeros(12, device=dev)
    out = _TrainOut()
    for i in range(8):
        out.act[i] = H[i].data_ptr()
        out.bits[i] = bits[i].data_ptr()
    out.act[8] = H[8].data_ptr()
    out.act[9] = HV.data_ptr()
    E = _act(64, P, dev)
    DV = _act(32, P, dev)
    out.act[10] = E.data_ptr()
    out.act[11] = DV.data_ptr()
    out.bits[8] = bits_v.data_ptr()
    out.amax = amax.data_ptr()
    out.ld = H[0].stride(0)
    st = _lib.stream_of(dev)

    def inf():
        call("nerf_mlp_forward_x3", ptr(sl_i), ptr(hd_i), ptr(pts), ptr(dirs), ptr(zero), 0, P, 1,
             ptr(raw), st)

    def train():
        call("nerf_mlp_train_forward_x3", ptr(sl_t), ptr(hd_t), ptr(pts), ptr(dirs), ptr(zero), P,
             ctypes.addressof(out), ptr(raw), st)

    ts = {"inference (65 slices)": [], "train (73 slices + stores)": []}
    for r in range(reps + 2):
        for name, fn in zip(ts, (inf, train)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts[name].append(e0.elapsed_time(e1))
    med = {k: float(np.median(v)) for k, v in ts.items()}
    for k, v in med.items():
        print(f"{k}: median {v * 1e3:.1f} us")
    a, b = med.values()
    print(f"per-slice cost ratio train/inference: {(b / 73) / (a / 65):.3f}")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
