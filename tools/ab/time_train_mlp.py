#!/usr/bin/env python3
"""Time the training MLP (nerfhip.train_mlp.NerfMLPFn) forward and backward on
P samples with the fused kernels on / off (NERF_TRAIN_FUSED_FORWARD /
_BACKWARD as module switches), HIP events on the launch stream around each
phase, medians over reps. The backward includes the batched weight gradients.

    python tools/ab/time_train_mlp.py [P] [reps]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))
sys.path.insert(0, REPO)


def main(P=196608, reps=20):
    import torch
    from nerfhip import train_mlp
    from nerfhip.synthetic import make_params
    from nerfhip.train_mlp import NerfMLPFn, mlp_params
    from src.models.nerf.network import NeRF
    dev = torch.device("cuda:0")
    params = make_params(0, 2.0, 0.1)
    m = NeRF().to(dev)
    with torch.no_grad():
        for k, p in m.named_parameters():
            p.copy_(torch.as_tensor(np.asarray(params["model." + k])))
    g = torch.Generator(device=dev).manual_seed(0)
    pts = (torch.rand((P, 3), device=dev, generator=g) * 3.0 - 1.5).requires_grad_(True)
    dirs = torch.nn.functional.normalize(torch.randn((P, 3), device=dev, generator=g), dim=1)
    d_raw = torch.randn((P, 4), device=dev, generator=g)
    ws = mlp_params(m)
    for ff, fb in ((False, False), (True, False), (True, True)):
        train_mlp.FUSED_FORWARD, train_mlp.FUSED_BACKWARD = ff, fb
        tf, tb = [], []
        for r in range(reps + 3):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
            out = NerfMLPFn.apply(pts, dirs, *ws)
            ev[1].record()
            torch.autograd.grad(out, [pts] + ws, d_raw)
            ev[2].record()
            torch.cuda.synchronize()
            if r >= 3:
                tf.append(ev[0].elapsed_time(ev[1]))
                tb.append(ev[1].elapsed_time(ev[2]))
        print(f"fused forward={ff!s:5} backward={fb!s:5}: forward {np.median(tf) * 1e3:8.1f} us  "
              f"backward {np.median(tb) * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
