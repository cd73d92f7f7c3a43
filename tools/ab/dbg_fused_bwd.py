#!/usr/bin/env python3
"""Debug: the fused training backward (nerf_mlp_train_backward_x3) against the
layer launches after one forward; prints, per output (d hv, DF, D0..D7,
d_enc), the relative error and where the worst rows / samples are."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))


def main(P=1000):
    from nerfhip import train_mlp
    from nerfhip.synthetic import make_params
    from nerfhip.train_mlp import NerfMLPFn, PARAM_NAMES, mlp_params
    from src.models.nerf.network import NeRF
    dev = torch.device("cuda:0")
    params = make_params(0, 2.0, 0.1)
    m = NeRF().to(dev)
    with torch.no_grad():
        for k, p in m.named_parameters():
            p.copy_(torch.as_tensor(np.asarray(params["model." + k])))
    g = torch.Generator().manual_seed(1)
    pts = (torch.rand((P, 3), generator=g) * 3.0 - 1.5).to(dev)
    dirs = torch.nn.functional.normalize(torch.randn((P, 3), generator=g), dim=1).to(dev)
    d_raw = torch.randn((P, 4), device=dev, generator=torch.Generator(device=dev).manual_seed(2))
    rec = {}
    for key, attr, di in ((True, "_backward_fused", 4), (False, "_backward_layers", 5)):
        fn = getattr(NerfMLPFn, attr)

        def w(*a, fn=fn, key=key, di=di):
            out = fn(*a)
            torch.cuda.synchronize()
            rows = [out[0], out[1], *out[2]] + (list(out[3]) if out[3] is not None else [])
            rec[key] = ([None if t is None else t.clone() for t in rows], a[di].clone())
            return out
        setattr(NerfMLPFn, attr, staticmethod(w))
    grads = {}
    for fused in (False, True):
        train_mlp.FUSED_BACKWARD = fused
        y = pts.clone().requires_grad_(True)
        out = NerfMLPFn.apply(y, dirs, *mlp_params(m))
        grads[fused] = torch.autograd.grad(out, [y] + mlp_params(m), d_raw)
        torch.cuda.synchronize()
    names = ["d_hv", "DF"] + [f"D{i}" for i in range(8)] + ["d_enc5", "d_enc0"]
    for name, a, b in zip(names, rec[True][0], rec[False][0]):
        if a is None:   # DF: the fused kernel folds the feature layer away
            continue
        e = (a - b).abs()
        rel = float(e.max() / b.abs().max().clamp_min(1e-30))
        bad = torch.isnan(a).sum().item()
        print(f"{name}: shape {tuple(a.shape)} rel {rel:.3e} nan {bad} "
              f"max|a| {float(a.abs().nan_to_num().max()):.3e} max|b| {float(b.abs().max()):.3e}")
        if rel > 1e-5 or bad:
            rows = (e.nan_to_num(1e30).amax(1) > 1e-5 * float(b.abs().max())).nonzero().reshape(-1)
            cols = (e.nan_to_num(1e30).amax(0) > 1e-5 * float(b.abs().max())).nonzero().reshape(-1)
            print(f"   bad rows {rows[:20].tolist()} ({rows.numel()}), bad samples "
                  f"{cols[:20].tolist()} ({cols.numel()})")
            r, c = divmod(int(e.nan_to_num(1e30).argmax()), e.shape[1])
            print(f"   worst [{r},{c}]: {a[r, c].item()} vs {b[r, c].item()}")
    print("dmax fused ", rec[True][1].tolist())
    print("dmax layers", rec[False][1].tolist())
    for name, a, b in zip(["pts"] + PARAM_NAMES, grads[True], grads[False]):
        rel = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        if not rel < 1e-5:
            print("grad", name, f"{rel:.3e}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1000)
