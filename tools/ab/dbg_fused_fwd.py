#!/usr/bin/env python3
"""Debug: the fused training forward against the layer launches (saved
tensors, ReLU bits, gradients) on one input set; prints where they differ."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main(P=3000):
    from nerfhip import train_mlp
    from nerfhip.synthetic import make_params
    from nerfhip.train import freq_encode
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
    x = pts.clone().requires_grad_(True)
    ref = m(torch.cat([freq_encode(x, 10), freq_encode(dirs, 4)], -1))
    ref_g = torch.autograd.grad(ref, [x] + mlp_params(m), d_raw)
    res = {}
    for fused in (False, True):
        train_mlp.FUSED_FORWARD = fused
        y = pts.clone().requires_grad_(True)
        out = NerfMLPFn.apply(y, dirs, *mlp_params(m))
        saved = [t.clone() for t in out.grad_fn.saved_tensors[:14]]
        grads = torch.autograd.grad(out, [y] + mlp_params(m), d_raw)
        res[fused] = (out.detach(), saved, grads)
    names = ["pts", "E", "h0", "h1", "h2", "h3", "h5", "h6", "h7", "V", "HV", "amax", "bits", "bits_v"]
    for i, n in enumerate(names):
        a, b = res[True][1][i], res[False][1][i]
        if a.dtype == torch.int16:
            d = (a != b)
            print(f"{n}: words differing {int(d.sum())} of {d.numel()}")
            if d.any():
                idx = torch.nonzero(d.reshape(-1))[:8].reshape(-1).tolist()
                print("   first", idx)
        else:
            rel = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
            print(f"{n}: rel {rel:.3e}")
            if rel > 1e-6 and a.dim() == 2:
                e = (a - b).abs()
                r, c = divmod(int(e.argmax()), e.shape[1])
                print(f"   worst at row {r} col {c}: {a[r, c].item()} vs {b[r, c].item()}")
    # ReLU decisions per valid sample: (h > 0) of each layer, fused vs layers
    Hs = {f: [res[f][1][i] for i in (2, 3, 4, 5)] + [res[f][1][1][64:320]] +
          [res[f][1][i] for i in (6, 7, 8)] for f in (False, True)}
    for L in range(8):
        a, b = Hs[True][L] > 0, Hs[False][L] > 0
        d = a != b
        if d.any():
            rows, cols = torch.nonzero(d, as_tuple=True)
            vals = torch.maximum(Hs[True][L][rows, cols].abs(), Hs[False][L][rows, cols].abs())
            print(f"h{L}: {int(d.sum())} ReLU flips at samples {sorted(set(cols.tolist()))[:10]}, "
                  f"max |h| there {float(vals.max()):.3e} (layer max {float(Hs[False][L].abs().max()):.3e})")
    for fused in (False, True):
        gp = res[fused][2][0]
        e = (gp - ref_g[0]).abs().max(1).values
        worst = torch.topk(e, 5)
        print(f"fused={fused}: pts grad rel {float(e.max() / ref_g[0].abs().max()):.3e}; worst samples",
              worst.indices.tolist(), [round(v, 4) for v in worst.values.tolist()])
    for k, (a, b) in enumerate(zip(res[True][2][1:], ref_g[1:])):
        rel = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        if rel > 1e-5:
            print("param grad", PARAM_NAMES[k], f"{rel:.3e}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3000)
