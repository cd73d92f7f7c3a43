"""GPU, one-off: the alpha head's gradient with d sigma 2^-30 x d hv, through
the fused forward + backward, with the views tile's d sigma row at its own
FP16 split range (a_split=128, shipped) and at the shared one (a_split=0, round
4): relative error of each gradient against torch FP32 autograd of the
reference module. tests/test_gpu_train_mlp.py::test_tiny_sigma_gradient_keeps_its_split_range
gates the shipped form."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "nerf-rep_for_test_amd"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "oracle")]


def main():
    import test_gpu_train_mlp as t
    from nerfhip import train_mlp
    from nerfhip.train import freq_encode
    from nerfhip.train_mlp import NerfMLPFn, PARAM_NAMES, mlp_params
    dev = torch.device("cuda:0")
    add = train_mlp.WgradBatch.add
    for P in (1024, 1000):
        for split in (True, False):
            train_mlp.WgradBatch.add = (add if split else
                                        lambda self, *a, a_split=0, **k: add(self, *a, **k))
            m = t._model(dev)
            pts, dirs = t._inputs(dev, P)
            d_raw = torch.randn((P, 4), device=dev, generator=torch.Generator(device=dev).manual_seed(3))
            d_raw[:, 3] *= 2.0 ** -30
            d_raw[t._relu_edge_samples(m, pts, dirs)] = 0.0
            x = pts.clone().requires_grad_(True)
            ref = m(torch.cat([freq_encode(x, 10), freq_encode(dirs, 4)], -1))
            rg = torch.autograd.grad(ref, [x] + mlp_params(m), d_raw)
            y = pts.clone().requires_grad_(True)
            out = NerfMLPFn.apply(y, dirs, *mlp_params(m))
            g = torch.autograd.grad(out, [y] + mlp_params(m), d_raw)
            e = {n: t._rel(a, b) for n, a, b in zip(["pts"] + PARAM_NAMES, g, rg)}
            print(f"P={P} own range={split}: alpha_linear.weight {e['alpha_linear.weight']:.3e} "
                  f"bias {e['alpha_linear.bias']:.3e}, max over all {max(e.values()):.3e}", flush=True)
    train_mlp.WgradBatch.add = add


if __name__ == "__main__":
    main()
