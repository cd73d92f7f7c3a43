"""Round-6 debug: the batched weight gradient on feature-major and T16
operands (train_mlp.WgradBatch) against FP64 matmul, weights and bias sums
separately, per shape, P and layout."""
import sys
import torch

sys.path.insert(0, "nerf-rep_for_test_amd")
from nerfhip.train_mlp import BlockRows, WgradBatch   # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(8)
for P in (1024, 4096):
    for lay in ("fm", "t16", "mixAt", "mixBt"):
        shapes = [(256, 256, None), (129, 256, 128), (256, 63, None), (147, 160, 144), (3, 128, None)]
        wb = WgradBatch(dev)
        ops = []
        for M, N, split in shapes:
            A = torch.randn((M, P), device=dev, generator=g)
            B = torch.relu(torch.randn((N, P), device=dev, generator=g))
            ta = lay in ("t16", "mixAt")
            tb = lay in ("t16", "mixBt")
            Ao = BlockRows.from_dense(A) if ta else A
            Bo = BlockRows.from_dense(B) if tb else B
            if split:
                aa = (A[:split].abs().max().reshape(1), A[split:].abs().max().reshape(1))
                wb.add(Ao, Bo, aa, B.abs().max().reshape(1), with_bias=True, a_split=split)
            else:
                wb.add(Ao, Bo, A.abs().max().reshape(1), B.abs().max().reshape(1), with_bias=True)
            ops.append((A, B))
        for (A, B), (gw, gb) in zip(ops, wb.results()):
            ref = A.double() @ B.double().t()
            sc = (A.double().abs() @ B.double().abs().t()).max().item()
            ew = ((gw.double() - ref).abs() / sc)
            rb = A.double().sum(1)
            eb = (gb.double() - rb).abs().max().item() / A.double().abs().sum(1).max().item()
            bad = (ew > 1e-6).nonzero()
            print(f"P {P} {lay:6s} {tuple(A.shape)[0]:4d}x{B.shape[0]:4d}: w {ew.max().item():.2e} "
                  f"b {eb:.2e} bad {bad.shape[0]} first {bad[:4].tolist()}", flush=True)
