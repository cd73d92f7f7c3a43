"""Timing: nerf_x3_chain vs the same layers as separate launches (C3 fine pass size)."""
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "nerf-rep_for_test_amd"))
from nerfhip.train_mlp import _chain, _layer, chain_perm, pack_x3_matrix, relu_bits_words  # noqa: E402

dev = torch.device("cuda:0")
P = 196608
g = torch.Generator(device=dev).manual_seed(0)
for k0, nl in ((8, 2), (8, 3), (2, 5)):
    K0 = 32 * k0
    Ws = [torch.randn((256, K0 if l == 0 else 256), device=dev, generator=g) * 0.06 for l in range(nl)]
    bs = [torch.randn(256, device=dev, generator=g) * 0.1 for _ in range(nl)]
    B = torch.randn((K0, P + 32), device=dev, generator=g)[:, :P]
    perm = chain_perm()
    packs = [pack_x3_matrix(W if l == 0 else W[:, perm]) for l, W in enumerate(Ws)]
    slices = torch.cat([pk for pk, _ in packs])
    Cs = [torch.empty((256, P + 32), device=dev)[:, :P] for _ in range(nl)]
    bits = [torch.empty(relu_bits_words(P, 16), device=dev, dtype=torch.int16) for _ in range(nl)]
    am = [torch.zeros(1, device=dev) for _ in range(nl)]
    nat = [pack_x3_matrix(W) for W in Ws]

    def chain():
        _chain(slices, [sw for _, sw in packs], bs, B, Cs, bits, P, am)

    def seq():
        src = B
        for l in range(nl):
            wp, sw = nat[l]
            _layer(wp, sw, 16, src.shape[0] // 32, src, Cs[l], P, bias=bs[l], relu=True,
                   amax=am[l], bits_out=bits[l])
            src = Cs[l]

    res = {}
    for name, fn in (("chain", chain), ("seq", seq)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / 20
    print(f"k0={k0} layers={nl} P={P}: chain {res['chain'] * 1e3:.1f} us, separate launches "
          f"{res['seq'] * 1e3:.1f} us", flush=True)
