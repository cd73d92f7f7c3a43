"""CPU: the x3 fragment packing of the training kernels (nerfhip/train_mlp.py)."""
import numpy as np
import torch


def test_pack_x3_matrix_layout_and_split():
    from nerfhip.train_mlp import pack_x3_matrix
    g = torch.Generator().manual_seed(0)
    M, K = 64, 96
    W = torch.randn((M, K), generator=g) * 0.37
    packed, sw = pack_x3_matrix(W)
    sw = int(sw.item())
    assert 2.0 ** 11 <= W.abs().max().item() * 2.0 ** sw < 2.0 ** 12
    h = packed.view(torch.float16).reshape(K // 32, M // 16, 2, 64, 8).double()
    Wr = np.zeros((M, K))
    for q in range(K // 32):
        for t in range(M // 16):
            for lane in range(64):
                r, gq = lane & 15, lane >> 4
                v = (h[q, t, 0, lane] + h[q, t, 1, lane]).numpy()
                Wr[16 * t + r, 32 * q + 8 * gq: 32 * q + 8 * gq + 8] = v
    Wr *= 2.0 ** -sw
    err = np.abs(Wr - W.double().numpy()).max() / W.abs().max().item()
    assert err < 2.0 ** -21, err
