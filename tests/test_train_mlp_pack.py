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


def test_side_wgrad_scope_keys_and_restore():
    """side_wgrad_scope (the trainer's side-stream weight gradients): keyed by
    each network's first weight, nested scopes restore the outer one, and the
    default scope (outside) is empty, so no backward outside the trainer uses a
    side stream. The backward-side plan (X3BwdStreamPacker) puts the fold's
    Wc^T first and leaves scale slot 1 (the unfolded feature layer's) unused:
    64 slices with the encoding products."""
    from nerfhip import train_mlp
    from nerfhip.train_mlp import PARAM_NAMES, X3BwdStreamPacker, side_wgrad_scope
    from src.models.nerf.network import NeRF
    a, b = NeRF(), NeRF()
    assert not train_mlp._SIDE_SCOPE[0]
    with side_wgrad_scope([a]):
        assert train_mlp._SIDE_SCOPE[0] == {a.pts_linears[0].weight.data_ptr()}
        with side_wgrad_scope([b.pts_linears[0].weight, a]):
            assert len(train_mlp._SIDE_SCOPE[0]) == 2
        assert train_mlp._SIDE_SCOPE[0] == {a.pts_linears[0].weight.data_ptr()}
    assert not train_mlp._SIDE_SCOPE[0]
    assert PARAM_NAMES[0] == "pts_linears.0.weight"
    plan, nsl = X3BwdStreamPacker.plan()
    assert nsl == 64 and plan[0][0] == "fold" and plan[0][3] == 0
    assert sorted(j for *_, j in plan) == [0, 2, 3, 4, 5, 6, 7, 8, 9, 10]
    assert plan[1][3] == 4   # W_7^T right after the 4 slices of Wc^T
