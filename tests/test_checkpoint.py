"""Checkpoints in the reference's format (net_utils.py:323-379): save, resolve,
prune, load into the torch Network, and pack the loaded weights (CPU)."""
import os

import numpy as np
import torch

from nerfhip import checkpoint as ck
from nerfhip.pack import pack_mlp, pack_mlp_x3
from nerfhip.synthetic import load_into_network, make_params


class _Recorder:
    def __init__(self):
        self.step = 7

    def state_dict(self):
        return {"step": self.step}


def _network():
    from src.config import reset
    from src.models.nerf.network import Network
    reset()
    return Network()


def test_save_resolve_prune_and_load(tmp_path):
    net = _network()
    p = make_params(3, 2.0, 0.5)
    load_into_network(net, p)
    opt = torch.optim.Adam(net.parameters(), lr=5e-4)
    sch = torch.optim.lr_scheduler.ExponentialLR(opt, 0.1)
    d = str(tmp_path / "trained")
    for epoch in range(8):
        ck.save_model(net, opt, sch, _Recorder(), d, epoch)
    nums = sorted(int(f.split(".")[0]) for f in os.listdir(d))
    assert nums == [3, 4, 5, 6, 7]                      # at most 5 numbered kept
    assert ck.resolve(d).endswith("7.pth")
    ck.save_model(net, opt, sch, _Recorder(), d, 8, last=True)
    assert ck.resolve(d).endswith("latest.pth")        # latest wins
    assert ck.resolve(d, epoch=5).endswith("5.pth")
    assert ck.resolve(str(tmp_path / "missing")) is None

    fresh = _network()
    assert ck.load_network(fresh, d) == 9               # next epoch
    for (k, a), b in zip(net.state_dict().items(), fresh.state_dict().values()):
        assert torch.equal(a, b), k
    assert ck.load_network(fresh, d, resume=False) == 0


def test_checkpoint_weights_pack_like_the_generator(tmp_path):
    net = _network()
    p = make_params(4, 2.0, 0.0)
    load_into_network(net, p)
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    sch = torch.optim.lr_scheduler.ExponentialLR(opt, 0.1)
    ck.save_model(net, opt, sch, _Recorder(), str(tmp_path), 0, last=True)
    params = ck.network_params(str(tmp_path))
    assert all(k.startswith(("model.", "model_fine.")) for k in params)
    for prefix in ("model", "model_fine"):
        for fn in (pack_mlp, pack_mlp_x3):
            a, ha = fn(params, prefix)
            b, hb = fn(p, prefix)
            assert np.array_equal(a, b) and np.array_equal(ha, hb)


GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _small_network():
    """The reference Network at width 16 (the width ckpt_ref was written at)."""
    from src.config import cfg, reset
    from src.models.nerf.network import Network
    reset()
    cfg.network.nerf.W = 16
    net = Network()
    reset()
    return net


def test_loads_a_checkpoint_written_by_the_reference():
    """tests/golden/ckpt_ref/ holds the files the reference's own save_model wrote
    (make_ckpt_golden.py): load_network reads them with weights_only=True into the
    Network (latest.pth preferred, next epoch returned, strict key match) and
    network_params hands the same tensors to the packer."""
    d = os.path.join(GOLD, "ckpt_ref")
    ref = np.load(os.path.join(GOLD, "ckpt_ref_state.npz"))
    assert ck.resolve(d).endswith("latest.pth")
    assert ck.resolve(d, epoch=7).endswith("7.pth")
    net = _small_network()
    assert ck.load_network(net, d) == int(ref["epoch"]) + 1
    for k, v in net.state_dict().items():
        assert np.array_equal(v.numpy(), ref["net__" + k]), k
    params = ck.network_params(d, epoch=7)
    assert sorted(params) == sorted(k[5:] for k in ref.files if k.startswith("net__"))
    raw = ck.load_checkpoint(os.path.join(d, "7.pth"))
    assert set(raw) == {"net", "optim", "scheduler", "recorder", "epoch"}
    assert raw["recorder"] == {"step": 1234}


def test_written_checkpoint_has_the_reference_layout(tmp_path):
    """save_model's file has the reference file's structure: the same top-level
    keys, the same net keys, an optimizer state_dict of the same shape."""
    net = _small_network()
    opt = torch.optim.Adam([{"params": [p], "lr": 5e-4, "weight_decay": 0.0, "eps": 1e-8}
                            for p in net.parameters()], 5e-4, weight_decay=0.0, eps=1e-8)
    net.model(torch.rand(4, 90)).sum().backward()
    opt.step()
    sch = torch.optim.lr_scheduler.ExponentialLR(opt, 0.1)
    ck.save_model(net, opt, sch, _Recorder(), str(tmp_path), 7)
    ours = ck.load_checkpoint(str(tmp_path / "7.pth"))
    theirs = ck.load_checkpoint(os.path.join(GOLD, "ckpt_ref", "7.pth"))
    assert set(ours) == set(theirs)
    assert list(ours["net"]) == list(theirs["net"])
    assert set(ours["optim"]) == set(theirs["optim"])
    assert len(ours["optim"]["param_groups"]) == len(theirs["optim"]["param_groups"])
    assert set(ours["optim"]["param_groups"][0]) == set(theirs["optim"]["param_groups"][0])
