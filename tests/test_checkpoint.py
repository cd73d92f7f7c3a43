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


def test_training_checkpoint_loads_into_reference_optimizer_and_scheduler(tmp_path):
    """tools/train_lego.py's resume file: the trainer's single-group Adam state
    re-laid out as the reference's make_optimizer builds it (one group per
    parameter in named_parameters() order, optimizer.py:8-28) loads with
    optim.load_state_dict, the ExponentialLR state with scheduler.load_state_dict
    (lr_scheduler.py:68-79), and the round trip back gives the trainer's state;
    the model dir holds only files the reference's listing parses."""
    import torch
    from nerfhip.checkpoint import (exponential_lr_state, reference_optim_state, save_model,
                                    single_group_optim_state)
    from src.models.nerf.network import Network
    torch.manual_seed(0)
    net = Network()
    order = [n for n, _ in net.named_parameters()]
    names = order[::-1]                                  # the trainer's own order differs
    params = dict(net.named_parameters())
    opt = torch.optim.Adam([params[n] for n in names], lr=5e-4, eps=1e-8)
    for p in net.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    ref_sd = reference_optim_state(opt, names, order)
    # the reference's make_optimizer over the same network
    ref_opt = torch.optim.Adam([{"params": [p], "lr": 5e-4, "weight_decay": 0.0, "eps": 1e-8}
                                for p in net.parameters()], 5e-4, weight_decay=0.0, eps=1e-8)
    ref_opt.load_state_dict(ref_sd)
    for name, p in net.named_parameters():
        a, b = ref_opt.state[p], opt.state[p]
        assert torch.equal(a["exp_avg"], b["exp_avg"]) and torch.equal(a["exp_avg_sq"], b["exp_avg_sq"])
    back = torch.optim.Adam([params[n] for n in names], lr=5e-4, eps=1e-8)
    back.load_state_dict(single_group_optim_state(ref_opt.state_dict(), names, order))
    for p in net.parameters():
        assert torch.equal(back.state[p]["exp_avg"], opt.state[p]["exp_avg"])

    class ExponentialLR(torch.optim.lr_scheduler.LRScheduler):   # lr_scheduler.py:68-79
        def __init__(self, optimizer, decay_epochs, gamma=0.1, last_epoch=-1):
            self.decay_epochs, self.gamma = decay_epochs, gamma
            super().__init__(optimizer, last_epoch)

        def get_lr(self):
            return [b * self.gamma ** (self.last_epoch / self.decay_epochs) for b in self.base_lrs]
    sched = ExponentialLR(ref_opt, decay_epochs=500, gamma=0.1)
    st = exponential_lr_state(5e-4, 0.1, 1000.0, 250, len(order))
    sched.load_state_dict(st)
    assert sched.last_epoch == 250 and abs(sched.get_lr()[0] - 5e-4 * 0.1 ** 0.25) < 1e-12

    class _S:
        def __init__(self, d):
            self.state_dict = lambda: d
    model_dir = tmp_path / "model"
    save_model(_S(net.state_dict()), _S(ref_sd), _S(st), _S({"step": 250}), str(model_dir), 250,
               last=True)
    save_model(_S(net.state_dict()), _S(ref_sd), _S(st), _S({"step": 250}), str(model_dir), 250)
    # net_utils.py:295-297: int(pth.split('.')[0]) for every file but latest.pth
    assert [int(f.split(".")[0]) for f in os.listdir(model_dir) if f != "latest.pth"] == [250]
    ck = torch.load(model_dir / "latest.pth", weights_only=True)
    assert set(ck) == {"net", "optim", "scheduler", "recorder", "epoch"}
