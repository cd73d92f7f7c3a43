"""Capture a checkpoint written by the reference's own save_model (survey container).

Imports the reference's ``save_model`` (src/utils/net_utils.py:323-343),
``make_optimizer`` (src/train/optimizer.py), ``make_lr_scheduler``
(src/train/scheduler.py) and ``Recorder`` (src/train/recorder.py) from
/root/reference with empty stand-ins for modules this image lacks and the
checkpoint does not involve (``termcolor.colored`` -> identity,
``tensorboardX.SummaryWriter`` -> no-op, ``imageio``/``cv2``/``imgaug``/
``plyfile``, imported by data_utils.py through src/train/__init__), builds the
reference ``Network`` at width 16 (same parameter names and nesting as the lego
8x256 network, a 160 KB file instead of 14 MB), takes one Adam step so the
optimizer state is populated, steps the scheduler, and lets ``save_model`` write
``<epoch>.pth`` and ``latest.pth``. Stores:

  tests/golden/ckpt_ref/7.pth, tests/golden/ckpt_ref/latest.pth  (the reference's files)
  tests/golden/ckpt_ref_state.npz   (net state_dict values + epoch, for comparison)

    python tests/golden/make_ckpt_golden.py
"""
from __future__ import annotations

import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

EPOCH = 7


def _stubs():
    tc = types.ModuleType("termcolor")
    tc.colored = lambda s, *a, **k: s
    sys.modules.setdefault("termcolor", tc)
    tb = types.ModuleType("tensorboardX")

    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

        def add_image(self, *a, **k):
            pass
    tb.SummaryWriter = SummaryWriter
    sys.modules.setdefault("tensorboardX", tb)
    # src/train/__init__ -> trainer.py -> data_utils.py imports these (augmentation,
    # PLY I/O); nothing on the checkpoint path uses them
    ia = types.ModuleType("imgaug")
    ia.augmenters = types.ModuleType("imgaug.augmenters")
    sys.modules.setdefault("imgaug", ia)
    sys.modules.setdefault("imgaug.augmenters", ia.augmenters)
    ply = types.ModuleType("plyfile")
    ply.PlyData = object
    sys.modules.setdefault("plyfile", ply)


def main():
    _stubs()
    cfg, Network, vr = mg._import_reference()
    import torch
    from src.utils.net_utils import save_model
    from src.train.optimizer import make_optimizer
    from src.train.scheduler import make_lr_scheduler
    from src.train.recorder import Recorder
    cfg.network.nerf.W = 16
    tmp = tempfile.mkdtemp()
    cfg.record_dir = os.path.join(tmp, "record")
    cfg.resume = True
    torch.manual_seed(0)
    net = Network()
    optim = make_optimizer(cfg, net)
    sched = make_lr_scheduler(cfg, optim)
    rec = Recorder(cfg)
    rec.step = 1234
    x = torch.rand(64, net.input_ch + net.input_ch_views)
    loss = net.model(x).square().mean() + net.model_fine(x).square().mean()
    loss.backward()
    optim.step()
    sched.step()
    model_dir = os.path.join(tmp, "model")
    save_model(net, optim, sched, rec, model_dir, EPOCH)
    save_model(net, optim, sched, rec, model_dir, EPOCH, last=True)
    out = os.path.join(HERE, "ckpt_ref")
    os.makedirs(out, exist_ok=True)
    for f in (f"{EPOCH}.pth", "latest.pth"):
        shutil.copy(os.path.join(model_dir, f), os.path.join(out, f))
    state = {k: v.detach().numpy() for k, v in net.state_dict().items()}
    np.savez_compressed(os.path.join(HERE, "ckpt_ref_state.npz"), epoch=EPOCH,
                        lr=np.array([g["lr"] for g in optim.param_groups]),
                        **{"net__" + k: v for k, v in state.items()})
    shutil.rmtree(tmp)
    print("wrote", out, sorted(os.listdir(out)), len(state), "tensors")


if __name__ == "__main__":
    main()
