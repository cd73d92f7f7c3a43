"""Checkpoints in the reference's format (src/utils/net_utils.py:323-372).

A checkpoint is ``{"net": state_dict, "optim": ..., "scheduler": ...,
"recorder": ..., "epoch": int}`` saved as ``<model_dir>/<epoch>.pth`` or
``latest.pth``; the network's keys are ``model.*`` (coarse) and
``model_fine.*`` (fine), the names ``nerfhip.pack`` reads. Loading never
unpickles code: ``torch.load(..., weights_only=True)`` only.
"""
from __future__ import annotations

import os

import torch


def _numbered(model_dir):
    out = []
    for f in os.listdir(model_dir):
        stem, ext = os.path.splitext(f)
        if ext == ".pth" and stem.isdigit():
            out.append(int(stem))
    return out


def save_model(net, optim, scheduler, recorder, model_dir, epoch, last=False):
    """net_utils.py:323-344: write the checkpoint; keep at most 5 numbered ones."""
    os.makedirs(model_dir, exist_ok=True)
    model = {"net": net.state_dict(), "optim": optim.state_dict(),
             "scheduler": scheduler.state_dict(), "recorder": recorder.state_dict(),
             "epoch": epoch}
    name = "latest.pth" if last else f"{epoch}.pth"
    torch.save(model, os.path.join(model_dir, name))
    pths = _numbered(model_dir)
    if len(pths) > 5:
        os.remove(os.path.join(model_dir, f"{min(pths)}.pth"))


def resolve(model_dir, epoch=-1):
    """The file load_network would read (net_utils.py:352-367), or None."""
    if not os.path.exists(model_dir):
        return None
    if not os.path.isdir(model_dir):
        return model_dir
    files = os.listdir(model_dir)
    pths = _numbered(model_dir)
    if not pths and "latest.pth" not in files:
        return None
    if epoch == -1:
        pth = "latest" if "latest.pth" in files else max(pths)
    else:
        pth = epoch
    return os.path.join(model_dir, f"{pth}.pth")


def load_checkpoint(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def load_network(net, model_dir, resume=True, epoch=-1, strict=True):
    """net_utils.py:347-379: load ``net`` from a checkpoint; returns the next epoch
    (0 when there is nothing to load)."""
    if not resume:
        return 0
    path = resolve(model_dir, epoch)
    if path is None:
        return 0
    ck = load_checkpoint(path)
    net.load_state_dict(ck["net"], strict=strict)
    return ck["epoch"] + 1 if "epoch" in ck else 0


def network_params(model_dir, epoch=-1):
    """The ``model.*`` / ``model_fine.*`` tensors of a checkpoint (for
    ``NerfPipeline.set_weights``)."""
    path = resolve(model_dir, epoch)
    if path is None:
        raise FileNotFoundError(f"no checkpoint under {model_dir}")
    net = load_checkpoint(path)["net"]
    return {k: v for k, v in net.items() if k.startswith(("model.", "model_fine."))}
