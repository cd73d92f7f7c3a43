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


def reference_optim_state(opt, names, order):
    """A single-param-group Adam state_dict (the trainer's: one fused multi-tensor
    step over ``names``, in that order) in the layout of the reference's
    ``make_optimizer`` (src/train/optimizer.py:8-28): one param group per
    parameter, in ``order`` (``net.named_parameters()`` order), so that the
    reference's ``load_model`` (net_utils.py:288-320) can call
    ``optim.load_state_dict`` on it. Group options are exported as plain floats
    (a capturable step keeps lr as a device tensor)."""
    sd = opt.state_dict()
    if len(sd["param_groups"]) != 1:
        raise ValueError("expected the trainer's single param group")
    g = sd["param_groups"][0]
    pos = {n: i for i, n in enumerate(names)}
    opts = {k: v for k, v in g.items() if k != "params"}
    opts["lr"] = float(opts["lr"])
    opts.update(capturable=False, fused=None, foreach=None)
    opts.setdefault("initial_lr", opts["lr"])
    opts["initial_lr"] = float(opts["initial_lr"])
    groups, state = [], {}
    for j, name in enumerate(order):
        i = g["params"][pos[name]]
        groups.append({**opts, "params": [j]})
        if i in sd["state"]:
            state[j] = {k: (v.detach().cpu().clone() if torch.is_tensor(v) else v)
                        for k, v in sd["state"][i].items()}
    return {"state": state, "param_groups": groups}


def single_group_optim_state(sd, names, order):
    """Inverse of reference_optim_state: a reference-layout (one group per
    parameter, ``order``) Adam state_dict for the trainer's single group over
    ``names``."""
    pos = {n: j for j, n in enumerate(order)}
    opts = {k: v for k, v in sd["param_groups"][0].items() if k != "params"}
    state = {}
    for i, name in enumerate(names):
        j = sd["param_groups"][pos[name]]["params"][0]
        if j in sd["state"]:
            state[i] = sd["state"][j]
    return {"state": state, "param_groups": [{**opts, "params": list(range(len(names)))}]}


def exponential_lr_state(base_lr, gamma, decay_epochs, last_epoch, n_groups):
    """The state_dict of the reference's ExponentialLR (src/utils/optimizer/
    lr_scheduler.py:68-79: lr = base_lr * gamma ** (last_epoch / decay_epochs);
    _LRScheduler.load_state_dict restores it as attributes)."""
    lr = base_lr * gamma ** (last_epoch / decay_epochs)
    return {"decay_epochs": decay_epochs, "gamma": gamma, "base_lrs": [base_lr] * n_groups,
            "last_epoch": int(last_epoch), "_step_count": int(last_epoch) + 1,
            "_get_lr_called_within_step": False, "_last_lr": [lr] * n_groups}
