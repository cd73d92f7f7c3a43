"""The training step's optimizer: torch.optim.Adam's update (src/train/
optimizer.py builds ``torch.optim.Adam(params, lr, weight_decay=0)``; eps 1e-8)
with ``clip_grad_value_`` (trainers/trainer.py:59) fused in front, over every
parameter in ONE ``nerf_adam_step`` launch (csrc/train_kernels.hip) instead of
torch's multi-tensor kernels (clamp + Adam: five launches, ~110 us per step).

The state stays torch's (``exp_avg``, ``exp_avg_sq``, ``step`` per parameter,
so ``state_dict`` / ``load_state_dict`` and nerfhip.checkpoint's reference
layout work unchanged); lr and the step count live on the device, so the
launch can be captured into a HIP graph and replayed.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call


class _AdamTensor(ctypes.Structure):
    """NerfAdamTensor (include/nerfhip.h)."""
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p),
                ("v", ctypes.c_void_p), ("n", ctypes.c_int64)]


class HipAdam(torch.optim.Adam):
    """Adam (weight decay 0, no amsgrad) + gradient value clipping at ``clip``
    (None: none; any clip >= 0 clamps the gradients in place to [-clip, clip]
    as clip_grad_value_ does, NaN kept), one parameter group, float32
    contiguous parameters on one ROCm device.

    One step count serves every parameter (it lives on the device for graph
    capture), so every parameter must have a gradient at every step (torch's
    Adam would skip one without and keep a separate count): ``step`` raises
    otherwise, and a loaded state dict must hold one common step value."""

    def __init__(self, params, lr=5e-4, betas=(0.9, 0.999), eps=1e-8, clip=None):
        params = list(params)
        dev = params[0].device
        if dev.type != "cuda":
            raise _lib.NerfHipError("HipAdam needs a ROCm GPU device (no CPU fallback)")
        super().__init__(params, lr=torch.tensor(lr, device=dev, dtype=torch.float32),
                         betas=betas, eps=eps, weight_decay=0.0, capturable=True,
                         foreach=False)
        if len(self.param_groups) != 1:
            raise ValueError("HipAdam takes one parameter group")
        if clip is not None and not clip >= 0:
            raise ValueError("HipAdam: clip must be None (no clipping) or >= 0")
        self.clip = -1.0 if clip is None else float(clip)   # < 0 tells the kernel: none
        self._count = torch.zeros(1, device=dev, dtype=torch.float32)   # shared step count
        self._key = None
        self._arr = None

    def _state_of(self, p):
        st = self.state[p]
        if not st:
            st["step"] = self._count.view(())
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        elif st["step"].data_ptr() != self._count.data_ptr():
            # a loaded state dict: every parameter must have been stepped together
            steps = {float(self.state[q]["step"]) for q in self.param_groups[0]["params"]
                     if q in self.state and "step" in self.state[q]
                     and self.state[q]["step"].data_ptr() != self._count.data_ptr()}
            if len(steps) > 1:
                raise ValueError(f"HipAdam: loaded state holds different step counts {steps}; "
                                 "it keeps one count for all parameters")
            self._count.copy_(st["step"].reshape(1).to(self._count))
            st["step"] = self._count.view(())
        return st

    @torch.no_grad()
    def step(self, closure=None):
        if closure is not None:
            raise ValueError("HipAdam.step takes no closure")
        g = self.param_groups[0]
        if g.get("amsgrad") or g.get("maximize") or g["weight_decay"] != 0:
            raise ValueError("HipAdam: amsgrad / maximize / weight decay are not supported")
        lr = g["lr"]
        if not torch.is_tensor(lr):   # a float lr set by someone else: back on the device
            lr = g["lr"] = torch.tensor(float(lr), device=self._count.device)
        rows = []
        missing = [p for p in g["params"] if p.grad is None]
        if missing and len(missing) != len(g["params"]):
            raise ValueError(f"HipAdam: {len(missing)} of {len(g['params'])} parameters have no "
                             "gradient; its shared step count needs all of them every step")
        for p in g["params"]:
            if p.grad is None:
                continue
            st = self._state_of(p)
            m, v, gr = st["exp_avg"], st["exp_avg_sq"], p.grad
            for t in (p, gr, m, v):
                if t.dtype != torch.float32 or not t.is_contiguous():
                    raise ValueError("HipAdam needs contiguous float32 tensors")
            rows.append((p.data_ptr(), gr.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel()))
        if not rows:
            return None
        key = tuple(rows)
        if key != self._key:
            self._arr = (_AdamTensor * len(rows))(*[_AdamTensor(*r) for r in rows])
            self._key = key
        b1, b2 = g["betas"]
        call("nerf_adam_step", ctypes.addressof(self._arr), len(rows), lr.data_ptr(),
             self._count.data_ptr(), None, float(b1), float(b2),
             float(g["eps"]), self.clip, _lib.stream_of(self._count.device))
        return None
