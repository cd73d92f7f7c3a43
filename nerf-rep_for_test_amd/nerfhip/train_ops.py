"""Differentiable compositing and importance sampling of the training step on
HIP kernels (csrc/train_kernels.hip, csrc/render_kernels.hip), as
``torch.autograd.Function`` s that ``train.render_train`` uses in place of the
torch-op versions.

* ``composite_hip(raw, z, rays_d, white)`` = ``_raw2outputs`` (VR:286-357,
  raw_noise_std 0): (rgb, disp, acc, weights, depth), backward to raw and z.
* ``sample_fine_hip(weights, z, u)`` = ``_sample_fine`` with training-mode u
  (VR:239-268) merged with the coarse depths by ``torch.sort(cat(z, z_f))``
  (VR:181-184): z_all [n, S + N_importance]; backward to the coarse weights
  (the reference does not detach the fine samples, so the fine loss reaches the
  coarse network through them).

* ``add_sigma_noise(raw, noise)``: raw with ``noise`` added to the density
  logit (raw_noise_std > 0, VR:310-314 / :1098-1103), gradient passed through.

None needs a host synchronisation, so a step built from them can be
captured into a HIP graph (``NerfTrainer(graph=True)``).
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import call, ptr


def _c(t):
    return None if t is None else t.contiguous()


class AddSigmaNoiseFn(torch.autograd.Function):
    """raw [..., 4] with noise [...] added to raw[..., 3] (nerf_add_sigma_noise);
    d raw = d out (the noise is a constant of the step)."""
    @staticmethod
    def forward(ctx, raw, noise):
        raw_c, nz = raw.detach().contiguous(), noise.detach().contiguous()
        assert nz.numel() * 4 == raw_c.numel()
        out = torch.empty_like(raw_c)
        call("nerf_add_sigma_noise", ptr(raw_c), ptr(nz), nz.numel(), ptr(out),
             _lib.stream_of(raw.device))
        return out

    @staticmethod
    def backward(ctx, g):
        return g, None


def add_sigma_noise(raw, noise):
    return AddSigmaNoiseFn.apply(raw, noise)


class CompositeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw, z, rays_d, white):
        n, S, _ = raw.shape
        dev = raw.device
        raw_c, z_c, rd = raw.detach().contiguous(), z.detach().contiguous(), \
            rays_d.detach().contiguous()
        f32 = torch.float32
        rgb = torch.empty((n, 3), device=dev, dtype=f32)
        disp = torch.empty((n,), device=dev, dtype=f32)
        acc = torch.empty((n,), device=dev, dtype=f32)
        depth = torch.empty((n,), device=dev, dtype=f32)
        w = torch.empty((n, S), device=dev, dtype=f32)
        T = torch.empty((n, S), device=dev, dtype=f32)
        call("nerf_composite_train_fwd", ptr(raw_c), ptr(z_c), ptr(rd), n, S, int(white), ptr(rgb),
             ptr(disp), ptr(acc), ptr(depth), ptr(w), ptr(T), _lib.stream_of(dev))
        ctx.save_for_backward(raw_c, z_c, rd, w, T, acc, depth)
        ctx.white = int(white)
        ctx.set_materialize_grads(False)
        return rgb, disp, acc, w, depth

    @staticmethod
    def backward(ctx, g_rgb, g_disp, g_acc, g_w, g_depth):
        raw, z, rd, w, T, acc, depth = ctx.saved_tensors
        n, S, _ = raw.shape
        d_raw = torch.empty_like(raw)
        d_z = torch.empty_like(z) if ctx.needs_input_grad[1] else None
        g_rgb, g_disp, g_acc, g_w, g_depth = map(_c, (g_rgb, g_disp, g_acc, g_w, g_depth))
        call("nerf_composite_train_bwd", ptr(raw), ptr(z), ptr(rd), ptr(w), ptr(T), ptr(acc),
             ptr(depth), n, S, ctx.white, ptr(g_rgb), ptr(g_disp), ptr(g_acc), ptr(g_depth),
             ptr(g_w), ptr(d_raw), ptr(d_z), _lib.stream_of(raw.device))
        return d_raw, d_z, None, None


class SampleFineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weights, z, u):
        n, S = z.shape
        NI = u.shape[1]
        w_c, z_c, u_c = weights.detach().contiguous(), z.detach().contiguous(), \
            u.detach().contiguous()
        zall = torch.empty((n, S + NI), device=z.device, dtype=torch.float32)
        call("nerf_sample_fine", ptr(z_c), S, ptr(w_c), ptr(u_c), NI, n, S, NI, ptr(zall),
             _lib.stream_of(z.device))
        ctx.save_for_backward(w_c, z_c, u_c, zall)
        ctx.set_materialize_grads(False)
        return zall

    @staticmethod
    def backward(ctx, g_zall):
        w, z, u, zall = ctx.saved_tensors
        if g_zall is None or not ctx.needs_input_grad[0]:
            return None, None, None
        n, S = z.shape
        d_w = torch.empty_like(w)
        g = g_zall.contiguous()
        call("nerf_sample_pdf_bwd", ptr(z), ptr(w), ptr(u), ptr(g), ptr(zall), n, S,
             u.shape[1], ptr(d_w), _lib.stream_of(z.device))
        return d_w, None, None


def composite_hip(raw, z, rays_d, white_bkgd=True):
    _lib.require_gpu(raw)
    return CompositeFn.apply(raw, z, rays_d, bool(white_bkgd))


def sample_fine_hip(weights, z, u):
    _lib.require_gpu(z)
    return SampleFineFn.apply(weights, z, u)


class MSEPairFn(torch.autograd.Function):
    """(loss_coarse, loss_fine, loss) = (mse(a, t), mse(b, t), their sum)
    (trainers/nerf.py:39-76) in one launch, its backward in one; b may be None
    (no fine pass: loss_fine = 0)."""

    @staticmethod
    def forward(ctx, a, b, target):
        a_c, t_c = a.detach().contiguous(), target.detach().contiguous()
        b_c = b.detach().contiguous() if b is not None else None
        out = torch.empty(3, device=a.device, dtype=torch.float32)
        call("nerf_mse_pair", ptr(a_c), ptr(b_c), ptr(t_c), a_c.numel(), ptr(out),
             _lib.stream_of(a.device))
        ctx.save_for_backward(a_c, b_c, t_c)
        ctx.has_b = b is not None
        ctx.set_materialize_grads(False)   # unused outputs' gradients stay None (= 0)
        return out[0], out[1], out[2]

    @staticmethod
    def backward(ctx, g0, g1, g2):
        a, b, t = ctx.saved_tensors
        gs = [None if x is None else x.to(torch.float32).contiguous() for x in (g0, g1, g2)]
        da = torch.empty_like(a)
        db = torch.empty_like(b) if ctx.has_b else None
        call("nerf_mse_pair_backward", ptr(a), ptr(b), ptr(t), a.numel(), *[ptr(x) for x in gs],
             ptr(da), ptr(db), _lib.stream_of(a.device))
        return da, db, None


def mse_losses_hip(out, target):
    """trainers/nerf.py:39-76 as mse_losses, on the fused loss kernel."""
    _lib.require_gpu(target)
    fine = out.get("rgb_map")
    lc, lf, loss = MSEPairFn.apply(out["rgb_map_0"], fine, target)
    res = {"loss_coarse": lc, "loss": loss}
    if fine is not None:
        res["loss_fine"] = lf
    return res
