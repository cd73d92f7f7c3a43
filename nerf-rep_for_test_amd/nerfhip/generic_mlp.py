"""The NeRF MLP for topologies other than lego's (reference ``network.py:9-74``
with ``use_viewdirs=True``: any depth D, width W, skip set and encoding widths),
layer by layer on ``nerf_linear_fm`` (FP32, feature-major activations) with the
frequency encodings from ``nerf_freq_encode_fm``. Lego's 8 x 256 / skip 4 never
comes here: it runs on the fused kernels (``mlp_x3.hip``, ``mlp_fused.hip``).

Per chunk of samples the activations live feature-major ([rows][P]); the skip
concatenation ``cat([input_pts, h])`` (NET:54-55) is a buffer whose first rows
hold the xyz encoding and whose lower rows receive the layer's output, and the
views input ``cat([feature, input_views])`` (NET:59) likewise, so nothing is
copied. rgb and alpha are written straight into raw [P][4] (NET:61-70)."""
from __future__ import annotations

import torch

from . import _lib
from ._lib import call, ptr

CHUNK = 1 << 18   # samples per pass: W x CHUNK x 4 B of activations
LEGO = (8, 256, (4,), 10, 4)   # (D, W, skips, L_xyz, L_dir): the fused kernels' topology


def topology(params, prefix):
    """(D, W, skips, L_xyz, L_dir) of a NeRF state dict (NET:9-43)."""
    D = 0
    while f"{prefix}.pts_linears.{D}.weight" in params:
        D += 1
    if D == 0:
        raise KeyError(f"{prefix}.pts_linears.0.weight missing")
    W, in_x = (int(v) for v in params[f"{prefix}.pts_linears.0.weight"].shape)
    skips = tuple(i for i in range(D - 1)
                  if int(params[f"{prefix}.pts_linears.{i + 1}.weight"].shape[1]) == W + in_x)
    in_v = int(params[f"{prefix}.views_linears.0.weight"].shape[1]) - W
    if (in_x - 3) % 6 or (in_v - 3) % 6:
        raise ValueError(f"{prefix}: encoding widths {in_x} / {in_v} are not 3 + 6 L")
    return D, W, skips, (in_x - 3) // 6, (in_v - 3) // 6


class GenericMLP:
    """One network (``prefix`` of a reference state dict) resident on ``device``."""

    def __init__(self, params, prefix, device):
        if f"{prefix}.output_linear.weight" in params:
            raise NotImplementedError(f"{prefix}: use_viewdirs=False (output_linear)")
        self.device = torch.device(device)
        self.D, self.W, self.skips, self.lx, self.ld = topology(params, prefix)
        self.nx, self.nd = 3 + 6 * self.lx, 3 + 6 * self.ld

        def t(name):
            return torch.as_tensor(params[f"{prefix}.{name}"]).to(
                device=self.device, dtype=torch.float32).contiguous()
        self.pts = [(t(f"pts_linears.{i}.weight"), t(f"pts_linears.{i}.bias")) for i in range(self.D)]
        self.alpha = (t("alpha_linear.weight"), t("alpha_linear.bias"))
        self.feature = (t("feature_linear.weight"), t("feature_linear.bias"))
        self.views = (t("views_linears.0.weight"), t("views_linears.0.bias"))
        self.rgb = (t("rgb_linear.weight"), t("rgb_linear.bias"))

    def _lin(self, wb, X, ldx, K, P, relu, Y, sym, syp, st):
        w, b = wb
        assert tuple(w.shape)[1] == K
        call("nerf_linear_fm", ptr(w), K, ptr(b), ptr(X), ldx, K, P, int(w.shape[0]), int(relu),
             ptr(Y), sym, syp, st)

    def forward(self, rays_o, rays_d, z, z_stride, n, S):
        """raw [n * S, 4] of the samples o + d z (VR:165) of n rays (z [n][S] with
        row stride z_stride, 0: one shared row)."""
        dev, st = self.device, _lib.stream_of(self.device)
        raw = torch.empty((n * S, 4), device=dev, dtype=torch.float32)
        zz = z.view(-1)[:S].expand(n, S) if z_stride == 0 else z.view(n, -1)[:, :S]
        W, nx, nd = self.W, self.nx, self.nd
        rpc = max(1, CHUNK // S)   # rays per pass
        for r0 in range(0, n, rpc):
            m = min(rpc, n - r0)
            P = m * S
            ro, rd = rays_o[r0:r0 + m], rays_d[r0:r0 + m]
            # VR:165 / :274-279: points and per-sample view directions, float32 as the reference
            pts = (ro[:, None, :] + rd[:, None, :] * zz[r0:r0 + m][..., None]).reshape(P, 3).contiguous()
            dirs = rd[:, None, :].expand(m, S, 3).reshape(P, 3).contiguous()
            # [xyz encoding | h] (the skip input) and [feature | dir encoding] (views input)
            skip = torch.empty((nx + W, P), device=dev, dtype=torch.float32)
            vin = torch.empty((W + nd, P), device=dev, dtype=torch.float32)
            call("nerf_freq_encode_fm", ptr(pts), 3, P, self.lx, ptr(skip), P, None, st)
            call("nerf_freq_encode_fm", ptr(dirs), 3, P, self.ld, ptr(vin[W:]), P, None, st)
            hs = [torch.empty((W, P), device=dev, dtype=torch.float32) for _ in range(2)]
            x, k = skip, nx                 # layer 0 reads the encoding rows
            for i in range(self.D):
                # a skip layer's output goes below the encoding rows (NET:54-55); two
                # skips in a row would read and write those rows: that one goes
                # through a free buffer
                direct = i not in self.skips or x is not skip
                y = skip[nx:] if i in self.skips and direct else hs[i & 1]
                self._lin(self.pts[i], x, P, k, P, True, y, P, 1, st)
                if not direct:
                    skip[nx:].copy_(y)
                x, k = (skip, nx + W) if i in self.skips else (y, W)
            # NET:57-70: alpha (raw[:, 3]), feature, views layer (+ ReLU), rgb (raw[:, :3])
            out = raw[r0 * S:(r0 + m) * S]
            self._lin(self.alpha, x, P, k, P, False, out[:, 3:], 1, 4, st)
            self._lin(self.feature, x, P, k, P, False, vin, P, 1, st)
            h = hs[(self.D + 1) & 1][:W // 2]   # (x's buffer: alpha / feature read it first)
            self._lin(self.views, vin, P, W + nd, P, True, h, P, 1, st)
            self._lin(self.rgb, h, P, W // 2, P, False, out, 1, 4, st)
        return raw
