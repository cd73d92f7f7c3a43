"""The reference's density-driven occupancy grid, captured (survey container).

``Renderer._populate_occupancy_grid_kilonerf_method`` (``volume_renderer.py:
875-961``) evaluates the coarse network's density at 3 x 3 x 3 sub-points of
every grid cell (offsets {0, 1/2, 1} of a cell, ``:913-920``) and marks a cell
occupied when the largest relu(sigma) of its 27 points exceeds 0.01
(``:943-947``). Two facts about it as written:

* it cannot run: it hands ``coarse_model`` the 63 xyz-encoding columns alone
  (``:930-936``) and ``NeRF.forward`` splits its input as 63 + 27
  (``network.py:49-51``), which raises -- as the reference's ``_query_network``
  does without view directions. The density does not depend on the view
  input (``network.py:59-61``: alpha comes from h before the views concat), so
  the capture calls the method with ``coarse_model`` wrapped to append a zero
  view encoding of 27 columns: every other line of the method is the
  reference's own;
* it writes the batch's decisions through ``list(set(batch_indices))``
  (``:950-953``), CPython's iteration order of a set of (x, y, z) tuples, not
  the batch's cell order: cell k of a 512-cell batch gets the decision of the
  k-th cell in that order. The drop-in reproduces this assignment (and offers
  the cells' own positions as an option).

Outputs ``tests/golden/kg_res<R>.npz`` for R in RESOLUTIONS: ``grid_bits``
(np.packbits of the [R, R, R] bool grid), ``cell_max_density`` (float32 per
cell in the method's flat order: z-major, x fastest; the largest relu(sigma) of
its 27 points, recorded from the wrapped model's outputs), ``res``,
``threshold``, ``bbox`` and the checkpoint's sha256. Only numbers are stored.

    python tests/golden/make_kilonerf_grid.py
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_ref_frames as MRF  # noqa: E402

RESOLUTIONS = (16, 32)


def main(argv):
    import torch
    cfg, Network, vr = MRF._import_reference()
    sd = torch.load(MRF.CKPT, map_location="cpu", weights_only=True)["net"]
    for res in [int(a) for a in argv] or RESOLUTIONS:
        cfg.enable_ess = True
        cfg.occupancy_grid_resolution = res
        net = Network()
        net.load_state_dict(sd)
        net.eval()
        torch.manual_seed(0)
        rend = vr.Renderer(net)
        rend.use_cuda_kernels = False
        sigmas = []

        class ZeroViews(torch.nn.Module):
            """coarse_model with a zero view encoding appended (density is view-free)."""

            def __init__(self, m):
                super().__init__()
                self.m = m

            def forward(self, x):
                out = self.m(torch.cat([x, torch.zeros((x.shape[0], 27), dtype=x.dtype)], -1))
                sigmas.append(out[..., 3].detach().clone())
                return out

        rend.coarse_model = ZeroViews(net.model)
        t0 = time.time()
        rend._populate_occupancy_grid_kilonerf_method()
        dt = time.time() - t0
        dens = torch.relu(torch.cat(sigmas)).view(-1, 27).max(1)[0].numpy().astype(np.float32)
        grid = rend.occupancy_grid.numpy().astype(bool)
        assert dens.shape == (res ** 3,) and grid.shape == (res, res, res)
        path = os.path.join(MRF.OUT, f"kg_res{res}.npz")
        np.savez_compressed(path, grid_bits=np.packbits(grid.reshape(-1)), res=res,
                            cell_max_density=dens, threshold=np.float32(0.01),
                            bbox=np.array([-2.0, -2.0, -2.0, 2.0, 2.0, 2.0], np.float32),
                            ckpt_sha256=MRF.ckpt_sha(), cpu_seconds=dt)
        occ_own = int((dens > np.float32(0.01)).sum())
        print(f"{path}: res {res}, {int(grid.sum())} cells occupied "
              f"({occ_own} by their own decision), {dt:.0f} s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
