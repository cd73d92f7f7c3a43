"""Frame sharding across GPUs: one process per GPU, row bands of the image,
one collective for the final pixels (RCCL over xGMI with backend "nccl").

The reference has no distributed render path; rays are
independent with ESS/ERT off, so rank r renders pixel rows
[r*H/P, (r+1)*H/P) and the 12 float32 maps per pixel (rgb_0, disp_0, acc_0,
depth_0, rgb, disp, acc, depth) are all-gathered as equal-size tiles. With
ERT/ESS on, chunk membership (2048 consecutive pixels) changes results, so
bands are cut on whole reference chunks instead (``chunk_aligned=True``), and
with ESS + ERT each rank replays the grid self-updates of the chunks outside
its band (NerfPipeline.render_band) so that every band sees the grid the
reference's sequential loop would have at its first chunk.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

MAP_ORDER = ("rgb_map_0", "disp_map_0", "acc_map_0", "depth_map_0",
             "rgb_map", "disp_map", "acc_map", "depth_map")
REF_CHUNK = 2048


def band(H, W, rank, world, chunk_aligned=False):
    """Pixel range [p0, p0+n) of this rank, plus the padded tile length."""
    total = H * W
    if chunk_aligned:
        nch = -(-total // REF_CHUNK)
        per = -(-nch // world)
        p0 = min(total, rank * per * REF_CHUNK)
        p1 = min(total, (rank + 1) * per * REF_CHUNK)
        return p0, p1 - p0, per * REF_CHUNK
    rows = -(-H // world)
    r0 = min(H, rank * rows)
    r1 = min(H, (rank + 1) * rows)
    return r0 * W, (r1 - r0) * W, rows * W


def pack_maps(maps, n, n_pad, device, n_importance=True):
    """[n_pad, 12] float32 tile of this rank's maps (zero padded)."""
    tile = torch.zeros((n_pad, 12), device=device, dtype=torch.float32)
    col = 0
    for k in MAP_ORDER:
        width = 3 if k.startswith("rgb") else 1
        if k in maps:
            tile[:n, col:col + width] = maps[k].reshape(n, width)
        col += width
    return tile


def unpack_maps(full, H, W, keys):
    out = {}
    col = 0
    for k in MAP_ORDER:
        width = 3 if k.startswith("rgb") else 1
        if k in keys:
            v = full[:H * W, col:col + width]
            out[k] = v.reshape(H, W, 3) if width == 3 else v.reshape(H, W)
        col += width
    return out


def render_frame_sharded(render_band, H, W, rank, world, device, group=None,
                         chunk_aligned=False):
    """render_band(p0, n) -> dict of flat maps for pixels [p0, p0+n) ({} when n
    is 0; it is called on every rank, so stateful renderers -- ESS + ERT,
    NerfPipeline.render_band -- advance their grid and counter everywhere).

    Returns the assembled frame (dict of [H,W(,3)] maps) on every rank."""
    p0, n, n_pad = band(H, W, rank, world, chunk_aligned)
    maps = render_band(p0, n) or {}
    keys = set(maps) if maps else set(MAP_ORDER)
    tile = pack_maps(maps, n, n_pad, device)
    if world == 1:
        full = tile
    else:
        full = torch.empty((world * n_pad, 12), device=device, dtype=torch.float32)
        dist.all_gather_into_tensor(full, tile, group=group)
        # bands are contiguous in pixel order except for the padding of each tile
        parts = []
        for r in range(world):
            q0, qn, _ = band(H, W, r, world, chunk_aligned)
            parts.append(full[r * n_pad:r * n_pad + qn])
        full = torch.cat(parts, 0)
    return unpack_maps(full, H, W, keys)
