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

With ERT's sample compaction a chunk's cost follows the scene (a chunk of
background retires nothing, one across the object retires most samples), so
contiguous bands load the ranks unevenly. ``render_frame_interleaved`` deals
the 2048-ray chunks out round-robin instead (chunk c -> rank
c mod P; NerfPipeline.render_chunks keeps the reference's sequential grid
semantics), gathers equal-size padded tiles and puts the chunks back in
pixel order with one index_select.
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


def _collective(world, group=None):
    """The gather runs for world > 1, and at world 1 whenever a one-rank
    process group is up, so the RCCL all-gather and the reassembly are
    exercised by a one-GPU run (tests/test_gpu_nccl.py: backend "nccl" at
    world 1, bit-equal to the one-pass frame). With no group (a plain
    one-process render), or a world-1 render inside a larger job, the tile is
    the frame."""
    if world > 1:
        return True
    return (dist.is_available() and dist.is_initialized()
            and dist.get_world_size(group) == 1)


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
    if not _collective(world, group):
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


def chunk_set(H, W, rank, world):
    """Chunks (2048 consecutive pixels, VR:147) rank `rank` owns under the
    interleaved assignment c -> c mod world, their pixel count, and the padded
    tile length (the most chunks any rank owns x 2048)."""
    total = H * W
    nch = -(-total // REF_CHUNK)
    mine = list(range(rank, nch, world))
    n = sum(min(REF_CHUNK, total - c * REF_CHUNK) for c in mine)
    return mine, n, -(-nch // world) * REF_CHUNK


_PERM = {}


def interleave_index(H, W, world, device):
    """Row of the gathered [world * n_pad] tiles holding each pixel, in pixel order."""
    key = (H, W, world, str(device))
    if key not in _PERM:
        total = H * W
        _, _, n_pad = chunk_set(H, W, 0, world)
        pix = torch.arange(total, dtype=torch.int64)
        c = pix // REF_CHUNK
        _PERM[key] = ((c % world) * n_pad + (c // world) * REF_CHUNK + pix % REF_CHUNK).to(device)
    return _PERM[key]


def render_frame_interleaved(render_chunks, H, W, rank, world, device, group=None):
    """render_chunks(chunks) -> dict of flat maps for the concatenated pixels of
    the given (ascending) chunk ids; called on every rank, also with an empty
    list, so stateful renderers (ESS + ERT, NerfPipeline.render_chunks) advance
    their grid and counter everywhere. Returns the assembled frame (dict of
    [H,W(,3)] maps) on every rank."""
    mine, n, n_pad = chunk_set(H, W, rank, world)
    maps = render_chunks(mine) or {}
    keys = set(maps) if maps else set(MAP_ORDER)
    tile = pack_maps(maps, n, n_pad, device)
    if not _collective(world, group):
        full = tile[:H * W]
    else:
        full = torch.empty((world * n_pad, 12), device=device, dtype=torch.float32)
        dist.all_gather_into_tensor(full, tile, group=group)
        full = full.index_select(0, interleave_index(H, W, world, device))
    return unpack_maps(full, H, W, keys)
