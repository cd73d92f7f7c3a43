"""Row-band / chunk-aligned frame sharding + the pixel all-gather (nerfhip.dist),
world_size 2 over gloo on the CPU. The per-band render is a deterministic
function of the pixel index, so the assembled frame must equal the
single-process frame exactly."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nerfhip import dist as nd


def fake_render(p0, n, with_fine=True):
    if n == 0:
        return {}
    p = torch.arange(p0, p0 + n, dtype=torch.float32)
    out = {"rgb_map_0": torch.stack([p, p + 0.25, p + 0.5], -1), "disp_map_0": -p,
           "acc_map_0": p * 0.5, "depth_map_0": p + 3.0}
    if with_fine:
        out.update({"rgb_map": torch.stack([2 * p, 2 * p + 1, 2 * p + 2], -1), "disp_map": p * 3,
                    "acc_map": p - 1, "depth_map": p * 7})
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def fake_render_chunks(chunks, total, with_fine=True):
    parts = [fake_render(c * nd.REF_CHUNK, min(nd.REF_CHUNK, total - c * nd.REF_CHUNK), with_fine)
             for c in chunks]
    if not parts:
        return {}
    return {k: torch.cat([p[k] for p in parts], 0) for k in parts[0]}


def _worker(rank, world, port, H, W, chunk_aligned, with_fine, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if chunk_aligned == "interleaved":
            frame = nd.render_frame_interleaved(
                lambda cs: fake_render_chunks(cs, H * W, with_fine), H, W, rank, world,
                torch.device("cpu"))
        else:
            frame = nd.render_frame_sharded(lambda p0, n: fake_render(p0, n, with_fine), H, W,
                                            rank, world, torch.device("cpu"),
                                            chunk_aligned=chunk_aligned)
        q.put((rank, {k: v.numpy().copy() for k, v in frame.items()}))  # by value, not fd
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("H,W,chunk_aligned,with_fine", [(8, 5, False, True), (7, 3, False, True),
                                                         (64, 80, True, True), (3, 1000, True, False),
                                                         (64, 80, "interleaved", True),
                                                         (3, 1000, "interleaved", False),
                                                         (9, 500, "interleaved", True),
                                                         (2, 3, "interleaved", True)])
def test_two_rank_frame_equals_single(H, W, chunk_aligned, with_fine):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, H, W, chunk_aligned, with_fine, q))
             for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = fake_render(0, H * W, with_fine)
    for rank in (0, 1):
        frame = got[rank]
        assert set(frame) == set(ref)
        for k, v in ref.items():
            shape = (H, W, 3) if k.startswith("rgb") else (H, W)
            assert torch.equal(torch.from_numpy(frame[k]), v.reshape(shape)), (rank, k)


def test_band_partition_covers_image():
    for H, W, world in [(800, 800, 8), (800, 800, 3), (5, 7, 8)]:
        for aligned in (False, True):
            seen = []
            for r in range(world):
                p0, n, pad = nd.band(H, W, r, world, aligned)
                assert n <= pad
                if aligned and p0 < H * W:
                    assert p0 % nd.REF_CHUNK == 0
                seen.extend(range(p0, p0 + n))
            assert seen == list(range(H * W))


def test_interleaved_chunk_sets_cover_image():
    """Chunk c -> rank c mod P: every chunk exactly once, tiles padded to the
    largest set, and the gather index maps each pixel to its rank's tile row."""
    for H, W, world in [(800, 800, 8), (800, 800, 3), (5, 7, 8), (100, 100, 2)]:
        total = H * W
        nch = -(-total // nd.REF_CHUNK)
        seen, npix = [], 0
        for r in range(world):
            mine, n, pad = nd.chunk_set(H, W, r, world)
            assert n <= pad and all(c % world == r for c in mine)
            seen += mine
            npix += n
        assert sorted(seen) == list(range(nch)) and npix == total
        idx = nd.interleave_index(H, W, world, torch.device("cpu"))
        assert idx.shape == (total,) and len(set(idx.tolist())) == total


def _grad_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerfhip.train import allreduce_mean
        grads = [torch.full((3, 4), float(rank + 1)), torch.arange(5, dtype=torch.float32) * (rank + 1)]
        allreduce_mean(grads, dist.group.WORLD)
        q.put((rank, [g.numpy().copy() for g in grads]))
    finally:
        dist.destroy_process_group()


def test_train_gradient_allreduce_mean():
    """Data-parallel C3 step: every rank ends with the mean of the ranks' gradients."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        a, b = got[rank]
        assert (a == 1.5).all()
        assert (b == torch.arange(5).numpy() * 1.5).all()


def _local_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        H, W = 7, 9
        local = nd.render_frame_sharded(lambda p0, n: fake_render(p0, n), H, W, 0, 1,
                                        torch.device("cpu"))
        inter = nd.render_frame_interleaved(lambda cs: fake_render_chunks(cs, H * W), H, W, 0, 1,
                                            torch.device("cpu"))
        q.put((rank, nd._collective(1), nd._collective(world),
               {k: v.numpy().copy() for k, v in local.items()},
               {k: v.numpy().copy() for k, v in inter.items()}))
    finally:
        dist.destroy_process_group()


def test_world_one_render_inside_larger_job_stays_local():
    """A world-1 frame rendered by one rank of a 2-rank job (its own full frame,
    e.g. an evaluation on every rank) takes no collective: the tile is the
    frame, equal to the single-process render; world 2 does gather."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_local_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = fake_render(0, 7 * 9)
    for rank in (0, 1):
        c1, c2, local, inter = got[rank]
        assert c1 is False and c2 is True
        for k, v in ref.items():
            want = v.numpy().reshape(local[k].shape)
            assert (local[k] == want).all() and (inter[k] == want).all(), k
