"""One rank of tests/test_gpu_dist.py: the real sharded render path of bench.py
(``bench.make_frame_fn``) in a fresh process, ranks sharing cuda:0 over gloo.

    RANK=r WORLD_SIZE=P MASTER_ADDR=127.0.0.1 MASTER_PORT=... \
        python tests/dist_frame_worker.py <out_dir>

Renders, on every rank, the C2 frame (lego test view 0, row bands,
``render_frame_sharded``) and C4 frames (test view 16, ESS + ERT threshold
0.01, 2048-ray chunks dealt round-robin, ``render_frame_interleaved``) at grid
call counters 0 and 498, so that grid self-updates (VR:1147-1157) fall inside
the frame on chunks owned by rank 0 (counter 0: chunks 0 and 250) and by
rank 1 (counter 498: chunks 1 and 251). Rank 0 then renders the same frames in
one pass (one process, NerfPipeline.render_image) and every rank writes
<out_dir>/rank<r>.npz: the gathered maps, its final grid and counter, and on
rank 0 the one-pass maps, grids and counters.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))

H = W = 800
C4_COUNTERS = (0, 498)


def main(out):
    import torch
    import torch.distributed as dist
    import bench
    from nerfhip.render import NerfPipeline
    from nerfhip.synthetic import make_occupancy_grid

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    ckpt = os.path.join(REPO, "checkpoints", "lego")

    def pipe(ess_ert, counter=0):
        p = NerfPipeline(dev, N_samples=64, N_importance=128, enable_ess=ess_ert,
                         enable_ert=ess_ert, ert_threshold=0.01, mlp_precision="f16x3")
        p.load_checkpoint(ckpt)
        if ess_ert:
            p.set_grid(make_occupancy_grid(0, 128, 1.2, 0.1))
            p.grid_update_counter = counter
        return p

    rec = {}
    pose0, K0 = bench.lego_camera(H, W, 0)
    p2 = pipe(False)
    maps = bench.make_frame_fn(p2, H, W, rank, world, dev, False)(pose0, K0)
    for k, v in maps.items():
        rec[f"c2_{k}"] = v.cpu().numpy()
    pose16, K16 = bench.lego_camera(H, W, 16)
    for c in C4_COUNTERS:
        p4 = pipe(True, c)
        maps = bench.make_frame_fn(p4, H, W, rank, world, dev, True)(pose16, K16)
        for k, v in maps.items():
            rec[f"c4_{c}_{k}"] = v.cpu().numpy()
        rec[f"c4_{c}_grid"] = p4.grid.cpu().numpy()
        rec[f"c4_{c}_counter"] = np.int64(p4.grid_update_counter)
        ev, _ = p4.evaluated_samples()
        rec[f"c4_{c}_evaluated"] = np.int64(ev)
        del p4
    dist.barrier()
    if rank == 0:              # the same frames in one pass, one process
        one = p2.render_image(H, W, pose0, K0)
        for k, v in one.items():
            rec[f"one_c2_{k}"] = v.cpu().numpy()
        for c in C4_COUNTERS:
            p4 = pipe(True, c)
            one = p4.render_image(H, W, pose16, K16)
            for k, v in one.items():
                rec[f"one_c4_{c}_{k}"] = v.cpu().numpy()
            rec[f"one_c4_{c}_grid"] = p4.grid.cpu().numpy()
            rec[f"one_c4_{c}_counter"] = np.int64(p4.grid_update_counter)
            ev, _ = p4.evaluated_samples()
            rec[f"one_c4_{c}_evaluated"] = np.int64(ev)
            del p4
    torch.cuda.synchronize()
    np.savez(os.path.join(out, f"rank{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
