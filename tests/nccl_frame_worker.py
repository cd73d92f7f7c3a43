"""The process of tests/test_gpu_nccl.py: RCCL (torch.distributed backend
"nccl", one rank on cuda:0 with device_id) under bench.py's own sharded frame
functions, so the collective branch of nerfhip.dist runs on the hardware:
``all_gather_into_tensor`` and the band / chunk reassembly
(``render_frame_sharded``, ``render_frame_interleaved`` with its
``index_select``), and the data-parallel train step's flat all-reduce.

    RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=... \
        python tests/nccl_frame_worker.py <out_dir>

Before the process group exists it renders the one-pass frames (C2 lego view
0; C4 view 16 with ESS + ERT at grid counter 0, chunk 0 updating the grid) and
one train step without a group; after ``init_process_group("nccl")`` the same
through the collective path. Writes <out_dir>/nccl.npz.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))

H = W = 800


def main(out):
    import torch
    import torch.distributed as dist
    import bench
    from nerfhip import dist as nd
    from nerfhip.render import NerfPipeline
    from nerfhip.synthetic import make_occupancy_grid, make_params
    from nerfhip.train import NerfTrainer
    from dist_train_worker import batch, flat_params

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ckpt = os.path.join(REPO, "checkpoints", "lego")

    def pipe(ess_ert):
        p = NerfPipeline(dev, N_samples=64, N_importance=128, enable_ess=ess_ert,
                         enable_ert=ess_ert, ert_threshold=0.01, mlp_precision="f16x3")
        p.load_checkpoint(ckpt)
        if ess_ert:
            p.set_grid(make_occupancy_grid(0, 128, 1.2, 0.1))
            p.grid_update_counter = 0
        return p

    rec = {}
    pose0, K0 = bench.lego_camera(H, W, 0)
    pose16, K16 = bench.lego_camera(H, W, 16)
    # one pass, no process group: the tile path
    assert not nd._collective(1)
    for k, v in pipe(False).render_image(H, W, pose0, K0).items():
        rec[f"one_c2_{k}"] = v.cpu().numpy()
    p4 = pipe(True)
    for k, v in p4.render_image(H, W, pose16, K16).items():
        rec[f"one_c4_{k}"] = v.cpu().numpy()
    rec["one_c4_grid"] = p4.grid.cpu().numpy()
    rec["one_c4_counter"] = np.int64(p4.grid_update_counter)
    params = make_params(0, 2.0, 0.0)
    tr = NerfTrainer(dev, params)
    tr.step(*batch(0, dev))
    rec["one_train"] = flat_params(tr)
    torch.cuda.synchronize()

    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    assert nd._collective(1)
    maps = bench.make_frame_fn(pipe(False), H, W, 0, 1, dev, False)(pose0, K0)
    for k, v in maps.items():
        rec[f"c2_{k}"] = v.cpu().numpy()
    p4 = pipe(True)
    maps = bench.make_frame_fn(p4, H, W, 0, 1, dev, True)(pose16, K16)
    for k, v in maps.items():
        rec[f"c4_{k}"] = v.cpu().numpy()
    rec["c4_grid"] = p4.grid.cpu().numpy()
    rec["c4_counter"] = np.int64(p4.grid_update_counter)
    # a direct all-gather of a known tile (the collective itself, not only its use)
    tile = torch.arange(12 * 2048, device=dev, dtype=torch.float32).reshape(2048, 12)
    full = torch.empty_like(tile)
    dist.all_gather_into_tensor(full, tile)
    rec["allgather_equal"] = np.bool_(torch.equal(full, tile))
    tr = NerfTrainer(dev, params)
    tr.step(*batch(0, dev), group=dist.group.WORLD)
    rec["train"] = flat_params(tr)
    torch.cuda.synchronize()
    np.savez(os.path.join(out, "nccl.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main(sys.argv[1])
