"""One rank of tests/test_gpu_dist.py's data-parallel training case: the C3
step of bench.py (``NerfTrainer.step(..., group=WORLD)``: forward, backward,
one flat all-reduce of the gradients, clip + Adam) in a fresh process, ranks
sharing cuda:0 over gloo.

    RANK=r WORLD_SIZE=P MASTER_ADDR=127.0.0.1 MASTER_PORT=... \
        python tests/dist_train_worker.py <out_dir>

Every rank starts from the same weights and steps once on its own 256-ray batch
(its own perturb / fine-u draws); rank 0 then recomputes the step in one
process: each batch's gradients (the same forward / backward), their mean,
then the same Adam. Writes <out_dir>/train_rank<r>.npz: the flattened
parameters after the step, and on rank 0 the one-process reference's.
Reference semantics: trainers/nerf.py:39-76, trainer.py:57-60 per rank; the
all-reduce is SURVEY §8e's data-parallel exchange.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))

NRAYS = 256


def batch(rank, dev):
    import torch
    g = np.random.default_rng(100 + rank)
    o = g.uniform(-0.5, 0.5, (NRAYS, 3)).astype(np.float32) + np.array([0, 0, 4.0], np.float32)
    d = g.normal(size=(NRAYS, 3)).astype(np.float32) * np.array([0.3, 0.3, 1.0], np.float32)
    d[:, 2] = -np.abs(d[:, 2]) - 0.5
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    target = g.uniform(0, 1, (NRAYS, 3)).astype(np.float32)
    t_rand = g.uniform(0, 1, (NRAYS, 64)).astype(np.float32)
    u = g.uniform(0, 1, (NRAYS, 128)).astype(np.float32)
    return [torch.from_numpy(a).to(dev) for a in (o, d, target, t_rand, u)]


def flat_params(tr):
    return np.concatenate([p.detach().cpu().numpy().reshape(-1) for p in tr.parameters()])


def main(out):
    import torch
    import torch.distributed as dist
    from nerfhip.synthetic import make_params
    from nerfhip.train import NerfTrainer
    from nerfhip.train_mlp import prepack

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    params = make_params(0, 2.0, 0.0)
    tr = NerfTrainer(dev, params)
    ro, rd, target, t_rand, u = batch(rank, dev)
    tr.step(ro, rd, target, t_rand, u, group=dist.group.WORLD)
    torch.cuda.synchronize()
    rec = {"params": flat_params(tr)}
    if rank == 0:   # the same step in one process: both batches' gradients, their mean
        ref = NerfTrainer(dev, params)
        grads = []
        for r in range(world):
            ro, rd, target, t_rand, u = batch(r, dev)
            ref.opt.zero_grad(set_to_none=True)
            prepack([ref.coarse, ref.fine])
            ref.loss(ref.forward(ro, rd, t_rand, u), target)["loss"].backward()
            grads.append([p.grad.detach().clone() for p in ref.parameters()])
        for i, p in enumerate(ref.parameters()):
            s = grads[0][i].clone()
            for r in range(1, world):
                s += grads[r][i]
            p.grad = s / world
        ref.opt.step()
        torch.cuda.synchronize()
        rec["ref_params"] = flat_params(ref)
    np.savez(os.path.join(out, f"train_rank{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
