"""GPU study: does a K step of the batched weight-gradient launch cost the same
for a light tile as for a full one? Times nerf_x3_wgrad_batch_z (via
WgradBatch, T16 operands, P = 1024 x 192) on batches of 11 tiles of one shape
each: full 256 x 256, 256 x 64 (the encoding tiles), 144 x 256 (the views
tile), 16 x 128 (an rgb-like head) -- same workgroup split (11 tiles x Z).

    python tools/ab/wgrad_tiles_bench.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))


def main():
    from nerfhip.train_mlp import BlockRows, WgradBatch
    dev = torch.device("cuda:0")
    P = 1024 * 192
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N in ((256, 256), (256, 64), (144, 256), (16, 128)):
        ops = []
        for _ in range(11):
            A = BlockRows.from_dense(torch.randn((M, P), device=dev, generator=g))
            B = BlockRows.from_dense(torch.relu(torch.randn((N, P), device=dev, generator=g)))
            ops.append((A, B))
        one = torch.ones(1, device=dev)

        def run():
            wb = WgradBatch(dev)
            for A, B in ops:
                wb.add(A, B, one, one, with_bias=True)
            return wb.results()
        run()
        ts = []
        for rep in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            if rep >= 2:
                ts.append(e0.elapsed_time(e1))
        ts.sort()
        ms = ts[len(ts) // 2]
        nbytes = 11 * (M + N) * P * 4
        print(f"11 tiles of {M:3d} x {N:3d}: {ms * 1e3:7.1f} us  "
              f"({nbytes / ms / 1e9:5.2f} TB/s of operands)", flush=True)
        del ops


if __name__ == "__main__":
    main()
