"""Round-6 study: the C4 frame's list-MLP launches (one per ERT depth segment,
NerfPipeline.mlp_ert) -- samples per launch, time per launch and the samples/s
each reaches, to size the persistent kernel's tail on small launches.
    python tools/ab/c4_launch_sizes.py [segment]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))
sys.path.insert(0, REPO)
from bench import DEFAULT_CKPT, lego_camera, make_frame_fn   # noqa: E402
from nerfhip.checkpoint import network_params                 # noqa: E402
from nerfhip.render import NerfPipeline                       # noqa: E402
from nerfhip.synthetic import make_occupancy_grid             # noqa: E402

seg = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
params = {k: v.numpy() for k, v in network_params(DEFAULT_CKPT).items()}
pipe = NerfPipeline(dev, N_samples=64, N_importance=128, near=2.0, far=6.0,
                    mlp_precision="f16x3", enable_ess=True, enable_ert=True,
                    ert_threshold=0.01, ert_segment=seg)
pipe.set_weights(params)
pipe.set_grid(make_occupancy_grid(0, 128, 1.2, 0.1))
frame = make_frame_fn(pipe, 800, 800, 0, 1, dev, True)
frame(*lego_camera(800, 800, 0))
torch.cuda.synchronize()
pipe.timer = []
frame(*lego_camera(800, 800, 1))
torch.cuda.synchronize()
rows = []
for e0, e1, cnt, _ in pipe.timer:
    n = int(cnt.item()) if torch.is_tensor(cnt) else int(cnt)
    rows.append((n, e0.elapsed_time(e1)))
pipe.timer = None
rows = np.array(rows, np.float64)
n, ms = rows[:, 0], rows[:, 1]
tiles = np.ceil(n / 128)
print(f"segment {seg}: {len(rows)} launches, {ms.sum():.1f} ms, {n.sum() / 1e6:.2f} M samples")
edges = [0, 256 * 128, 2 * 256 * 128, 8 * 256 * 128, 32 * 256 * 128, 1e12]
for a, b in zip(edges[:-1], edges[1:]):
    m = (n >= a) & (n < b)
    if m.any():
        print(f"  samples [{int(a):>9d}, {b:>9.0f}): {m.sum():3d} launches, {ms[m].sum():7.1f} ms, "
              f"{n[m].sum() / ms[m].sum() / 1e3:7.2f} Msamples/ms... per launch "
              f"{ms[m].mean():6.3f} ms, tiles/WG {tiles[m].mean() / 256:6.2f}")
best = (n / ms).max()
print(f"  time at the best launch's rate: {(n / best).sum():.1f} ms of {ms.sum():.1f}")
