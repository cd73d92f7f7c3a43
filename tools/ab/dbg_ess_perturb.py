"""debug: does t_rand reach the ESS sampler through render_image / render_chunks?"""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from nerfhip.render import NerfPipeline
from nerfhip.synthetic import make_occupancy_grid, make_params
from goldlib import load
dev = torch.device("cuda:0")
H = W = 96
params = make_params(0, 3.0, 1.0)
grid = make_occupancy_grid(4, 128, 0.5, 0.01)
cams = load("lego_test_cameras")
f = 0.5 * 800 / np.tan(0.5 * float(cams["camera_angle_x"]))
K = np.array([[f, 0, 400 - 352], [0, f, 400 - 352], [0, 0, 1]], np.float32)
pose = cams["poses"][0]
tr = torch.rand((H * W, 64), device=dev, generator=torch.Generator(device=dev).manual_seed(5))
for ess in (False, True):
    outs = []
    for t in (None, tr):
        p = NerfPipeline(dev, N_samples=64, N_importance=128, enable_ess=ess, enable_ert=ess, ert_threshold=0.01)
        p.set_weights(params)
        p.set_grid(grid)
        p.grid_update_counter = 496
        p.capture_zall = []
        o = p.render_image(H, W, pose, K, t_rand=t)
        outs.append((o, torch.cat(p.capture_zall)))
    (a, za), (b, zb) = outs
    print("ess", ess, "zall equal", torch.equal(za, zb), "rgb0 equal", torch.equal(a["rgb_map_0"], b["rgb_map_0"]),
          "rgb equal", torch.equal(a["rgb_map"], b["rgb_map"]), "acc0 mean", float(a["acc_map_0"].mean()),
          "max |d rgb0|", float((a["rgb_map_0"] - b["rgb_map_0"]).abs().max()))
