"""Capture the reference's spiral camera path (run in the survey container).

Calls the reference ``Renderer.generate_spiral_poses`` (volume_renderer.py:359-419,
plain numpy) on the lego test poses and stores the result.

    python tests/golden/make_path_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def main():
    cfg, Network, vr = mg._import_reference()
    meta = json.load(open(os.path.join(mg.REF, "data/nerf_synthetic/lego/transforms_test.json")))
    poses = np.array([f["transform_matrix"] for f in meta["frames"]], np.float32)
    rend = vr.Renderer.__new__(vr.Renderer)     # the method only reads its arguments
    out = {}
    for n, rots, zr in ((30, 2, 0.5), (7, 1, 0.25)):
        out[f"spiral_{n}_{rots}_{zr}"] = vr.Renderer.generate_spiral_poses(rend, poses, n, rots, zr)
    np.savez_compressed(os.path.join(HERE, "p1_spiral_poses.npz"), **out)
    print("wrote", list(out))


if __name__ == "__main__":
    main()
