#!/usr/bin/env python3
"""Per-fixture end-to-end parity report of the HIP renderer (GPU box).

For every golden fixture and both MLP precisions: coarse-map max errors vs the
reference's golden render and the fine-map per-ray gate report
(``tests/goldlib.py fine_gate``) next to the reference's own reparametrisation
floor. One JSON object per line; ``--out FILE`` also writes the list.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "nerf-rep_for_test_amd"), REPO):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    from conftest import golden_names
    from goldlib import fine_gate, grid_of, load, max_err, params_of, rel_err
    from nerfhip.render import NerfPipeline
    dev = torch.device("cuda:0")
    rows = []
    for name in golden_names():
        z = load(name)
        s = load("s_" + name)
        for prec in ("fp32", "f16x3"):
            pipe = NerfPipeline(dev, N_samples=int(z["N_samples"]),
                                N_importance=int(z["N_importance"]), near=float(z["near"]),
                                far=float(z["far"]), lindisp=bool(z["lindisp"]),
                                white_bkgd=bool(z["white_bkgd"]), enable_ess=bool(z["enable_ess"]),
                                enable_ert=bool(z["enable_ert"]),
                                ert_threshold=float(z["ert_threshold"]), mlp_precision=prec)
            pipe.set_weights(params_of(z))
            g = grid_of(z)
            if g is not None:
                pipe.set_grid(g)
            pipe.grid_update_counter = int(z["grid_counter_in"])
            tr = (torch.from_numpy(z["t_rand"]).to(dev) if "t_rand" in z else None)
            res = {k: v.cpu().numpy() for k, v in
                   pipe.render_image(int(z["H"]), int(z["W"]), z["pose"], z["K"],
                                     t_rand=tr).items()}
            n = int(z["H"]) * int(z["W"])
            row = {"fixture": name, "precision": prec, "rays": n,
                   "coarse_rgb_max_abs": max_err(res["rgb_map_0"], z["out_rgb_map_0"].reshape(n, 3)),
                   "coarse_depth_max_rel": rel_err(res["depth_map_0"],
                                                   z["out_depth_map_0"].reshape(n))}
            if int(z["N_importance"]) > 0:
                ok, rep = fine_gate(res, z, s)
                row.update({"fine_gate_ok": bool(ok), **rep})
            rows.append(row)
            print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
