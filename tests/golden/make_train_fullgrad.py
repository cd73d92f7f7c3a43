"""Element-wise gradient fixtures of the reference training step (survey container).

The train goldens (make_train_golden.py) keep each gradient's norm, sum and
first 64 values. This script re-runs the reference training step of each of
them (asserting the same norms bit for bit) and stores every gradient tensor,
plus the reference's own element-wise noise floor: the step is re-run on
K = 16 exact reparametrisations of the network (hidden units permuted, half
with a +-1-ulp libm; make_train_sensitivity.py), each variant's gradients are
compared with the golden's gradients permuted the same way (a permutation of
the units permutes the gradient exactly in real arithmetic), and per tensor
the largest relative L2 distance ||g_variant - P g_gold|| / ||g_gold|| is kept:

  tests/golden/tg_<fixture>.npz: g__<param> float32 (full loss),
      gc__<param> float32 (coarse loss), gdist__<param> / gcdist__<param>
      (float64: the reference's largest relative L2 distance from itself),
      k_variants

Only numbers are stored.

    python tests/golden/make_train_fullgrad.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402
import make_sensitivity as MS  # noqa: E402
import make_train_golden as MT  # noqa: E402
from make_train_sensitivity import K_VARIANTS, _ulp_libm_ad  # noqa: E402


def _rel(a, b):
    nb = float(np.linalg.norm(b))
    return float(np.linalg.norm(a - b)) / max(nb, 1e-30)


def main():
    import torch
    cfg, Network, vr = MG._import_reference()
    with open(os.path.join(MG.REF, "data", "nerf_synthetic", "lego", "transforms_test.json")) as f:
        meta = json.load(f)
    for name, spec in MT.SPECS.items():
        gold = dict(np.load(os.path.join(HERE, name + ".npz")))
        params = MG.make_params(*spec["w"])
        rec = MT.capture(name, spec, cfg, Network, vr, meta, params=params, write=False, full=True)
        names = [str(k) for k in gold["param_names"]]
        for k in names:
            assert float(rec["gnorm__" + k]) == float(gold["gnorm__" + k]), k
        g = {k: rec["gfull__" + k] for k in names}
        gc = {k: rec["gcfull__" + k] for k in names if "gcfull__" + k in rec}
        dist = {k: 0.0 for k in g}
        cdist = {k: 0.0 for k in gc}
        for v in range(K_VARIANTS):
            orig = _ulp_libm_ad(torch, 300 + v) if v >= K_VARIANTS // 2 else None
            try:
                rv = MT.capture(name, spec, cfg, Network, vr, meta,
                                params=MS.permute_params(params, 100 + v), write=False, full=True)
            finally:
                for k, fn in (orig or {}).items():
                    setattr(torch, k, fn)
            pg = MS.permute_params(g, 100 + v)       # the golden's gradients, permuted alike
            pgc = MS.permute_params({**g, **gc}, 100 + v)
            for k in g:
                dist[k] = max(dist[k], _rel(rv["gfull__" + k], pg[k]))
            for k in gc:
                cdist[k] = max(cdist[k], _rel(rv["gcfull__" + k], pgc[k]))
        out = {"g__" + k: v.astype(np.float32) for k, v in g.items()}
        out.update({"gc__" + k: v.astype(np.float32) for k, v in gc.items()})
        out.update({"gdist__" + k: np.float64(v) for k, v in dist.items()})
        out.update({"gcdist__" + k: np.float64(v) for k, v in cdist.items()})
        out["k_variants"] = K_VARIANTS
        path = os.path.join(HERE, "tg_" + name + ".npz")
        np.savez_compressed(path, **out)
        worst = sorted(dist.items(), key=lambda kv: -kv[1])[:4]
        print(path, f"{os.path.getsize(path) / 2**20:.1f} MiB; worst full-loss distances",
              [(k, round(v, 5)) for k, v in worst], flush=True)


if __name__ == "__main__":
    main()
