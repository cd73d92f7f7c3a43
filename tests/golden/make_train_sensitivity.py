"""The reference training step's own float32 noise floor per gradient tensor
(survey container).

The gradient of the full loss reaches the coarse network through the fine
samples (VR:239-268, not detached): d loss_fine / d z_fine is a derivative of
the fine MLP along the ray, where the encoding's sin(2^9 x) makes it a
rapidly varying function of the sample position, and d z_fine / d weights
carries 1 / (cdf[above] - cdf[below]) (down to 1e-5). Those norms are
ill-conditioned in the reference's own float32 rounding. This script re-runs
the reference training step of each train golden (make_train_golden.py) on 16
exact reparametrisations of the network (hidden units permuted, as
make_sensitivity.py; half of them with a +-1-ulp libm whose perturbation is
transparent to autograd) and stores per parameter tensor the largest relative
deviation of its gradient norm (full loss and coarse loss) from the golden's:

  tests/golden/ts_<fixture>.npz: gnorm_spread__<param>, gcnorm_spread__<param>,
                                 loss_spread, k_variants

Permutation leaves every gradient norm unchanged in real arithmetic. Only
numbers are stored.

    python tests/golden/make_train_sensitivity.py
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

K_VARIANTS = 16


def _ulp_libm_ad(torch, seed):
    """sin/cos/exp/sigmoid moved by +-1 ulp at random; the gradient is the
    unperturbed function's (the shift is a constant to autograd)."""
    gen = torch.Generator().manual_seed(seed)
    orig = {k: getattr(torch, k) for k in ("sin", "cos", "exp", "sigmoid")}

    def wrap(fn):
        def f(x, *a, **kw):
            y = fn(x, *a, **kw)
            d = torch.randint(0, 3, y.shape, generator=gen) - 1
            to = torch.where(d > 0, torch.full_like(y, float("inf")),
                             torch.full_like(y, float("-inf")))
            yn = torch.where(d == 0, y.detach(), torch.nextafter(y.detach(), to))
            return y + (yn - y.detach())
        return f
    for k, fn in orig.items():
        setattr(torch, k, wrap(fn))
    return orig


def main():
    import torch
    cfg, Network, vr = MG._import_reference()
    with open(os.path.join(MG.REF, "data", "nerf_synthetic", "lego", "transforms_test.json")) as f:
        meta = json.load(f)
    for name, spec in MT.SPECS.items():
        gold = dict(np.load(os.path.join(HERE, name + ".npz")))
        params = MG.make_params(*spec["w"])
        names = [str(k) for k in gold["param_names"]]
        spread = {k: 0.0 for k in names}
        cspread = {k: 0.0 for k in names if "gcnorm__" + k in gold}
        lspread = 0.0
        for v in range(K_VARIANTS):
            orig = _ulp_libm_ad(torch, 300 + v) if v >= K_VARIANTS // 2 else None
            try:
                rec = MT.capture(name, spec, cfg, Network, vr, meta,
                                 params=MS.permute_params(params, 100 + v), write=False)
            finally:
                for k, fn in (orig or {}).items():
                    setattr(torch, k, fn)
            for k in names:
                ref = float(gold["gnorm__" + k])
                spread[k] = max(spread[k], abs(float(rec["gnorm__" + k]) - ref) / max(ref, 1e-30))
            for k in cspread:
                ref = float(gold["gcnorm__" + k])
                cspread[k] = max(cspread[k],
                                 abs(float(rec["gcnorm__" + k]) - ref) / max(ref, 1e-30))
            lspread = max(lspread, abs(float(rec["loss"]) - float(gold["loss"])) / float(gold["loss"]))
        out = {"gnorm_spread__" + k: np.float64(v) for k, v in spread.items()}
        out.update({"gcnorm_spread__" + k: np.float64(v) for k, v in cspread.items()})
        out.update(loss_spread=np.float64(lspread), k_variants=K_VARIANTS)
        np.savez_compressed(os.path.join(HERE, "ts_" + name + ".npz"), **out)
        worst = sorted(spread.items(), key=lambda kv: -kv[1])[:4]
        print(name, "loss spread %.2e" % lspread, "worst full-loss norm spreads",
              [(k, round(v, 4)) for k, v in worst], flush=True)


if __name__ == "__main__":
    main()
