"""Training step (C3): the differentiable pieces match the oracle on the CPU;
the device-only trainer refuses a CPU device. GPU parity: tests/test_gpu_train.py."""
import numpy as np
import pytest
import torch

from nerfhip import train as T
from nerfhip._lib import NerfHipError
from goldlib import load, params_of
from oracle import nerf_oracle as O


def test_freq_encode_matches_oracle():
    x = np.random.default_rng(0).uniform(-3, 3, (50, 3)).astype(np.float32)
    for L in (10, 4):
        got = T.freq_encode(torch.from_numpy(x), L).numpy()
        np.testing.assert_allclose(got, O.embed(x, L), atol=2e-6, rtol=0)


@pytest.mark.parametrize("white", [True, False])
def test_composite_matches_oracle(white):
    rng = np.random.default_rng(1)
    n, S = 40, 64
    raw = rng.normal(0, 2, (n, S, 4)).astype(np.float32)
    z = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    got = T.composite(torch.from_numpy(raw), torch.from_numpy(z), torch.from_numpy(d), white)
    ref = O.raw2outputs(raw, z, d, white)
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g.numpy(), r, atol=2e-6, rtol=1e-5)


def test_sample_pdf_matches_oracle_and_has_gradients():
    rng = np.random.default_rng(2)
    n = 30
    z = np.sort(rng.uniform(2, 6, (n, 64)), 1).astype(np.float32)
    mids = (np.float32(0.5) * (z[:, 1:] + z[:, :-1])).astype(np.float32)
    w = (rng.random((n, 64)) ** 3).astype(np.float32)
    u = rng.random((n, 128)).astype(np.float32)
    wt = torch.from_numpy(w[:, 1:-1].copy()).requires_grad_(True)
    got = T.sample_pdf(torch.from_numpy(mids), wt, torch.from_numpy(u))
    ref = O.sample_fine(mids, w[:, 1:-1], u)
    np.testing.assert_allclose(got.detach().numpy(), ref, atol=1e-5, rtol=0)
    got.sum().backward()             # no detach: the fine loss reaches the coarse net
    assert torch.isfinite(wt.grad).all() and wt.grad.abs().sum() > 0


def test_trainer_refuses_cpu():
    with pytest.raises(NerfHipError):
        T.NerfTrainer("cpu", {})


def test_train_math_matches_reference_backward():
    """The trainer's differentiable core on the CPU reproduces the reference's
    own training forward/backward (t1 golden): the loss bit-for-bit, every
    parameter gradient to 1e-5 relative."""
    from src.models.nerf.network import NeRF
    z = load("t1_train_step")
    p = params_of(z)
    nets = {"model": NeRF(), "model_fine": NeRF()}
    with torch.no_grad():
        for pref, m in nets.items():
            for k, q in m.named_parameters():
                q.copy_(torch.from_numpy(np.asarray(p[f"{pref}.{k}"])))
    ro, rd = O.camera_rays(int(z["H"]), int(z["W"]), z["pose"], z["K"])
    zc = O.stratify(np.broadcast_to(O.coarse_depths(2.0, 6.0, 64, False), (ro.shape[0], 64)),
                    z["t_rand"])
    out = T.render_train(nets["model"], nets["model_fine"], torch.from_numpy(ro),
                         torch.from_numpy(rd), torch.from_numpy(zc), torch.from_numpy(z["u"]))
    losses = T.mse_losses(out, torch.from_numpy(z["gt"].reshape(-1, 3)))
    assert losses["loss"].item() == float(z["loss"])
    losses["loss"].backward()
    for pref, m in nets.items():
        for k, q in m.named_parameters():
            name = f"{pref}.{k}"
            ref = float(z["gnorm__" + name])
            assert abs(q.grad.double().norm().item() - ref) <= 1e-5 * ref, name
            np.testing.assert_allclose(q.grad.reshape(-1)[:64].numpy(), z["ghead__" + name],
                                       atol=1e-5 * ref, rtol=0)


@pytest.mark.parametrize("white", [True, False])
def test_composite_ert_matches_oracle_per_chunk(white):
    """nerfhip.train.composite_ert (the training-mode ERT, autograd) vs the
    oracle's VR:1089-1133 over 2048-ray chunks: a chunk with terminating rays
    (argmax quirk), one where a single ray terminates, one where none does."""
    rng = np.random.default_rng(3)
    n, S = 2048 * 2 + 300, 48
    raw = rng.normal(0, 2, (n, S, 4)).astype(np.float32)
    raw[..., 3] = rng.normal(2.0, 3.0, (n, S)).astype(np.float32)
    raw[2048:, :, 3] = -5.0
    raw[2048 + 9, :, 3] = 40.0
    z = np.sort(rng.uniform(2, 6, (n, S)), 1).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t_raw = torch.from_numpy(raw).requires_grad_(True)
    got = T.composite_ert(t_raw, torch.from_numpy(z), torch.from_numpy(d), 0.01, white)
    for c0 in range(0, n, 2048):
        sl = slice(c0, min(n, c0 + 2048))
        ref = O.raw2outputs_ert(raw[sl], z[sl], d[sl], 0.01, white)
        for g, r in zip(got, ref):
            np.testing.assert_allclose(g.detach().numpy()[sl], r, atol=2e-6, rtol=1e-5)
    got[0].sum().backward()
    assert torch.isfinite(t_raw.grad).all()
    g1 = torch.cat([t_raw.grad[2048:2048 + 9], t_raw.grad[2048 + 10:4096]])
    assert (g1 == 0).all()          # chunk 1: every other ray's weights zeroed (quirk 1)


@pytest.mark.parametrize("name", ["t1_train_step", "t2_train_ess_ert"])
def test_full_gradient_fixture_consistent(name):
    """tg_<name>.npz (make_train_fullgrad.py) holds the golden step's gradients
    element by element: their norms / sums / first values are the golden's, and
    the reference's self-distance under reparametrisation is a sane fraction."""
    from goldlib import load
    z, tg = load(name), load("tg_" + name)
    for k in [str(s) for s in z["param_names"]]:
        g = tg["g__" + k].astype(np.float64)
        assert abs(np.linalg.norm(g) - float(z["gnorm__" + k])) <= 1e-6 * float(z["gnorm__" + k]) + 1e-12
        assert np.allclose(g.reshape(-1)[:64], z["ghead__" + k], rtol=0, atol=1e-30 + 1e-7 * np.abs(g).max())
        assert 0.0 <= float(tg["gdist__" + k]) < 0.2
        if "gcnorm__" + k in z:
            gc = tg["gc__" + k].astype(np.float64)
            assert abs(np.linalg.norm(gc) - float(z["gcnorm__" + k])) <= 1e-6 * float(z["gcnorm__" + k]) + 1e-12
