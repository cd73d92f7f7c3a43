"""Deterministic NeRF parameter generator.

Synthetic weights for the 8x256 coarse+fine NeRF MLP, defined by a formula
(splitmix64 counter hash -> uniform in [-1, 1) -> scaled by gain/sqrt(fan_in)),
so the same parameters can be rebuilt bit-for-bit in the fixture-capture
container, in the CPU tests and on the GPU box without shipping a checkpoint.

Parameter names and shapes follow the reference state_dict of
``Network`` (reference ``src/models/nerf/network.py:9-74``, ``:126-159``):
``model.pts_linears.{0..7}``, ``model.views_linears.0``,
``model.feature_linear``, ``model.alpha_linear``, ``model.rgb_linear`` and the
same under ``model_fine.``. The default bound 1/sqrt(fan_in) matches the range
of torch's default ``nn.Linear`` initialisation.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict

import numpy as np

W = 256
D = 8
SKIPS = (4,)
XYZ_FREQ = 10
DIR_FREQ = 4
IN_XYZ = 3 * (1 + 2 * XYZ_FREQ)   # 63
IN_DIR = 3 * (1 + 2 * DIR_FREQ)   # 27


def layer_shapes(prefix: str = "model"):
    """(name, out_features, in_features) in state_dict order for one NeRF MLP."""
    out = []
    for i in range(D):
        if i == 0:
            fin = IN_XYZ
        elif (i - 1) in SKIPS:
            fin = W + IN_XYZ
        else:
            fin = W
        out.append((f"{prefix}.pts_linears.{i}", W, fin))
    out.append((f"{prefix}.views_linears.0", W // 2, W + IN_DIR))
    out.append((f"{prefix}.feature_linear", W, W))
    out.append((f"{prefix}.alpha_linear", 1, W))
    out.append((f"{prefix}.rgb_linear", 3, W // 2))
    return out


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return z ^ (z >> np.uint64(31))


def _uniform(seed: int, tensor_id: int, n: int) -> np.ndarray:
    """n exact float32 values in [-1, 1) with 24-bit resolution."""
    idx = np.arange(n, dtype=np.uint64)
    key = np.uint64((seed & 0xFFFFFFFF) << 32 | (tensor_id & 0xFFFFFFFF))
    with np.errstate(over="ignore"):
        h = _splitmix64(idx ^ _splitmix64(np.full(1, key, dtype=np.uint64))[0])
    top = (h >> np.uint64(40)).astype(np.int64)          # 24 bits
    return ((top.astype(np.float64) / float(1 << 23)) - 1.0).astype(np.float32)


def make_params(seed: int = 0, gain: float = 1.0, alpha_bias: float = 0.0,
                prefixes=("model", "model_fine")) -> "OrderedDict[str, np.ndarray]":
    """Return an ordered dict name -> float32 array with the reference's shapes.

    ``gain`` scales every weight and bias bound; ``alpha_bias`` is added to the
    density head's bias (a dense medium exercises early termination).
    """
    params: "OrderedDict[str, np.ndarray]" = OrderedDict()
    tid = 0
    for p_i, prefix in enumerate(prefixes):
        for name, fout, fin in layer_shapes(prefix):
            bound = np.float32(gain / np.sqrt(fin))
            w = (_uniform(seed, tid, fout * fin) * bound).reshape(fout, fin)
            tid += 1
            b = _uniform(seed, tid, fout) * bound
            tid += 1
            if name.endswith("alpha_linear"):
                b = (b + np.float32(alpha_bias)).astype(np.float32)
            params[name + ".weight"] = w.astype(np.float32)
            params[name + ".bias"] = b.astype(np.float32)
    return params


def params_digest(params) -> str:
    """sha256 over the concatenated little-endian float32 bytes, in order."""
    h = hashlib.sha256()
    for k, v in params.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v, dtype="<f4").tobytes())
    return h.hexdigest()


def load_into_network(net, params) -> None:
    """Copy generated params into a torch Network (``model.*``/``model_fine.*``)."""
    import torch
    sd = net.state_dict()
    missing = [k for k in sd if k not in params]
    if missing:
        raise KeyError(f"generated params lack {missing[:4]}")
    with torch.no_grad():
        for k, t in sd.items():
            src = torch.from_numpy(np.ascontiguousarray(params[k]))
            if tuple(src.shape) != tuple(t.shape):
                raise ValueError(f"{k}: shape {tuple(src.shape)} != {tuple(t.shape)}")
            t.copy_(src)


def make_occupancy_grid(seed: int = 0, res: int = 128, radius: float = 1.2,
                        noise: float = 0.1) -> np.ndarray:
    """Deterministic stand-in for the reference's ESS grid initialisation.

    Reference ``VR:830-873``: bool[res^3] = (|normalised coord| <= 1.2) OR
    (rand < 0.1). The random term here is the counter hash instead of
    ``torch.rand`` so the grid is reproducible everywhere.
    """
    ax = np.arange(res, dtype=np.float32)
    g = (ax / np.float32(res - 1)) * np.float32(2.0) - np.float32(1.0)
    x, y, z = np.meshgrid(g, g, g, indexing="ij")
    dist = np.sqrt(x * x + y * y + z * z)
    sphere = dist <= np.float32(radius)
    r = (_uniform(seed, 0x6D1D, res ** 3).reshape(res, res, res) + np.float32(1.0)) * np.float32(0.5)
    return sphere | (r < np.float32(noise))
