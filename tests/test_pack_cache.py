"""The packing launch's device-table cache (nerfhip.train_mlp._launch_packs),
on the CPU: every packer rebuild allocates new output buffers (the streams,
scales, maxima, the fold's Wc / bc, the head), so the cached table of an
earlier build must never serve a later one -- also when the parameter
addresses repeat (A, then B, then A again). A stale table would make the
device pack kernels write into the freed buffers of the old build (a
use-after-free: silent corruption of whatever reuses that memory, e.g. another
table of device pointers, then an illegal address) and leave the live stream
unpacked. The launch itself is replaced by a recorder here."""
import torch

from nerfhip import train_mlp as T


def test_rebuild_never_reuses_an_old_builds_table(monkeypatch):
    from src.models.nerf.network import NeRF
    launched = []
    monkeypatch.setattr(T, "call", lambda name, *a: launched.append((name, a)))
    monkeypatch.setattr(T, "_fold", lambda packers: None)
    monkeypatch.setattr(T, "_PACK_TABLES", {})
    monkeypatch.setattr(T._lib, "stream_of", lambda device=None: 0)
    torch.manual_seed(0)
    pa = dict(zip(T.PARAM_NAMES, T.mlp_params(NeRF())))
    pb = dict(pa, **{"rgb_linear.weight": pa["rgb_linear.weight"].detach().clone()})
    net = T.X3NetPacker("cpu")
    tables, streams = [], []
    for p in (pa, pb, pa):
        net._ensure_built(p)
        T._launch_packs([net])
        tables.append(launched[-1][1][0])      # the descriptor table's address
        streams.append(net.fwd.stream.data_ptr())
    assert net.gen == 3
    # the third build owns new buffers, and its launch got a table made for it
    assert tables[2] != tables[0] and tables[2] != tables[1]
    # every output address in the live table lies in the live build's buffers
    import numpy as np
    descs = T._PACK_TABLES[((id(net), net.gen),)][0]
    recs = np.frombuffer(descs.numpy().tobytes(), dtype=np.dtype(T._DESC_FIELDS))
    live = [(t.data_ptr(), t.data_ptr() + t.numel() * t.element_size())
            for t in (net.fwd.stream, net.bwd.stream) + tuple(
                o for o, _, _ in getattr(net.bwd, "out", {}).values())]
    for r in recs:
        o = int(r["out"])
        assert any(a <= o < b for a, b in live), hex(o)


def test_unchanged_parameters_reuse_the_table(monkeypatch):
    from src.models.nerf.network import NeRF
    launched = []
    monkeypatch.setattr(T, "call", lambda name, *a: launched.append((name, a)))
    monkeypatch.setattr(T, "_fold", lambda packers: None)
    monkeypatch.setattr(T, "_PACK_TABLES", {})
    monkeypatch.setattr(T._lib, "stream_of", lambda device=None: 0)
    pa = dict(zip(T.PARAM_NAMES, T.mlp_params(NeRF())))
    net = T.X3NetPacker("cpu")
    for _ in range(3):
        net._ensure_built(pa)
        T._launch_packs([net])
    assert net.gen == 1 and len(T._PACK_TABLES) == 1
    assert len({a[0] for _, a in launched}) == 1
