"""The real sharded render path (and the data-parallel training step) on the
GPU: two fresh processes (ranks over
gloo, both on cuda:0) run bench.py's own frame function
(``bench.make_frame_fn``: C2 row bands + all-gather; C4 2048-ray chunks dealt
round-robin with the ESS grid's self-updates replayed) and the
gathered frames must be bit-equal to the one-pass frame of one process.

Reference semantics: the sequential chunk loop VR:147-205, the grid
self-update VR:1147-1157 and the chunk-wide ERT rule VR:1115-1123. C4 runs at
grid call counters 0 and 498, so updating chunks fall inside the frame on
either rank (tests/dist_frame_worker.py). RCCL itself needs one GPU per rank:
the multi-GPU runs are the driver's; this covers every other part of the N > 1
path on the HIP renderer (band / chunk partition, replays, gather, reassembly).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))
WORLD = 2
KEYS = ("rgb_map_0", "disp_map_0", "acc_map_0", "depth_map_0",
        "rgb_map", "disp_map", "acc_map", "depth_map")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def ranks(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    out = str(tmp_path_factory.mktemp("dist"))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE=str(WORLD))
    procs = []
    for r in range(WORLD):
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(HERE, "dist_frame_worker.py"), out],
            env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
            stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=100)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, log) in enumerate(zip(procs, logs)):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{log[-3000:]}"
    return [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(WORLD)]


def _equal(a, b):
    a = np.asarray(a)
    return np.array_equal(a.reshape(-1), np.asarray(b).reshape(-1), equal_nan=True)


def test_c2_row_bands_equal_one_pass_frame(ranks):
    one = ranks[0]
    for r, rec in enumerate(ranks):
        for k in KEYS:
            assert _equal(rec[f"c2_{k}"], one[f"one_c2_{k}"]), (r, k)


@pytest.mark.parametrize("counter", [0, 498])
def test_c4_interleaved_chunks_equal_one_pass_frame(ranks, counter):
    one = ranks[0]
    p = f"c4_{counter}_"
    for r, rec in enumerate(ranks):
        for k in KEYS:
            assert _equal(rec[p + k], one["one_" + p + k]), (r, k)
        # every rank leaves the frame with the sequential loop's grid and counter
        assert np.array_equal(rec[p + "grid"], one["one_" + p + "grid"]), r
        assert int(rec[p + "counter"]) == int(one["one_" + p + "counter"]) == counter + 2 * 313
    # the ranks' own chunks partition the frame: their evaluated samples add up
    assert sum(int(rec[p + "evaluated"]) for rec in ranks) == int(one["one_" + p + "evaluated"])
    # the C4 frame really terminates rays (acc = 0, disp = NaN from the chunk rule)
    assert np.isnan(one["one_" + p + "disp_map"]).any()


@pytest.fixture(scope="module")
def train_ranks(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    out = str(tmp_path_factory.mktemp("dist_train"))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE=str(WORLD))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_train_worker.py"), out],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(WORLD)]
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=100)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, log) in enumerate(zip(procs, logs)):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{log[-3000:]}"
    return [dict(np.load(os.path.join(out, f"train_rank{r}.npz"))) for r in range(WORLD)]


def test_data_parallel_train_step_equals_mean_gradient_step(train_ranks):
    """bench.py's C3 step at world 2 (each rank its own batch and draws, the
    gradients all-reduced in one flat bucket, then clip + Adam): every rank ends
    with the same parameters, bit for bit those of one process that averages
    the two batches' gradients itself before the same Adam step."""
    ref = train_ranks[0]["ref_params"]
    for r, rec in enumerate(train_ranks):
        assert np.array_equal(rec["params"], ref), r
    assert np.isfinite(ref).all()
