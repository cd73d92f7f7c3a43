"""RCCL on the hardware and bench.py's own N-rank launch on a one-GPU box.

* ``init_process_group("nccl", device_id=cuda:0)`` at world 1 forces
  nerfhip.dist's collective branch (it gathers whenever a group is up): the C2
  row-band frame through ``all_gather_into_tensor`` and the C4 interleaved-chunk
  frame through the all-gather + ``index_select`` reassembly must be bit-equal
  to the one-pass frames rendered before the group existed, with the final
  occupancy grid and counter equal; the data-parallel train step's flat
  all-reduce over RCCL leaves the parameters bit-equal to the step without a
  group (tests/nccl_frame_worker.py, a fresh process).
* ``NERF_DIST_BACKEND=gloo python bench.py --gpus 2 --config c3`` starts its
  own two ranks (sharing the one GPU) and reports n_gpus 2; with RCCL the same
  command exits non-zero on a one-GPU box instead of timing one rank.

Reference: SURVEY §8e (rows shard by image tile, one gather of final pixels);
the reference's only NCCL use is train.py:115-120 (DDP's gradient all-reduce).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
KEYS = ("rgb_map_0", "disp_map_0", "acc_map_0", "depth_map_0",
        "rgb_map", "disp_map", "acc_map", "depth_map")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _clean_env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                        "NERF_DIST_BACKEND")}
    env.update(kw)
    return env


@pytest.fixture(scope="module")
def nccl(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    out = str(tmp_path_factory.mktemp("nccl"))
    env = _clean_env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                     MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, os.path.join(HERE, "nccl_frame_worker.py"), out],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    return dict(np.load(os.path.join(out, "nccl.npz")))


def _equal(a, b):
    return np.array_equal(np.asarray(a).reshape(-1), np.asarray(b).reshape(-1), equal_nan=True)


def test_rccl_allgather_of_a_tile(nccl):
    assert bool(nccl["allgather_equal"])


def test_rccl_row_band_frame_equals_one_pass(nccl):
    for k in KEYS:
        assert _equal(nccl[f"c2_{k}"], nccl[f"one_c2_{k}"]), k


def test_rccl_interleaved_chunk_frame_equals_one_pass(nccl):
    for k in KEYS:
        assert _equal(nccl[f"c4_{k}"], nccl[f"one_c4_{k}"]), k
    assert np.array_equal(nccl["c4_grid"], nccl["one_c4_grid"])
    assert int(nccl["c4_counter"]) == int(nccl["one_c4_counter"]) == 2 * 313
    assert np.isnan(nccl["one_c4_disp_map"]).any()   # the frame terminates rays


def test_rccl_train_allreduce_equals_step_without_group(nccl):
    assert np.array_equal(nccl["train"], nccl["one_train"])


def test_bench_self_launches_two_ranks_on_one_gpu():
    """The driver's `python bench.py --gpus N` form: no torchrun, the script
    starts N ranks itself (gloo rehearsal: both ranks on the one GPU)."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--config", "c3", "--steps", "3", "--warmup", "3"],
                       env=_clean_env(NERF_DIST_BACKEND="gloo"), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["scaling"] == "weak"
    assert rec["value"] > 0 and np.isfinite(rec["loss_last"])


def test_bench_refuses_more_rccl_ranks_than_gpus():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    n = torch.cuda.device_count() + 1
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n),
                        "--steps", "1"], env=_clean_env(), capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 2 and "visible GPU" in r.stderr, r.stderr[-2000:]
    assert not r.stdout.strip()
