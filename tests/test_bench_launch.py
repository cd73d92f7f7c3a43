"""bench.py's own multi-rank launch, on the CPU (the driver's
`python bench.py --gpus N`): with no torchrun environment the script starts N
rank processes itself, rank 0 prints the one JSON line with n_gpus = N, and a
--gpus the launch cannot honour exits non-zero instead of timing fewer ranks.
`--config dist-check` is the timed region's skeleton (process group, barriers,
max over ranks) without a render, so gloo runs it here; tests/test_gpu_nccl.py
runs the real configs on the GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                        "NERF_DIST_BACKEND")}
    env.update(kw)
    return env


def _run(args, env, timeout=180):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_reports_every_rank(n):
    r = _run(["--gpus", str(n), "--config", "dist-check", "--steps", "4", "--warmup", "1"],
             _env(NERF_DIST_BACKEND="gloo"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 alone prints
    rec = lines[0]
    assert rec["n_gpus"] == n and rec["steps"] == 4 and rec["allreduce_ok"]
    assert rec["config"]["backend"] == "gloo"
    # the ranks are children of the launcher, not the launcher itself
    assert rec["config"]["ranks_pid"] != os.getpid()


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "2", "--config", "dist-check"],
             _env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", NERF_DIST_BACKEND="gloo"))
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
    assert not r.stdout.strip()


def test_more_rccl_ranks_than_gpus_exits_nonzero():
    """Here no GPU is visible: RCCL ranks cannot get one each, so the launcher
    refuses before it starts any rank (and before any GPU call)."""
    torch = pytest.importorskip("torch")
    if torch.cuda.device_count() >= 2:
        pytest.skip("a host with 2+ GPUs would run the frames")
    r = _run(["--gpus", "2", "--steps", "1"], _env())
    assert r.returncode == 2 and "visible GPU" in r.stderr
    assert not r.stdout.strip()


def test_failing_rank_fails_the_launch():
    """A rank that dies takes the launch down with its status (the others are
    stopped, not left waiting in a collective)."""
    r = _run(["--gpus", "2", "--config", "dist-check", "--steps", "-1"],
             _env(NERF_DIST_BACKEND="bogus"))
    assert r.returncode != 0
