"""bench.py --gpus N without a launcher starts N rank processes itself.

The stub workload (--stub) runs the launcher and the process-group path on CPU with gloo: every
rank joins, checks in with an all-reduce, and rank 0 prints one JSON line. The GPU bench uses the
same launch_ranks / init_ranks with the nccl (RCCL) backend."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=180):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_flag_starts_n_ranks(n):
    p = _run(["--gpus", str(n), "--stub", "--envs", "1024"])
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == d["pg_world_size"] == d["ranks_reported"] == n
    assert d["replicas_total"] == n * 1024
    assert len(set(d["rank_pids"])) == n


def test_single_rank_default():
    p = _run(["--stub"])
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["ranks_reported"] == 1


def test_gpus_mismatch_with_launcher_fails_loudly():
    p = _run(["--gpus", "2", "--stub"], env=dict(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode != 0
    assert "launcher started 1 rank" in p.stderr


def test_failed_rank_fails_the_launch():
    # rank 1 exits before joining; rank 0 would wait for it in the rendezvous: the launcher must stop
    # rank 0 and return non-zero instead of hanging
    p = _run(["--gpus", "2", "--stub"], env=dict(MS_STUB_FAIL_RANK="1"), timeout=120)
    assert p.returncode == 3
