"""bench.py's rank launcher (``--gpus N`` without torchrun): N fresh rank processes, rank 0's JSON line forwarded as
the only stdout line, a failing rank's exit code propagated. Runs a CPU stand-in rank (``--standin-worker``: gloo over
the launcher's rendezvous, no GPU) so that it runs here; the real ranks take the same path into bench.main()."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=REPO)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_runs_every_rank_and_prints_one_json_line(n):
    r = _run("--gpus", str(n), "--standin-worker")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # rank 0's non-JSON line went to stderr, the other ranks print no JSON
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["rank_sum"] == n * (n + 1) // 2
    for k in range(n):  # every rank ran and joined the collective
        assert f"standin rank {k} of {n}: sum {n * (n + 1) // 2}" in r.stderr
    assert "not a json line from rank 0" in r.stderr


def test_launcher_propagates_a_failing_rank():
    """Rank 1 exits 3 before the rendezvous; rank 0 would block in it forever: the launcher stops it, prints no JSON
    line and returns 3 (the driver sees the failure instead of a hang)."""
    r = _run("--gpus", "2", "--standin-worker", "--standin-fail-rank", "1", timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == ""
    assert "rank 1 exited with 3" in r.stderr


def test_gpus_1_has_no_launcher():
    """--gpus 1 (the driver's BENCH form) runs in this process: the stand-in reports world 1 without children."""
    r = _run("--gpus", "1", "--standin-worker")
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
    assert "[rank" not in r.stderr
