"""bench.py --gpus N starts N ranks itself when no launcher did,
and refuses a WORLD_SIZE that disagrees with --gpus.  CPU only: the ranks run
the --stub-rank body (a gloo group, no GPU work) through the same launcher."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_launch_plan():
    assert bench.launch_plan(1, {}) == ("here", None)
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}) == ("here", None)
    kind, msg = bench.launch_plan(8, {"WORLD_SIZE": "1"})
    assert kind == "error" and "WORLD_SIZE=1" in msg
    assert bench.launch_plan(1, {"WORLD_SIZE": "2"})[0] == "error"
    assert bench.launch_plan(0, {})[0] == "error"


def _run(args, env, timeout=180):
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=str(ROOT))


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2])
def test_bare_gpus_flag_starts_the_ranks(n):
    p = _run(["--gpus", str(n), "--stub-rank"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == n
    assert d["per_rank"]["rank"] == list(range(n))


def test_world_size_mismatch_exits_nonzero():
    p = _run(["--gpus", "4", "--stub-rank"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
