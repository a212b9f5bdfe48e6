"""bench.py's multi-rank launcher on the CPU: `--gpus 2` started without a launcher spawns 2
ranks itself (torch.distributed.run as a child process), the ranks form a world of 2 over
gloo, the timed region takes the max over ranks, and rank 0 prints ONE JSON line."""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _run(*args):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_spawns_two_ranks():
    d = _run("--gpus", "2", "--selftest", "--steps", "5", "--warmup", "1")
    assert d["n_gpus"] == 2 and d["world_size_seen"] == 2 and d["backend"] == "gloo"
    assert d["ranks_reporting"] == [0, 1]
    assert d["steps"] == 5 and d["value"] > 0 and d["selftest"] is True
    assert d["config"]["parallelism"] == "dp2"


def test_bench_single_rank_selftest():
    d = _run("--selftest", "--steps", "3", "--warmup", "0")
    assert d["n_gpus"] == 1 and d["world_size_seen"] == 1 and d["backend"] is None
    assert "rehearsal" not in d
