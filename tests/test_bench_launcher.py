"""bench.py's entry point: `python bench.py --gpus N` starts N ranks itself, an
outer launcher's WORLD_SIZE must agree with --gpus, and n_gpus is the process group's size.  Driven
with the GPU-free `dpcheck` workload over gloo."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=180):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 4])
def test_gpus_flag_starts_n_ranks(n):
    r = _run(["--gpus", str(n), "--workload", "dpcheck"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == n
    assert line["rank_sum"] == line["expected"] == n * (n + 1) / 2


def test_outer_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--workload", "dpcheck"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)
