"""CPU: bench.py's own multi-rank launcher.  `python bench.py --gpus N` must start N rank
processes that really form one process group and all-reduce (here over gloo with the
--stub per-rank function, no GPU), report n_gpus from the group that ran, and refuse --
non-zero exit, nothing timed -- when it cannot give every rank a GPU or when a launcher's
WORLD_SIZE disagrees with --gpus."""

import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=180):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_forms_n_ranks_and_all_reduces(n):
    r = _run(["--gpus", str(n), "--backend", "gloo", "--stub", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_seen"] == list(range(n))
    assert out["allreduce_ok"] is True and out["backend"] == "gloo"


def test_launcher_refuses_more_ranks_than_gpus():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])  # no GPU in this container
    assert r.returncode == 2
    assert "refusing" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "3", "--stub", "--backend", "gloo"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
