"""bench.py --gpus N run as a plain command (no torch.distributed launcher):
the parent starts N fresh rank processes itself, before torch is imported
and without exec, and rank 0 prints one line whose timing is the max over
ranks (the driver's scaling runs depend on this).  --dry-run replaces the
search with rank-dependent sleeps over gloo, so this runs on CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


@pytest.mark.timeout(180)
def test_launcher_starts_ranks_and_reports_max():
    steps = 4
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", str(steps), "--warmup", "1"],
                       env=_env(), capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout  # exactly one JSON line on stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps
    ranks = d["ranks"]
    assert sorted(x["rank"] for x in ranks) == [0, 1]
    assert sorted(x["local_rank"] for x in ranks) == [0, 1]
    assert len({x["pid"] for x in ranks}) == 2
    # max over ranks: rank 1 sleeps 20 ms per step
    worst = max(x["elapsed"] for x in ranks)
    assert abs(d["ms_per_step"] - worst / steps * 1e3) < 1e-6
    assert d["ms_per_step"] >= 20.0


@pytest.mark.timeout(60)
def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-run"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=50)
    assert r.returncode != 0
    assert "--gpus 3 but WORLD_SIZE=2" in r.stderr


@pytest.mark.timeout(180)
def test_failing_rank_fails_the_run():
    # rank 1 cannot join: its WORLD_SIZE disagrees (set by a bad launcher);
    # simulated by asking for a step count the dry run rejects on rank 1 only
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "2"],
                       env=_env(NGT_BENCH_DRYRUN_FAIL_RANK="1"), capture_output=True, text=True, timeout=170)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
