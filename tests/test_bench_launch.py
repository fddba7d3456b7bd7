"""bench.py's rank launch (CPU, gloo): ``--gpus N`` without a launcher starts N ranks itself, and a
launcher whose WORLD_SIZE disagrees with --gpus is refused.  ``--check-launch`` stops after the
process group is up, so no GPU is touched."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env.update(DSP_BENCH_BACKEND="gloo", DSP_BENCH_ONE_DEVICE="1", OMP_NUM_THREADS="1", **kw)
    return env


def test_bench_spawns_requested_ranks():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--check-launch"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["ranks_seen"] == 2 and lines[0]["world_size_env"] == 2 and lines[0]["gpus_flag"] == 2


def test_bench_refuses_world_size_mismatch():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--check-launch"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 2
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr
