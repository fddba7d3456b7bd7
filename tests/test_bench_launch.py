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


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_multirank_line_carries_both_values():
    """N > 1: ``value`` is extraction + all-gather per step, ``value_extract_only`` the graph-replayed
    extraction alone; N = 1 has only ``value``."""
    m = _bench_module()
    args = m.parse([])
    args.steps, args.clips = 10, 100000
    r2 = m.assemble_result(args, 2, 2, True, "gloo", 50000, 4.0e8, 0.02, 0.03, 1.4)
    assert r2["value"] == round(4.0e8 / 0.03, 1) and r2["value_extract_only"] == round(4.0e8 / 0.02, 1)
    assert r2["ms_per_step"] == 3.0 and r2["ms_per_step_extract_only"] == 2.0
    assert r2["rehearsal"] is True and r2["backend"] == "gloo" and r2["n_gpus"] == 2
    r1 = m.assemble_result(args, 1, 1, False, None, 100000, 4.0e8, 0.02, None, 2.8)
    assert "value_extract_only" not in r1 and r1["value"] == round(4.0e8 / 0.02, 1)
    assert r1["config"]["parallelism"].startswith("dp1")
    # both exchange loops timed (RCCL): value from the faster, both reported
    r8 = m.assemble_result(args, 8, 8, False, "RCCL", 12500, 4.0e8, 0.004, 0.0045, 0.35, None, 0.005, 0.0045, True)
    assert r8["value"] == round(4.0e8 / 0.0045, 1) and r8["ms_per_step"] == 0.45
    assert r8["ms_per_step_serial_exchange"] == 0.5 and r8["ms_per_step_pipelined_exchange"] == 0.45
    assert r8["exchange_own_block_equal"] is True and "pipelined" in r8["config"]["launch"]


def test_committed_pipelined_rehearsal_line():
    """The committed 2-rank rehearsal of both exchange loops (gloo, DSP_BENCH_PIPELINE=1)."""
    p = os.path.join(REPO, "profiles", "r06z_rehearsal_pipelined.json")
    with open(p) as f:
        d = json.loads([l for l in f.read().splitlines() if l.startswith("{")][-1])
    assert d["rehearsal"] is True and d["n_gpus"] == 2
    assert d["exchange_own_block_equal"] is True and d["timed_outputs_equal"] is True
    assert d["ms_per_step"] == min(d["ms_per_step_serial_exchange"], d["ms_per_step_pipelined_exchange"])


def test_committed_rehearsal_line():
    """The committed 2-rank rehearsal (gloo, one GPU) carries both values."""
    p = os.path.join(REPO, "profiles", "r05_multirank_rehearsal_bench.json")
    if not os.path.exists(p):
        import pytest
        pytest.skip("no round-5 rehearsal record yet")
    with open(p) as f:
        d = json.loads([l for l in f.read().splitlines() if l.startswith("{")][-1])
    assert d["rehearsal"] is True and d["n_gpus"] == 2 and d["ranks_seen"] == 2
    assert d["value"] > 0 and d["value_extract_only"] >= d["value"] * 0.5
    assert d["allgather"]["collectives"] == 1
