"""bench.py's own multi-rank launcher (CPU, no GPU touched): ``python bench.py --gpus N`` without
WORLD_SIZE spawns N ranks with torch.distributed.run's environment and exits with the worst child
status; a WORLD_SIZE that disagrees with --gpus is refused.  ``--dry-launch`` stops every rank
before GPU initialisation (VERDICT r1 "next round" item 1)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def _port(k: int) -> str:
    """A rendezvous port per test and xdist worker, below the ephemeral range: a port picked free by
    binding and releasing can be taken by a concurrently running test before the ranks bind it."""
    w = os.environ.get("PYTEST_XDIST_WORKER", "gw0")
    return str(21000 + 40 * int(w[2:] or 0) + k)


def _run(args, env, timeout=120):
    return subprocess.run([sys.executable, BENCH, *args], env=env, capture_output=True, text=True, timeout=timeout)


def test_spawns_ranks_with_launch_env():
    p = _run(["--gpus", "3", "--dry-launch"], _env())
    assert p.returncode == 0, p.stderr
    recs = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert sorted(int(r["RANK"]) for r in recs) == [0, 1, 2]
    assert {r["WORLD_SIZE"] for r in recs} == {"3"} and {r["LOCAL_WORLD_SIZE"] for r in recs} == {"3"}
    assert {r["MASTER_ADDR"] for r in recs} == {"127.0.0.1"}
    assert len({r["MASTER_PORT"] for r in recs}) == 1
    assert all(r["LOCAL_RANK"] == r["RANK"] for r in recs)
    assert len({r["pid"] for r in recs}) == 3          # separate processes, none is the parent
    assert all(r["pid"] != p.args for r in recs)


def test_worst_child_status_propagates():
    p = _run(["--gpus", "2", "--dry-launch"], _env(NKV_DRY_RC_RANK1="3"))
    assert p.returncode == 3
    p = _run(["--gpus", "4", "--dry-launch"], _env(NKV_DRY_RC_RANK0="1", NKV_DRY_RC_RANK2="5"))
    assert p.returncode == 5


def test_failed_rank_ends_hung_peers():
    # rank 0 "hangs" (as in a collective whose peer died); rank 1 fails -> the launcher stops rank 0
    t0 = time.monotonic()
    p = _run(["--gpus", "2", "--dry-launch"], _env(NKV_DRY_SLEEP_RANK0="100", NKV_DRY_RC_RANK1="7",
                                                   NKV_LAUNCH_GRACE_S="1"), timeout=90)
    assert time.monotonic() - t0 < 60
    assert p.returncode == 128 + 15 or p.returncode == 7, p.returncode   # SIGTERM'd rank 0, or rank 1's 7
    assert p.returncode >= 7


def test_world_size_mismatch_refused():
    p = _run(["--gpus", "8", "--dry-launch"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr


def test_torchrun_style_env_passes():
    p = _run(["--gpus", "2", "--dry-launch"], _env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1",
                                                   MASTER_ADDR="127.0.0.1", MASTER_PORT="29999"))
    assert p.returncode == 0
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["RANK"] == "1" and rec["MASTER_PORT"] == "29999"


def test_single_gpu_default_runs_in_process():
    p = _run(["--dry-launch"], _env())
    assert p.returncode == 0
    recs = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(recs) == 1 and recs[0]["WORLD_SIZE"] is None


# ---- round 3: bounded collectives, wall clocks, per-rank device identity ----

def test_collective_probe_gathers_devices():
    p = _run(["--gpus", "2", "--collective-probe"], _env(NKV_BACKEND="gloo", MASTER_PORT=_port(1)), timeout=120)
    assert p.returncode == 0, p.stderr
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["world"] == 2 and rec["backend"] == "gloo" and rec["sum"] == 3.0
    assert len(rec["devices"]) == 2
    # CPU ranks have no GPU identity: distinct_devices is undecidable, not true
    assert rec["distinct_devices"] is None


def test_rank_missing_from_allreduce_ends_every_rank():
    """One rank never joins the all-reduce: its peer's collective times out (bounded by
    NKV_COLLECTIVE_TIMEOUT_S instead of torch's 10 min), that rank exits non-zero, and the
    launcher ends the absent rank and exits non-zero — all within the bound.  The bound also covers
    the rendezvous (init_process_group), so it must exceed a loaded host's `import torch` in the
    late rank (a 4 s bound failed the rendezvous under pytest -n 4)."""
    t0 = time.monotonic()
    p = _run(["--gpus", "2", "--collective-probe"],
             _env(NKV_BACKEND="gloo", NKV_PROBE_HANG_RANK="1", NKV_COLLECTIVE_TIMEOUT_S="20", MASTER_PORT=_port(2),
                  NKV_LAUNCH_GRACE_S="2", NKV_RANK_WALL_S="0"), timeout=150)
    dt = time.monotonic() - t0
    assert dt < 90, dt
    assert p.returncode != 0
    assert "probe rank 0: all-reduce failed" in p.stderr, p.stderr[-2000:]
    assert "bench launcher: rank 0 exited with 3" in p.stderr


def test_rank_watchdog_ends_a_hung_rank():
    """Under torch.distributed.run (no launcher of ours): the per-rank wall clock alone ends a rank
    that never returns, with status 124 and a stack dump."""
    t0 = time.monotonic()
    p = _run(["--gpus", "2", "--collective-probe"],
             _env(NKV_BACKEND="gloo", NKV_PROBE_HANG_RANK="1", NKV_COLLECTIVE_TIMEOUT_S="600", MASTER_PORT=_port(3),
                  NKV_LAUNCH_GRACE_S="600", NKV_RANK_WALL_S="6", NKV_LAUNCH_WALL_S="0"), timeout=120)
    assert time.monotonic() - t0 < 60
    assert p.returncode == 124, (p.returncode, p.stderr[-2000:])
    assert "wall clock of 6 s exceeded" in p.stderr


def test_launcher_wall_clock_ends_an_all_ranks_hang():
    """Every rank blocked (no rank exits, so no grace period starts): the launcher's wall clock
    terminates them all and exits 124."""
    t0 = time.monotonic()
    p = _run(["--gpus", "3", "--dry-launch"],
             _env(NKV_DRY_SLEEP_RANK0="300", NKV_DRY_SLEEP_RANK1="300", NKV_DRY_SLEEP_RANK2="300",
                  NKV_LAUNCH_WALL_S="3", NKV_RANK_WALL_S="0"), timeout=120)
    assert time.monotonic() - t0 < 40
    assert p.returncode == 124, p.returncode
    assert "wall clock of 3 s exceeded" in p.stderr
