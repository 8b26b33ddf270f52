"""CPU: `bench.py --gpus N` as a bare command (no torch.distributed.run around it) spawns its
N ranks itself, before anything imports torch or initialises HIP, relays rank 0's JSON line
and fails when any rank fails. The ranks run in
MAXK_BENCH_SELFTEST mode: they report the launcher environment they were given and exit,
without torch, so this runs in seconds on a machine with no GPU."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(n, spec, timeout=60, extra_env=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR")}
    env["MAXK_BENCH_SELFTEST"] = spec
    env.update(extra_env or {})
    t0 = time.time()
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "3"], env=env,
                       capture_output=True, text=True, timeout=timeout)
    return p, time.time() - t0


@pytest.mark.parametrize("n", [2, 3, 8])
def test_bare_gpus_n_spawns_and_relays_rank0(n):
    p, _ = _run(n, "ok")
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout              # exactly rank 0's JSON line
    rec = json.loads(lines[0])
    assert rec == {"selftest": True, "world": n, "rank": 0, "local_rank": 0,
                   "master": rec["master"], "spawned": True}
    assert rec["master"].startswith("127.0.0.1:")
    assert "parent imports no torch" in p.stderr


def test_failing_rank_fails_the_job_and_stops_the_others():
    # rank 1 exits 3; rank 0 would otherwise sleep 600 s (a rank stuck in a collective)
    p, dt = _run(2, "fail:1")
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert dt < 30, dt
    assert "rank 1 exited with 3" in p.stderr


def test_parent_never_imports_torch():
    """The spawning process must not initialise HIP: importing bench and spawning leaves
    torch out of sys.modules (spawn_ranks also asserts it)."""
    code = (
        "import os, sys, json\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "os.environ['MAXK_BENCH_SELFTEST'] = 'ok'\n"
        "for v in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT'):\n"
        "    os.environ.pop(v, None)\n"
        "import bench\n"
        "assert 'torch' not in sys.modules\n"
        "rc = bench.spawn_ranks(2, ['--gpus', '2'])\n"
        "assert 'torch' not in sys.modules\n"
        "print('RC', rc)\n")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert "RC 0" in p.stdout


def test_launcher_env_runs_as_a_rank():
    """Under torch.distributed.run (WORLD_SIZE in the environment) bench.py is a rank and does
    not spawn again."""
    env = dict(os.environ, MAXK_BENCH_SELFTEST="ok", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    rec = json.loads(p.stdout.strip())
    assert rec["spawned"] is False and rec["world"] == 2
    assert "spawning" not in p.stderr


def test_straggler_limit_ends_ranks_left_behind():
    """rank 1 exits 0 while rank 0 hangs (as in a collective its peer left); the
    parent stops it after MAXK_BENCH_STRAGGLER_S and fails the job with 124."""
    p, dt = _run(2, "exit0:1", extra_env={"MAXK_BENCH_STRAGGLER_S": "2"})
    assert p.returncode == 124, (p.returncode, p.stderr)
    assert dt < 30, dt
    assert "still running" in p.stderr


def test_topology_gathered_from_every_rank():
    """rank 0's line carries torch.distributed's world size and backend,
    every rank's device identity (all-gathered) and the RCCL version (selftest ranks: a gloo
    group with made-up, distinct device identities)."""
    p, _ = _run(3, "topology", timeout=120)
    assert p.returncode == 0, p.stderr
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]   # gloo logs its own
    assert len(line) == 1, p.stdout
    topo = json.loads(line[0])["topology"]
    assert topo["world_size"] == 3 and topo["launcher_world_size"] == 3
    assert topo["backend"] == "gloo"
    assert [r["rank"] for r in topo["ranks"]] == [0, 1, 2]
    assert len({r["pci_bus_id"] for r in topo["ranks"]}) == 3
    assert topo["rccl_version"].count(".") == 2


def test_two_nccl_ranks_on_one_device_are_refused():
    """Two ranks whose identities resolve to one device fail the one-GPU-per-rank check that
    every nccl run makes before any work: non-zero exit, the reason on stderr."""
    p, _ = _run(2, "topology:dup", timeout=120)
    assert p.returncode != 0, p.stdout
    assert "resolve to the same device" in p.stderr
