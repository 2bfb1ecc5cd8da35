"""bench.py --gpus N starts its own ranks when no launcher set WORLD_SIZE: one child
process per rank before any GPU call, RANK = LOCAL_RANK = i, the shard rendezvous, rank
0 prints the line with n_gpus = N (tlsrecordlayer.py:27-37: the connection is the shard
unit, so ranks never exchange data).  --dry-run runs the plumbing without a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=180)


def test_spawner_distinct_local_ranks():
    r = _run(["--gpus", "4", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4
    assert [x["rank"] for x in d["ranks"]] == [0, 1, 2, 3]
    assert [x["local_rank"] for x in d["ranks"]] == [0, 1, 2, 3]
    assert [x["device"] for x in d["ranks"]] == [0, 1, 2, 3]
    assert len({x["pid"] for x in d["ranks"]}) == 4 and os.getpid() not in {x["pid"] for x in d["ranks"]}
    assert d["t_max"] == 0.004 and d["devices_shared"] is False


def test_spawner_refuses_more_ranks_than_devices():
    r = _run(["--gpus", "3", "--dry-run"], TLSGPU_DRYRUN_DEVICES="2")
    assert r.returncode != 0 and "--share-devices" in r.stderr


def test_spawner_shared_devices_round_robin():
    r = _run(["--gpus", "3", "--dry-run", "--share-devices"], TLSGPU_DRYRUN_DEVICES="2")
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 3 and [x["device"] for x in d["ranks"]] == [0, 1, 0] and d["devices_shared"] is True


def test_spawner_fails_when_a_rank_fails():
    r = _run(["--gpus", "3", "--dry-run"], TLSGPU_DRYRUN_FAIL_RANK="1")
    # rank 1 exits 3; rank 0 may notice the lost peer first and exit 1: either way non-zero
    assert r.returncode != 0
    assert "exited with" in r.stderr


def test_single_gpu_needs_no_spawn():
    r = _run(["--gpus", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 1 and d["ranks"][0]["pid"] != os.getpid()


def test_dry_run_parity_is_reduced_over_ranks():
    """bench.py's N > 1 parity: every rank checks its whole shard
    against the CPU oracle (shard_parity, its share of the host cores) and bit_exact is
    the AND over the ranks.  --dry-run --records R stands the oracle's own output in for
    the GPU's; a byte flipped on one rank must turn rank 0's bit_exact false."""
    r = _run(["--gpus", "3", "--dry-run", "--records", "48"])
    assert r.returncode == 0, r.stderr[-2000:]
    p = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])["parity"]
    assert p["bit_exact"] is True and p["bit_exact_ranks"] == [True, True, True]
    assert p["threads_per_rank"] >= 1
    r = _run(["--gpus", "3", "--dry-run", "--records", "48"], TLSGPU_DRYRUN_CORRUPT_RANK="2")
    assert r.returncode == 0, r.stderr[-2000:]
    p = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])["parity"]
    assert p["bit_exact"] is False and p["bit_exact_ranks"] == [True, True, False]
