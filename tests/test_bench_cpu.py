"""bench.py's own launcher (`python bench.py --gpus N` with no torchrun): the rank processes
it starts and their environment, checked with --dry-run (no torch, no GPU in the children).
The reference drives every GPU from one command (utils/trainer.py:28-30, nn.DataParallel)."""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _clean_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "LOCAL_WORLD_SIZE", "BENCH_DRY_RUN_FAIL_RANK")}
    env.update(extra)
    return env


def _run(args, **extra):
    return subprocess.run([sys.executable, BENCH] + args, env=_clean_env(**extra),
                          capture_output=True, text=True, timeout=60)


def test_launcher_starts_one_process_per_gpu():
    r = _run(["--gpus", "4", "--steps", "7", "--warmup", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 4
    assert sorted(int(d["RANK"]) for d in lines) == [0, 1, 2, 3]
    for d in lines:
        assert d["LOCAL_RANK"] == d["RANK"]
        assert d["WORLD_SIZE"] == "4"
        assert d["MASTER_ADDR"] == "127.0.0.1"
        assert int(d["MASTER_PORT"]) > 0
        # the children run the same command line (same timed region, steps and warmup)
        assert d["argv"] == ["--gpus", "4", "--steps", "7", "--warmup", "2", "--dry-run"]
    assert len({d["MASTER_PORT"] for d in lines}) == 1


def test_single_gpu_runs_in_process():
    r = _run(["--gpus", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1 and lines[0]["WORLD_SIZE"] is None


def test_launcher_rank_count_must_match_gpus():
    # under torchrun (WORLD_SIZE set) --gpus must equal the number of ranks
    r = _run(["--gpus", "4", "--dry-run"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "n_gpus must equal" in r.stderr


def test_launcher_failure_stops_other_ranks():
    t0 = time.time()
    r = _run(["--gpus", "3", "--dry-run"], BENCH_DRY_RUN_FAIL_RANK="1")
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "stopping the other ranks" in r.stderr
    assert time.time() - t0 < 30  # the waiting ranks were terminated, not waited for


def test_rank_envs():
    sys.path.insert(0, REPO)
    import bench
    envs = bench.rank_envs(2, 12345, base={"X": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1"]
    assert all(e["X"] == "1" and e["MASTER_PORT"] == "12345" for e in envs)


def test_launcher_forwards_sigterm_to_ranks():
    """the ranks run in sessions of their own, so a SIGTERM to the launcher (a
    scheduler's timeout) must be forwarded to them, or they keep their GPUs and wait in a
    collective.  Every dry-run rank sleeps (no rank fails); SIGTERM the launcher: it exits
    128 + 15 and no rank survives it."""
    import signal
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "3", "--dry-run"],
                         env=_clean_env(BENCH_DRY_RUN_FAIL_RANK="99"), stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    pids = []
    t0 = time.time()
    while len(pids) < 3 and time.time() - t0 < 30:
        line = p.stdout.readline()
        if line.startswith("{"):
            pids.append(json.loads(line)["pid"])
    assert len(pids) == 3
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    time.sleep(0.5)
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive, pid
