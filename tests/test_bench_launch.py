"""bench.py's self-launch (`--gpus N` with no torch.distributed.run around
it): N fresh rank processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*,
rank 0's line relayed, a failing rank failing the run.  The rank body here
is the CPU stub (gloo barriers and the max-over-ranks wall time), so no GPU
is touched."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, timeout=120):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3",
                           "--warmup", "1", "--stub", *extra],
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


def test_two_rank_self_launch_prints_one_line():
    p = _run("--gpus", "2")
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1
    # the max over ranks: rank 1 sleeps longer than rank 0
    assert rec["ms_per_step"] >= 20.0 / 3 * 0.9


def test_failing_rank_fails_the_run():
    p = _run("--gpus", "2", "--stub-fail-rank", "1")
    assert p.returncode != 0
    assert "rank failed" in p.stderr


def test_stalled_ranks_are_killed():
    # rank 1 fails before joining the rendezvous is the fail case; a stall
    # is a rank that never finishes: a timeout shorter than gloo's wait
    p = _run("--gpus", "2", "--stub-fail-rank", "-1", "--rank-timeout", "0.01")
    assert p.returncode == 124, (p.returncode, p.stderr)
    assert "stalled" in p.stderr


def test_single_gpu_runs_in_process():
    p = _run("--gpus", "1")
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_eight_rank_self_launch_binds_local_ranks_and_reduces():
    """The driver's 8-GPU run, rehearsed on the CPU: eight fresh ranks, each
    with its own LOCAL_RANK (the device it binds), one line from rank 0,
    the readout reduce (gloo here, RCCL on the GPUs) summing every rank's
    counters and reported as reduce_ms."""
    p = _run("--gpus", "8", timeout=240)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8
    assert rec["local_ranks"] == list(range(8))
    assert "reduce_error" not in rec and rec["reduce_ms"] >= 0
    # the max over ranks: rank 7 sleeps 80 ms in its timed region
    assert rec["ms_per_step"] >= 80.0 / 3 * 0.9


def test_eight_ranks_one_stalled_fails_the_run():
    p = _run("--gpus", "8", "--stub-stall-rank", "5", "--rank-timeout", "20", timeout=240)
    assert p.returncode == 124, (p.returncode, p.stderr)
    assert "stalled" in p.stderr


def test_eight_ranks_stalled_reduce_is_reported():
    """A reduce that never completes on one rank: rank 0 still prints its
    line, with reduce_error, and the run exits non-zero (status 3)."""
    p = _run("--gpus", "8", "--stub-reduce-stall-rank", "3", "--reduce-timeout", "3",
             timeout=240)
    assert p.returncode == 3, (p.returncode, p.stderr)
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.strip()][-1])
    assert rec["n_gpus"] == 8 and rec["reduce_error"] == "timed out"
    assert "reduce_ms" not in rec
