"""bench.py's own launcher: ``python3 bench.py --gpus N`` (the driver's command form) starts N ranks.

Run here without a GPU, the ranks take the CPU dry-run path (gloo): the launch, the rendezvous on
127.0.0.1, the product partitioner (cep_shard_plan + the host cep_partition / cep_gather) and the
per-rank totals.  Nothing is matched (that needs the device), so the line's ``value`` is null."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, K = 40_000, 2_000


def _run(*args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_2_launches_two_ranks():
    r = _run("--gpus", "2", "--events", str(N), "--keys", str(K), "--steps", "1", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                      # one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] is None and d["dry_run"]
    ev = d["config"]["events_per_rank"]
    assert len(ev) == 2 and sum(ev) == 2 * N               # weak scaling: N events per GPU, node-wide 2N
    assert d["config"]["shard"]["planned_events"] == ev     # the partitioner's plan, realised on every rank
    assert abs(ev[0] - ev[1]) <= 100                        # rebalanced toward equal events
    # every key on exactly one rank: the per-rank distinct keys add up to the node's keys present
    from kcep import synth
    key, _, _ = synth.c2_stream_np(2 * N, 2 * K)
    assert sum(d["config"]["keys_per_rank"]) == len(np.unique(key))


def test_failing_rank_fails_the_run():
    r = _run("--gpus", "2", "--events", str(N), "--keys", str(K), "--steps", "1", "--warmup", "0",
             env_extra={"KCEP_BENCH_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr


def test_single_rank_dry_run():
    r = _run("--events", str(N), "--keys", str(K), "--steps", "1", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 1 and d["config"]["events_per_rank"] == [N]
