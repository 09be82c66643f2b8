"""Headline benchmark: BASELINE.json metric on config C2.

  events/sec (whole node) of the 3-stage strict A->B->C query over 1M keys x
  100M synthetic int events per GPU, match phase with the batch resident in
  HBM (SoA key_id i32 + value i32, grouped by key), plus achieved HBM GB/s of
  the dominant kernel.

One process per GPU (torch.distributed over RCCL when launched with
torch.distributed.run).  Keys are sharded across ranks (weak scaling: every
rank owns 1M keys and 100M events); the only collective is the all-gather of
per-rank (events, matches) and the max-reduction of the timed interval.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kafkastreams-cep_amd"))

PEAK_HBM_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--events", type=int, default=100_000_000, help="events per GPU")
    ap.add_argument("--keys", type=int, default=1_000_000, help="keys per GPU")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-steps", action="store_true", help="minimal run for rocprofv3")
    return ap.parse_args()


def shard(rank: int, n: int, K: int):
    """Rank r owns keys [r*K, (r+1)*K) and the counter range [r*n, (r+1)*n) of the
    C2 generator: disjoint key sets, so per-key NFAs never cross ranks."""
    return rank * K, rank * n


def gather_stats(stats, world: int):
    """The path's one exchange step: all-gather per-rank (events, matches, seconds);
    returns (total events, total matches, max seconds over ranks)."""
    if world > 1:
        import torch
        import torch.distributed as dist
        allg = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allg, stats)
        return (sum(float(x[0]) for x in allg), sum(float(x[1]) for x in allg), max(float(x[2]) for x in allg))
    return float(stats[0]), float(stats[1]), float(stats[2])


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    from kcep import native as N, synth, Schema

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)

    n, K = args.events, args.keys
    # rank r owns keys [r*K, (r+1)*K) and the counter range [r*n, (r+1)*n) of the
    # C2 generator (key-hash sharding of one node-wide stream)
    key_offset, lo = shard(rank, n, K)
    key, val, order = synth.c2_stream_torch(n, K, dev, key_offset=key_offset, lo=lo)
    torch.cuda.synchronize(dev)

    ir = synth.c2_pattern().to_ir(Schema([("value", "i32")]))
    pat = N.CompiledPattern(ir)
    sess = N.Session(pat, n, mode=N.MODE_PROCESSOR, device=local)
    assert sess.path == N.PATH_STENCIL

    def step():
        sess.push(n, key.data_ptr(), [val.data_ptr()], mem=N.MEM_DEVICE, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in ev]
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)

    n_matches, csum = sess.checksum()
    stats = torch.tensor([float(n), float(n_matches), elapsed], dtype=torch.float64, device=dev)
    tot_events, tot_matches, t_max = gather_stats(stats, world)

    if rank == 0:
        algo_bytes = 8.0 * n + 4.0 * 3 * n_matches         # 8 B/event + 12 B/match
        achieved = algo_bytes / (avg_kernel_ms * 1e-3) / 1e9
        value = tot_events * args.steps / t_max
        traffic = _pmc_traffic(n)
        line = {
            "metric": "events/sec (whole node), 3-stage A->B->C over 1M keys; achieved HBM GB/s",
            "value": value,
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (splitmix64 counter RNG, BASELINE.md §3 C2)",
            "config": {"workload": "C2: 3-stage strict A->B->C, processor mode", "events_per_gpu": n,
                       "keys_per_gpu": K, "matches_per_gpu": int(n_matches), "matches_total": int(tot_matches),
                       "path": "stencil",
                       "parallelism": f"key-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                         "kernel_ms": avg_kernel_ms, "algo_bytes_per_launch": algo_bytes},
            "cpu_baseline": None,
            "checksum": f"{csum:016x}",
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = _cpu_baseline(key, val, order, ir, args.cpu_threads, n_matches, csum)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _pmc_traffic(n):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (if any),
    FETCH_SIZE doubled per the gfx950 correction (MI355X_MICROARCH.md §HBM)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if int(d.get("events")) != n:
            return None
        return float(d["hbm_bytes_per_launch"])
    except Exception:
        return None


def _cpu_baseline(key, val, order, ir, threads, gpu_matches, gpu_csum):
    """The oracle (C restatement of the reference NFA) on the host cores over
    the full workload (same arrays), plus a 1-core figure on a 4M-event prefix."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    hk, hv, ho = key.cpu().numpy(), val.cpu().numpy(), order.cpu().numpy()
    p = O.OraclePattern(ir)
    b = O.BatchArrays(hk, [hv], [1], offset=ho, ts=ho)
    threads = max(1, min(threads, os.cpu_count() or 1))
    t0 = time.perf_counter()
    nm, cs = O.baseline(p, b, O.MODE_PROCESSOR, threads)
    dt = time.perf_counter() - t0
    m1 = min(len(hk), 4_000_000)
    while 0 < m1 < len(hk) and hk[m1] == hk[m1 - 1]:
        m1 += 1
    b1 = O.BatchArrays(hk[:m1], [hv[:m1]], [1], offset=ho[:m1], ts=ho[:m1])
    t1 = time.perf_counter()
    O.baseline(p, b1, O.MODE_PROCESSOR, 1)
    dt1 = time.perf_counter() - t1
    return {"value": len(hk) / dt, "unit": "events/s", "cores": threads, "kind": "port",
            "sample": f"full C2 workload ({len(hk)} events) on {threads} threads; 1-core figure on a "
                      f"{m1}-event whole-key prefix",
            "value_1core": m1 / dt1, "parity": bool(nm == gpu_matches and cs == gpu_csum),
            "oracle_matches": int(nm)}


if __name__ == "__main__":
    main()
