"""Headline benchmark: BASELINE.json metric on config C2.

  events/sec (whole node) of the 3-stage strict A->B->C query over 1M keys x
  100M synthetic int events per GPU, match phase with the batch resident in
  HBM (SoA key_id i32 + value i32, grouped by key), plus achieved HBM GB/s of
  the dominant kernel.

One process per GPU (torch.distributed over RCCL when launched with
torch.distributed.run).  With N > 1 every rank generates the node-wide stream
(counter RNG, identical on every rank), splits it with the product partitioner
(kcep/shard.py: cep_shard_plan + cep_partition on the device, keys by hash
rebalanced to equal events) and matches only its shard.  C2/C3/C4 keep the
per-GPU shape (weak scaling: N x 1M keys x 100M events for C2); C5 is the
node-wide 10M keys x 100 events split over N GPUs (strong scaling).  The one
collective is kcep/shard.py's CountExchange: after every step the rank's
device-resident match count is all-gathered over RCCL with its event count and
scanned into the rank's global match offset, on a side stream that overlaps the
next step.

``--config c3|c4|c5`` measures the other BASELINE configs (not the headline
line; DESIGN.md reports them).

Launch.  ``python3 bench.py --gpus N`` with N > 1 and no ``WORLD_SIZE`` in the
environment starts the N ranks itself (``launch``: N child processes with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT, rank 0's
line relayed, a failing rank fails the run); the parent never touches the GPU.
Under ``torch.distributed.run`` (WORLD_SIZE set) each process is one rank.
Without a visible GPU the ranks run a dry run on CPU (gloo): the launch, the
partitioner and the per-rank totals, nothing matched, ``value`` null.

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
METRIC = "events/sec (whole node), 3-stage A->B->C over 1M keys; achieved HBM GB/s"

# per-GPU shapes (BASELINE.md §3 / SURVEY §8(d)); C5's 10M keys are the node-wide
# total over 8 GPUs, so one GPU owns 1.25M keys x 100 events
CONFIGS = {
    "c2": dict(keys=1_000_000, events=100_000_000, desc="C2: 3-stage strict A->B->C, processor mode"),
    "c3": dict(keys=100_000, per_key=100, desc="C3: stock oneOrMore + sum/count state + within(60s)"),
    "c4": dict(keys=100_000, per_key=12, desc="C4: skip-till-any times(3) + zeroOrMore"),
    "c5": dict(keys=10_000_000, per_key=100, node_wide=True,
               desc="C5: AND/OR + optional(), strict, 10M keys x 100 events node-wide, key-hash sharded"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal (gloo): launch, partitioner and per-rank totals, nothing matched; "
                         "automatic when no GPU is visible")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--events", type=int, default=None, help="events per GPU (c2)")
    ap.add_argument("--keys", type=int, default=None, help="keys per GPU")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="oracle threads for cpu_baseline (default: nproc, every CPU this process may run on)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-input", action="store_true", help="skip the PCIe-inclusive (host buffer) figure")
    ap.add_argument("--processor-batch", type=lambda x: [int(v) for v in x.split(",") if v], default=[1 << 16, 1 << 20],
                    help="stencil/chain: record counts per host batch for the processor-batch legs (comma list)")
    ap.add_argument("--carry-batches", type=int, default=10,
                    help="stencil/chain: also stream the batch through a carry session in this many batches")
    ap.add_argument("--force-path", choices=["stencil", "chain", "runs", "general"], default=None,
                    help="run the workload on this path (e.g. C3 on the general NFA), not the fastest exact one")
    ap.add_argument("--nfa-kernel", choices=["auto", "wave", "lane"], default="auto",
                    help="general path: one key per wave (CEP_SESSION_WAVE_NFA) or per lane (CEP_SESSION_LANE_NFA); "
                         "auto: the library's choice")
    ap.add_argument("--handoff-cap", type=int, default=16384,
                    help="C4: per-key workspace cap (words) of the hand-off leg -- keys over it continue on the "
                         "CPU (the oracle) from their exported state; 0 skips the leg")
    ap.add_argument("--gather-matches", action="store_true",
                    help="N > 1: after the timed steps, gather every rank's matches to rank 0 (12 B/match) and "
                         "time it")
    return ap.parse_args(argv)


def gather_stats(stats, world: int):
    """All-gather per-rank (events, matches, seconds) after the timed region; returns (total
    events, total matches, max seconds over ranks)."""
    if world > 1:
        import torch
        import torch.distributed as dist
        allg = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allg, stats)
        return (sum(float(x[0]) for x in allg), sum(float(x[1]) for x in allg), max(float(x[2]) for x in allg))
    return float(stats[0]), float(stats[1]), float(stats[2])


def node_stream(cfg: str, K: int, n: int | None, dev):
    """The stream one GPU (world 1) or the whole node (world > 1) matches, device-resident:
    (key, [cols], ts, ir)."""
    from kcep import synth, Schema
    I32 = Schema([("value", "i32")])
    if cfg == "c2":
        key, val, order = synth.c2_stream_torch(n, K, dev)
        return key, [val], order, synth.c2_pattern().to_ir(I32)
    L = CONFIGS[cfg]["per_key"]
    gen_t = {"c3": synth.c3_stream_torch, "c4": synth.c4_stream_torch, "c5": synth.c5_stream_torch}[cfg]
    pat = {"c3": synth.c3_pattern, "c4": synth.c4_pattern, "c5": synth.c5_pattern}[cfg]()
    key, val, ts = gen_t(K, dev, L=L)
    return key, [val], ts, pat.to_ir(I32)


def workload(cfg: str, rank: int, world: int, K: int, n: int | None, dev, stream):
    """This rank's device-resident batch: (key, [cols], ts, ir, shard info).  World 1: the
    per-GPU config.  World > 1: the node-wide stream split by the product partitioner -- keys
    planned by hash, rebalanced to equal events (cep_shard_plan), split on the device
    (cep_partition + cep_gather)."""
    import torch
    from kcep import shard as S
    node_wide = CONFIGS[cfg].get("node_wide", False)
    if world == 1:
        key, cols, ts, ir = node_stream(cfg, K, n, dev)
        return key, cols, ts, ir, None
    NK = K if node_wide else K * world
    NN = None if n is None else (n if node_wide else n * world)
    key, cols, ts, ir = node_stream(cfg, NK, NN, dev)
    t0 = time.perf_counter()
    counts = torch.bincount(key, minlength=NK).cpu().numpy()
    table, loads = S.shard_plan(counts, world, rebalance=True)
    sh = S.split(rank, world, key, cols, table=torch.from_numpy(table).to(dev),
                 stream=stream.cuda_stream if stream is not None else None, ts=ts)
    if key.is_cuda:
        torch.cuda.synchronize(dev)
    info = {"node_events": int(key.numel()), "node_keys": NK, "planned_events": loads.tolist(),
            "partition_s": time.perf_counter() - t0, "partitioner": "cep_shard_plan(rebalance) + cep_partition"}
    del key, cols, ts
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    return sh.key, sh.cols, sh.extra["ts"], ir, (sh, info)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n: int, argv) -> int:
    """``--gpus n`` without a launcher: one child process per rank (this script again, never an exec),
    each with RANK / LOCAL_RANK / WORLD_SIZE and a 127.0.0.1 rendezvous.  Rank 0's stdout (the JSON line)
    is relayed; the other ranks' stdout goes to stderr.  The first rank to fail ends the run: the others
    are killed by PID and its exit status is returned.  This process imports neither torch nor the
    library, so it never touches a GPU; each rank checks ``n`` against the devices it sees."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.kill()
            if live:
                time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    return rc


def dry_run(args, world: int, rank: int):
    """No GPU visible: the multi-rank path up to the device, on CPU.  Every rank builds the node-wide
    stream, takes its shard with the product partitioner (kcep/shard.py on CPU tensors: cep_shard_plan +
    the host cep_partition / cep_gather) and the ranks all-gather their event counts over gloo.  Nothing is
    matched (the kernels need a GPU), so ``value`` is null.  Sizes default to 1/100 of the config's."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    C = CONFIGS[args.config]
    K = args.keys or max(1, C["keys"] // 100)
    n_req = args.events or (C["events"] // 100 if C.get("events") else None)
    key, cols, ts, ir, shard_info = workload(args.config, rank, world, K, n_req, torch.device("cpu"), None)
    n = int(key.numel())
    mine = torch.tensor([float(n), float(torch.unique(key).numel())], dtype=torch.float64)
    per = [torch.zeros_like(mine) for _ in range(world)] if world > 1 else [mine]
    if world > 1:
        dist.all_gather(per, mine)
    if rank == 0:
        line = {"metric": METRIC if args.config == "c2" else f"events/sec (whole node), {C['desc']}",
                "value": None, "unit": "events/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": None, "higher_is_better": True,
                "scaling": "strong" if C.get("node_wide") and world > 1 else "weak", "vs_baseline": None,
                "dtype": "int32", "data": "synthetic (splitmix64 counter RNG, BASELINE.md §3)",
                "config": {"workload": C["desc"], "keys_per_gpu": K,
                           "parallelism": f"key-hash sharded x{world}" if world > 1 else "1 GPU",
                           "events_per_rank": [int(p[0]) for p in per], "keys_per_rank": [int(p[1]) for p in per]},
                "roofline": None, "cpu_baseline": None,
                "dry_run": "no GPU visible: launch, partitioner and per-rank totals on CPU (gloo); nothing matched"}
        if shard_info is not None:
            line["config"]["shard"] = shard_info[1]
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus, argv))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: running {world} ranks", file=sys.stderr)
    if os.environ.get("KCEP_BENCH_FAIL_RANK") == str(rank):      # tests/test_bench_launch.py: a failing rank
        sys.exit(3)
    if args.dry_run or not torch.cuda.is_available():
        return dry_run(args, world, rank)
    if world > torch.cuda.device_count():
        raise SystemExit(f"bench.py: {world} ranks but only {torch.cuda.device_count()} GPUs visible")
    from kcep import native as N
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)

    C = CONFIGS[args.config]
    K = args.keys or C["keys"]
    n_req = args.events or C.get("events")
    key, cols, ts, ir, shard_info = workload(args.config, rank, world, K, n_req, dev, stream)
    n = int(key.numel())
    torch.cuda.synchronize(dev)
    exchange = None
    if world > 1:
        from kcep import shard as S
        exchange = S.CountExchange(dev)

    pat = N.CompiledPattern(ir)
    force = {"stencil": N.PATH_STENCIL, "chain": N.PATH_CHAIN, "runs": N.PATH_RUNS,
             "general": N.PATH_GENERAL}.get(args.force_path, 0)
    sess = N.Session(pat, n, mode=N.MODE_PROCESSOR, device=local, force_path=force,
                     lane_nfa={"auto": None, "wave": False, "lane": True}[args.nfa_kernel])
    if args.config == "c2" and not force:
        assert sess.path == N.PATH_STENCIL

    def step():
        sess.push(n, key.data_ptr(), [c.data_ptr() for c in cols], mem=N.MEM_DEVICE, stream=stream.cuda_stream)
        if exchange is not None:             # the path's one exchange: counts -> global match offsets
            exchange.post(sess, n, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kernel_ms, batch_ms = [], []
    if sess.path in (N.PATH_STENCIL, N.PATH_CHAIN):
        sess.set_timing(False)        # no event packets in the timed steps; kernel time is a separate pass
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if sess.path in (N.PATH_GENERAL, N.PATH_RUNS):   # these pushes sync internally; read the kernel time
            kernel_ms.append(sess.last_kernel_ms())
            batch_ms.append(sess.last_batch_ms())
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if sess.path in (N.PATH_STENCIL, N.PATH_CHAIN):
        # one more pass per step under HIP events on the launch stream (cep_last_kernel_ms)
        sess.set_timing(True)
        for _ in range(args.steps):
            step()
            kernel_ms.append(sess.last_kernel_ms())
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)

    n_matches, csum = sess.checksum()
    stats = torch.tensor([float(n), float(n_matches), elapsed], dtype=torch.float64, device=dev)
    tot_events, tot_matches, t_max = gather_stats(stats, world)
    exch = None
    if exchange is not None:
        off, node_ev, node_m = exchange.result((exchange.posted - 1) % exchange.slots)
        exch = {"collective": "RCCL all_gather of (events, matches) + exclusive scan, per step, side stream",
                "rank0_match_offset": off, "node_events": node_ev, "node_matches": node_m,
                "consistent": bool(node_ev == int(tot_events) and node_m == int(tot_matches))}
        if args.gather_matches:
            from kcep import shard as S
            out = sess.collect()
            dist.barrier()
            tg = time.perf_counter()
            merged = S.gather_matches(out, shard_info[0].perm, dst=0)
            dist.barrier()
            exch["gather_s"] = time.perf_counter() - tg
            if rank == 0:
                exch["gathered_matches"] = int(len(merged["match_record"]))

    if rank == 0:
        plain = (sess.path == N.PATH_STENCIL and pat.info.stencil_k <= 7
                 and os.environ.get("KCEP_STENCIL_KEYED") != "1")
        if sess.path in (N.PATH_STENCIL, N.PATH_CHAIN):
            k = pat.info.stencil_k
            algo_bytes = 8.0 * n + 4.0 * k * n_matches          # 8 B/event + 4k B/match
            # the plain kernel writes one int per match (its first record); stencil_gather writes
            # the k-int rows: the kernel's own algorithmic bytes are 8 B/event + 4 B/match
            kernel_bytes = 8.0 * n + 4.0 * n_matches if plain else algo_bytes
        else:
            out = sess.collect(raise_on_error=False)
            n_ent = len(out["ent_record"])
            # 8 B/event in (key + i32 value); CSR out: 20 B/match + 12 B/entry
            algo_bytes = 8.0 * n + 20.0 * n_matches + 12.0 * n_ent
            kernel_bytes = algo_bytes
        if sess.path in (N.PATH_STENCIL, N.PATH_CHAIN):
            # the plain kernel runs strict fixed-length patterns of k <= 7 (C2); the keyed one chains (C5)
            roof_ms, roof_kernel = avg_kernel_ms, "stencil_plain_kernel" if plain else "stencil_kernel"
        else:
            # these paths write their CSR in later launches (runs_write / nfa_compact), so the bytes
            # are divided by the whole step's device time (HIP events around cep_push_batch)
            roof_ms = sum(batch_ms) / len(batch_ms)
            roof_kernel = "whole cep_push_batch (" + ("runs_sim + runs_emit" if sess.path == N.PATH_RUNS
                                                       else "nfa kernel + compaction") + ")"
        achieved = kernel_bytes / (roof_ms * 1e-3) / 1e9
        value = tot_events * args.steps / t_max
        build = N.lib().cep_version().decode().rsplit(" ", 1)[-1]
        traffic, traffic_src = _pmc_traffic(args.config, n, build)
        line = {
            "metric": METRIC if args.config == "c2" else f"events/sec (whole node), {C['desc']}",
            "value": value,
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if C.get("node_wide") and world > 1 else "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (splitmix64 counter RNG, BASELINE.md §3)",
            "config": {"workload": C["desc"], "events_per_gpu": n, "keys_per_gpu": K,
                       "matches_per_gpu": int(n_matches), "matches_total": int(tot_matches),
                       "path": {N.PATH_STENCIL: "stencil", N.PATH_CHAIN: "chain", N.PATH_RUNS: "runs"}.get(sess.path, "general"),
                       "parallelism": f"key-hash sharded x{world}" if world > 1 else "1 GPU",
                       "kernels": "compiled for the pattern (hiprtc)" if sess.jit else "built-in",
                       "forced_path": args.force_path, "nfa_kernel": args.nfa_kernel},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": roof_kernel, "kernel_ms": roof_ms, "algo_bytes_per_launch": kernel_bytes,
                         "algo_bytes_per_step": algo_bytes},
            "cpu_baseline": None,
            "checksum": f"{csum:016x}",
            "build": build,
        }
        if shard_info is not None:
            line["config"]["shard"] = shard_info[1]
            line["config"]["exchange"] = exch
        if sess.path in (N.PATH_GENERAL, N.PATH_RUNS):
            line["batch_ms"] = roof_ms
            gname = ("kcep_nfa_wave" if sess.wave else "kcep_nfa_kernel") if sess.jit else (
                "nfa_wave_kernel" if sess.wave else "nfa_kernel")
            line["first_kernel"] = {"name": {N.PATH_GENERAL: gname,
                                             N.PATH_RUNS: "kcep_runs_sim" if sess.jit else "runs_sim"}[sess.path],
                                    "ms": avg_kernel_ms}
        if sess.path == N.PATH_GENERAL:
            line["config"]["live_run_hwm"] = sess.live_run_hwm()     # run-explosion high-water mark
            # keys the resident (uncapped) run handed back: they outgrew even the whole device pool
            erec, ecode = sess.batch_errors()
            line["config"]["keys_over_device_pool"] = int(sum(1 for c in ecode if c == N.E_RUN_CAPACITY))
        if world == 1 and args.config == "c4" and args.handoff_cap > 0 and not force:
            line["handoff"] = _handoff_leg(ir, key, cols[0], ts, K, C["per_key"], args.handoff_cap, stream)
            line["config"]["keys_on_cpu"] = line["handoff"]["keys_on_cpu"]
        if world == 1 and sess.path in (N.PATH_STENCIL, N.PATH_CHAIN) and not args.no_host_input:
            line["pcie_inclusive"], host = _pcie_inclusive(sess, n, key, cols, stream, csum)
            # the processor's own batch sizes (CEPStream.query batch_size defaults to 1 << 16): host
            # batches over PCIe, each collected, through a carry session
            line["processor_batches"] = [
                _carry_stream(pat, n, K, key, cols, stream, 0, n_matches, csum, value / world, reps=1, per=b,
                              host=host, collect=True) for b in args.processor_batch]
            del host
            # the same from pageable host memory, as a JVM heap array reaches the library through JNI
            # (GetPrimitiveArrayCritical): cep_push_batch copies it into the session's pinned ring
            pageable = (key.cpu().numpy(), [c.cpu().numpy() for c in cols])
            line["processor_batches"] += [
                _carry_stream(pat, n, K, key, cols, stream, 0, n_matches, csum, value / world, reps=1, per=b,
                              host=pageable, collect=True) for b in args.processor_batch]
            del pageable
            # the records as a Kafka partition delivers them: keys interleaved, in generation order (the C2
            # stream's ts column is each record's arrival position); the library groups each batch on the
            # device (CEP_BATCH_ARRIVAL_ORDER) and hands the matches back in arrival order
            line["processor_batches"] += [
                _arrival_batches(pat, n, K, key, cols, ts, stream, n_matches, csum, value / world, per=b, pipelined=p)
                for b in args.processor_batch for p in (False, True)]
        if world == 1 and sess.path in (N.PATH_STENCIL, N.PATH_CHAIN, N.PATH_RUNS) and args.carry_batches > 1:
            line["carry_stream"] = _carry_stream(pat, n, K, key, cols, stream, args.carry_batches, n_matches, csum,
                                                 value / world)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = _cpu_baseline(args.config, key, cols, ts, ir, args.cpu_threads, n_matches, csum,
                                                 sess, stream)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _pcie_inclusive(sess, n, key, cols, stream, csum, steps=3):
    """The same batch handed over in (pinned) host memory, as the JNI boundary would: each push
    stages the columns over PCIe before the kernels.  Reported beside `value`, never as it."""
    from kcep import native as N
    hk = key.cpu().pin_memory()
    hc = [c.cpu().pin_memory() for c in cols]
    sess.set_timing(False)

    def push():
        sess.push(n, hk.data_ptr(), [c.data_ptr() for c in hc], mem=N.MEM_HOST, stream=stream.cuda_stream)
    push()
    stream.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        push()
    stream.synchronize()
    dt = (time.perf_counter() - t0) / steps
    sess.set_timing(True)
    _, c2 = sess.checksum()
    return {"value": n / dt, "unit": "events/s", "ms_per_step": dt * 1e3, "host_memory": "pinned",
            "bytes_per_step": int(hk.numel() * hk.element_size() + sum(c.numel() * c.element_size() for c in hc)),
            "parity": c2 == csum}, (hk, hc)


def _carry_stream(pat, n, K, key, cols, stream, nb, n_matches, csum, resident, reps=3, per=None, host=None,
                  collect=False):
    """The same stream pushed through a CEP_SESSION_CARRY session (the GpuCEPProcessor route) in
    consecutive batches (`nb` of them, or of `per` records): keys cut at batch boundaries continue
    from their carried halos.  `host` = pinned host copies of (key, cols): every push stages its
    batch over PCIe, as the JNI boundary hands it; `collect`: every batch's CSR is materialised on
    the host (cep_collect), as the processor's flush does.  Parity: the batches' matches and
    checksums (over stream positions) add up to the one-batch run.  Reported beside `value`, never
    as it."""
    import torch
    from kcep import native as N
    if per is None:
        per = -(-n // nb)
        per = -(-per // 4096) * 4096                 # 16-B aligned batch starts
    bounds = list(range(0, n, per)) + [n]
    cs = N.Session(pat, per, mode=N.MODE_PROCESSOR, carry=True, max_keys=K)
    cs.set_timing(False)
    src_k, src_c = host if host is not None else (key, cols)
    mem = N.MEM_HOST if host is not None else N.MEM_DEVICE
    pageable = host is not None and not hasattr(src_k, "data_ptr")     # numpy arrays: pageable memory

    def addr(a):
        return a.ctypes.data if pageable else a.data_ptr()

    def esize(a):
        return a.itemsize if pageable else a.element_size()

    def one_pass(check):
        tot_m, tot_c = 0, 0
        for a, b in zip(bounds[:-1], bounds[1:]):
            cs.push(b - a, addr(src_k) + 4 * a, [addr(c) + esize(c) * a for c in src_c],
                    mem=mem, stream=stream.cuda_stream,
                    flags=N.BATCH_OFFSETS_MONOTONE | (N.BATCH_DELIVER if collect else 0))
            if check:
                m, c = cs.checksum()
                tot_m, tot_c = tot_m + m, (tot_c + c) & 0xFFFFFFFFFFFFFFFF
            elif collect:
                cs.collect()
        return tot_m, tot_c

    m, c = one_pass(True)
    stream.synchronize()
    times = []
    for _ in range(reps):
        cs.state_clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        one_pass(False)
        stream.synchronize()
        times.append(time.perf_counter() - t0)
    dt = min(times)
    nbat = len(bounds) - 1
    out = {"value": n / dt, "unit": "events/s", "batches": nbat, "events_per_batch": per,
           "ms_per_pass": dt * 1e3, "vs_resident": n / dt / resident,
           "path": {N.PATH_STENCIL: "stencil", N.PATH_CHAIN: "chain", N.PATH_RUNS: "runs"}.get(cs.path, "general"),
           "parity": bool(m == n_matches and c == csum), "matches": int(m)}
    if host is not None or collect:
        # per-batch cost above streaming the batch's records at the resident rate
        out.update({"host_memory": ("pageable" if pageable else "pinned") if host is not None else None,
                    "collect_per_batch": collect,
                    "us_per_batch": dt * 1e6 / nbat,
                    "overhead_us_per_batch": (dt - n / resident) * 1e6 / nbat})
    cs.close()
    return out


def _mix64(x):
    import numpy as np
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xff51afd7ed558ccd)
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xc4ceb9fe1a85ec53)
        return x ^ (x >> np.uint64(33))


def _csr_checksum(mrec, ent_off, ent_name, ent_rec, pos_map):
    """cep_checksum's order-independent sum (per match: mix64 over its record and traversal entries) of a
    host CSR, its record positions first mapped through pos_map (numpy, vectorised over matches)."""
    import numpy as np
    if len(mrec) == 0:
        return 0
    lens = np.diff(ent_off)
    with np.errstate(over="ignore"):
        h = _mix64(pos_map[mrec].astype(np.uint64) * np.uint64(0x9e3779b97f4a7c15))
        for t in range(int(lens.max())):
            sel = lens > t
            e = ent_off[:-1][sel] + t
            v = (pos_map[ent_rec[e]].astype(np.uint64) << np.uint64(8)) ^ ent_name[e].astype(np.uint64)
            h[sel] = _mix64(h[sel] ^ v)
        return int(h.sum(dtype=np.uint64))


def _arrival_batches(pat, n, K, key, cols, ts, stream, n_matches, csum, resident, per, pipelined=False):
    """The processor's flushes as a Kafka partition delivers the records: the C2 stream in its generation
    (arrival) order -- keys interleaved -- in pinned host batches of `per` records through a carry session,
    CEP_BATCH_ARRIVAL_ORDER | CEP_BATCH_DELIVER, each collected: the library groups every batch by key on
    the device and returns its matches in arrival order of the completing record, so no host sorts.
    Parity: the batches' matches, their stream (arrival) positions mapped back to the resident batch's
    positions, give the resident run's match count and checksum; and every batch's matches come in
    non-decreasing arrival order of their completing record (the reference's forward order).
    pipelined: batch i + 1 is pushed before batch i is collected (cep_collect_batch: double-buffered
    delivery), so the host's copy-in of the next batch overlaps the device's work on this one."""
    import numpy as np
    import torch
    from kcep import native as N
    ka = torch.empty_like(key)
    ka[ts] = key
    ca = []
    for c in cols:
        x = torch.empty_like(c)
        x[ts] = c
        ca.append(x)
    hk, hc = ka.cpu().pin_memory(), [c.cpu().pin_memory() for c in ca]
    del ka, ca
    pos_map = ts.cpu().numpy().copy()                      # arrival position -> resident batch position
    pos_map[pos_map.copy()] = np.arange(n)
    cs = N.Session(pat, per, mode=N.MODE_PROCESSOR, carry=True, max_keys=K)
    cs.set_timing(False)
    flags = N.BATCH_OFFSETS_MONOTONE | N.BATCH_DELIVER | N.BATCH_ARRIVAL_ORDER
    bounds = list(range(0, n, per)) + [n]

    def one_pass(check):
        parts, ordered = [], True

        def take(out):
            nonlocal ordered
            if check:
                mr = out["match_record"]
                ordered = ordered and bool(np.all(mr[1:] >= mr[:-1]))
                parts.append(out)
        prev = None
        for a, b in zip(bounds[:-1], bounds[1:]):
            cs.push(b - a, hk.data_ptr() + 4 * a, [c.data_ptr() + c.element_size() * a for c in hc], mem=N.MEM_HOST,
                    stream=stream.cuda_stream, flags=flags)
            if not pipelined:
                take(cs.collect())
                continue
            if prev is not None:
                take(cs.collect(batch_id=prev))
            prev = cs.batch_id()
        if pipelined and prev is not None:
            take(cs.collect(batch_id=prev))
        return parts, ordered

    parts, ordered = one_pass(True)
    m = sum(len(p["match_record"]) for p in parts)
    c = 0
    for p in parts:
        c = (c + _csr_checksum(p["match_record"], p["ent_off"], p["ent_name"], p["ent_record"], pos_map)) & ((1 << 64) - 1)
    del parts
    cs.state_clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    one_pass(False)
    stream.synchronize()
    dt = time.perf_counter() - t0
    cs.close()
    nbat = len(bounds) - 1
    return {"value": n / dt, "unit": "events/s", "batches": nbat, "events_per_batch": per, "ms_per_pass": dt * 1e3,
            "vs_resident": n / dt / resident, "path": "stencil" if cs.path == N.PATH_STENCIL else "chain",
            "parity": bool(m == n_matches and c == csum), "forward_order": ordered, "matches": int(m),
            "host_memory": "pinned", "collect_per_batch": True, "arrival_order": True, "pipelined": pipelined,
            "us_per_batch": dt * 1e6 / nbat, "overhead_us_per_batch": (dt - n / resident) * 1e6 / nbat}


def _kcrf_events(blob):
    """(offset, first column) of every event a KCRF state holds (include/kcep.h, cep_state_to_reference)."""
    import struct
    ncols = struct.unpack_from("<i", blob, 12)[0]
    at = 24
    (nh,) = struct.unpack_from("<i", blob, at)
    at += 4 + 12 * nh
    (ne,) = struct.unpack_from("<i", blob, at)
    at += 4
    evs = []
    for _ in range(ne):
        _, _, _, off, _ = struct.unpack_from("<qiiqq", blob, at)
        at += 32
        (c0,) = struct.unpack_from("<q", blob, at)
        at += 8 * ncols
        evs.append((off, c0))
    return evs


def _handoff_leg(ir, key, val, ts, K, L, cap, stream, nb=4):
    """BASELINE.md §3 C4's CPU-fallback count, measured: the workload through a CEP_SESSION_CARRY session
    (the GpuCEPProcessor route) in `nb` batches -- batch b holds records [b*L/nb, (b+1)*L/nb) of every key
    -- with the per-key workspace capped at `cap` words (cep_opts.max_key_words).  A key over the cap is
    handed back (CEP_E_RUN_CAPACITY, its state as of the batch start); as GpuCEPProcessor.handOff does,
    its state is evicted, rewritten in the reference's terms (cep_state_to_reference) and the key
    continues on the CPU -- here the oracle, the C restatement of the reference NFA, resumed from that
    form -- over the rest of its records.  Parity: every key's joined matches (device, then CPU) against
    the oracle's uninterrupted run, in the reference's per-key emission order.  C4's ts column is each
    record's index within its key, pushed as its offset too, so the CPU side maps back by offset."""
    import numpy as np
    import torch
    from kcep import native as N
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    per = L // nb
    pat = N.CompiledPattern(ir)
    s = N.Session(pat, K * per, mode=N.MODE_PROCESSOR, carry=True, max_keys=K, max_key_words=cap)
    kk, vv, tt = key.view(K, L), val.view(K, L), ts.view(K, L)
    keep = torch.ones(K, dtype=torch.bool, device=key.device)
    hv = val.cpu().numpy().reshape(K, L)
    pos2idx = np.zeros(K * L, np.int64)          # stream position -> index in the key-grouped stream
    dev_out, cpu_m, handed = [], {}, {}
    t_dev = t_cpu = 0.0
    for b in range(nb):
        rows = torch.nonzero(keep).flatten()
        bk = kk[rows, b * per:(b + 1) * per].contiguous().view(-1)
        bv = vv[rows, b * per:(b + 1) * per].contiguous().view(-1)
        bt = tt[rows, b * per:(b + 1) * per].contiguous().view(-1)
        rk = rows.cpu().numpy()
        base = s.stream_position()
        j = np.arange(len(rk) * per)
        pos2idx[base:base + len(j)] = rk[j // per] * L + b * per + j % per
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.push(bk.numel(), bk.data_ptr(), [bv.data_ptr()], ts=bt.data_ptr(), offset=bt.data_ptr(), mem=N.MEM_DEVICE,
               stream=stream.cuda_stream, flags=N.BATCH_OFFSETS_MONOTONE)
        out = s.collect(raise_on_error=False)
        erec, ecode = s.batch_errors()
        t_dev += time.perf_counter() - t0
        assert all(c == N.E_RUN_CAPACITY for c in ecode), "C4 raises no reference exception"
        cap_keys = sorted({int(rk[(int(r) - base) // per]) for r in erec})
        dev_out.append((out, set(cap_keys)))
        if not cap_keys:
            continue
        blobs = s.state_evict(cap_keys)
        keep[torch.tensor(cap_keys, device=key.device)] = False
        t1 = time.perf_counter()
        for k, blob in zip(cap_keys, blobs):                    # the reference continues the key
            handed[k] = b
            ref = pat.state_to_reference(blob) if blob else None
            evs = _kcrf_events(ref) if ref else []
            o_ = np.array([e[0] for e in evs] + list(range(b * per, L)), np.int64)
            v_ = np.array([e[1] for e in evs] + [int(hv[k, i]) for i in range(b * per, L)], np.int32)
            r = O.OracleRun(O.OraclePattern(ir), O.MODE_PROCESSOR)
            bat = O.BatchArrays(np.full(len(o_), k, np.int32), [v_], [1], offset=o_, ts=o_)
            if ref:
                r.resume(bat, ref)
            else:
                r.process(bat)
            cpu_m[k] = [(k * L + int(o_[m.record]), [(nm, k * L + int(o_[e])) for nm, e in m.traversal])
                        for m in r.matches(with_groups=False)]
        t_cpu += time.perf_counter() - t1
    got = {}
    for out, cap_keys in dev_out:                               # device matches, batch by batch
        mk, mr, eo = out["match_key"], pos2idx[out["match_record"]], out["ent_off"]
        en, er = out["ent_name"], pos2idx[out["ent_record"]]
        for m in range(len(mk)):
            k = int(mk[m])
            if k not in cap_keys:
                got.setdefault(k, []).append((int(mr[m]), list(zip(en[eo[m]:eo[m + 1]].tolist(),
                                                                    er[eo[m]:eo[m + 1]].tolist()))))
    for k, ms in cpu_m.items():                                 # then the CPU's, after the hand-off
        got.setdefault(k, []).extend(ms)
    hk = key.cpu().numpy()
    want_csr = O.baseline_csr(O.OraclePattern(ir), O.BatchArrays(hk, [val.cpu().numpy()], [1],
                                                                 ts=ts.cpu().numpy()), O.MODE_PROCESSOR,
                              max(1, min(16, os.cpu_count() or 1)))
    want = {}
    wk, wr, wo, wn, we = (want_csr[f] for f in ("match_key", "match_record", "ent_off", "ent_name", "ent_record"))
    for m in range(len(wk)):
        want.setdefault(int(wk[m]), []).append((int(wr[m]), list(zip(wn[wo[m]:wo[m + 1]].tolist(),
                                                                      we[wo[m]:wo[m + 1]].tolist()))))
    parity = all(got.get(k, []) == want.get(k, []) for k in set(got) | set(want))
    s.close()
    diff = None
    if not parity:                                              # the first key that differs, for the record
        k = next(k for k in sorted(set(got) | set(want)) if got.get(k, []) != want.get(k, []))
        diff = {"key": k, "handed_back_in_batch": handed.get(k), "device_or_cpu": got.get(k, [])[:4],
                "reference": want.get(k, [])[:4], "n_got": len(got.get(k, [])), "n_want": len(want.get(k, []))}
    return {"cap_words": cap, "batches": nb, "keys_on_cpu": len(handed),
            "handed_back_per_batch": [sum(1 for v in handed.values() if v == b) for b in range(nb)],
            "device_s": t_dev, "cpu_continuation_s": t_cpu,
            "matches": int(sum(len(v) for v in got.values())), "parity": bool(parity), "first_difference": diff,
            "how": "keys over the cap: cep_state_evict -> cep_state_to_reference -> oracle resume (GpuCEPProcessor.handOff)"}


def _pmc_traffic(cfg, n, build):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (if any), FETCH_SIZE doubled per
    the gfx950 correction (MI355X_MICROARCH.md §HBM), and where they come from: the summary file, the
    library build (source hash, cep_version) and commit its counters were taken on, and whether that is
    the build this run measures.  rocprofv3 --pmc cannot run inside this process (tools/gpu_prof.sh
    collects it in separate passes of the same command)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json" if cfg == "c2" else f"pmc_traffic_{cfg}.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if int(d.get("events")) != n:
            return None, None
        return float(d["hbm_bytes_per_launch"]), {
            "file": os.path.relpath(p, ROOT), "pmc": d.get("source"), "build": d.get("build"),
            "commit": d.get("commit"), "same_build_as_this_run": d.get("build") == build}
    except Exception:
        return None, None


def host_cpu():
    """The host the CPU baseline runs on: CPU model, logical CPUs, physical cores (distinct
    (package, core) pairs of /proc/cpuinfo), the CPUs this process may run on (nproc) and the
    cgroup CPU quota, if any (a GPU box may grant a share of a larger machine)."""
    model, phys, cur = None, set(), {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and model is None:
                    model = v
                elif k in ("physical id", "core id"):
                    cur[k] = v
                elif not k and cur:
                    phys.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"model": model, "logical_cpus": os.cpu_count(), "physical_cores": len(phys) or None,
            "nproc": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota}


def _cpu_baseline(cfg, key, cols, ts, ir, threads, gpu_matches, gpu_csum, sess, stream):
    """The oracle (C restatement of the reference NFA) on the host cores.

    The full workload (same arrays) on ``threads`` threads (default: the CPUs this
    process may use, capped by the cgroup quota), parity by match count + checksum
    against the GPU's run of the same batch.  Plus a 1-core figure on a whole-key
    prefix of ~4M events."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from kcep import native as N
    hk = key.cpu().numpy()
    hc = [c.cpu().numpy() for c in cols]
    ho = ts.cpu().numpy()
    p = O.OraclePattern(ir)
    cpu = host_cpu()
    # every CPU this process may run on (nproc), capped by the cgroup CPU quota: a GPU box grants
    # a share of a larger machine, and threads beyond the quota only time-slice (measured slower)
    usable = cpu["nproc"] if not cpu["cgroup_cpu_quota"] else min(cpu["nproc"], max(1, int(cpu["cgroup_cpu_quota"])))
    threads = max(1, threads or usable)

    def prefix(m):
        m = min(len(hk), m)
        while 0 < m < len(hk) and hk[m] == hk[m - 1]:
            m += 1
        return m

    m_all = len(hk)                     # the whole workload (<= ~10 s on the box's CPU share)
    b = O.BatchArrays(hk[:m_all], [c[:m_all] for c in hc], [1] * len(hc), offset=ho[:m_all] if cfg == "c2" else None,
                      ts=ho[:m_all])
    t0 = time.perf_counter()
    nm, cs = O.baseline(p, b, O.MODE_PROCESSOR, threads)
    dt = time.perf_counter() - t0
    m1 = prefix(4_000_000)
    b1 = O.BatchArrays(hk[:m1], [c[:m1] for c in hc], [1] * len(hc), offset=ho[:m1] if cfg == "c2" else None,
                       ts=ho[:m1])
    t1 = time.perf_counter()
    O.baseline(p, b1, O.MODE_PROCESSOR, 1)
    dt1 = time.perf_counter() - t1
    return {"value": m_all / dt, "unit": "events/s", "cores": threads, "kind": "port",
            "sample": f"full workload ({m_all} events) on {threads} threads (key-sharded; nproc "
                      f"{cpu['nproc']}, cgroup CPU quota {cpu['cgroup_cpu_quota']}); 1-core figure on a {m1}-event "
                      f"whole-key prefix",
            "model": cpu["model"], "host": cpu, "seconds": dt,
            "value_1core": m1 / dt1, "parity": bool(nm == gpu_matches and cs == gpu_csum),
            "oracle_matches": int(nm)}


if __name__ == "__main__":
    main()
