"""Key-hash sharding of the NFA path across the GPUs of one node.

The reference scales through Kafka: the producer partitions records by key hash,
each stream task owns the NFAs of its keys, and tasks never exchange state
(``README.md:348-355``; the run counter is per key, ``NFAStates.java:36``; buffer
nodes and aggregates are keyed per record key).  A node does the same with one
process per GPU:

* **Partitioner** -- ``shard_plan`` assigns every key a shard (``fmix32(key) %
  G``, optionally rebalanced to equal event counts, sticky across batches) and
  ``partition``/``take`` split a batch by a stable counting sort on the device or
  on the host (``cep_partition`` / ``cep_gather``), so each shard keeps the
  batch's key grouping and per-key arrival order.
* **Matching** -- each rank pushes its shard to its own session.  No data
  crosses GPUs while matching.
* **Exchange** -- the only collective: an all-gather of every rank's
  ``(n_events, n_matches)`` and an exclusive scan of the match counts, which
  gives each rank the global offset of its matches (``CountExchange`` runs it on
  a side stream so it overlaps the next batch).  ``gather_matches`` optionally
  sends the ranks' match CSRs to one rank, renumbered to global record
  positions and merged into the single-GPU order.

Collectives go through ``torch.distributed``: ``nccl`` (RCCL over xGMI) on GPUs,
``gloo`` in the CPU tests.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import native as N


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def key_shard(key_id: int, n_shards: int) -> int:
    """Default shard of a key: ``fmix32(key_id) % n_shards`` (``cep_key_shard``)."""
    return int(N.lib().cep_key_shard(int(key_id), int(n_shards)))


def shard_plan(key_events, n_shards: int, rebalance: bool = True):
    """Key -> shard table for dense key ids ``[0, len(key_events))`` (``cep_shard_plan``).

    Returns ``(table int32[n_keys], shard_events int64[n_shards])``.  Compute it once and pass it
    to every ``partition`` of a carry deployment: a key must stay on its GPU across batches."""
    ev = np.ascontiguousarray(key_events, dtype=np.int64)
    table = np.zeros(len(ev), np.int32)
    loads = np.zeros(n_shards, np.int64)
    N.check(N.lib().cep_shard_plan(ev.ctypes.data if len(ev) else None, len(ev), int(n_shards),
                                   1 if rebalance else 0, table.ctypes.data if len(ev) else None,
                                   loads.ctypes.data))
    return table, loads


def partition(key, n_shards: int, table=None, stream=None):
    """Stable split of a batch by shard (``cep_partition``).

    ``key`` is a numpy int32 array (host path) or an int32 CUDA tensor (device path: kernels on
    ``stream``, no host sync; ``table`` must then be a device tensor too).  Returns ``(perm,
    shard_off)`` of the same kind: shard ``s`` owns ``perm[shard_off[s]:shard_off[s+1]]``, the
    batch positions of its records in batch order."""
    if _is_torch(key) and not key.is_cuda:                 # CPU tensors: the host path
        import torch
        perm, off = partition(key.numpy(), n_shards, None if table is None else np.asarray(table))
        return torch.from_numpy(perm), torch.from_numpy(off)
    if _is_torch(key):
        import torch
        n = int(key.numel())
        perm = torch.empty(n, dtype=torch.int64, device=key.device)
        off = torch.empty(n_shards + 1, dtype=torch.int64, device=key.device)
        tp = table.data_ptr() if table is not None else None
        nk = int(table.numel()) if table is not None else 0
        N.check(N.lib().cep_partition(key.data_ptr() if n else None, n, int(n_shards), tp, nk,
                                      perm.data_ptr() if n else None, off.data_ptr(), N.MEM_DEVICE,
                                      C.c_void_p(stream) if stream else None))
        return perm, off
    key = np.ascontiguousarray(key, dtype=np.int32)
    n = len(key)
    perm = np.empty(n, np.int64)
    off = np.empty(n_shards + 1, np.int64)
    tab = None if table is None else np.ascontiguousarray(table, dtype=np.int32)
    N.check(N.lib().cep_partition(key.ctypes.data if n else None, n, int(n_shards),
                                  tab.ctypes.data if tab is not None else None, 0 if tab is None else len(tab),
                                  perm.ctypes.data if n else None, off.ctypes.data, N.MEM_HOST, None))
    return perm, off


def take(src, perm, stream=None):
    """``src[perm]`` through ``cep_gather`` (host numpy arrays or CUDA tensors, 1/4/8-byte
    elements): one column of a shard."""
    if _is_torch(src) and not src.is_cuda:
        import torch
        return torch.from_numpy(take(src.numpy(), perm.numpy() if _is_torch(perm) else perm))
    if _is_torch(src):
        import torch
        n = int(perm.numel())
        dst = torch.empty(n, dtype=src.dtype, device=src.device)
        N.check(N.lib().cep_gather(src.data_ptr() if src.numel() else None, src.element_size(),
                                   perm.data_ptr() if n else None, n, dst.data_ptr() if n else None, N.MEM_DEVICE,
                                   C.c_void_p(stream) if stream else None))
        return dst
    src = np.ascontiguousarray(src)
    perm = np.ascontiguousarray(perm, dtype=np.int64)
    dst = np.empty(len(perm), src.dtype)
    if len(perm):
        N.check(N.lib().cep_gather(src.ctypes.data, src.itemsize, perm.ctypes.data, len(perm), dst.ctypes.data,
                                   N.MEM_HOST, None))
    return dst


class Shard:
    """One rank's share of a node-wide batch: its columns and the batch positions they came from."""

    def __init__(self, rank: int, perm, key, cols, extra: Optional[Dict[str, object]] = None):
        self.rank = rank
        self.perm = perm          # positions of this shard's records in the node-wide batch
        self.key = key
        self.cols = list(cols)
        self.extra = extra or {}  # valid / topic / partition / offset / ts, when the batch has them

    @property
    def n(self) -> int:
        return int(self.perm.numel() if _is_torch(self.perm) else len(self.perm))


def split(rank: int, n_shards: int, key, cols: Sequence, table=None, stream=None, **extra) -> Shard:
    """The shard of ``rank`` of a batch (every array host numpy or every array CUDA tensors)."""
    perm, off = partition(key, n_shards, table, stream)
    if _is_torch(off):
        lo, hi = (int(x) for x in off[rank:rank + 2].cpu())
    else:
        lo, hi = int(off[rank]), int(off[rank + 1])
    p = perm[lo:hi]
    if _is_torch(p):
        p = p.contiguous()
    return Shard(rank, p, take(key, p, stream), [take(c, p, stream) for c in cols],
                 {k: take(v, p, stream) for k, v in extra.items() if v is not None})


# ---- the one exchange step ----
def _backend_device(device=None):
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        return device if device is not None else torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def exchange_counts(n_events: int, n_matches: int, device=None):
    """All-gather every rank's ``(n_events, n_matches)``; returns ``(counts int64[world, 2], match
    offset of this rank, total events, total matches)`` -- the exclusive scan of the match counts."""
    import torch
    import torch.distributed as dist
    dev = _backend_device(device)
    world, rank = dist.get_world_size(), dist.get_rank()
    mine = torch.tensor([int(n_events), int(n_matches)], dtype=torch.int64, device=dev)
    allc = torch.empty(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allc, mine)
    allc = allc.view(world, 2).cpu()
    offs = torch.cumsum(allc[:, 1], 0) - allc[:, 1]
    return allc.numpy(), int(offs[rank]), int(allc[:, 0].sum()), int(allc[:, 1].sum())


class CountExchange:
    """Per-batch count exchange that overlaps the next batch: after a push, the session's
    device-resident match count is copied into a slot on the launch stream; a side stream waits
    for it and all-gathers ``(n_events, n_matches)`` of every rank over RCCL, then scans the match
    counts into each rank's global match offset -- all device-side, no host sync."""

    def __init__(self, device, slots: int = 64):
        import torch
        import torch.distributed as dist
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.device = device
        self.slots = slots
        self.mine = torch.zeros(slots, 2, dtype=torch.int64, device=device)
        self.allc = torch.zeros(slots, self.world, 2, dtype=torch.int64, device=device)
        self.offset = torch.zeros(slots, dtype=torch.int64, device=device)   # this rank's global match offset
        self.total = torch.zeros(slots, 2, dtype=torch.int64, device=device)  # node-wide (events, matches)
        self.side = torch.cuda.Stream(device=device)
        self.done = [None] * slots       # per slot: the side-stream event of its last exchange
        self.posted = 0

    def post(self, session: "N.Session", n_events: int, stream) -> int:
        """Enqueue the exchange of the session's last batch; returns its slot.  Everything the
        slot's inputs need is ordered on ``stream`` (the launch stream), after the slot's previous
        exchange has finished reading them."""
        import torch
        import torch.distributed as dist
        k = self.posted % self.slots
        self.posted += 1
        if self.done[k] is not None:     # the slot is reused: its last all-gather must have read it
            stream.wait_event(self.done[k])
        with torch.cuda.stream(stream):
            self.mine[k, 0].fill_(int(n_events))
        session.match_count_to(self.mine[k, 1].data_ptr(), stream.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(stream)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ev)
            dist.all_gather_into_tensor(self.allc[k].view(-1), self.mine[k])
            c = self.allc[k, :, 1]
            self.offset[k] = (torch.cumsum(c, 0) - c)[self.rank]
            self.total[k] = self.allc[k].sum(0)
            self.done[k] = torch.cuda.Event()
            self.done[k].record(self.side)
        return k

    def wait(self):
        self.side.synchronize()

    def result(self, slot: int):
        """(this rank's global match offset, node events, node matches) of a posted slot."""
        self.wait()
        return int(self.offset[slot]), int(self.total[slot, 0]), int(self.total[slot, 1])


def globalize(out: dict, perm) -> dict:
    """A shard's collected CSR (``Session.collect``) with batch positions renumbered to positions of
    the node-wide batch (non-carry sessions: record positions are shard batch indices)."""
    p = perm.cpu().numpy() if _is_torch(perm) else np.asarray(perm)
    g = dict(out)
    g["match_record"] = p[out["match_record"]] if len(out["match_record"]) else np.zeros(0, np.int64)
    g["ent_record"] = p[out["ent_record"]] if len(out["ent_record"]) else np.zeros(0, np.int64)
    return g


def merge(outs: List[dict]) -> dict:
    """Merge globalized shard CSRs into the order one GPU emits for the whole batch: matches by key
    in batch order, per key in emission order.  Keys are contiguous in the batch and a key's matches
    complete at its own records in non-decreasing order, so a stable sort by the emitting record
    is that order (several matches of one record keep ``matchPattern``'s order)."""
    mr = np.concatenate([o["match_record"] for o in outs]) if outs else np.zeros(0, np.int64)
    mk = np.concatenate([o["match_key"] for o in outs]) if outs else np.zeros(0, np.int32)
    lens = np.concatenate([np.diff(o["ent_off"]) for o in outs]) if outs else np.zeros(0, np.int64)
    starts = np.concatenate([o["ent_off"][:-1] + sum(len(x["ent_name"]) for x in outs[:i])
                             for i, o in enumerate(outs)]) if outs else np.zeros(0, np.int64)
    en = np.concatenate([o["ent_name"] for o in outs]) if outs else np.zeros(0, np.int32)
    er = np.concatenate([o["ent_record"] for o in outs]) if outs else np.zeros(0, np.int64)
    order = np.argsort(mr, kind="stable")
    lens_o = lens[order]
    ent_off = np.zeros(len(order) + 1, np.int64)
    np.cumsum(lens_o, out=ent_off[1:])
    idx = (np.concatenate([np.arange(s, s + l) for s, l in zip(starts[order], lens_o)])
           if len(order) else np.zeros(0, np.int64)).astype(np.int64)
    return dict(match_record=mr[order], match_key=mk[order], ent_off=ent_off, ent_name=en[idx],
                ent_record=er[idx])


def _pack(out: dict):
    nm, ne = len(out["match_record"]), len(out["ent_name"])
    return np.concatenate([np.array([nm, ne], np.int64), out["match_record"].astype(np.int64),
                           out["match_key"].astype(np.int64), out["ent_off"].astype(np.int64),
                           out["ent_name"].astype(np.int64), out["ent_record"].astype(np.int64)])


def _unpack(a: np.ndarray) -> dict:
    nm, ne = int(a[0]), int(a[1])
    at = 2
    def cut(k, dt):
        nonlocal at
        x = a[at:at + k].astype(dt)
        at += k
        return x
    return dict(match_record=cut(nm, np.int64), match_key=cut(nm, np.int32), ent_off=cut(nm + 1, np.int64),
                ent_name=cut(ne, np.int32), ent_record=cut(ne, np.int64))


def gather_matches(out: dict, perm, dst: int = 0, device=None) -> Optional[dict]:
    """Send every rank's CSR (renumbered to node-wide batch positions) to rank ``dst``, which returns
    them merged into the single-GPU order; other ranks return None.  Point-to-point over RCCL (or
    gloo): per match its emitting record, key and entries -- for a k-stage strict pattern 12 B/match
    of record indices plus the bookkeeping words."""
    import torch
    import torch.distributed as dist
    dev = _backend_device(device)
    world, rank = dist.get_world_size(), dist.get_rank()
    mine = _pack(globalize(out, perm))
    if rank != dst:
        dist.send(torch.tensor([len(mine)], dtype=torch.int64, device=dev), dst)
        dist.send(torch.from_numpy(mine).to(dev), dst)
        return None
    parts = []
    for r in range(world):
        if r == rank:
            parts.append(_unpack(mine))
            continue
        ln = torch.zeros(1, dtype=torch.int64, device=dev)
        dist.recv(ln, r)
        buf = torch.zeros(int(ln.item()), dtype=torch.int64, device=dev)
        dist.recv(buf, r)
        parts.append(_unpack(buf.cpu().numpy()))
    return merge(parts)
