"""GpuCEPProcessor: batching host mirror of the reference ``CEPProcessor``.

Reference: ``cep/processor/CEPProcessor.java:46-171``.  The reference steps one
key's NFA per ``process(key, value)`` call, loading and saving the key's state in
its stores around each record (``loadNFA`` ``:111-124``, ``nfaStore.put``
``:144-147``) and forwarding the completed ``Sequence``s at once (``:148``).

This processor keeps the same contract but hands the records to the device in
batches: ``process`` appends the record to a host buffer and a
flush -- on ``batch_size`` records, ``punctuate`` or ``close`` -- does one
``cep_push_batch`` on a carry session (``CEP_SESSION_CARRY``), whose device-side
per-key state (run queue, runs counter, high-water marks, buffer nodes, fold
registers) plays the role of the reference's three stores.

* **Null filter** (``:135-138``): a record with a null key or value is dropped
  before anything else, so it neither touches state nor moves the high-water
  mark.
* **High-water mark** (``:140, 152-160``): evaluated on the device per key and
  topic, across batches.
* **Keys and topics** are interned to dense ids (``key_id`` for the carry
  session, topic ids from the pattern's ``Schema`` so that ``withTopic`` filters
  keep their ids).  The session holds ``max_keys`` key ids; a batch that needs
  more spills the least recently used keys' state to the host
  (``cep_state_evict``) and re-admits a spilled key under a free id when it
  returns (``cep_state_import_keys``), so the number of distinct keys over the
  stream's life is unbounded, like the reference's ``NFAStore``
  (``NFAStoreImpl.java:34-85``).
* **Capacity hand-off.**  A key the device hands back with ``CEP_E_RUN_CAPACITY``
  (over ``max_key_words``) keeps its state as of the batch start; its records of
  the batch are pushed again with the per-key cap lifted, so every record is
  processed (``:134-150``).  Only a key that outgrows the whole device pool fails
  the task.
* **Values** are decoded into the schema's typed columns by a
  ``kcep.ingest.ColumnDecoder``.
* **Forward order.**  Each batch goes to the device in arrival order
  (``CEP_BATCH_ARRIVAL_ORDER``): the library groups it by key on the device and
  returns the matches in arrival order of their completing record (one record's
  matches in ``matchPattern``'s order), so the host sorts nothing.  The forwarded
  stream is therefore exactly the reference's, record for record -- only delayed
  to the flush.
* **Errors.**  Where the reference throws out of ``process()`` (user-predicate
  exceptions, ``UnknownAggregateException``, the buffer's ``IllegalStateException``)
  the flush forwards the matches of the records that arrived before the failing
  one and raises ``CepError``; the processor is then failed, as the reference's
  stream task is.  The device reports every failing key of the batch
  (``cep_batch_errors``), so the failure picked is the first in arrival order,
  where the reference's ``process()`` throws.
* **Query name** normalisation copies ``:83``: ``toLowerCase()`` then
  ``String.replace("\\\\s+", "")``, which is a *literal* replace in Java (no regex).
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import numpy as np

from . import native as N
from .ingest import ColumnDecoder
from .pattern import Pattern, Schema
from .sequence import Event, Sequence, sequence_from_traversal


class ProcessorFailed(RuntimeError):
    pass


# carry blob layout (csrc/kcep_dev.h CB_*, nfa_dev.h export_state): per key a header of CB_HDR
# words, then 3 words per high-water mark, 4 per queued run, then the carried events, each
# carry_evw(ncols) = 8 + 2*ncols words starting with its stream position (int64)
_CB_HDR, _CB_NHWM, _CB_QLEN, _CB_NEV, _CB_NCOLS = 12, 3, 4, 5, 10


def carried_positions(blob: bytes) -> set:
    """Stream positions of every event a ``cep_state_export`` blob carries: the general path's
    "KCST" blobs (run queues, buffer nodes, events) or the stencil path's "KCSH" halos (each key's
    last K-1 records)."""
    hdr = np.frombuffer(blob, np.int32, 5, 0)
    nkeys = int(hdr[4])
    out = set()
    at = 20
    if blob[:4] == b"KCSH":
        for _ in range(nkeys):
            cnt = int(np.frombuffer(blob, np.int32, 1, at + 4)[0])
            out.update(int(x) for x in np.frombuffer(blob, np.int64, cnt, at + 16))
            at += 16 + 8 * cnt
        return out
    for _ in range(nkeys):
        w = int(np.frombuffer(blob, np.int32, 1, at + 4)[0])
        words = np.frombuffer(blob, np.int32, w, at + 8)
        nev = int(words[_CB_NEV])
        if nev:
            evw = 8 + 2 * int(words[_CB_NCOLS])
            e0 = _CB_HDR + 3 * int(words[_CB_NHWM]) + 4 * int(words[_CB_QLEN])
            ev = words[e0:e0 + nev * evw].reshape(nev, evw)
            pos = ev[:, 0].astype(np.uint32).astype(np.int64) | (ev[:, 1].astype(np.int64) << 32)
            out.update(int(x) for x in pos)
        at += 8 + 4 * w
    return out


class GpuCEPProcessor:
    """One stream task's processor for one query (``CEPProcessor`` equivalent)."""

    def __init__(self, queryName: str, pattern: Union[Pattern, bytes], schema: Schema, decoder: ColumnDecoder,
                 batch_size: int = 1 << 16, max_keys: int = 1 << 20, device: int = 0,
                 mode: int = N.MODE_PROCESSOR, prune_at: int = 1 << 20, max_key_words: int = 0):
        if decoder.schema is not schema and decoder.schema.columns != schema.columns:
            raise ValueError("decoder and pattern use different schemas")
        self.queryName = queryName.lower().replace("\\s+", "")
        self.schema = schema
        self.decoder = decoder
        self.batch_size = int(batch_size)
        self.max_keys = int(max_keys)
        self.max_key_words = int(max_key_words)
        self.device = device
        self.mode = mode
        ir = pattern if isinstance(pattern, (bytes, bytearray)) else pattern.to_ir(schema)
        self.compiled = N.CompiledPattern(bytes(ir))
        self.session: Optional[N.Session] = None
        self._forward: Optional[Callable[[Any, Sequence], None]] = None
        # record key -> device key id.  The session holds max_keys ids; when a batch needs more, the
        # least recently used keys are spilled to the host (cep_state_evict) and re-admitted under a
        # free id when they come back (cep_state_import_keys): the reference's NFAStore is unbounded
        # (NFAStoreImpl.java:34-85).
        self._keys: Dict[Any, int] = {}
        self._id_key: Dict[int, Any] = {}
        self._free: List[int] = []
        self._next_id = 0
        self._used = np.zeros(0, np.int64)        # per key id: the flush that last used it (LRU)
        self._flushes = 0
        self._spilled: Dict[Any, Tuple[bytes, np.ndarray]] = {}   # key -> (single-key blob, positions)
        self._pending: List[Tuple[Any, tuple, int, int, int, int, Event]] = []
        self._log: Dict[int, Event] = {}          # stream position -> Event (carried runs point back here)
        self._failed: Optional[Exception] = None
        self._hwm: Dict[Tuple[Any, int], int] = {}  # stencil sessions: (record key, topic id) -> high-water mark
        self._prune_at = max(int(prune_at), 2 * self.batch_size)   # _log size that triggers a prune
        self._prune_min = self._prune_at
        self.capacity_reruns = 0                  # keys re-run with the per-key workspace cap lifted
        self._arrived = 0                         # non-null records flushed so far (error records are numbered so)

    # ---- Processor API (CEPProcessor.init/process/punctuate/close, :88-170) ----
    def init(self, forward: Callable[[Any, Sequence], None], session=None):
        """``forward(key, sequence)`` is ``ProcessorContext.forward`` (``:148``).  ``session``
        defaults to a carry ``kcep.native.Session`` on ``device`` (tests pass a stand-in to
        check the host logic without a GPU)."""
        self._forward = forward
        self.session = session or N.Session(self.compiled, self.batch_size, mode=self.mode, device=self.device,
                                            carry=True, max_keys=self.max_keys, max_key_words=self.max_key_words)

    def process(self, key, value, topic: str, partition: int, offset: int, timestamp: int):
        """One record with its ``ProcessorContext`` metadata."""
        self._check()
        if key is None or value is None:                  # :135-138
            return
        row = self.decoder.row(value)
        ev = Event(key, value, int(timestamp), topic, int(partition), int(offset))
        self._pending.append((key, row, self.schema.topic_id(topic), int(partition), int(offset), int(timestamp), ev))
        if len(self._pending) >= self.batch_size:
            self.flush()

    def punctuate(self, timestamp: int):
        self.flush()

    def close(self):
        try:
            if self._failed is None and self.session is not None:
                self.flush()
        finally:
            if self.session is not None:
                self.session.close()
                self.session = None

    # ---- key ids ----
    def _key_ids(self, recs) -> np.ndarray:
        """Device key id of every record: interned keys keep theirs; new and spilled keys take free
        ids, spilling the least recently used keys of earlier batches when none is left."""
        self._flushes += 1
        want = list(dict.fromkeys(r[0] for r in recs))    # distinct keys, first-arrival order
        if len(want) > self.max_keys:
            raise N.CepError(11, f"one batch holds {len(want)} distinct keys, more than max_keys={self.max_keys}")
        new = [k for k in want if k not in self._keys]
        short = len(new) - len(self._free) - (self.max_keys - self._next_id)
        if short > 0:
            self._spill(max(short, self.max_keys // 8), set(want))
        admit_keys, admit_ids, admit_blobs = [], [], []
        for k in new:
            kid = self._free.pop() if self._free else self._take_id()
            self._keys[k] = kid
            self._id_key[kid] = k
            sp = self._spilled.pop(k, None)
            if sp is not None:
                admit_keys.append(k)
                admit_ids.append(kid)
                admit_blobs.append(sp[0])
        if admit_ids:
            self.session.state_import_keys(admit_blobs, admit_ids)
        ids = np.fromiter((self._keys[r[0]] for r in recs), np.int32, len(recs))
        if len(self._used) < self._next_id:
            self._used = np.concatenate([self._used, np.zeros(self._next_id - len(self._used), np.int64)])
        self._used[ids] = self._flushes
        return ids

    def _take_id(self) -> int:
        self._next_id += 1
        return self._next_id - 1

    def _spill(self, count: int, busy: set):
        """Move the ``count`` least recently used keys not in this batch to the host."""
        cand = [kid for kid in np.argsort(self._used[:self._next_id], kind="stable")
                if int(kid) in self._id_key and self._id_key[int(kid)] not in busy][:count]
        if not cand:
            return
        blobs = self.session.state_evict(cand)
        for kid, blob in zip(cand, blobs):
            kid = int(kid)
            k = self._id_key.pop(kid)
            del self._keys[k]
            self._free.append(kid)
            if blob:                                      # a key without state starts afresh anyway
                self._spilled[k] = (blob, N.state_positions(blob))

    # ---- batching ----
    def _run(self, recs, idx):
        """One cep_push_batch of the records ``recs[i] for i in idx`` (arrival indices, ascending), in
        arrival order (the device groups them by key).  Returns ``(matches, errors)``: per match (arrival
        index of the completing record, key id, traversal entries as (name id, stream position)) in
        forward order, and per failing key (arrival index, code)."""
        n = len(idx)
        perm = np.asarray(idx, np.int64)                  # arrival index of batch position
        sorted_recs = [recs[i] for i in perm]
        cols = self.decoder.columns([r[1] for r in sorted_recs])
        topic = np.fromiter((r[2] for r in sorted_recs), np.int32, n)
        part = np.fromiter((r[3] for r in sorted_recs), np.int32, n)
        off = np.fromiter((r[4] for r in sorted_recs), np.int64, n)
        ts = np.fromiter((r[5] for r in sorted_recs), np.int64, n)
        base = self.session.stream_position()
        for i, r in enumerate(sorted_recs):
            self._log[base + i] = r[6]
        try:
            self.session.push(n, np.ascontiguousarray(self._kid[perm]), cols, topic=topic, partition=part, offset=off,
                              ts=ts, flags=self._flags | N.BATCH_DELIVER | N.BATCH_ARRIVAL_ORDER)
            out = self.session.collect(raise_on_error=False)
        except N.CepError as e:                           # no state was committed for this batch:
            self._failed = e                              # the task fails, as the reference's does
            raise
        mrec = out["match_record"] - base                 # stream position -> batch position
        matches = []
        for m in range(len(mrec)):
            a, b = int(out["ent_off"][m]), int(out["ent_off"][m + 1])
            matches.append((int(perm[mrec[m]]), int(out["match_key"][m]),
                            [(int(out["ent_name"][i]), int(out["ent_record"][i])) for i in range(a, b)]))
        errors = []
        if out["err"]:
            erec, ecode = self.session.batch_errors()
            errors = [(int(perm[r - base]), int(c)) for r, c in zip(erec, ecode)]
        return matches, errors

    def flush(self) -> int:
        """Push the buffered records as one batch and forward its matches; returns how many."""
        self._check()
        if not self._pending:
            return 0
        recs, self._pending = self._pending, []
        base = self._arrived                              # non-null records handed to process() before this flush
        self._arrived += len(recs)
        arrival = list(range(len(recs)))                  # the processor-wide arrival index of recs[i] is base + this
        self._flags = 0
        if self.session.path in (N.PATH_STENCIL, N.PATH_CHAIN, N.PATH_RUNS):
            # the stencil / chain / runs paths carry each key's records (its last K-1, or those
            # from its oldest open run on), not its NFA: the high-water-mark rule
            # (CEPProcessor.checkHighWaterMark :152-160) is applied here, in arrival order, and the
            # batch handed over has increasing offsets per key and topic.  Every admitted record is
            # processed and moves the mark (a record that throws fails the task anyway).
            kept, arrival = [], []
            for i, r in enumerate(recs):
                hk = (r[0], r[2])
                if r[4] < self._hwm.get(hk, -1):
                    continue
                self._hwm[hk] = r[4] + 1
                kept.append(r)
                arrival.append(i)
            recs = kept
            self._flags = N.BATCH_OFFSETS_MONOTONE
            if not recs:
                return 0
        self._kid = self._key_ids(recs)
        matches, errors = self._run(recs, np.arange(len(recs)))
        # keys over the per-key workspace cap (CEP_E_RUN_CAPACITY) are handed back with their state as
        # of the batch start: re-run exactly their records with the cap lifted, so that every record
        # is processed, as the reference's process() does (CEPProcessor.java:134-150)
        cap = {self._kid[a] for a, c in errors if c == 9}
        if cap:
            matches = [m for m in matches if m[1] not in cap]
            errors = [e for e in errors if e[1] != 9]
            idx = np.flatnonzero(np.isin(self._kid, np.fromiter(cap, np.int32, len(cap))))
            self.session.set_max_key_words(0)
            try:
                m2, e2 = self._run(recs, idx)
            finally:
                self.session.set_max_key_words(self.max_key_words)
            self.capacity_reruns += len(cap)
            if any(c == 9 for _, c in e2):
                self._failed = N.CepError(9, "a key outgrew the whole device pool",
                                          base + arrival[min(a for a, c in e2 if c == 9)])
                raise self._failed
            matches += m2
            errors += e2
        if cap:                                           # (each push's matches already come in arrival order)
            matches.sort(key=lambda m: m[0])              # arrival order of the completing record (stable)
        limit = err_code = None
        if errors:                                        # the first failure in ARRIVAL order (cep_batch_errors)
            limit, err_code = min(errors)
        names = self.compiled.names
        sent = 0
        for a, _, ents in matches:
            if limit is not None and a >= limit:
                break
            seq = sequence_from_traversal(ents, names, self._log.__getitem__)
            self._forward(recs[a][6].key, seq)
            sent += 1
        if not errors and len(self._log) >= self._prune_at:
            self._prune()
        if errors:
            # the failing record by its arrival index over the processor's life (non-null records)
            self._failed = N.CepError(err_code, N.ERRORS.get(err_code, "exception") + " in process()",
                                      base + arrival[limit])
            raise self._failed
        return sent

    def _prune(self):
        """Drop the records no live run can reach any more: the device's carried state lists, per
        key, the events its runs and buffer nodes still reference (``cep_state_export``), each with
        its stream position; spilled keys keep theirs.  Runs only when the log has doubled since the
        last prune."""
        keep = set(int(x) for x in N.state_positions(self.session.state_export()))
        for _, pos in self._spilled.values():
            keep.update(int(x) for x in pos)
        self._log = {p: ev for p, ev in self._log.items() if p in keep}
        self._prune_at = max(self._prune_min, 2 * len(self._log))

    # ---- checkpoint / restore (the NFAStore / buffer / aggregates stores) ----
    def checkpoint(self) -> dict:
        """Flushes, then returns the device state (``cep_state_export``) with the host's key table
        and the records carried runs may still reference."""
        self.flush()
        return {"state": self.session.state_export(), "keys": dict(self._keys), "log": dict(self._log),
                "topics": dict(self.schema.topics), "hwm": dict(self._hwm),
                "spilled": {k: v[0] for k, v in self._spilled.items()}, "next_id": self._next_id,
                "free": list(self._free)}

    def restore(self, snap: dict):
        self._check()
        if self._pending:
            raise ProcessorFailed("restore() with buffered records")
        # carried high-water marks are (interned topic id, offset) pairs (NFAStates.latestOffsets,
        # NFAStates.java:37): the topic ids must mean the same topics as when the snapshot was taken
        topics = dict(snap.get("topics", {}))
        ids = {i: t for t, i in self.schema.topics.items()}
        for t, i in topics.items():
            if self.schema.topics.get(t, i) != i or ids.get(i, t) != t:
                raise ProcessorFailed(f"snapshot topic ids conflict with this processor's schema: {t!r} -> {i}")
        for t, i in sorted(topics.items(), key=lambda x: x[1]):
            self.schema.topics[t] = i
        self.session.state_clear()
        self.session.state_import(snap["state"])
        self._keys = dict(snap["keys"])
        self._id_key = {i: k for k, i in self._keys.items()}
        self._next_id = int(snap.get("next_id", max(self._keys.values(), default=-1) + 1))
        self._free = list(snap.get("free", []))
        self._used = np.zeros(self._next_id, np.int64)
        self._spilled = {k: (b, N.state_positions(b)) for k, b in snap.get("spilled", {}).items()}
        self._log = dict(snap["log"])
        self._hwm = dict(snap.get("hwm", {}))

    def _check(self):
        if self._failed is not None:
            raise ProcessorFailed(f"processor failed earlier: {self._failed}")
        if self.session is None:
            raise ProcessorFailed("processor not initialised (call init())")
