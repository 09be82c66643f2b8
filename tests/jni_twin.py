"""Drives jni/kcep_jni.c (compiled unchanged against tests/jni_stub/) the way
java/com/github/fhuss/kafka/streams/cep/processor/GpuCEPProcessor.java does -- test infrastructure, no JVM in the image.

``JniLib`` wraps every ``native`` method of GpuCEPProcessor.java as a ctypes call of its
``Java_..._GpuCEPProcessor_*`` symbol with a mock ``JNIEnv`` (Java arrays are mock objects over
numpy buffers).  ``JavaTwin`` restates GpuCEPProcessor's ``process``/``flush`` call for call: the
host high-water mark and ``CEP_BATCH_OFFSETS_MONOTONE`` on stencil/chain sessions, the key-id
spill (``cepStateEvict``/``cepStateImportKeys``), one ``cepPushBatch`` (push + the one
``cep_collect``) and two ``cepCollect`` reads per push, the capacity re-run with
``cepSetMaxKeyWords(0)``, forwarding in arrival order, pruning by ``cepStatePositions``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "jni_stub", "libkcep_jni_test.so")
PFX = "Java_com_github_fhuss_kafka_streams_cep_processor_GpuCEPProcessor_"

# every native method of java/com/github/fhuss/kafka/streams/cep/processor/GpuCEPProcessor.java
NATIVES = ["cepCompile", "cepStageNames", "cepSessionOpen", "cepSessionPath", "cepPushBatch", "cepCollect",
           "cepBatchErrors", "cepStreamPosition", "cepStateExport", "cepStateImport", "cepStateEvict",
           "cepStateImportKeys", "cepStatePositions", "cepSetMaxKeyWords", "cepSessionClose", "cepPatternFree",
           "cepLastError", "cepStateToReference"]

CEP_MODE_PROCESSOR, CEP_SESSION_CARRY, CEP_E_RUN_CAPACITY = 1, 1, 9
CEP_PATH_STENCIL, CEP_PATH_CHAIN, CEP_PATH_RUNS, CEP_BATCH_OFFSETS_MONOTONE, CEP_BATCH_DELIVER = 1, 3, 4, 1, 2
CEP_BATCH_ARRIVAL_ORDER = 4


class JniLib:
    def __init__(self, path=LIB):
        L = C.CDLL(path)
        P = C.c_void_p
        self.L = L
        L.mock_env.restype = P
        L.mock_prim_array.restype = P
        L.mock_prim_array.argtypes = [P, C.c_int32, C.c_int32]
        L.mock_obj_array.restype = P
        L.mock_obj_array.argtypes = [C.c_int32]
        L.mock_obj_set.argtypes = [P, C.c_int32, P]
        L.mock_obj_get.restype = P
        L.mock_obj_get.argtypes = [P, C.c_int32]
        L.mock_data.restype = P
        L.mock_data.argtypes = [P]
        L.mock_len.restype = C.c_int32
        L.mock_len.argtypes = [P]
        L.mock_pins.restype = C.c_long
        self.env = L.mock_env()
        self._keep = []
        sig = {
            "cepCompile": (C.c_int64, [P]),
            "cepStageNames": (P, [C.c_int64]),
            "cepSessionOpen": (C.c_int64, [C.c_int64, C.c_int32, C.c_int32, C.c_int64, C.c_int32, C.c_int64,
                                           C.c_int64, C.c_int64]),
            "cepSessionPath": (C.c_int32, [C.c_int64]),
            "cepPushBatch": (C.c_int32, [C.c_int64, C.c_int32, P, P, P, P, P, P, P, C.c_int32]),
            "cepCollect": (C.c_int64, [C.c_int64, P, P, P, P, P, P]),
            "cepBatchErrors": (P, [C.c_int64]),
            "cepStreamPosition": (C.c_int64, [C.c_int64]),
            "cepStateExport": (P, [C.c_int64, C.c_int32, C.c_int32]),
            "cepStateImport": (C.c_int32, [C.c_int64, P]),
            "cepStateEvict": (P, [C.c_int64, P]),
            "cepStateImportKeys": (C.c_int32, [C.c_int64, P, P]),
            "cepStatePositions": (P, [P]),
            "cepSetMaxKeyWords": (C.c_int32, [C.c_int64, C.c_int64]),
            "cepSessionClose": (None, [C.c_int64]),
            "cepPatternFree": (None, [C.c_int64]),
            "cepLastError": (P, []),
            "cepStateToReference": (P, [C.c_int64, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, PFX + name)
            f.restype = res
            f.argtypes = [P, P] + args                    # JNIEnv*, jclass
            setattr(self, "_" + name, f)

    # ---- Java arrays ----
    def arr(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        self._keep.append(a)
        return self.L.mock_prim_array(a.ctypes.data, len(a), a.itemsize)

    def objs(self, items):
        o = self.L.mock_obj_array(len(items))
        for i, x in enumerate(items):
            self.L.mock_obj_set(o, i, x)
        return o

    def to_np(self, jarr, dtype):
        if not jarr:
            return None
        n = self.L.mock_len(jarr)
        if n == 0:
            return np.zeros(0, dtype)
        return np.ctypeslib.as_array(C.cast(self.L.mock_data(jarr), C.POINTER(np.ctypeslib.as_ctypes_type(dtype))),
                                     shape=(n,)).copy()

    def string(self, jstr) -> str:
        return C.string_at(self.L.mock_data(jstr)).decode()

    def pins(self) -> int:
        return self.L.mock_pins()

    # ---- the natives, Java-typed ----
    def cepCompile(self, ir: bytes) -> int:
        return self._cepCompile(self.env, None, self.arr(np.frombuffer(ir, np.int8)))

    def cepStageNames(self, pattern: int):
        o = self._cepStageNames(self.env, None, pattern)
        return [self.string(self.L.mock_obj_get(o, i)) for i in range(self.L.mock_len(o))]

    def cepSessionOpen(self, pattern, device, mode, max_events, flags, max_keys, max_key_words, max_pool_bytes=0) -> int:
        return self._cepSessionOpen(self.env, None, pattern, device, mode, max_events, flags, max_keys, max_key_words,
                                    max_pool_bytes)

    def cepSessionPath(self, session) -> int:
        return self._cepSessionPath(self.env, None, session)

    def cepPushBatch(self, session, n, key, topic, part, off, ts, types, cols, flags) -> int:
        return self._cepPushBatch(self.env, None, session, n, self.arr(key), self.arr(topic), self.arr(part),
                                  self.arr(off), self.arr(ts), self.arr(types), self.objs([self.arr(c) for c in cols]),
                                  flags)

    def cepCollect(self, session, sizes, mrec=None, mkey=None, eoff=None, ename=None, erec=None) -> int:
        a = [self.arr(x) if x is not None else None for x in (sizes, mrec, mkey, eoff, ename, erec)]
        return self._cepCollect(self.env, None, session, *a)

    def cepBatchErrors(self, session):
        return self.to_np(self._cepBatchErrors(self.env, None, session), np.int64)

    def cepStreamPosition(self, session) -> int:
        return self._cepStreamPosition(self.env, None, session)

    def cepStateExport(self, session, lo, hi):
        a = self.to_np(self._cepStateExport(self.env, None, session, lo, hi), np.int8)
        return None if a is None else a.tobytes()

    def cepStateEvict(self, session, keys):
        o = self._cepStateEvict(self.env, None, session, self.arr(np.asarray(keys, np.int32)))
        if not o:
            return None
        return [self.to_np(self.L.mock_obj_get(o, i), np.int8).tobytes() for i in range(self.L.mock_len(o))]

    def cepStateImportKeys(self, session, blobs, keys) -> int:
        return self._cepStateImportKeys(self.env, None, session,
                                        self.objs([self.arr(np.frombuffer(b, np.int8)) for b in blobs]),
                                        self.arr(np.asarray(keys, np.int32)))

    def cepStatePositions(self, blob: bytes):
        return self.to_np(self._cepStatePositions(self.env, None, self.arr(np.frombuffer(blob, np.int8))), np.int64)

    def cepSetMaxKeyWords(self, session, words) -> int:
        return self._cepSetMaxKeyWords(self.env, None, session, words)

    def cepSessionClose(self, session):
        self._cepSessionClose(self.env, None, session)

    def cepPatternFree(self, pattern):
        self._cepPatternFree(self.env, None, pattern)

    def cepStateToReference(self, pattern, blob: bytes):
        a = self.to_np(self._cepStateToReference(self.env, None, pattern, self.arr(np.frombuffer(blob, np.int8))),
                       np.int8)
        return None if a is None else a.tobytes()

    def cepLastError(self) -> str:
        return self.string(self._cepLastError(self.env, None))


class JavaTwin:
    """GpuCEPProcessor.java's host logic, call for call, over the JNI shim.  Records are
    (key, [column values], topic, partition, offset, timestamp); the decoder is the identity on
    the per-column values with Java types ``types`` (1 int32, 2 int64, 3 double)."""

    def __init__(self, jl: JniLib, ir: bytes, types, batch_size, max_keys, max_key_words=0, prune_at=None,
                 max_pool_bytes=0):
        self.j = jl
        self.types = list(types)
        self.batch_size = batch_size
        self.max_keys = max_keys
        self.max_key_words = max_key_words
        self.pattern = self._check(jl.cepCompile(ir))
        self.names = jl.cepStageNames(self.pattern)
        self.session = self._check(jl.cepSessionOpen(self.pattern, 0, CEP_MODE_PROCESSOR, batch_size,
                                                     CEP_SESSION_CARRY, max_keys, max_key_words, max_pool_bytes))
        self.path = jl.cepSessionPath(self.session)
        self.key_ids, self.id_keys, self.free_ids = {}, {}, []
        self.next_id = 0
        self.last_used = {}
        self.flushes = 0
        self.spilled, self.spilled_pos = {}, {}
        self.topic_ids = {}
        self.high_water = {}
        self.pending = []
        self.log = {}
        self.prune_at = prune_at or max(1 << 20, 2 * batch_size)
        self.forwarded = []                                 # (key, [(stage name, [record offsets])])
        self.pushes = 0
        self.reruns = 0

    def _check(self, h):
        if h < 0:
            raise RuntimeError(self.j.cepLastError())
        return h

    def process(self, key, vals, topic, partition, offset, ts):
        if key is None or vals is None:
            return
        self.pending.append((key, vals, topic, partition, offset, ts))
        if len(self.pending) >= self.batch_size:
            self.flush()

    def close(self):
        self.flush()
        self.j.cepSessionClose(self.session)
        self.j.cepPatternFree(self.pattern)

    def _topic(self, t):
        return self.topic_ids.setdefault(t, len(self.topic_ids))

    def _run(self, recs, kid, idx, flags):
        j = self.j
        n = len(idx)
        order = list(idx)                                   # arrival order: the device groups by key
        key_id = np.array([kid[a] for a in order], np.int32)
        topic = np.array([self._topic(recs[a][2]) for a in order], np.int32)
        part = np.array([recs[a][3] for a in order], np.int32)
        off = np.array([recs[a][4] for a in order], np.int64)
        ts = np.array([recs[a][5] for a in order], np.int64)
        np_t = {1: np.int32, 2: np.int64, 3: np.float64}
        cols = [np.array([recs[a][1][c] for a in order], np_t[t]) for c, t in enumerate(self.types)]
        base = j.cepStreamPosition(self.session)
        for jj, a in enumerate(order):
            self.log[base + jj] = recs[a]
        rc = j.cepPushBatch(self.session, n, key_id, topic, part, off, ts, np.array(self.types, np.int32), cols,
                            flags | CEP_BATCH_DELIVER | CEP_BATCH_ARRIVAL_ORDER)
        self.pushes += 1
        if rc != 0:
            raise RuntimeError(f"cepPushBatch {rc}: {j.cepLastError()}")
        sizes = np.zeros(2, np.int64)
        j.cepCollect(self.session, sizes)
        nm, ne = int(sizes[0]), int(sizes[1])
        mrec, mkey = np.zeros(nm, np.int64), np.zeros(nm, np.int32)
        eoff, ename, erec = np.zeros(nm + 1, np.int64), np.zeros(ne, np.int32), np.zeros(ne, np.int64)
        r = j.cepCollect(self.session, sizes, mrec, mkey, eoff, ename, erec)
        matches = [(order[int(mrec[m] - base)], int(mkey[m]), ename[eoff[m]:eoff[m + 1]].copy(),
                    erec[eoff[m]:eoff[m + 1]].copy()) for m in range(nm)]
        errors = []
        if r < 0:
            errs = j.cepBatchErrors(self.session)
            errors = [(order[int(errs[i] - base)], int(errs[i + 1])) for i in range(0, len(errs), 2)]
        return matches, errors

    def _key_ids(self, recs):
        self.flushes += 1
        want = list(dict.fromkeys(r[0] for r in recs))
        assert len(want) <= self.max_keys
        fresh = [k for k in want if k not in self.key_ids]
        short = len(fresh) - len(self.free_ids) - (self.max_keys - self.next_id)
        if short > 0:
            self._spill(max(short, self.max_keys // 8), set(want))
        blobs, ids = [], []
        for k in fresh:
            kid = self.free_ids.pop() if self.free_ids else self.next_id
            if kid == self.next_id:
                self.next_id += 1
            self.key_ids[k] = kid
            self.id_keys[kid] = k
            b = self.spilled.pop(k, None)
            self.spilled_pos.pop(k, None)
            if b is not None:
                blobs.append(b)
                ids.append(kid)
        if ids and self.j.cepStateImportKeys(self.session, blobs, ids) != 0:
            raise RuntimeError(self.j.cepLastError())
        kid = [self.key_ids[r[0]] for r in recs]
        for x in kid:
            self.last_used[x] = self.flushes
        return kid

    def _spill(self, count, busy):
        cand = sorted((i for i, k in self.id_keys.items() if k not in busy), key=lambda i: (self.last_used[i], i))
        cand = cand[:count]
        if not cand:
            return
        blobs = self.j.cepStateEvict(self.session, cand)
        if blobs is None:
            raise RuntimeError(self.j.cepLastError())
        for i, b in zip(cand, blobs):
            k = self.id_keys.pop(i)
            del self.key_ids[k]
            self.free_ids.append(i)
            if b:
                self.spilled[k] = b
                self.spilled_pos[k] = self.j.cepStatePositions(b)

    def flush(self):
        if not self.pending:
            return
        arrived, self.pending = self.pending, []
        host_mark = self.path in (CEP_PATH_STENCIL, CEP_PATH_CHAIN, CEP_PATH_RUNS)
        recs, at = [], []                                   # the device's records and their arrival indices
        for i, r in enumerate(arrived):                     # (keys on the reference: the Java's hand-off only)
            if host_mark:
                hw = self.high_water.setdefault(r[0], {})
                t = self._topic(r[2])
                if t in hw and r[4] < hw[t]:
                    continue
                hw[t] = r[4] + 1
            recs.append(r)
            at.append(i)
        matches, errors = [], []
        if recs:
            m, e = self._run_device(recs, CEP_BATCH_OFFSETS_MONOTONE if host_mark else 0)
            matches = [(at[a],) + tuple(x) for a, *x in m]
            errors = [(at[a], c) for a, c in e]
        limit = min(errors)[0] if errors else None
        matches.sort(key=lambda m: m[0])
        for a, _, en, er in matches:
            if limit is not None and a >= limit:
                break
            groups = {}
            for nm, pos in zip(en, er):                     # Sequence.Builder.add, then build(true)
                groups.setdefault(self.names[nm], []).append(self.log[int(pos)][4])
            self.forwarded.append((arrived[a][0], [(s, sorted(v)) for s, v in reversed(list(groups.items()))]))
        if errors:
            raise RuntimeError(f"reference exception {min(errors)[1]} at record {limit}")
        if len(self.log) >= self.prune_at:
            self._prune()

    def _run_device(self, recs, flags):
        kid = self._key_ids(recs)
        allidx = list(range(len(recs)))
        matches, errors = self._run(recs, kid, allidx, flags)
        cap = {kid[a] for a, c in errors if c == CEP_E_RUN_CAPACITY}
        if cap:
            matches = [m for m in matches if m[1] not in cap]
            errors = [e for e in errors if e[1] != CEP_E_RUN_CAPACITY]
            idx = [i for i in allidx if kid[i] in cap]
            self.j.cepSetMaxKeyWords(self.session, 0)
            try:
                m2, e2 = self._run(recs, kid, idx, flags)
            finally:
                self.j.cepSetMaxKeyWords(self.session, self.max_key_words)
            self.reruns += len(cap)
            assert not any(c == CEP_E_RUN_CAPACITY for _, c in e2), "a key outgrew the whole device pool"
            matches += m2
            errors += e2
        return matches, errors

    def _prune(self):
        state = self.j.cepStateExport(self.session, 0, 2 ** 31 - 1)
        keep = set(int(x) for x in self.j.cepStatePositions(state))
        for ps in self.spilled_pos.values():
            keep.update(int(x) for x in ps)
        self.log = {p: r for p, r in self.log.items() if p in keep}
        self.prune_at = max(max(1 << 20, 2 * self.batch_size), 2 * len(self.log))
