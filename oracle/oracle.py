"""ctypes wrapper around the C oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  The product path (kafkastreams-cep_amd/kcep, libkcep.so)
never does.  Parity status: pinned by the reference's own test vectors
(tests/golden/); see cep_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcep_oracle.so")

MODE_NFA_SINGLE = 0
MODE_PROCESSOR = 1
MODE_NFA_PER_KEY = 2

T_I32, T_I64, T_F64 = 1, 2, 3
_NP = {T_I32: np.int32, T_I64: np.int64, T_F64: np.float64}


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P, I64, I32 = C.c_void_p, C.c_int64, C.c_int32
        L.orc_compile.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(P), C.c_char_p, C.c_size_t]
        L.orc_pattern_free.argtypes = [P]
        L.orc_n_stages.argtypes = [P]
        L.orc_n_names.argtypes = [P]
        L.orc_name.argtypes = [P, C.c_int]
        L.orc_name.restype = C.c_char_p
        L.orc_stage_info.argtypes = [P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(I64),
                                     C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_run_new.argtypes = [P, C.c_int]
        L.orc_run_new.restype = P
        L.orc_run_free.argtypes = [P]
        L.orc_run_batch.argtypes = [P, P]
        L.orc_run_resume.argtypes = [P, P, C.c_char_p, C.c_size_t]
        L.orc_baseline_csr.argtypes = [P, P, C.c_int, C.c_int]
        L.orc_baseline_csr.restype = P
        L.orc_csr_sizes.argtypes = [P, C.POINTER(I64), C.POINTER(I64), C.POINTER(C.c_int)]
        L.orc_csr_copy.argtypes = [P, P, P, P, P, P]
        L.orc_csr_free.argtypes = [P]
        L.orc_err_record.argtypes = [P]
        L.orc_err_record.restype = I64
        L.orc_err_msg.argtypes = [P]
        L.orc_err_msg.restype = C.c_char_p
        L.orc_n_matches.argtypes = [P]
        L.orc_n_matches.restype = I64
        L.orc_match.argtypes = [P, I64, C.POINTER(I64), C.POINTER(I32), C.POINTER(I64), C.POINTER(I64)]
        L.orc_entry.argtypes = [P, I64, C.POINTER(I32), C.POINTER(I64)]
        L.orc_seq_groups.argtypes = [P, I64, C.POINTER(I32), C.POINTER(I64), I64]
        L.orc_seq_groups.restype = I64
        L.orc_seq_events.argtypes = [P, I64, C.POINTER(I64), I64]
        L.orc_seq_events.restype = I64
        L.orc_inst_state.argtypes = [P, I32, C.POINTER(I64), C.POINTER(I64)]
        L.orc_queue_entry.argtypes = [P, I32, I64, C.POINTER(I32), C.POINTER(I32), C.POINTER(I64),
                                      C.POINTER(I64), C.c_char_p, C.c_size_t]
        L.orc_baseline.argtypes = [P, P, C.c_int, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_int)]
        L.orc_baseline.restype = I64
        L.orc_svb_bind.argtypes = [P, P]
        L.orc_svb_bind.restype = None
        L.orc_svb_put.argtypes = [P, C.c_int, I64, C.c_int, I64, C.c_char_p]
        L.orc_svb_get.argtypes = [P, C.c_int, I64, C.c_char_p, C.c_int]
        L.orc_dewey_compatible.argtypes = [C.c_char_p, C.c_char_p]
        L.orc_dewey_add_run.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_size_t]
        L.orc_dewey_add_stage.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
        _lib = L
    return _lib


class OracleError(Exception):
    def __init__(self, code, msg, record=-1):
        super().__init__(f"oracle error {code}: {msg} (record {record})")
        self.code = code
        self.record = record


class _Batch(C.Structure):
    _fields_ = [("n", C.c_int64), ("key", C.c_void_p), ("valid", C.c_void_p), ("topic", C.c_void_p),
                ("partition", C.c_void_p), ("offset", C.c_void_p), ("ts", C.c_void_p),
                ("ncols", C.c_int32), ("cols", C.POINTER(C.c_void_p))]


def _ptr(a):
    return None if a is None else a.ctypes.data


class BatchArrays:
    """Keeps numpy arrays alive while the C side reads them."""

    def __init__(self, key, cols, coltypes, valid=None, topic=None, partition=None, offset=None, ts=None):
        self.key = np.ascontiguousarray(key, dtype=np.int32)
        n = len(self.key)
        self.cols = [np.ascontiguousarray(c, dtype=_NP[t]) for c, t in zip(cols, coltypes)]
        for c in self.cols:
            assert len(c) == n
        self.valid = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
        self.topic = None if topic is None else np.ascontiguousarray(topic, dtype=np.int32)
        self.partition = None if partition is None else np.ascontiguousarray(partition, dtype=np.int32)
        self.offset = None if offset is None else np.ascontiguousarray(offset, dtype=np.int64)
        self.ts = None if ts is None else np.ascontiguousarray(ts, dtype=np.int64)
        self._colptrs = (C.c_void_p * max(1, len(self.cols)))(*[c.ctypes.data for c in self.cols])
        self.s = _Batch(n, _ptr(self.key), _ptr(self.valid), _ptr(self.topic), _ptr(self.partition),
                        _ptr(self.offset), _ptr(self.ts), len(self.cols), self._colptrs)


@dataclass
class Match:
    record: int
    key: int
    traversal: list            # [(name_id, event_record)] final -> begin
    groups: list = field(default_factory=list)   # [(stage_name, [event_record...])]


class OraclePattern:
    def __init__(self, ir: bytes):
        L = lib()
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = L.orc_compile(ir, len(ir), C.byref(h), err, 512)
        if rc:
            raise OracleError(rc, err.value.decode())
        self.h = h
        self.names = [L.orc_name(h, i).decode() for i in range(L.orc_n_names(h))]
        self.coltypes = list(ir[10:10 + int.from_bytes(ir[8:10], "little")])

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_pattern_free(self.h)
            self.h = None

    def stages(self):
        """[(name, type, window, [(op, target)])] in Stages list order."""
        L = lib()
        out = []
        for s in range(L.orc_n_stages(self.h)):
            nm, ty = C.c_int(), C.c_int()
            w = C.c_int64()
            ops = (C.c_int * 8)()
            tg = (C.c_int * 8)()
            ne = L.orc_stage_info(self.h, s, C.byref(nm), C.byref(ty), C.byref(w), ops, tg)
            out.append((self.names[nm.value], ty.value, w.value, [(ops[i], tg[i]) for i in range(ne)]))
        return out


class OracleRun:
    def __init__(self, pattern: OraclePattern, mode: int):
        self.p = pattern
        self.h = lib().orc_run_new(pattern.h, mode)
        self._keep = []

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_run_free(self.h)
            self.h = None

    def process(self, batch: BatchArrays):
        self._keep.append(batch)
        L = lib()
        rc = L.orc_run_batch(self.h, C.byref(batch.s))
        if rc:
            raise OracleError(rc, L.orc_err_msg(self.h).decode(), L.orc_err_record(self.h))

    def resume(self, batch: BatchArrays, state: bytes):
        """Continue one key from its state in the reference's terms ("KCRF", cep_state_to_reference):
        the batch's first records are the state's events, the rest are processed."""
        self._keep.append(batch)
        L = lib()
        rc = L.orc_run_resume(self.h, C.byref(batch.s), state, len(state))
        if rc:
            raise OracleError(rc, L.orc_err_msg(self.h).decode(), L.orc_err_record(self.h))

    def matches(self, with_groups=True):
        L = lib()
        out = []
        rec, ebeg, eend = C.c_int64(), C.c_int64(), C.c_int64()
        key = C.c_int32()
        nm = C.c_int32()
        ev = C.c_int64()
        for m in range(L.orc_n_matches(self.h)):
            L.orc_match(self.h, m, C.byref(rec), C.byref(key), C.byref(ebeg), C.byref(eend))
            trav = []
            for e in range(ebeg.value, eend.value):
                L.orc_entry(self.h, e, C.byref(nm), C.byref(ev))
                trav.append((nm.value, ev.value))
            mt = Match(rec.value, key.value, trav)
            if with_groups:
                ng = L.orc_seq_groups(self.h, m, None, None, 0)
                names = (C.c_int32 * max(ng, 1))()
                cnts = (C.c_int64 * max(ng, 1))()
                L.orc_seq_groups(self.h, m, names, cnts, ng)
                ne = L.orc_seq_events(self.h, m, None, 0)
                evs = (C.c_int64 * max(ne, 1))()
                L.orc_seq_events(self.h, m, evs, ne)
                k = 0
                for g in range(ng):
                    mt.groups.append((self.p.names[names[g]], [evs[k + i] for i in range(cnts[g])]))
                    k += cnts[g]
            out.append(mt)
        return out

    # ---- SharedVersionedBufferTest: direct buffer operations on a bound batch ----
    def svb_bind(self, batch: BatchArrays):
        self._keep.append(batch)
        lib().orc_svb_bind(self.h, C.byref(batch.s))

    def svb_put(self, sid, ev, psid, pev, version):
        rc = lib().orc_svb_put(self.h, sid, ev, -1 if psid is None else psid, -1 if pev is None else pev,
                               version.encode())
        if rc:
            raise OracleError(rc, lib().orc_err_msg(self.h).decode())

    def svb_get(self, sid, ev, version, remove=False):
        rc = lib().orc_svb_get(self.h, sid, ev, version.encode(), 1 if remove else 0)
        if rc:
            raise OracleError(rc, lib().orc_err_msg(self.h).decode())
        return self.matches()[-1]

    def state(self, key=0):
        runs, qs = C.c_int64(), C.c_int64()
        if lib().orc_inst_state(self.h, key, C.byref(runs), C.byref(qs)):
            return None
        return runs.value, qs.value

    def queue(self, key=0):
        L = lib()
        st = self.state(key)
        out = []
        if st is None:
            return out
        sid, eps = C.c_int32(), C.c_int32()
        seq, ev = C.c_int64(), C.c_int64()
        buf = C.create_string_buffer(4096)
        for i in range(st[1]):
            L.orc_queue_entry(self.h, key, i, C.byref(sid), C.byref(eps), C.byref(seq), C.byref(ev), buf, 4096)
            out.append(dict(stage=sid.value, eps=eps.value, seq=seq.value, event=ev.value,
                            version=buf.value.decode()))
        return out


def baseline(pattern: OraclePattern, batch: BatchArrays, mode=MODE_PROCESSOR, threads=1):
    cs = C.c_uint64()
    err = C.c_int()
    n = lib().orc_baseline(pattern.h, C.byref(batch.s), mode, threads, C.byref(cs), C.byref(err))
    if err.value:
        raise OracleError(err.value, "baseline failed")
    return n, cs.value


def baseline_csr(pattern: OraclePattern, batch: BatchArrays, mode=MODE_PROCESSOR, threads=1):
    """The baseline run keeping every match: dict of numpy arrays in cep_collect's layout and order
    (key order of the grouped batch, per key in emission order)."""
    import numpy as np
    L = lib()
    h = L.orc_baseline_csr(pattern.h, C.byref(batch.s), mode, threads)
    try:
        nm, ne, err = C.c_int64(), C.c_int64(), C.c_int()
        L.orc_csr_sizes(h, C.byref(nm), C.byref(ne), C.byref(err))
        if err.value:
            raise OracleError(err.value, "baseline failed")
        out = dict(match_record=np.zeros(nm.value, np.int64), match_key=np.zeros(nm.value, np.int32),
                   ent_off=np.zeros(nm.value + 1, np.int64), ent_name=np.zeros(ne.value, np.int32),
                   ent_record=np.zeros(ne.value, np.int64))
        L.orc_csr_copy(h, *[out[k].ctypes.data for k in ("match_record", "match_key", "ent_off", "ent_name",
                                                           "ent_record")])
        return out
    finally:
        L.orc_csr_free(h)


def dewey_compatible(a, b):
    return bool(lib().orc_dewey_compatible(a.encode(), b.encode()))


def dewey_add_run(v, off=1):
    buf = C.create_string_buffer(256)
    rc = lib().orc_dewey_add_run(v.encode(), off, buf, 256)
    if rc:
        raise OracleError(rc, "addRun")
    return buf.value.decode()


def dewey_add_stage(v):
    buf = C.create_string_buffer(256)
    lib().orc_dewey_add_stage(v.encode(), buf, 256)
    return buf.value.decode()
