"""ctypes binding of libkcep.so (include/kcep.h).

This is the only way the Python host reaches the matcher: there is no Python
or CPU evaluation path behind it.  If the shared library is missing the
import of the binding fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("KCEP_LIB") or os.path.join(PKG_ROOT, "libkcep.so")   # KCEP_LIB: experiment builds

CEP_OK = 0
ERRORS = {
    1: "InvalidPatternException", 2: "UnknownAggregateException", 3: "IllegalStateException",
    4: "NullPointerException", 5: "ArithmeticException", 6: "ClassCastException",
    7: "ArrayIndexOutOfBoundsException", 8: "BadIR", 9: "RunCapacity", 10: "HipError", 11: "BadArgument",
    12: "Unsupported",
}
E_RUN_CAPACITY = 9         # a key over its device workspace, handed back per key (cep_batch_errors)
MODE_NFA, MODE_PROCESSOR = 0, 1
PATH_STENCIL, PATH_GENERAL, PATH_CHAIN, PATH_RUNS = 1, 2, 3, 4
MEM_HOST, MEM_DEVICE = 0, 1
BATCH_OFFSETS_MONOTONE = 1
BATCH_DELIVER = 2          # the push is collected at once: matches handed to pinned host memory by the device
BATCH_ARRIVAL_ORDER = 4    # records in arrival order: grouped by key on the device, matches back in arrival order
SESSION_CARRY = 1
SESSION_INTERPRET = 2
SESSION_PROFILE = 4
SESSION_LANE_NFA = 8
SESSION_WAVE_NFA = 16


class CepError(RuntimeError):
    def __init__(self, code: int, msg: str, record: int = -1):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}" + (f" (record {record})" if record >= 0 else ""))
        self.code = code
        self.record = record


class PatternInfo(C.Structure):
    _fields_ = [("n_stages", C.c_int32), ("n_names", C.c_int32), ("n_patterns", C.c_int32),
                ("n_cols", C.c_int32), ("stencil_ok", C.c_int32), ("stencil_k", C.c_int32),
                ("chain_ok", C.c_int32), ("runs_ok", C.c_int32)]


class Opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("mode", C.c_int32), ("force_path", C.c_int32), ("flags", C.c_int32),
                ("max_events", C.c_int64), ("max_keys", C.c_int64), ("arena_scale", C.c_double),
                ("max_key_words", C.c_int64), ("max_pool_bytes", C.c_int64)]


class Batch(C.Structure):
    _fields_ = [("n", C.c_int64), ("key_id", C.c_void_p), ("valid", C.c_void_p), ("topic", C.c_void_p),
                ("partition", C.c_void_p), ("offset", C.c_void_p), ("ts", C.c_void_p), ("n_cols", C.c_int32),
                ("mem", C.c_int32), ("cols", C.POINTER(C.c_void_p)), ("flags", C.c_uint32),
                ("reserved", C.c_uint32)]


class Matches(C.Structure):
    _fields_ = [("n_matches", C.c_int64), ("n_entries", C.c_int64), ("match_record", C.POINTER(C.c_int64)),
                ("match_key", C.POINTER(C.c_int32)), ("ent_off", C.POINTER(C.c_int64)),
                ("ent_name", C.POINTER(C.c_int32)), ("ent_record", C.POINTER(C.c_int64)),
                ("path", C.c_int32), ("err", C.c_int32), ("err_record", C.c_int64)]


SYMBOLS = ["cep_compile", "cep_pattern_free", "cep_pattern_get_info", "cep_pattern_name", "cep_pattern_stage",
           "cep_session_open",
           "cep_session_close", "cep_session_path", "cep_push_batch", "cep_device_match_count", "cep_collect",
           "cep_checksum", "cep_last_kernel_ms", "cep_last_batch_ms", "cep_last_error", "cep_version",
           "cep_state_export", "cep_state_import", "cep_state_clear", "cep_key_state", "cep_stream_position",
           "cep_session_jit", "cep_session_wave", "cep_pattern_kernel_source", "cep_pattern_build_kernels", "cep_live_run_hwm",
           "cep_batch_errors", "cep_session_set_timing",
           "cep_key_profile", "cep_key_hash", "cep_key_shard", "cep_shard_plan", "cep_partition", "cep_gather",
           "cep_match_count_to", "cep_state_evict", "cep_state_import_keys", "cep_state_positions",
           "cep_session_set_max_key_words", "cep_state_to_reference", "cep_pattern_check", "cep_batch_attempts",
           "cep_csr_check", "cep_batch_id", "cep_batch_ready", "cep_collect_batch"]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C kafkastreams-cep_amd` "
                          "(there is no CPU fallback)")
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7.  Load
    # it first so that libkcep.so binds to the same runtime (same SONAME) and
    # torch tensors, streams and our sessions share one device context.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    L.cep_compile.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(P)]
    L.cep_pattern_free.argtypes = [P]
    L.cep_pattern_free.restype = None
    L.cep_pattern_get_info.argtypes = [P, C.POINTER(PatternInfo)]
    L.cep_pattern_name.argtypes = [P, C.c_int32]
    L.cep_pattern_name.restype = C.c_char_p
    L.cep_pattern_stage.argtypes = [P, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                    C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int32]
    L.cep_pattern_stage.restype = C.c_int32
    L.cep_session_open.argtypes = [P, C.POINTER(Opts), C.POINTER(P)]
    L.cep_session_close.argtypes = [P]
    L.cep_session_close.restype = None
    L.cep_session_path.argtypes = [P]
    L.cep_push_batch.argtypes = [P, C.POINTER(Batch), P]
    L.cep_device_match_count.argtypes = [P]
    L.cep_device_match_count.restype = C.c_void_p
    L.cep_collect.argtypes = [P, C.POINTER(Matches)]
    L.cep_checksum.argtypes = [P, C.POINTER(C.c_uint64), C.POINTER(C.c_int64)]
    L.cep_last_kernel_ms.argtypes = [P, C.POINTER(C.c_float)]
    L.cep_last_batch_ms.argtypes = [P, C.POINTER(C.c_float)]
    L.cep_state_export.argtypes = [P, C.c_int32, C.c_int32, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    L.cep_state_import.argtypes = [P, C.c_void_p, C.c_size_t]
    L.cep_state_clear.argtypes = [P]
    L.cep_key_state.argtypes = [P, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.cep_stream_position.argtypes = [P]
    L.cep_stream_position.restype = C.c_int64
    L.cep_session_jit.argtypes = [P]
    L.cep_session_wave.argtypes = [P]
    L.cep_batch_attempts.argtypes = [P]
    L.cep_csr_check.argtypes = [C.POINTER(Matches), C.c_int64, C.c_int32]
    L.cep_batch_id.argtypes = [P]
    L.cep_batch_id.restype = C.c_int64
    L.cep_batch_ready.argtypes = [P, C.c_int64]
    L.cep_collect_batch.argtypes = [P, C.c_int64, C.POINTER(Matches)]
    L.cep_live_run_hwm.argtypes = [P, C.POINTER(C.c_int64)]
    L.cep_session_set_timing.argtypes = [P, C.c_int32]
    L.cep_batch_errors.argtypes = [P, C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
    L.cep_key_profile.argtypes = [P, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
    L.cep_pattern_kernel_source.argtypes = [P, C.c_int32, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]
    L.cep_pattern_build_kernels.argtypes = [P, C.c_int32]
    L.cep_key_hash.argtypes = [C.c_int32]
    L.cep_key_hash.restype = C.c_uint32
    L.cep_key_shard.argtypes = [C.c_int32, C.c_int32]
    L.cep_key_shard.restype = C.c_int32
    L.cep_shard_plan.argtypes = [P, C.c_int64, C.c_int32, C.c_int32, P, P]
    L.cep_partition.argtypes = [P, C.c_int64, C.c_int32, P, C.c_int64, P, P, C.c_int32, P]
    L.cep_gather.argtypes = [P, C.c_int32, P, C.c_int64, P, C.c_int32, P]
    L.cep_match_count_to.argtypes = [P, P, P]
    if hasattr(L, "cep_state_evict"):       # (KCEP_LIB A/B runs may load an older build)
        L.cep_state_evict.argtypes = [P, P, C.c_int64, C.POINTER(C.c_void_p), P]
        L.cep_state_import_keys.argtypes = [P, P, P, P, C.c_int64]
        L.cep_state_positions.argtypes = [P, C.c_size_t, P, C.c_int64, C.POINTER(C.c_int64)]
        L.cep_session_set_max_key_words.argtypes = [P, C.c_int64]
    L.cep_state_to_reference.argtypes = [P, C.c_char_p, C.c_size_t, P, C.c_size_t, C.POINTER(C.c_size_t)]
    L.cep_last_error.restype = C.c_char_p
    L.cep_version.restype = C.c_char_p
    _lib = L
    return L


def check(rc: int):
    if rc != CEP_OK:
        raise CepError(rc, lib().cep_last_error().decode())


def state_positions(blob: bytes) -> np.ndarray:
    """cep_state_positions: stream positions of the records a state blob still references."""
    n = C.c_int64()
    check(lib().cep_state_positions(blob, len(blob), None, 0, C.byref(n)))
    out = np.zeros(n.value, np.int64)
    if n.value:
        check(lib().cep_state_positions(blob, len(blob), out.ctypes.data, n.value, C.byref(n)))
    return out


class CompiledPattern:
    """``cep_compile`` handle: the device-side equivalent of ``Stages``."""

    def __init__(self, ir: bytes):
        L = lib()
        self.h = C.c_void_p()
        check(L.cep_compile(ir, len(ir), C.byref(self.h)))
        info = PatternInfo()
        check(L.cep_pattern_get_info(self.h, C.byref(info)))
        self.info = info
        self.names = [L.cep_pattern_name(self.h, i).decode() for i in range(info.n_names)]

    def stages(self):
        """[(name, type, window, [(op, target)])] in Stages list order."""
        L = lib()
        out = []
        nm, ty = C.c_int32(), C.c_int32()
        w = C.c_int64()
        ops = (C.c_int32 * 16)()
        tg = (C.c_int32 * 16)()
        for s in range(self.info.n_stages):
            ne = L.cep_pattern_stage(self.h, s, C.byref(nm), C.byref(ty), C.byref(w), ops, tg, 16)
            out.append((self.names[nm.value], ty.value, w.value, [(ops[i], tg[i]) for i in range(ne)]))
        return out

    def state_to_reference(self, blob: bytes) -> bytes:
        """cep_state_to_reference: a single-key KCST blob (Session.state_evict) in the reference's own
        terms ("KCRF"): NFA.runs, high-water marks, run queue, buffer nodes, aggregates, their events."""
        L = lib()
        n = C.c_size_t()
        check(L.cep_state_to_reference(self.h, blob, len(blob), None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        check(L.cep_state_to_reference(self.h, blob, len(blob), buf, n.value, C.byref(n)))
        return buf.raw[:n.value]

    def kernel_source(self, path=PATH_RUNS) -> str:
        """HIP source of the kernels compiled for this pattern (cep_pattern_kernel_source)."""
        n = C.c_size_t()
        check(lib().cep_pattern_kernel_source(self.h, path, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        check(lib().cep_pattern_kernel_source(self.h, path, buf, n.value, C.byref(n)))
        return buf.value.decode()

    def build_kernels(self, path=PATH_RUNS):
        """Generate and compile (hiprtc, gfx950) the pattern's kernels; raises CepError on failure."""
        check(lib().cep_pattern_build_kernels(self.h, path))

    def close(self):
        if self.h:
            lib().cep_pattern_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Session:
    """One ``cep_session`` (one stream task's processor on one GPU)."""

    def __init__(self, pattern: CompiledPattern, max_events: int, mode=MODE_PROCESSOR, device=0, force_path=0,
                 carry=False, max_keys=0, interpret=False, profile=False, max_key_words=0, lane_nfa=None,
                 max_pool_bytes=0):
        """``carry=True``: every key's NFA state continues across batches (CEP_SESSION_CARRY);
        key ids must then be dense in [0, max_keys) and record positions are stream positions.
        ``interpret=True``: the built-in interpreting kernels instead of kernels compiled for the
        pattern (CEP_SESSION_INTERPRET); ``self.jit`` says which run.  ``max_key_words``: the
        general path's per-key workspace cap -- a key over it is handed back per key
        (``batch_errors`` lists it with RunCapacity), every other key completes.  ``max_pool_bytes``:
        how far the general path's workspace pool may grow for a batch (0: a quarter of the HBM)."""
        self.pattern = pattern
        self.h = C.c_void_p()
        # lane_nfa: None = the library's choice, True = one key per lane, False = one key per wave
        flags = ((SESSION_CARRY if carry else 0) | (SESSION_INTERPRET if interpret else 0) |
                 (SESSION_PROFILE if profile else 0) | (SESSION_LANE_NFA if lane_nfa else 0) |
                 (SESSION_WAVE_NFA if lane_nfa is False else 0))
        o = Opts(device, mode, force_path, flags, max_events, max_keys, 0.0, max_key_words, max_pool_bytes)
        check(lib().cep_session_open(pattern.h, C.byref(o), C.byref(self.h)))
        self.path = lib().cep_session_path(self.h)
        self.jit = bool(lib().cep_session_jit(self.h))
        self.wave = bool(lib().cep_session_wave(self.h))
        self._keep = None

    def close(self):
        if self.h:
            lib().cep_session_close(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push(self, n, key, cols, valid=None, topic=None, partition=None, offset=None, ts=None, mem=MEM_HOST,
             flags=0, stream=None):
        """Arrays are numpy arrays (mem=MEM_HOST) or integer device pointers (mem=MEM_DEVICE)."""
        def ptr(a):
            if a is None:
                return None
            if isinstance(a, int):
                return a
            return a.ctypes.data

        colptrs = (C.c_void_p * max(1, len(cols)))(*[ptr(c) for c in cols])
        b = Batch(int(n), ptr(key), ptr(valid), ptr(topic), ptr(partition), ptr(offset), ptr(ts), len(cols), mem,
                  colptrs, flags, 0)
        self._keep = (key, cols, valid, topic, partition, offset, ts, colptrs, b)
        check(lib().cep_push_batch(self.h, C.byref(b), C.c_void_p(stream) if stream else None))

    def batch_id(self) -> int:
        """cep_batch_id: the number of the last pushed batch."""
        return int(lib().cep_batch_id(self.h))

    def batch_ready(self, batch_id: int) -> bool:
        """cep_batch_ready: whether the batch's matches are complete (no wait)."""
        rc = lib().cep_batch_ready(self.h, int(batch_id))
        if rc not in (0, 1):                               # (CEP_E_ARG / CEP_E_HIP)
            check(rc)
        return rc == 1

    def collect(self, raise_on_error=True, batch_id=None):
        """Matches of the last batch (or, ``batch_id``: of the delivered batch before it, cep_collect_batch)
        as numpy arrays.  When the reference would have thrown inside ``process()`` this raises
        ``CepError`` (code, record); with ``raise_on_error=False`` the dict carries ``err``/``err_record``
        instead, and the matches emitted before ``err_record`` are the ones the reference forwarded."""
        m = Matches()
        if batch_id is None:
            check(lib().cep_collect(self.h, C.byref(m)))
        else:
            check(lib().cep_collect_batch(self.h, int(batch_id), C.byref(m)))
        nm, ne = m.n_matches, m.n_entries

        def arr(p, n, dt):                                # one copy out of the library-owned CSR
            if n == 0:
                return np.zeros(0, dt)
            return np.frombuffer(C.string_at(p, n * np.dtype(dt).itemsize), dt)

        out = dict(match_record=arr(m.match_record, nm, np.int64), match_key=arr(m.match_key, nm, np.int32),
                   ent_off=arr(m.ent_off, nm + 1, np.int64), ent_name=arr(m.ent_name, ne, np.int32),
                   ent_record=arr(m.ent_record, ne, np.int64), path=m.path, err=m.err,
                   err_record=m.err_record)
        if m.err and raise_on_error:
            raise CepError(m.err, lib().cep_last_error().decode(), m.err_record)
        return out

    def checksum(self):
        s = C.c_uint64()
        n = C.c_int64()
        check(lib().cep_checksum(self.h, C.byref(s), C.byref(n)))
        return n.value, s.value

    def live_run_hwm(self) -> int:
        """General path: the most live runs any key held during the last batch (-1: other path)."""
        v = C.c_int64()
        check(lib().cep_live_run_hwm(self.h, C.byref(v)))
        return v.value

    def attempts(self) -> int:
        """General path: kernel attempts of the last batch (1 + pool regrowth re-runs; 0: other path)."""
        return int(lib().cep_batch_attempts(self.h))

    def set_timing(self, on: bool):
        """cep_session_set_timing: per-batch HIP event timing on/off."""
        check(lib().cep_session_set_timing(self.h, 1 if on else 0))

    def batch_errors(self):
        """Every failing key's (stream position, code) of the last batch, ascending (cep_batch_errors)."""
        n = C.c_int64()
        check(lib().cep_batch_errors(self.h, None, None, 0, C.byref(n)))
        rec = np.zeros(n.value, np.int64)
        code = np.zeros(n.value, np.int32)
        if n.value:
            check(lib().cep_batch_errors(self.h, rec.ctypes.data, code.ctypes.data, n.value, C.byref(n)))
        return rec, code

    def key_profile(self):
        """``profile=True`` sessions: int64 array [n_keys, 25] (cep_key_profile): key, live-run max, run
        evaluations, wall clock (100 MHz), 8 phase clocks, 3 scan counters, 0, workspace words, then the
        words per allocation kind (first workspace, match output, heap, run queues, private lists,
        aggregates, other) and the batch pool's share of them (kcep_dev.h NFA_PROFILE_W)."""
        import numpy as np
        n = C.c_int64()
        check(lib().cep_key_profile(self.h, None, 0, C.byref(n)))
        out = np.zeros((n.value, 25), np.int64)
        check(lib().cep_key_profile(self.h, out.ctypes.data, out.size, C.byref(n)))
        return out

    # ---- carried state (CEP_SESSION_CARRY) ----
    def state_export(self, key_lo=0, key_hi=2**31 - 1) -> bytes:
        L = lib()
        need = C.c_size_t()
        check(L.cep_state_export(self.h, key_lo, key_hi, None, 0, C.byref(need)))
        buf = C.create_string_buffer(need.value)
        check(L.cep_state_export(self.h, key_lo, key_hi, buf, need.value, C.byref(need)))
        return buf.raw[:need.value]

    def state_import(self, blob: bytes):
        check(lib().cep_state_import(self.h, blob, len(blob)))

    def state_clear(self):
        check(lib().cep_state_clear(self.h))

    def state_evict(self, keys) -> list:
        """cep_state_evict: the listed key ids' state as single-key blobs (b"" for a key without
        state), dropped from the device so that the ids are free."""
        k = np.ascontiguousarray(keys, np.int32)
        offs = np.zeros(len(k) + 1, np.int64)
        p = C.c_void_p()
        check(lib().cep_state_evict(self.h, k.ctypes.data, len(k), C.byref(p), offs.ctypes.data))
        if not len(k) or offs[-1] == 0:
            return [b""] * len(k)
        raw = C.string_at(p.value, int(offs[-1]))
        return [raw[int(offs[i]):int(offs[i + 1])] for i in range(len(k))]

    def state_import_keys(self, blobs, keys):
        """cep_state_import_keys: single-key blobs restored under new key ids."""
        k = np.ascontiguousarray(keys, np.int32)
        bufs = [C.create_string_buffer(b, max(1, len(b))) for b in blobs]
        ptrs = (C.c_void_p * max(1, len(bufs)))(*[C.cast(b, C.c_void_p) for b in bufs])
        lens = (C.c_size_t * max(1, len(bufs)))(*[len(b) for b in blobs])
        check(lib().cep_state_import_keys(self.h, ptrs, lens, k.ctypes.data, len(k)))

    def set_max_key_words(self, words: int):
        check(lib().cep_session_set_max_key_words(self.h, int(words)))

    def key_state(self, key: int):
        """(NFA.getRuns(), run-queue length) of a key, or None if it has no state yet."""
        runs, q = C.c_int64(), C.c_int64()
        check(lib().cep_key_state(self.h, key, C.byref(runs), C.byref(q)))
        return None if q.value < 0 else (runs.value, q.value)

    def stream_position(self):
        return lib().cep_stream_position(self.h)

    def match_count_to(self, dst_ptr: int, stream=None):
        """Enqueue a copy of the last batch's device match count (int64) to device address dst_ptr."""
        check(lib().cep_match_count_to(self.h, C.c_void_p(dst_ptr), C.c_void_p(stream) if stream else None))

    def last_kernel_ms(self):
        ms = C.c_float()
        check(lib().cep_last_kernel_ms(self.h, C.byref(ms)))
        return ms.value

    def last_batch_ms(self):
        ms = C.c_float()
        check(lib().cep_last_batch_ms(self.h, C.byref(ms)))
        return ms.value
