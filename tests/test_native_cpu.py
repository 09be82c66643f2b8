"""CPU-side checks of libkcep.so: it loads, exports every symbol of
include/kcep.h, and its pattern compiler (csrc/compile.cpp, an independent
restatement of StagesFactory) produces the same stage tables as the oracle.
No HIP compute call is made here."""
import ctypes
import os
import re

import pytest

from kcep import native as N
from kcep import synth, Schema, QueryBuilder, Event, Selected
import oracle as O
from golden_util import scenarios, load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "kcep.h")).read()
    return sorted(set(re.findall(r"\b(cep_[a-z_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    L = N.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), f"libkcep.so does not export {s}"
    assert set(N.SYMBOLS) <= set(syms)
    assert b"gfx950" in L.cep_version()


ALL_IR = [(f["name"], f["ir"]) for f in scenarios()] + [(f["name"], f["ir"]) for f in load("stages_factory.json")]


@pytest.mark.parametrize("name,ir", ALL_IR, ids=[n for n, _ in ALL_IR])
def test_compiler_matches_oracle(name, ir):
    ir = bytes.fromhex(ir)
    try:
        want = O.OraclePattern(ir)
    except O.OracleError as e:
        with pytest.raises(N.CepError) as ei:
            N.CompiledPattern(ir)
        assert ei.value.code == e.code
        return
    got = N.CompiledPattern(ir)
    assert got.names == want.names
    assert got.stages() == want.stages()


def test_stencil_eligibility():
    sch = Schema([("value", "i32")])
    p = N.CompiledPattern(synth.c2_pattern().to_ir(sch))
    assert p.info.stencil_ok == 1 and p.info.stencil_k == 3
    for fx in scenarios():
        cp = N.CompiledPattern(bytes.fromhex(fx["ir"]))
        eligible = fx["name"] in ("nfa_strict3", "readme_letters", "proc_high_water_mark", "proc_null_key_value")
        assert bool(cp.info.stencil_ok) == eligible, fx["name"]


def test_chain_eligibility():
    """Strict patterns whose middle stages are optional() take the chain path (k <= 4)."""
    sch = Schema([("value", "i32")])
    p = N.CompiledPattern(synth.c5_pattern().to_ir(sch))
    assert p.info.chain_ok == 1 and p.info.stencil_ok == 0 and p.info.stencil_k == 3
    assert N.CompiledPattern(synth.c2_pattern().to_ir(sch)).info.chain_ok == 0
    for fx in scenarios():
        cp = N.CompiledPattern(bytes.fromhex(fx["ir"]))
        assert bool(cp.info.chain_ok) == (fx["name"] == "nfa_optional_strict"), fx["name"]
    v = Event.value()
    five = QueryBuilder().select("a").where(v == 0)
    for i in range(1, 5):
        five = five.then().select(f"s{i}").optional().where(v == i) if i < 4 else five.then().select("z").where(v == 9)
    assert N.CompiledPattern(five.build().to_ir(sch)).info.chain_ok == 0    # 5 stages: general path
    first_opt = (QueryBuilder().select("a").optional().where(v == 0).then().select("b").where(v == 1).build())
    assert N.CompiledPattern(first_opt.to_ir(sch)).info.chain_ok == 0


def test_bad_ir_rejected():
    sch = Schema([("value", "i32")])
    ir = synth.c2_pattern().to_ir(sch)
    for bad in (b"", b"XXXX" + ir[4:], ir[:-1], ir + b"\x00"):
        with pytest.raises(N.CepError) as ei:
            N.CompiledPattern(bad)
        assert ei.value.code == 8


def test_null_strategy_is_npe():
    sch = Schema([("value", "i32")], topics=["t"])
    p = (QueryBuilder().select("a").where(Event.value() == 0).then()
         .select("b", Selected.fromTopic("t")).where(Event.value() == 1).build())
    with pytest.raises(N.CepError) as ei:
        N.CompiledPattern(p.to_ir(sch))
    assert ei.value.code == 4
    with pytest.raises(O.OracleError) as eo:
        O.OraclePattern(p.to_ir(sch))
    assert eo.value.code == 4


def test_runs_kernels_build():
    """Every runs-path pattern of the golden scenarios (and C3) gets kernels compiled for it
    (jit.cpp): one straight-line function per predicate / fold entry, built by hiprtc for gfx950."""
    import re
    sch = Schema([("value", "i32")])
    irs = [synth.c3_pattern().to_ir(sch)] + [bytes.fromhex(f["ir"]) for f in scenarios()]
    built = 0
    for ir in irs:
        cp = N.CompiledPattern(ir)
        if not cp.info.runs_ok:
            with pytest.raises(N.CepError):
                cp.kernel_source(N.PATH_RUNS)
            continue
        src = cp.kernel_source(N.PATH_RUNS)
        fns = set(re.findall(r"bool jf_(\d+)\(", src))
        cases = set(re.findall(r"case (\d+): return jf_", src))
        assert fns and fns == cases
        assert "kcep_runs_sim" in src and "kcep_runs_write" in src
        cp.build_kernels(N.PATH_RUNS)
        built += 1
    assert built >= 8


def test_general_kernels_build():
    """The general path's kernel compiled for C4 and for a golden scenario with state,
    getOrElse-free folds and topics (hiprtc, gfx950)."""
    sch = Schema([("value", "i32")])
    for ir in (synth.c4_pattern().to_ir(sch), bytes.fromhex([f for f in scenarios() if f["name"] == "stock_demo"][0]["ir"])):
        cp = N.CompiledPattern(ir)
        assert "kcep_nfa_kernel" in cp.kernel_source(N.PATH_GENERAL)
        cp.build_kernels(N.PATH_GENERAL)


def test_runs_eligibility():
    """Deterministic strict patterns take the runs path (compile.cpp analyse_runs): C3's
    oneOrMore predicate and its successor's are complementary comparisons."""
    sch = Schema([("value", "i32")])
    assert N.CompiledPattern(synth.c3_pattern().to_ir(sch)).info.runs_ok == 1
    assert N.CompiledPattern(synth.c4_pattern().to_ir(sch)).info.runs_ok == 0     # skip-till-any
    v = Event.value()
    overlapping = (QueryBuilder().select("a").where(v == 0).then().select("b").oneOrMore().where(v >= 1)
                   .then().select("c").where(v <= 2).build())                      # TAKE and PROCEED can both match
    assert N.CompiledPattern(overlapping.to_ir(sch)).info.runs_ok == 0
    runs = {f["name"] for f in scenarios() if N.CompiledPattern(bytes.fromhex(f["ir"])).info.runs_ok}
    assert {"nfa_stateful_condition", "nfa_one_or_more", "nfa_times3", "nfa_strict3"} <= runs
    assert not runs & {"nfa_sequence_condition", "nfa_zero_or_more", "nfa_any_any", "stock_demo"}


def _kcst(words, key=0):
    """A single-key KCST blob (cep_state_evict's format) around the key's state words."""
    import struct
    w = list(words)
    return struct.pack("<IIqi", 0x5453434B, 1, 0, 1) + struct.pack("<ii", key, len(w)) + struct.pack("<%di" % len(w), *w)


def test_state_to_reference_host_only():
    """cep_state_to_reference (host-only): a minimal carried state -- one run on the begin stage with
    version [1], one high-water mark -- becomes the KCRF form (runs counter, hwm, queue with its Dewey
    digits), and malformed blobs are refused with CEP_E_ARG instead of read out of bounds."""
    import struct
    cp = N.CompiledPattern(synth.c4_pattern().to_ir(Schema([("value", "i32")])))
    begin = [i for i, st in enumerate(cp.stages()) if st[1] == 0][0]      # StateType BEGIN
    CB_HDR = 12
    # header: words, runs lo/hi, nhwm, qlen, nev, nnode, npred, nver, nseq, ncols, nstates
    hdr = [0, 5, 0, 1, 1, 0, 0, 0, 2, 0, 1, 0]
    hwm = [0, 7, 0]                                   # topic 0, offset 7
    queue = [begin | (0xFF << 8), 0, -1, 1]          # begin stage, version at 0, no event, seq 1
    vers = [1, 1]                                     # [len 1, digit 1]
    words = hdr + hwm + queue + vers
    words[0] = len(words)
    out = cp.state_to_reference(_kcst(words, key=3))
    magic, ver, key, ncols, runs = struct.unpack_from("<IIiiq", out, 0)
    assert (magic, ver, key, ncols, runs) == (0x4652434B, 1, 3, 1, 5)
    nh, = struct.unpack_from("<i", out, 24)
    assert nh == 1 and struct.unpack_from("<iq", out, 28) == (0, 7)
    assert struct.unpack_from("<i", out, 40) == (0,)             # no events
    qlen, sid, eps, flags, seq, last, ts, nd, d0 = struct.unpack_from("<iiiiqiqii", out, 44)
    assert (qlen, sid, eps, flags, seq, last, ts, nd, d0) == (1, begin, -1, 0, 1, -1, -1, 1, 1)
    bad = list(words)
    bad[3] = -1                                       # negative hwm count
    with pytest.raises(N.CepError):
        cp.state_to_reference(_kcst(bad))
    bad = list(words)
    bad[CB_HDR + 3 + 1] = 40                          # the run's version outside the version section
    with pytest.raises(N.CepError):
        cp.state_to_reference(_kcst(bad))
    with pytest.raises(N.CepError):
        cp.state_to_reference(_kcst(words)[:-4])      # truncated
    bad = list(words)
    bad[CB_HDR + 3 + 2] = 0                           # the run's last event: there are no events
    with pytest.raises(N.CepError):
        cp.state_to_reference(_kcst(bad))
    # a pattern with aggregates: one run sequence, its two states (sum, count) as (type, lo, hi)
    cs = N.CompiledPattern(synth.c3_pattern().to_ir(Schema([("value", "i32")])))
    begin = [i for i, st in enumerate(cs.stages()) if st[1] == 0][0]
    hdr = [0, 5, 0, 0, 1, 0, 0, 0, 2, 1, 1, 2]
    aggs = [1, 10, 0, 1, 2, 0]                        # sum = 10 (int), count = 2 (int)
    words = hdr + [begin | (0xFF << 8), 0, -1, 0] + [1, 1] + aggs
    words[0] = len(words)
    assert cs.state_to_reference(_kcst(words))
    for t in (4, -1):                                 # a boxed type outside int / long / double
        bad = list(words)
        bad[-6] = t
        with pytest.raises(N.CepError):
            cs.state_to_reference(_kcst(bad))


def test_csr_check_rejects_corrupt_csr():
    """cep_csr_check: the host walk of a device-written CSR is guarded -- a CSR with
    decreasing offsets, offsets not ending at n_entries, or a record / stage name out of range fails
    with CEP_E_HIP (the reference fails the task with an exception, never a crash)."""
    import ctypes as C
    import numpy as np

    def check(mrec, eoff, ename, erec, n_records=10, n_names=4):
        mrec, eoff = np.asarray(mrec, np.int64), np.asarray(eoff, np.int64)
        ename, erec = np.asarray(ename, np.int32), np.asarray(erec, np.int64)
        key = np.zeros(len(mrec), np.int32)
        m = N.Matches(len(mrec), len(erec), mrec.ctypes.data_as(C.POINTER(C.c_int64)),
                      key.ctypes.data_as(C.POINTER(C.c_int32)), eoff.ctypes.data_as(C.POINTER(C.c_int64)),
                      ename.ctypes.data_as(C.POINTER(C.c_int32)), erec.ctypes.data_as(C.POINTER(C.c_int64)),
                      2, 0, -1)
        return N.lib().cep_csr_check(C.byref(m), n_records, n_names)

    assert check([2, 5], [0, 2, 3], [1, 2, 1], [2, 1, 5]) == 0
    assert check([], [0], [], []) == 0
    assert check([2, 5], [0, 3, 2], [1, 2, 1], [2, 1, 5]) == 10        # offsets decrease
    assert check([2, 5], [1, 2, 3], [1, 2, 1], [2, 1, 5]) == 10        # does not start at 0
    assert check([2, 5], [0, 2, 2], [1, 2, 1], [2, 1, 5]) == 10        # does not end at n_entries
    assert check([2, 11], [0, 2, 3], [1, 2, 1], [2, 1, 5]) == 10       # match record past the batch
    assert check([2, 5], [0, 2, 3], [1, 2, 1], [2, -7, 5]) == 10       # entry record negative
    assert check([2, 5], [0, 2, 3], [1, 4, 1], [2, 1, 5]) == 10        # stage name id past the names
    assert "inconsistent" in N.lib().cep_last_error().decode()
