"""The Java lowering of the reference DSL, without a JVM or a GPU.

java/com/github/fhuss/kafka/streams/cep/pattern/PatternIR.java walks a reference Pattern chain and feeds
the IR builder of include/kcep.h (cep_irb_*) through jni/kcep_jni.c.  Here the shim is compiled
unchanged against tests/jni_stub/jni.h and driven call for call as PatternIR.encode drives it
(tests/patternir_twin.py).  The bytes it produces must equal kcep/pattern.py's encode_pattern -- the
IR every GPU parity test compiles -- for every golden fixture (the reference's own tests, transcribed
in tests/golden/gen_golden.py), the StagesFactoryTest shapes and BASELINE configs C1-C5.  Queries with
an opaque matcher or aggregator, and IR no device path takes, get the CPU decision."""
import ctypes as C
import importlib.util
import os
import re
import sys

import numpy as np
import pytest

from jni_twin import JniLib, LIB
import patternir_twin as T
import patterns_lib as PL

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "com", "github", "fhuss", "kafka", "streams", "cep")

from kcep import QueryBuilder, Selected, Schema, Event, States, SequenceAgg, TimeUnit  # noqa: E402
from kcep import pattern as KP, synth  # noqa: E402
from kcep import native as N  # noqa: E402


@pytest.fixture(scope="module")
def ij():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: build it with `make -C tests/jni_stub` (__graft_entry__.build does)")
    return T.IrJni(JniLib())


def captured_patterns():
    """Every (pattern, schema, topics-before, bytes) gen_golden.py encodes: Pattern.to_ir is wrapped
    while the fixture builders run, so each call's own inputs and output are recorded."""
    spec = importlib.util.spec_from_file_location("gen_golden", os.path.join(ROOT, "tests", "golden", "gen_golden.py"))
    gg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gg)
    seen = []
    real = KP.Pattern.to_ir

    def spy(self, schema):
        before = sorted(schema.topics, key=lambda t: schema.topics[t])
        ir = real(self, schema)
        seen.append((self, schema, before, ir))
        return ir

    KP.Pattern.to_ir = spy
    try:
        fx = gg.nfa_fixtures() + gg.processor_fixtures()
        sf = gg.stages_factory_fixtures()
    finally:
        KP.Pattern.to_ir = real
    return seen, fx, sf


def test_java_natives_match_the_shim(ij):
    src = open(os.path.join(JAVA, "pattern", "PatternIR.java")).read()
    java = re.findall(r"private static native [\w\[\]]+ (\w+)\(", src)
    assert sorted(java) == sorted(T.NATIVES_IR)
    c = open(os.path.join(ROOT, "jni", "kcep_jni.c")).read()
    assert sorted(re.findall(r"JNICALL IRB\((\w+)\)", c)) == sorted(T.NATIVES_IR)
    for n in T.NATIVES_IR:
        assert hasattr(ij.jl.L, T.PFX_IR + n)


def test_java_expr_kinds_are_the_twins():
    """Every node kind the twin dispatches on exists in Expr.java with its builder call."""
    src = open(os.path.join(JAVA, "pattern", "ir", "Expr.java")).read()
    for kind, call in [("Const", "out.constant"), ("Column", "out.field"), ("EventField", "out.event"),
                       ("TopicEq", "out.topicEq"), ("State", "out.state"), ("Curr", "out.curr"),
                       ("Seq", "out.seq"), ("Bin", "out.op"), ("Un", "out.op"), ("Cmp", "out.op"),
                       ("Logic", "out.op"), ("Cast", "out.cast")]:
        m = re.search(r"static final class %s extends Expr \{(.*?)\n    \}\n" % kind, src, re.S)
        assert m, kind
        assert call in m.group(1), (kind, call)


def test_every_golden_fixture_lowers_byte_identical(ij):
    seen, fx, sf = captured_patterns()
    assert len(fx) == 24
    by_ir = {f["ir"] for f in fx}
    n_gpu = 0
    for pat, schema, before, want in seen:
        got = T.encode(ij, pat, schema, pre_topics=before)
        if got.gpu():
            assert got.ir == want
            n_gpu += 1
        else:                                     # only the patterns the reference itself rejects
            assert got.status == T.CEP_E_INVALID_PATTERN, got.reason
    # all 24 scenario fixtures (the IR the GPU parity tests compile) came out of the JNI builder
    assert n_gpu >= 24
    built = {T.encode(ij, p, s, pre_topics=b).ir.hex() for p, s, b, _ in seen if T.encode(ij, p, s, pre_topics=b).gpu()}
    assert by_ir <= built
    assert ij.jl.pins() == 0


def test_stages_factory_rejections_route_to_the_cpu(ij):
    """StagesFactoryTest's invalid patterns: the IR is built, cep_compile rejects it with the
    reference's InvalidPatternException, and the query stays on CEPProcessor (which then throws it)."""
    _, _, sf = captured_patterns()
    bad = [f for f in sf if f.get("expected", {}).get("error") == 1]
    assert bad
    seen, _, _ = captured_patterns()
    rejected = [T.encode(ij, p, s, pre_topics=b) for p, s, b, ir in seen if ir.hex() in {f["ir"] for f in bad}]
    assert rejected and all(not r.gpu() and r.status == T.CEP_E_INVALID_PATTERN for r in rejected)


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4", "c5", "stock", "next_one_or_more", "any_any"])
def test_baseline_configs_lower_byte_identical(ij, name):
    I32 = Schema([("value", "i32")])
    pats = {
        "c1": (QueryBuilder().select("stage-1").where(Event.value() == ord("A")).then()
               .select("stage-2").where(Event.value() == ord("B")).then()
               .select("stage-3").where(Event.value() == ord("C")).build(), Schema([("value", "i32")], ["Letters"])),
        "c2": (synth.c2_pattern(), I32), "c3": (synth.c3_pattern(), I32), "c4": (synth.c4_pattern(), I32),
        "c5": (synth.c5_pattern(), I32), "stock": (PL.stock_demo(), PL.STOCK_SCHEMA),
        "next_one_or_more": (PL.next_one_or_more(), I32), "any_any": (PL.any_any(), I32),
    }
    pat, schema = pats[name]
    before = sorted(schema.topics, key=lambda t: schema.topics[t])
    want = pat.to_ir(schema)
    got = T.encode(ij, pat, schema, pre_topics=before)
    assert got.gpu(), got.reason
    assert got.ir == want
    # the processor's topic ids are the builder's: topic i is got.topics[i]
    assert got.topics == sorted(schema.topics, key=lambda t: schema.topics[t])
    assert N.CompiledPattern(got.ir).info.n_patterns == len(pat.chain())


def test_sequence_matchers_topics_and_windows_lower(ij):
    sch = Schema([("price", "i64"), ("volume", "f64")], topics=["a"])
    p = (QueryBuilder().select("s1", Selected.withStrictContiguity().withTopic("b"))
         .where((Event.field("price") > 10) & ~(Event.field("volume") < 0.5)).fold("n", Event.field("price") * 2)
         .then().select("s2", Selected.withSkipTilNextMatch()).oneOrMore()
         .where((SequenceAgg.avg("price") < Event.field("price")) | (SequenceAgg.count("s1") >= 3))
         .or_(SequenceAgg.sum("volume") > 2.5)
         .within(3, TimeUnit.MINUTES).then()
         .select(Selected.withSkipTilAnyMatch().withTopic("a"))
         .where(SequenceAgg.last("price", "s2") != SequenceAgg.first("price", "s1")).build())
    want = p.to_ir(sch)
    got = T.encode(ij, p, sch, pre_topics=["a"])
    assert got.gpu(), got.reason
    assert got.ir == want
    assert got.topics == ["a", "b"]


def test_opaque_matcher_or_aggregator_routes_to_the_cpu(ij):
    I32 = Schema([("value", "i32")])
    p = synth.c2_pattern()
    p.ancestor.predicate = T.Opaque(lambda e: e.value() == 1)          # stage 2: a Java lambda
    got = T.encode(ij, p, I32)
    assert not got.gpu() and "opaque" in got.reason
    q = PL.stock_demo()
    q.ancestor.aggregates[0].aggregate = T.Opaque()                    # a lambda Aggregator
    got = T.encode(ij, q, PL.STOCK_SCHEMA)
    assert not got.gpu() and "Aggregator" in got.reason
    assert ij.jl.pins() == 0


def test_type_errors_are_bad_ir_at_the_call(ij):
    """A body the IR types reject (a non-boolean matcher) fails at the builder call, not later."""
    I32 = Schema([("value", "i32")])
    p = QueryBuilder().select("a").where(Event.value() == 0).build()
    p.predicate = Event.value() + 1                                    # an int, not a boolean
    got = T.encode(ij, p, I32)
    assert not got.gpu() and got.status == T.CEP_E_BAD_IR and "boolean" in got.reason


def test_unlowerable_device_shape_routes_to_the_cpu(ij):
    """An IR that compiles but that no carry session can run (cep_pattern_check) stays on the CPU."""
    I32 = Schema([("value", "i32")])
    # too many stages for the device NFA tables (NFA_MAX_STAGES = 64)
    qb = QueryBuilder().select("s0").where(Event.value() == 0)
    for i in range(1, 40):
        qb = qb.then().select(f"s{i}").oneOrMore().where(Event.value() == i % 4)
    p = qb.then().select("last").where(Event.value() == 3).build()
    got = T.encode(ij, p, I32)
    assert not got.gpu() and got.status == T.CEP_E_UNSUPPORTED, (got.status, got.reason)


# ---- the C-ABI itself (ctypes, no JNI) ----
def _lib():
    L = N.lib()
    P = C.c_void_p
    L.cep_irb_new.argtypes = [P, C.c_int32, C.POINTER(P)]
    L.cep_irb_free.argtypes = [P]
    L.cep_irb_free.restype = None
    L.cep_irb_select.argtypes = [P, C.c_char_p, C.c_int32, C.c_int32, C.c_char_p]
    L.cep_irb_const.argtypes = [P, C.c_int32, C.c_int64, C.c_double]
    L.cep_irb_field.argtypes = [P, C.c_int32]
    L.cep_irb_op.argtypes = [P, C.c_int32]
    L.cep_irb_where.argtypes = [P, C.c_int32]
    L.cep_irb_fold.argtypes = [P, C.c_char_p, C.c_int32]
    L.cep_irb_finish.argtypes = [P, P, C.c_size_t, C.POINTER(C.c_size_t)]
    L.cep_irb_state.argtypes = [P, C.c_char_p, C.c_int32, C.c_int32]
    L.cep_pattern_check.argtypes = [P, C.c_int32]
    return L


def test_irb_c_abi_error_paths():
    L = _lib()
    b = C.c_void_p()
    assert L.cep_irb_new((C.c_int32 * 1)(1), 1, C.byref(b)) == 0
    need = C.c_size_t()
    assert L.cep_irb_finish(b, None, 0, C.byref(need)) == 8                # no select yet
    assert L.cep_irb_where(b, 1) == 11                                    # select first
    assert L.cep_irb_select(b, b"a", 0, 0, None) == 0
    assert L.cep_irb_where(b, 1) == 11                                    # stack underflow
    assert L.cep_irb_field(b, 3) == 8                                     # unknown column
    assert L.cep_irb_const(b, 0, 1, 0.0) == 0
    assert L.cep_irb_const(b, 1, 5, 0.0) == 0
    assert L.cep_irb_op(b, 0x40) == 8                                     # boolean + int
    assert L.cep_irb_state(b, b"s", 2, 0) == 0                            # the failed op consumed its operands
    assert L.cep_irb_finish(b, None, 0, C.byref(need)) == 11              # unconsumed expression
    assert L.cep_irb_where(b, 1) == 8                                     # a long is not a matcher
    assert L.cep_irb_finish(b, None, 0, C.byref(need)) == 0
    L.cep_irb_free(b)


def test_irb_matches_encode_for_a_hand_built_query():
    """select("a").where(value == 0).then().select().times(3).where(value > 1).fold("s", value) -- by hand."""
    L = _lib()
    b = C.c_void_p()
    assert L.cep_irb_new((C.c_int32 * 1)(1), 1, C.byref(b)) == 0
    L.cep_irb_quantifier.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]
    assert L.cep_irb_select(b, b"a", 0, 0, None) == 0
    assert L.cep_irb_field(b, 0) == 0 and L.cep_irb_const(b, 1, 0, 0.0) == 0 and L.cep_irb_op(b, 0x50) == 0
    assert L.cep_irb_where(b, 1) == 0
    assert L.cep_irb_select(b, None, 1, 0, None) == 0
    assert L.cep_irb_quantifier(b, 0, 0, 3) == 0
    assert L.cep_irb_field(b, 0) == 0 and L.cep_irb_const(b, 1, 1, 0.0) == 0 and L.cep_irb_op(b, 0x54) == 0
    assert L.cep_irb_where(b, 1) == 0
    assert L.cep_irb_field(b, 0) == 0 and L.cep_irb_fold(b, b"s", 0) == 0
    need = C.c_size_t()
    assert L.cep_irb_finish(b, None, 0, C.byref(need)) == 0
    buf = (C.c_uint8 * need.value)()
    assert L.cep_irb_finish(b, buf, need.value, C.byref(need)) == 0
    L.cep_irb_free(b)
    want = (QueryBuilder().select("a").where(Event.value() == 0).then().select().times(3)
            .where(Event.value() > 1).fold("s", Event.value()).build()).to_ir(Schema([("value", "i32")]))
    assert bytes(buf) == want
    pat = N.CompiledPattern(want)
    assert L.cep_pattern_check(pat.h, 1) == 0


# ComplexStreamsBuilder's public surface (core/src/main/java/com/github/fhuss/kafka/streams/cep/
# ComplexStreamsBuilder.java:31-106): constructors, the stream(...) overloads and build()
REFERENCE_BUILDER = {
    "ctors": [[], ["StreamsBuilder"]],
    "stream": [["Collection<String>", "Consumed<K, V>"], ["String", "Consumed<K, V>"], ["String"], ["KStream<K, V>"]],
}


def _params(sig):
    """Parameter types of a Java signature (commas inside <...> belong to the type)."""
    parts, depth, cur = [], 0, ""
    for ch in sig:
        depth += {"<": 1, ">": -1}.get(ch, 0)
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    return [" ".join(p.replace("final ", "").split()[:-1]) for p in parts if p.strip()]


def test_gpu_streams_builder_mirrors_the_reference_entry_point():
    """GpuComplexStreamsBuilder is the drop-in for ComplexStreamsBuilder (no reference file
    needs a hand edit): every reference constructor and stream(...) overload exists with the same
    parameters, each stream(...) has a twin taking the value's IrSchema last, every route ends in
    new GpuCEPStreamImpl<>(stream, schema, options), and GpuCEPStreamImpl has that constructor."""
    src = open(os.path.join(JAVA, "GpuComplexStreamsBuilder.java")).read()
    ctors = [_params(m) for m in re.findall(r"public GpuComplexStreamsBuilder\(([^)]*)\)", src)]
    streams = [_params(m) for m in re.findall(r"public <K, V> CEPStream<K, V> stream\(([^)]*)\)", src)]
    for c in REFERENCE_BUILDER["ctors"]:
        assert c in ctors, c
    for sig in REFERENCE_BUILDER["stream"]:
        assert sig in streams, sig
        assert sig + ["IrSchema<V>"] in streams, sig
    assert "public Topology build()" in src
    assert src.count("new GpuCEPStreamImpl<>(stream, schema, options)") == 1
    assert "new CEPStreamImpl" not in src                 # the CPU route is GpuCEPStreamImpl's decision
    impl = open(os.path.join(ROOT, "java", "org", "apache", "kafka", "streams", "kstream", "internals",
                             "GpuCEPStreamImpl.java")).read()
    assert re.search(r"public GpuCEPStreamImpl\(final KStream<K, V> stream, final IrSchema<V> schema, "
                     r"final GpuOptions options\)", impl)
    integ = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "GpuComplexStreamsBuilder" in integ
