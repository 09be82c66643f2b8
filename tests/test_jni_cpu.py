"""The JNI shim (jni/kcep_jni.c) without a GPU: compiled unchanged against tests/jni_stub/jni.h, it
exports one symbol per ``native`` method of java/com/github/fhuss/kafka/streams/cep/processor/GpuCEPProcessor.java, and its host-only calls
(pattern compile, stage names, blob positions) work through a mock JNIEnv with every pinned array
released."""
import os
import re
import struct

import numpy as np
import pytest

from jni_twin import JniLib, LIB, NATIVES, PFX
import patterns_lib as PL

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def jl():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: build it with `make -C tests/jni_stub` (__graft_entry__.build does)")
    return JniLib()


def test_java_natives_match_the_shim(jl):
    src = open(os.path.join(ROOT, "java", "com", "github", "fhuss", "kafka", "streams", "cep", "processor", "GpuCEPProcessor.java")).read()
    java = re.findall(r"private static native [\w\[\]]+ (\w+)\(", src)
    assert sorted(java) == sorted(NATIVES)
    c = open(os.path.join(ROOT, "jni", "kcep_jni.c")).read()
    assert sorted(re.findall(r"JNICALL CLS\((\w+)\)", c)) == sorted(NATIVES)
    for n in NATIVES:
        assert hasattr(jl.L, PFX + n)


def test_compile_and_stage_names_through_the_shim(jl):
    ir = PL.c5_optional().to_ir(PL.I32)
    p = jl.cepCompile(ir)
    assert p > 0
    names = jl.cepStageNames(p)
    assert names[0] == "$final" and len(names) >= 4
    jl.cepPatternFree(p)
    assert jl.cepCompile(b"\x00\x01") < 0 and jl.cepLastError()
    assert jl.pins() == 0


def test_state_positions_through_the_shim(jl):
    # a KCSH blob (stencil carry): two keys with 2 and 1 carried records
    blob = struct.pack("<IIqi", 0x4853434B, 1, 10, 2)
    blob += struct.pack("<iiQqq", 3, 2, 0, 7, 9) + struct.pack("<iiQq", 5, 1, 0, 8)
    assert list(jl.cepStatePositions(blob)) == [7, 9, 8]
    assert jl.pins() == 0


def _java_body(src, signature_re):
    m = re.search(signature_re, src)
    assert m, signature_re
    i = src.index("{", m.end() - 1)
    depth = 0
    for k in range(i, len(src)):
        depth += {"{": 1, "}": -1}.get(src[k], 0)
        if depth == 0:
            return src[i:k + 1]
    raise AssertionError("unbalanced " + signature_re)


def _twin_body(src, name):
    m = re.search(r"\n    def " + re.escape(name) + r"\(.*?(?=\n    def |\Z)", src, re.S)
    assert m, name
    return m.group(0)


@pytest.mark.parametrize("java_sig,twin", [
    (r"public void init\(ProcessorContext context\)", "__init__"),
    (r"public void close\(\)", "close"),
    (r"private void run\(", "_run"),
    (r"private int\[\] keyIds\(", "_key_ids"),
    (r"private void spill\(", "_spill"),
    (r"public void flush\(\)", "flush"),
    (r"private void runDevice\(", "_run_device"),
    (r"private void prune\(\)", "_prune"),
])
def test_java_methods_call_the_natives_the_twin_calls(java_sig, twin):
    """The mechanical link between GpuCEPProcessor.java and its twin (tests/jni_twin.py, which the GPU
    tests drive): each method makes the same native calls in the same order (cepLastError, the error
    text, aside).  The Java's reference hand-off (handOff) has no twin: it continues a key on the
    reference classes, which test_handoff_gpu.py checks through the oracle."""
    jsrc = open(os.path.join(ROOT, "java", "com", "github", "fhuss", "kafka", "streams", "cep", "processor",
                             "GpuCEPProcessor.java")).read()
    tsrc = open(os.path.join(ROOT, "tests", "jni_twin.py")).read()
    tsrc = tsrc[tsrc.index("class JavaTwin"):]
    jcalls = [c for c in re.findall(r"\b(cep[A-Z]\w*)\(", _java_body(jsrc, java_sig)) if c != "cepLastError"]
    tcalls = [c for c in re.findall(r"\.(cep[A-Z]\w*)\(", _twin_body(tsrc, twin)) if c != "cepLastError"]
    assert jcalls == tcalls, (java_sig, jcalls, tcalls)
