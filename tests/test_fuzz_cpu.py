"""Random patterns (tests/fuzz_patterns.py): the product's pattern compiler (libkcep.so, host code)
accepts exactly the patterns the oracle accepts, with the same error class for the rest
(StagesFactory.java InvalidPatternException), and the generator is deterministic."""
import pytest

import oracle as O
from kcep import native as N
import fuzz_patterns as F
import patterns_lib as PL

SEEDS = range(300)


def test_generator_is_deterministic():
    for seed in (0, 5, 123):
        a, b = F.random_pattern(seed), F.random_pattern(seed)
        assert a[0].to_ir(PL.I32) == b[0].to_ir(PL.I32) and a[1:] == b[1:]
        ka, va, ta = F.random_stream(seed)
        kb, vb, tb = F.random_stream(seed)
        assert (ka == kb).all() and (va == vb).all() and (ta == tb).all()


def test_compile_validity_matches_oracle():
    seen = {"ok": 0, "invalid": 0}
    for seed in SEEDS:
        pat, desc, _ = F.random_pattern(seed)
        ir = pat.to_ir(PL.I32)
        oerr = None
        try:
            O.OraclePattern(ir)
        except O.OracleError as e:
            oerr = e.code
        gerr = None
        try:
            N.CompiledPattern(ir)
        except N.CepError as e:
            gerr = e.code
        assert oerr == gerr, (seed, desc, oerr, gerr)
        seen["ok" if oerr is None else "invalid"] += 1
    assert seen["ok"] > 200 and seen["invalid"] > 5, seen
