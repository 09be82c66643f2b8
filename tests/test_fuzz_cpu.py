"""Random patterns (tests/fuzz_patterns.py): the product's pattern compiler (libkcep.so, host code)
accepts exactly the patterns the oracle accepts, with the same error class for the rest
(StagesFactory.java InvalidPatternException), the generator is deterministic, and the default GPU
suite's seeds stay small per key."""
import numpy as np
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


@pytest.mark.parametrize("variant", ["mixed", "strict", "runs"])
def test_default_seeds_stay_bounded(variant):
    """The default GPU suite's seeds (test_fuzz_gpu.py, 0-11) run in seconds: the device evaluates
    every key even where the reference task would stop at an earlier key's exception, so each key on
    its own must stay small (the generator keeps skipping strategies off open-ended repeats on long
    keys; one unbounded seed once took the device past its test timeout)."""
    for seed in range(12):
        pat, desc, _ = F.pattern_for(seed, variant)
        ir = pat.to_ir(PL.I32)
        try:
            p = O.OraclePattern(ir)
        except O.OracleError:
            continue
        key, val, ts = F.stream_for(seed, variant)
        worst = 0
        for k in np.unique(key):
            m = key == k
            r = O.OracleRun(p, O.MODE_NFA_PER_KEY)
            try:
                r.process(O.BatchArrays(key[m], [val[m]], [1], ts=ts[m]))
            except O.OracleError:
                pass
            worst = max(worst, len(r.matches(with_groups=False)))
        assert worst < 5000, (seed, desc, worst)
