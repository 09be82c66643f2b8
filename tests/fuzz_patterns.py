"""Seeded random patterns and streams for the parity fuzz tests (tests/test_fuzz_gpu.py,
tests/test_fuzz_cpu.py).

A pattern is 1-5 stages built through the reference's builder surface (QueryBuilder.java:25-60,
StageBuilder / PatternBuilder): each stage picks a contiguity (strict / skip-till-next /
skip-till-any, Selected.java), a cardinality (one, optional, oneOrMore, zeroOrMore, times(n),
StagesFactory.java), a predicate over the record's value (comparisons, modulo tests, and/or/not), and
sometimes a fold into a state the next stage reads (the stock demo's shape, Patterns.java:11-25) or
a window (within).  The same seed always gives the same pattern and stream."""
import numpy as np

from kcep import QueryBuilder, Selected, TimeUnit, Event, States, Curr, Long, Int, Schema

VMAX = 6                     # values 0..VMAX-1: small, so that predicates hit often
# the rich variant: three typed columns and two topics (Selected.withTopic, Selected.java:19-67)
RICH = Schema([("value", "i32"), ("px", "i64"), ("r", "f64")], topics=["A", "B"])


def _pred_rich(rng):
    kind = rng.integers(0, 5)
    if kind == 0:
        return Event.field("px") > int(rng.integers(0, 6)) * 1000
    if kind == 1:
        return Event.field("r") < float(rng.choice([0.25, 0.5, 0.75]))
    if kind == 2:
        return (Event.field("px") % 3) == (Event.value() % 3)
    if kind == 3:
        return (Event.field("r") * 4 > Event.value()) | (Event.field("px") < 500)
    return _pred(rng)


def _pred(rng, lowerable=False):
    """A value predicate; `lowerable`: comparisons and their and/or/not only (the stencil lowering,
    compile.cpp, takes no arithmetic)."""
    v = Event.value()
    kind = rng.choice([0, 1, 2, 4, 5]) if lowerable else rng.integers(0, 6)
    c = int(rng.integers(0, VMAX))
    if kind == 0:
        return v == c
    if kind == 1:
        return v < max(1, c)
    if kind == 2:
        return v > min(VMAX - 2, c)
    if kind == 3:
        return (v % 2) == int(rng.integers(0, 2))
    if kind == 4:
        d = int(rng.integers(0, VMAX))
        return (v == c) | (v == d)
    return ~(v == c) & (v < VMAX - 1)


def random_pattern(seed, rich=False):
    """(builder pattern, description, window) for `seed`; `rich`: predicates over the RICH schema's
    columns and stages reading one topic."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 6))
    cls = seed % 3                   # the stream's key length class (random_stream)
    n_any = n_rep = 0
    desc = []
    fold_state = None
    b = None
    for s in range(n):
        name = f"s{s}"
        strat = int(rng.choice([0, 1, 2], p=[0.35, 0.4, 0.25])) if s > 0 else 0
        card = int(rng.choice([0, 1, 2, 3, 4], p=[0.5, 0.12, 0.15, 0.1, 0.13])) if s > 0 else int(
            rng.choice([0, 2, 4], p=[0.7, 0.15, 0.15]))
        if s == n - 1 and rng.random() < 0.9:
            card = 0                 # mostly valid: a final stage may be neither optional nor repeated
                                     # (StagesFactory.java InvalidPatternException); the rest checks the error
        # Skipping strategies over open-ended repeats enumerate subsets of a key's records (as the
        # reference does, exponentially): so that every seed runs in seconds (the device evaluates
        # every key, the task stops at the first exception), skip-till-any repeats and skip-till-any
        # after a repeat only on the short keys, at most two skip-till-any stages and no open-ended
        # repeat on the long keys (checked by the per-key oracle over seeds 0-299: <= 3.2 k matches a key)
        if strat == 2 and card in (2, 3) and cls > 0 and s < n - 1:
            card = 0
        if strat == 2 and (n_any >= 2 and cls == 2 or n_rep >= 1 and cls > 0):
            strat = 1
        if card in (2, 3) and cls == 2:
            card = 4 if s < n - 1 else 0
        n_any += strat == 2
        n_rep += card in (2, 3)
        sel = [Selected.withStrictContiguity, Selected.withSkipTilNextMatch, Selected.withSkipTilAnyMatch][strat]()
        if rich and rng.random() < 0.25:
            sel = sel.withTopic(str(rng.choice(["A", "B"])))
        st = (QueryBuilder().select(name, sel) if b is None else b.then().select(name, sel))
        if card == 1:
            st = st.optional()
        elif card == 2:
            st = st.oneOrMore()
        elif card == 3:
            st = st.zeroOrMore()
        elif card == 4:
            st = st.times(int(rng.integers(2, 4)))
        if fold_state is not None and rng.random() < 0.6:
            p = Event.value() >= States.getOrElse(fold_state, Long(0)).asLong() % VMAX
            desc.append(f"{name}:{strat}/{card}/state")
        else:
            p = _pred_rich(rng) if rich else _pred(rng)
            desc.append(f"{name}:{strat}/{card}")
        b = st.where(p)
        if rng.random() < 0.2:
            b = b.or_(Event.value() == int(rng.integers(0, VMAX)))
        fold_state = None
        if s < n - 1 and rng.random() < 0.2:
            fold_state = f"f{s}"
            b = b.fold(fold_state, Curr.long() + Event.value())
    window = None
    if rng.random() < 0.25:
        window = int(rng.integers(3, 20))
        b = b.within(window, TimeUnit.MILLISECONDS)
        desc.append(f"within {window} ms")
    return b.build(), " ".join(desc), window


def random_stream(seed, n_keys=None, per_key=None):
    """Key-grouped (key, value, timestamp) arrays for `seed`: Poisson record counts per key (short,
    medium or long keys by seed), values 0..VMAX-1, timestamps strictly increasing by 1-3 ms."""
    rng = np.random.default_rng(seed + 7919)
    if per_key is None:
        n_keys, per_key = [(300, 4), (120, 12), (40, 30)][seed % 3]
    lens = rng.poisson(per_key, n_keys) + 1
    key = np.repeat(np.arange(n_keys, dtype=np.int32), lens)
    val = rng.integers(0, VMAX, len(key)).astype(np.int32)
    ts = np.cumsum(rng.integers(1, 4, len(key))).astype(np.int64)
    return key, val, ts


def rich_columns(seed, key, val, ts, processor):
    """Columns and record metadata of the rich variant for a key-grouped `key`: px (i64), r (f64),
    topic 0/1, ~5 % null records, and in processor mode ~5 % re-deliveries, which the processor's
    high-water mark drops when it has seen the offset (CEPProcessor.java:152-160).  A re-delivery is
    the record 3 positions back delivered again (same key, offset and contents: an offset names one
    record of a partition; buffer nodes are keyed by it, Matched.java:31-35).  Returns
    (val, ts, px, r, topic, valid, offset)."""
    rng = np.random.default_rng(seed + 15485863)
    n = len(key)
    val, ts = val.copy(), ts.copy()
    px = rng.integers(0, 6000, n).astype(np.int64)
    r = rng.random(n)
    topic = rng.integers(0, 2, n).astype(np.int32)
    valid = (rng.random(n) > 0.05).astype(np.uint8)
    offset = np.arange(n, dtype=np.int64)
    if processor:
        dup = rng.random(n) < 0.05
        for i in np.nonzero(dup)[0]:
            if i >= 3 and key[i - 3] == key[i]:
                for a in (val, ts, px, r, topic, valid, offset):
                    a[i] = a[i - 3]
    return val, ts, px, r, topic, valid, offset


def random_strict_pattern(seed):
    """A pattern of the stencil / chain paths' class (compile.cpp analyse_stencil): 1-8 strict
    stages on value predicates (ranges, sets, complements, and/or), optional middle stages in
    patterns of <= 4 stages (the chain path), sometimes a window.  Returns (pattern, desc, window)."""
    rng = np.random.default_rng(seed + 31337)
    n = int(rng.choice(np.arange(1, 9), p=[.1, .2, .2, .2, .1, .08, .06, .06]))
    chain = n <= 4 and rng.random() < 0.5
    b, desc = None, []
    for s in range(n):
        st = QueryBuilder().select(f"s{s}") if b is None else b.then().select(f"s{s}")
        opt = chain and 0 < s < n - 1 and rng.random() < 0.6
        if opt:
            st = st.optional()
        b = st.where(_pred(rng, lowerable=True))
        if rng.random() < 0.15:
            b = b.or_(Event.value() == int(rng.integers(0, VMAX)))
        desc.append(f"s{s}{'?' if opt else ''}")
    window = None
    if rng.random() < 0.2:
        window = int(rng.integers(3, 20))
        b = b.within(window, TimeUnit.MILLISECONDS)
        desc.append(f"within {window} ms")
    return b.build(), " ".join(desc), window


def random_runs_pattern(seed):
    """A pattern of the runs path's class (compile.cpp analyse_runs): 2-6 strict stages, the first
    plain; later ones plain, optional, times(n) or oneOrMore, a oneOrMore stage's successor reading
    the complement of its predicate (provably exclusive, so no run branches); folds into states
    (sums, counts, last values) that later predicates compare against, C3's shape
    (NFATest.java:66-87).  Returns (pattern, desc, window)."""
    rng = np.random.default_rng(seed + 271828)
    n = int(rng.integers(2, 7))
    b, desc, prev, folded = None, [], None, []
    for s in range(n):
        st = QueryBuilder().select(f"s{s}") if b is None else b.then().select(f"s{s}")
        card = 0 if s == 0 or s == n - 1 else int(rng.choice([0, 1, 2, 3], p=[0.35, 0.15, 0.35, 0.15]))
        if card == 1:
            st = st.optional()
        elif card == 2:
            st = st.oneOrMore()
        elif card == 3:
            st = st.times(int(rng.integers(2, 4)))
        if prev is not None:                     # successor of a oneOrMore stage
            p = ~prev if rng.random() < 0.5 else (~prev & (Event.value() < VMAX - 1))
        elif card == 2:
            p = Event.value() >= int(rng.integers(1, VMAX)) if rng.random() < 0.6 else Event.value() == int(rng.integers(0, VMAX))
        elif folded and rng.random() < 0.5:
            nm = str(rng.choice(folded))
            if rng.random() < 0.5:
                p = Event.value() * 2 >= States.getOrElse(nm, Long(0)).asLong() % (2 * VMAX)
            else:
                p = (States.getInt("sum") / States.getInt("count")).asDouble() < Event.value() if (
                    "sum" in folded and "count" in folded) else Event.value() != States.getOrElse(nm, Long(-1)).asLong()
        else:
            p = _pred(rng)
        prev = p if card == 2 else None
        b = st.where(p)
        desc.append(f"s{s}{['', '?', '+', '{n}'][card]}")
        if s < n - 1 and rng.random() < 0.35:
            kind = int(rng.integers(0, 3))
            if kind == 0:
                b = b.fold("sum", (Curr.int() + Event.value()) if "sum" in folded else Event.value())
                b = b.fold("count", (Curr.int() + 1) if "count" in folded else Int(1))
                folded += [x for x in ("sum", "count") if x not in folded]
            elif kind == 1:
                b = b.fold("last", Event.value().asLong())
                folded += [] if "last" in folded else ["last"]
            else:
                b = b.fold("tot", Curr.long() + Event.value()) if "tot" in folded else b.fold("tot", Event.value().asLong())
                folded += [] if "tot" in folded else ["tot"]
    window = None
    if rng.random() < 0.3:
        window = int(rng.integers(5, 40))
        b = b.within(window, TimeUnit.MILLISECONDS)
        desc.append(f"within {window} ms")
    return b.build(), " ".join(desc), window


def pattern_for(seed, variant):
    return {"strict": random_strict_pattern, "runs": random_runs_pattern}.get(variant, random_pattern)(seed)


def stream_for(seed, variant):
    """The strict variant's streams span several 4096-record stencil tiles (12-30 k records), so
    that tile, super-tile and batch boundaries fall inside keys' runs."""
    if variant in ("strict", "runs"):
        n_keys, per_key = [(3000, 4), (2000, 12), (500, 60)][seed % 3]
        return random_stream(seed, n_keys, per_key)
    return random_stream(seed)
