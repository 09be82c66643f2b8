"""Synthetic keyed event streams of BASELINE.md §3 (configs C2-C5).

Counter-based RNG so that every GPU and the CPU see identical data:
``rng(seed, i) = splitmix64(seed + i)`` where ``splitmix64(x)`` is one step of
the SplitMix64 generator from state ``x`` (state += 0x9e3779b97f4a7c15, then
the Stafford variant-13 finaliser).  Events are stable-sorted by
``(key_id, ts)`` with ``ts = offset = i`` (the pre-sort index).

Two implementations with identical output: numpy (CPU, used by tests and the
CPU baseline sample) and torch (GPU tensors for bench.py; int64 arithmetic
wraps like uint64 and shifts are masked to be logical).
"""
from __future__ import annotations

import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB

C2_KEY_SEED = 0xCE9
C2_VAL_SEED = 0xCE9A


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z = x + np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
        z = z ^ (z >> np.uint64(31))
    return z


def rng_np(seed: int, lo: int, hi: int) -> np.ndarray:
    i = np.arange(lo, hi, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return splitmix64_np(i + np.uint64(seed))


def c2_stream_np(n: int, n_keys: int, nvals: int = 4, key_seed=C2_KEY_SEED, val_seed=C2_VAL_SEED,
                 key_offset: int = 0, lo: int = 0):
    """C2: key = rng % K, value = rng % 4 (0=A 1=B 2=C 3=other),
    stable-sorted by key; returns (key int32, value int32, ts/offset int64).
    ``lo`` selects the counter range [lo, lo+n) (one shard of a larger stream)."""
    key = (rng_np(key_seed, lo, lo + n) % np.uint64(n_keys)).astype(np.int64)
    val = (rng_np(val_seed, lo, lo + n) % np.uint64(nvals)).astype(np.int32)
    order = np.argsort(key, kind="stable")
    return ((key[order] + key_offset).astype(np.int32), val[order], order.astype(np.int64) + lo)


def _srl(x, k):
    """logical right shift of int64 tensor (uint64 bits)."""
    import torch
    return (x >> k) & ((1 << (64 - k)) - 1)


def _mul_u64(x, c):
    """x * c mod 2^64 on int64 tensors (c given as an unsigned python int)."""
    if c >= 1 << 63:
        c -= 1 << 64
    return x * c


def splitmix64_torch(x):
    z = x + (GOLDEN - (1 << 64))
    z = _mul_u64(z ^ _srl(z, 30), M1)
    z = _mul_u64(z ^ _srl(z, 27), M2)
    return z ^ _srl(z, 31)


def umod_torch(x, m: int):
    """unsigned 64-bit x mod m (m < 2^31) on int64 tensors."""
    import torch
    hi = _srl(x, 32)
    lo = x & 0xFFFFFFFF
    r32 = (1 << 32) % m
    return ((hi % m) * r32 + (lo % m)) % m


def rng_torch(seed: int, lo: int, hi: int, device):
    import torch
    i = torch.arange(lo, hi, dtype=torch.int64, device=device)
    s = seed if seed < (1 << 63) else seed - (1 << 64)
    return splitmix64_torch(i + s)


def c2_stream_torch(n: int, n_keys: int, device, nvals: int = 4, key_seed=C2_KEY_SEED, val_seed=C2_VAL_SEED,
                    key_offset: int = 0, lo: int = 0, chunk: int = 1 << 25):
    """Same stream as c2_stream_np, generated on ``device``."""
    import torch
    key = torch.empty(n, dtype=torch.int32, device=device)
    val = torch.empty(n, dtype=torch.int32, device=device)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        key[a:b] = umod_torch(rng_torch(key_seed, lo + a, lo + b, device), n_keys).to(torch.int32)
        val[a:b] = umod_torch(rng_torch(val_seed, lo + a, lo + b, device), nvals).to(torch.int32)
    skey, order = torch.sort(key, stable=True)
    sval = val[order]
    del key, val
    return (skey + key_offset).contiguous(), sval.contiguous(), order + lo


def c2_pattern():
    """3-stage strict A -> B -> C (BASELINE C2; README Letters shape)."""
    from .pattern import QueryBuilder
    from .expr import Event
    return (QueryBuilder().select("A").where(Event.value() == 0).then()
            .select("B").where(Event.value() == 1).then()
            .select("C").where(Event.value() == 2).build())


# ---- C3-C5: fixed-length key segments ----
# Records are laid out key-major: record i belongs to key i // L and is that
# key's (i % L)-th event, so the batch is already grouped by (key, ts).

C3_SEED, C4_SEED, C5_SEED = 0xC3, 0xC4, 0xC5


def _segmented(n_keys, L, key_offset, lo):
    """global counter range of this shard's records and their key ids."""
    first = lo * L
    return first, first + n_keys * L


def c3_stream_np(n_keys: int, L: int = 100, key_offset: int = 0, lo: int = 0):
    """C3 stock ticker: per key, ts += 1 + rng % 30000 (ms), price = 100 + random
    walk of steps rng % 11 - 5 (i32).  ``lo`` = index of this shard's first key."""
    a, b = _segmented(n_keys, L, key_offset, lo)
    r = rng_np(C3_SEED, a, b)
    dts = (r % np.uint64(30000)).astype(np.int64) + 1
    step = ((r >> np.uint64(32)) % np.uint64(11)).astype(np.int64) - 5
    ts = np.cumsum(dts.reshape(n_keys, L), axis=1).reshape(-1)
    price = (100 + np.cumsum(step.reshape(n_keys, L), axis=1)).reshape(-1).astype(np.int32)
    key = (np.repeat(np.arange(n_keys, dtype=np.int64), L) + key_offset).astype(np.int32)
    return key, price, ts


def c4_stream_np(n_keys: int, L: int = 12, key_offset: int = 0, lo: int = 0):
    """C4 run-explosion stress: v = rng % 4, L events per key (kept small, Q6)."""
    a, b = _segmented(n_keys, L, key_offset, lo)
    val = (rng_np(C4_SEED, a, b) % np.uint64(4)).astype(np.int32)
    key = (np.repeat(np.arange(n_keys, dtype=np.int64), L) + key_offset).astype(np.int32)
    return key, val, np.tile(np.arange(L, dtype=np.int64), n_keys)


def c5_stream_np(n_keys: int, L: int = 100, key_offset: int = 0, lo: int = 0):
    """C5 AND/OR + optional: v = rng % 64, L events per key."""
    a, b = _segmented(n_keys, L, key_offset, lo)
    val = (rng_np(C5_SEED, a, b) % np.uint64(64)).astype(np.int32)
    key = (np.repeat(np.arange(n_keys, dtype=np.int64), L) + key_offset).astype(np.int32)
    return key, val, np.tile(np.arange(L, dtype=np.int64), n_keys)


def _key_torch(n_keys, L, key_offset, device):
    import torch
    return (torch.arange(n_keys, dtype=torch.int32, device=device).repeat_interleave(L) + key_offset).contiguous()


def c3_stream_torch(n_keys: int, device, L: int = 100, key_offset: int = 0, lo: int = 0):
    import torch
    a, b = _segmented(n_keys, L, key_offset, lo)
    r = rng_torch(C3_SEED, a, b, device)
    dts = umod_torch(r, 30000) + 1
    step = umod_torch(_srl(r, 32), 11) - 5
    ts = torch.cumsum(dts.view(n_keys, L), dim=1).reshape(-1)
    price = (100 + torch.cumsum(step.view(n_keys, L), dim=1)).reshape(-1).to(torch.int32)
    return _key_torch(n_keys, L, key_offset, device), price.contiguous(), ts.contiguous()


def _uniform_stream_torch(seed, m, n_keys, L, key_offset, lo, device):
    import torch
    a, b = _segmented(n_keys, L, key_offset, lo)
    val = umod_torch(rng_torch(seed, a, b, device), m).to(torch.int32)
    ts = torch.arange(L, dtype=torch.int64, device=device).repeat(n_keys)
    return _key_torch(n_keys, L, key_offset, device), val.contiguous(), ts.contiguous()


def c4_stream_torch(n_keys: int, device, L: int = 12, key_offset: int = 0, lo: int = 0):
    return _uniform_stream_torch(C4_SEED, 4, n_keys, L, key_offset, lo, device)


def c5_stream_torch(n_keys: int, device, L: int = 100, key_offset: int = 0, lo: int = 0):
    return _uniform_stream_torch(C5_SEED, 64, n_keys, L, key_offset, lo, device)


def c3_pattern():
    """C3: first v>0 (sum=v, count=1) -> second.oneOrMore (avg >= v; sum+=v, count+=1)
    -> latest (avg < v), within(60 s).  Shape of NFATest.java:66-87."""
    from .pattern import QueryBuilder, TimeUnit
    from .expr import Event, States, Curr
    avg = (States.getInt("sum") / States.getInt("count")).asDouble()
    return (QueryBuilder().select("first").where(Event.value() > 0)
            .fold("sum", Event.value()).fold("count", 1).then()
            .select("second").oneOrMore().where(avg >= Event.value())
            .fold("sum", Curr.int() + Event.value()).fold("count", Curr.int() + 1).then()
            .select("latest").where(avg < Event.value()).within(60, TimeUnit.SECONDS).build())


def c4_pattern():
    """C4: a strict v==0 -> b skip-till-any times(3) v==1 -> c skip-till-any
    zeroOrMore v==2 -> d skip-till-any v==3."""
    from .pattern import QueryBuilder, Selected
    from .expr import Event
    return (QueryBuilder().select("a").where(Event.value() == 0).then()
            .select("b", Selected.withSkipTilAnyMatch()).times(3).where(Event.value() == 1).then()
            .select("c", Selected.withSkipTilAnyMatch()).zeroOrMore().where(Event.value() == 2).then()
            .select("d", Selected.withSkipTilAnyMatch()).where(Event.value() == 3).build())


def c5_pattern():
    """C5: s1 10<=v<20 -> s2.optional() v==5 or v==6 -> s3 (30<=v<40) or v==63, strict."""
    from .pattern import QueryBuilder
    from .expr import Event
    v = Event.value()
    return (QueryBuilder().select("s1").where((v >= 10) & (v < 20)).then()
            .select("s2").optional().where((v == 5) | (v == 6)).then()
            .select("s3").where(((v >= 30) & (v < 40)) | (v == 63)).build())
