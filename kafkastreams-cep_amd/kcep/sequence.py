"""Event / Sequence — host mirror of the reference output types.

* ``Event``     reference ``cep/Event.java:27-123``: identity is
  (topic, partition, offset); ``compareTo`` orders by offset within one
  topic-partition and by timestamp across them.
* ``Sequence``  reference ``cep/Sequence.java:36-225``: stage groups in the
  reversed first-seen order of the buffer traversal (``Builder.build(true)``),
  each group a ``TreeSet<Event>``.

``sequences_from_matches`` turns the CSR returned by ``cep_collect`` into
these objects.  The per-stage TreeSet is emulated exactly, including
java.util.TreeMap's red-black insertion (its shape decides which duplicates
collapse when the comparator is inconsistent across topics).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, List


@dataclass(frozen=True)
class Event:
    key: Any
    value: Any
    timestamp: int
    topic: str
    partition: int
    offset: int

    def compareTo(self, that: "Event") -> int:
        if self.topic != that.topic or self.partition != that.partition:
            return (self.timestamp > that.timestamp) - (self.timestamp < that.timestamp)
        return (self.offset > that.offset) - (self.offset < that.offset)

    def __eq__(self, o):          # Event.equals: (topic, partition, offset)
        return isinstance(o, Event) and (self.topic, self.partition, self.offset) == (o.topic, o.partition, o.offset)

    def __hash__(self):
        return hash((self.topic, self.partition, self.offset))


class _Node:
    __slots__ = ("ev", "l", "r", "p", "red")

    def __init__(self, ev, p):
        self.ev, self.l, self.r, self.p, self.red = ev, None, None, p, False


class TreeSet:
    """java.util.TreeSet<Event> with natural ordering (TreeMap.put +
    fixAfterInsertion)."""

    def __init__(self):
        self.root = None
        self.size = 0

    def add(self, ev: Event):
        t = self.root
        if t is None:
            self.root = _Node(ev, None)
            self.size = 1
            return True
        while True:
            parent = t
            c = ev.compareTo(t.ev)
            if c < 0:
                t = t.l
            elif c > 0:
                t = t.r
            else:
                return False
            if t is None:
                break
        e = _Node(ev, parent)
        if c < 0:
            parent.l = e
        else:
            parent.r = e
        self._fix(e)
        self.size += 1
        return True

    @staticmethod
    def _par(x):
        return x.p if x else None

    @staticmethod
    def _left(x):
        return x.l if x else None

    @staticmethod
    def _right(x):
        return x.r if x else None

    @staticmethod
    def _red(x):
        return x.red if x else False

    @staticmethod
    def _set(x, red):
        if x:
            x.red = red

    def _rot_left(self, p):
        if p is None:
            return
        r = p.r
        p.r = r.l
        if r.l:
            r.l.p = p
        r.p = p.p
        if p.p is None:
            self.root = r
        elif p.p.l is p:
            p.p.l = r
        else:
            p.p.r = r
        r.l = p
        p.p = r

    def _rot_right(self, p):
        if p is None:
            return
        lft = p.l
        p.l = lft.r
        if lft.r:
            lft.r.p = p
        lft.p = p.p
        if p.p is None:
            self.root = lft
        elif p.p.r is p:
            p.p.r = lft
        else:
            p.p.l = lft
        lft.r = p
        p.p = lft

    def _fix(self, x):
        P, L, R = self._par, self._left, self._right
        x.red = True
        while x is not None and x is not self.root and x.p.red:
            if P(x) is L(P(P(x))):
                y = R(P(P(x)))
                if self._red(y):
                    self._set(P(x), False); self._set(y, False); self._set(P(P(x)), True)
                    x = P(P(x))
                else:
                    if x is R(P(x)):
                        x = P(x)
                        self._rot_left(x)
                    self._set(P(x), False); self._set(P(P(x)), True)
                    self._rot_right(P(P(x)))
            else:
                y = L(P(P(x)))
                if self._red(y):
                    self._set(P(x), False); self._set(y, False); self._set(P(P(x)), True)
                    x = P(P(x))
                else:
                    if x is L(P(x)):
                        x = P(x)
                        self._rot_right(x)
                    self._set(P(x), False); self._set(P(P(x)), True)
                    self._rot_left(P(P(x)))
        self.root.red = False

    def __iter__(self):
        out, stack, n = [], [], self.root
        while stack or n:
            while n:
                stack.append(n)
                n = n.l
            n = stack.pop()
            out.append(n.ev)
            n = n.r
        return iter(out)

    def __len__(self):
        return self.size


class Staged:
    def __init__(self, stage: str):
        self.stage = stage
        self.events = TreeSet()

    def getStage(self):
        return self.stage

    def getEvents(self) -> List[Event]:
        return list(self.events)

    def __eq__(self, o):
        return isinstance(o, Staged) and self.stage == o.stage and self.getEvents() == o.getEvents()

    def __repr__(self):
        return f"{{stage='{self.stage}', events={self.getEvents()}}}"


class Sequence:
    """Ordered stage groups (Sequence.java:330-519)."""

    def __init__(self, matched: List[Staged]):
        self._matched = list(matched)
        self._indexed = {s.stage: s for s in self._matched}

    def getByName(self, stage: str):
        return self._indexed.get(stage)

    def getByIndex(self, i: int):
        return self._matched[i]

    def matched(self):
        return list(self._matched)

    def size(self):
        return sum(len(s.events) for s in self._matched)

    def __iter__(self):
        for s in self._matched:
            yield from s.getEvents()

    def __eq__(self, o):
        return isinstance(o, Sequence) and self._matched == o._matched

    def __repr__(self):
        return repr(self._matched)

    class Builder:
        def __init__(self):
            self._groups = {}

        def add(self, stage: str, event: Event):
            g = self._groups.get(stage)
            if g is None:
                g = self._groups[stage] = Staged(stage)
            g.events.add(event)
            return self

        def build(self, reversed_: bool = True):
            gs = list(self._groups.values())
            return Sequence(gs[::-1] if reversed_ else gs)

    @staticmethod
    def newBuilder():
        return Sequence.Builder()


def sequence_from_traversal(entries, names, event_of) -> Sequence:
    """entries: [(name_id, record)] final stage first; event_of(record) -> Event."""
    b = Sequence.Builder()
    for nm, rec in entries:
        b.add(names[nm], event_of(rec))
    return b.build(True)


def sequences_from_matches(out, names, event_of):
    """CSR of cep_collect -> [(record, key, Sequence)] in emission order."""
    res = []
    for m in range(len(out["match_record"])):
        a, b = int(out["ent_off"][m]), int(out["ent_off"][m + 1])
        ents = [(int(out["ent_name"][i]), int(out["ent_record"][i])) for i in range(a, b)]
        res.append((int(out["match_record"][m]), int(out["match_key"][m]), sequence_from_traversal(ents, names, event_of)))
    return res
