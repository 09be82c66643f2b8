"""Helpers shared by the golden-vector tests (test infrastructure)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def scenarios():
    return load("scenarios.json")


TYPES = {1: np.int32, 2: np.int64, 3: np.float64}


def event_arrays(fx):
    ev = fx["events"]
    coltypes = [t for _, t in fx["columns"]]
    cols = [np.asarray(c, dtype=TYPES[t]) for c, t in zip(ev["cols"], coltypes)]
    out = dict(key=np.asarray(ev["key"], np.int32), cols=cols, coltypes=coltypes,
               topic=np.asarray(ev["topic"], np.int32), partition=np.asarray(ev["partition"], np.int32),
               offset=np.asarray(ev["offset"], np.int64), ts=np.asarray(ev["ts"], np.int64))
    out["valid"] = np.asarray(ev["valid"], np.uint8) if "valid" in ev else None
    return out


def seq_repr(groups):
    """[(stage, [records])] -> comparable list."""
    return [(g["stage"], list(g["events"])) if isinstance(g, dict) else (g[0], list(g[1])) for g in groups]
