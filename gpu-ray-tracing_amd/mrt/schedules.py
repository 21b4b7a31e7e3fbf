"""Saved launch schedules of the tracer's autotuner.

The autotuner (cfg.autotune, csrc/mrt_api.cpp) times up to ten ray-distribution
schedules on the first ~90 launches of every (batch size, kernel variant) and
keeps the fastest. Which one wins depends on the BVH and the frame, and two
candidates within a few per cent of each other could settle differently from run
to run. A ScheduleStore keeps the settled choices per BVH — keyed by a content
fingerprint of the Compact2 buffers, like the reference's bvhcache keys its
.dat files by the scene (Renderer.cc:157-217) — so a later run on the same BVH
locks them at bind time: no exploring launches, the same schedule every run.

The package ships one store (tuned_schedules.json, written by tools/tune_db.py on
an MI355X for the bench's workloads); callers may keep their own next to their
.dat cache.
"""
from __future__ import annotations

import json
import os

import numpy as np

from . import _lib

DEFAULT_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned_schedules.json")


def bvh_fingerprint(nodes, woop, tri_index) -> str:
    """Content hash of the three Compact2 buffers (numpy arrays or tensors)."""
    import xxhash

    h = xxhash.xxh64()
    for a in (nodes, woop, tri_index):
        if not isinstance(a, np.ndarray):
            a = a.detach().cpu().numpy()
        a = np.ascontiguousarray(a)
        h.update(np.int64(a.nbytes).tobytes())
        h.update(memoryview(a).cast("B"))
    return h.hexdigest()


class ScheduleStore:
    """{fingerprint: [[num_rays, variant, candidate, version], ...]} in a JSON file."""

    def __init__(self, path: str = DEFAULT_PATH):
        self.path = path
        self.table = {}
        if path and os.path.exists(path):
            with open(path) as f:
                doc = json.load(f)
            if doc.get("version") == _lib.MRT_TUNE_VERSION:
                self.table = {k: [tuple(e) for e in v] for k, v in doc.get("bvhs", {}).items()}

    def entries(self, fingerprint: str) -> list:
        return list(self.table.get(fingerprint, []))

    def apply(self, tracer, fingerprint: str) -> int:
        """Lock the saved schedules of this BVH in `tracer` (after set_bvh). Returns how many."""
        e = self.entries(fingerprint)
        if e:
            tracer.load_schedules(e)
        return len(e)

    def update(self, fingerprint: str, entries) -> int:
        """Merge a tracer's settled schedules (Tracer.schedules()); returns how many are new."""
        cur = {(n, v): (n, v, c, ver) for n, v, c, ver in self.table.get(fingerprint, [])}
        new = 0
        for n, v, c, ver in entries:
            if ver != _lib.MRT_TUNE_VERSION:
                continue
            new += (n, v) not in cur
            cur[(n, v)] = (n, v, c, ver)
        self.table[fingerprint] = sorted(cur.values())
        return new

    def save(self, path: str | None = None) -> None:
        path = path or self.path
        doc = {"version": _lib.MRT_TUNE_VERSION,
               "note": "autotuner schedules per BVH fingerprint: [num_rays, variant, candidate, version]; "
                       "variant | 512 = a batch of secondary rays (MRT_TRACE_SECONDARY)",
               "bvhs": {k: [list(e) for e in v] for k, v in sorted(self.table.items())}}
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(doc, f, indent=1)
        os.replace(tmp, path)
