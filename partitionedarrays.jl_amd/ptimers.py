"""PTimer (PTimers.jl:17-148): wall-clock sections per part, reported as
min/max/avg over the parts on MAIN.

On HIP parts a section ends when the device work the host enqueued inside it
has finished: `tic_`/`toc_` synchronise the streams of the local parts before
reading the clock (the reference's kernels are synchronous; ours are not).
`tic_(barrier=True)` also waits for the other processes (MPI.Barrier in
PTimers.jl:69-74)."""
from __future__ import annotations

import time

from .backends import MAIN, PData, gather, map_parts


def _sync_parts(parts: PData):
    be = parts.backend
    if hasattr(be, "context"):
        for p in parts.part_ids:
            be.context(p).sync()


class PTimer:
    """PTimer(parts; verbose) (PTimers.jl:32-38)."""

    def __init__(self, parts: PData, verbose: bool = False):
        self.parts = parts
        self.timings = {}          # name -> PData of seconds (one per local part)
        self.verbose = verbose
        self.current = time.perf_counter()

    def tic_(self, barrier: bool = False):
        """tic!(t; barrier) (PTimers.jl:65-74)"""
        _sync_parts(self.parts)
        if barrier:
            self.parts.backend.barrier()
        self.current = time.perf_counter()
        return self

    def toc_(self, name: str):
        """toc!(t, name) (PTimers.jl:76-87)"""
        _sync_parts(self.parts)
        now = time.perf_counter()
        dt = now - self.current
        self.timings[name] = map_parts(lambda _: dt, self.parts)
        if self.verbose and MAIN in self.parts.part_ids:
            print(f"[{dt:12.3e} s in MAIN] {name}", flush=True)
        self.current = time.perf_counter()
        return self

    @property
    def data(self):
        """t.data (PTimers.jl:40-59): on MAIN, {name: {min, max, avg}} over
        the parts; an empty dict elsewhere."""
        out = {}
        for name, timing in self.timings.items():
            g = gather(timing)
            if MAIN in g.part_ids:
                ns = list(g.local(MAIN))
                out[name] = {"min": min(ns), "max": max(ns), "avg": sum(ns) / len(ns)}
        return out

    def report(self, linechars: str = "unicode") -> str:
        """print_timer (PTimers.jl:93-148): sections by decreasing max."""
        data = self.data
        if not data:
            return ""
        rule = "─" if linechars == "unicode" else "-"
        w = 12
        ln = max(len("Section"), max(len(k) for k in data))
        head = "Section".ljust(ln) + "max".rjust(w) + "min".rjust(w) + "avg".rjust(w)
        lines = [rule * len(head), head, rule * len(head)]
        for name, d in sorted(data.items(), key=lambda kv: -kv[1]["max"]):
            lines.append(name.ljust(ln) + f"{d['max']:12.3e}{d['min']:12.3e}{d['avg']:12.3e}")
        lines.append(rule * (ln + 3 * w))
        return "\n".join(lines)
