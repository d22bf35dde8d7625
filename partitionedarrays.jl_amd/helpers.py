"""Table and ptr utilities (Helpers.jl:63-156), numpy, 1-based ptrs as in Julia."""
from __future__ import annotations

import numpy as np


class Table:
    """Table{T}: `data` + 1-based Int32 `ptrs` (Helpers.jl:63-94)."""

    __slots__ = ("data", "ptrs")

    def __init__(self, data, ptrs):
        self.data = np.asarray(data)
        self.ptrs = np.asarray(ptrs, dtype=np.int32)

    def __len__(self):
        return len(self.ptrs) - 1

    def __getitem__(self, i):  # 1-based, Helpers.jl:73-82
        return self.data[self.ptrs[i - 1] - 1: self.ptrs[i] - 1]

    def tolist(self):
        return [self[i].tolist() for i in range(1, len(self) + 1)]

    def copy(self):
        return Table(self.data.copy(), self.ptrs.copy())

    def __eq__(self, other):
        return (isinstance(other, Table) and np.array_equal(self.ptrs, other.ptrs)
                and np.array_equal(self.data, other.data))

    def __repr__(self):
        return f"Table({self.tolist()})"

    @staticmethod
    def from_lists(vv, dtype=np.int32):
        """Table(a::AbstractArray{<:AbstractArray}) Helpers.jl:85-88"""
        ptrs = counts_to_ptrs([len(v) for v in vv])
        data = np.concatenate([np.asarray(v, dtype=dtype) for v in vv]) if vv else np.zeros(0, dtype)
        return Table(data.astype(dtype, copy=False), ptrs)


def counts_to_ptrs(counts):
    """Helpers.jl:133-141 (length_to_ptrs! over the counts)"""
    counts = np.asarray(counts, dtype=np.int64)
    ptrs = np.empty(len(counts) + 1, dtype=np.int64)
    ptrs[0] = 1
    np.cumsum(counts, out=ptrs[1:])
    ptrs[1:] += 1
    if ptrs[-1] > np.iinfo(np.int32).max:
        raise OverflowError("Table larger than Int32 ptrs")
    return ptrs.astype(np.int32)


def ptrs_to_counts(ptrs):
    """Helpers.jl:143-149"""
    return np.diff(np.asarray(ptrs, dtype=np.int64))


def trace_setup():
    """PA_TRACE_SETUP=1: phase times of the matrix setup on stderr"""
    import os
    import sys
    import time
    on = bool(os.environ.get("PA_TRACE_SETUP"))

    def mark(what=None, t0=None):
        t = time.perf_counter()
        if on and what is not None:
            print(f"[pa setup] {what:28s} {1e3 * (t - t0):8.2f} ms", file=sys.stderr, flush=True)
        return t
    return mark
