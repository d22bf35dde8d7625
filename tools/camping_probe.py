"""Partition camping?  FE27 256^3 F64 one part: x and y are exactly 128 MiB
each.  Allocate y after a dummy buffer of `gap` bytes so the x/y address
offset changes; time mul! per gap (HIP-event span).  Prints the x and y
device addresses.   python tools/camping_probe.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402
import torch  # noqa: E402

be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
A = pamd.drivers.stencil_operator(parts, (256,) * 3, 27)
x = pamd.PVector.from_host(pamd.map_parts(lambda s: np.random.default_rng(1).uniform(-1, 1, s.num_lids),
                                          A.cols.partition), A.cols)
ctx = be.context(1)


def addr(v):
    return int(pamd._lib.vec_ptr(v.values.local(1).h)) if hasattr(pamd._lib, "vec_ptr") else None


def t(y, reps=30):
    for _ in range(3):
        pamd.mul_(y, A, x)
    ctx.sync()
    ctx.span_start()
    for _ in range(reps):
        pamd.mul_(y, A, x)
    ctx.span_stop()
    return round(ctx.span_ms() / reps, 4)


keep = []
for gap in (0, 4096, 65536, 1 << 20, 3 << 20, 7 << 20, 64 << 20, (64 << 20) + 4096):
    if gap:
        keep.append(torch.empty(gap, dtype=torch.uint8, device="cuda:0"))
    y = pamd.PVector.undef(A.rows)
    keep.append(y)
    print(json.dumps({"gap_bytes": gap, "ms_per_mul": [t(y), t(y)]}), flush=True)
# x re-uploaded into a fresh buffer after the gaps (moves x instead of y)
x2 = pamd.PVector.from_host(pamd.map_parts(lambda s: np.random.default_rng(1).uniform(-1, 1, s.num_lids),
                                           A.cols.partition), A.cols)
x = x2
print(json.dumps({"x_moved": True, "ms_per_mul": [t(keep[-1]), t(keep[-1])]}), flush=True)
