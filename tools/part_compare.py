"""Why does a 256³ part of the (2,2,2) partition of 512³ run faster than the
one-part 256³ operator?  Same process: each operator's format info, traffic
and its merged mul! timed alone (pa_spmv_all on one part, no halo), HIP-event
span over --reps calls.   python tools/part_compare.py [--reps 30]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--merge", type=int, default=1, help="pa_tune spmv_merge (0: one launch per slice kind)")
ap.add_argument("--idlist", type=int, default=1, help="0: keep identity slice lists (spmv_flags bit 4 off)")
a = ap.parse_args()
pamd._lib.tune("spmv_merge", a.merge)
if not a.idlist:
    pamd._lib.tune("spmv_flags", pamd._lib.tune("spmv_flags", 0) & ~16)
be = pamd.HIPBackend(devices=[0])


def alone(A, x, y, p):
    c = be.context(p)
    ix = pamd.device.device_index(c, A.cols.partition.local(p))
    iy = pamd.device.device_index(c, A.rows.partition.local(p))
    one, zero = pamd._lib.scalar_buf(1.0, np.float64), pamd._lib.scalar_buf(0.0, np.float64)
    args = (1, pamd._lib.ptr_array([A.values.local(p).h]), pamd._lib.ptr_array([y.values.local(p).h]),
            pamd._lib.ptr_array([iy.h]), pamd._lib.ptr_array([x.values.local(p).h]), pamd._lib.ptr_array([ix.h]),
            None, one[1], zero[1])
    for _ in range(3):
        pamd._lib.call("pa_spmv_all", *args)
    c.sync()
    c.span_start()
    for _ in range(a.reps):
        pamd._lib.call("pa_spmv_all", *args)
    c.span_stop()
    return round(c.span_ms() / a.reps, 4)


for shape in ((1, 1, 1), (2, 2, 2)):
    parts = be.get_part_ids(shape)
    N = tuple(a.n * s for s in shape)
    A = pamd.drivers.stencil_operator(parts, N, 27)
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids),
                                              A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows)
    for p in (parts.part_ids[0], parts.part_ids[-1]):
        M = A.values.local(p)
        rec = {"shape": list(shape), "part": p, "ms_alone": alone(A, x, y, p), "info": M.info(), "traffic": M.traffic(),
               "nlids_cols": int(A.cols.partition.local(p).num_lids)}
        print(json.dumps(rec), flush=True)
    del A, x, y
