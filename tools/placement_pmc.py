"""Counter-level look at the placement spread: K copies of
the one-part FE27 256³ operator and K x vectors, every (A_i, x_j) pairing
run `--reps` times in a fixed schedule that is printed as JSON (one entry
per mul! call).  Run under `rocprofv3 --kernel-trace --pmc <ctrs>` (one
pass per counter group); `--analyze DIR...` then maps each pass's SpMV
dispatches onto the schedule and prints, per pairing, the median kernel
time and the median of every counter collected.

    python tools/placement_pmc.py [--k 2] [--reps 6]             (the profiled child)
    python tools/placement_pmc.py --analyze gpurun_out/x/pmc1 gpurun_out/x/pmc2 ...
"""
import argparse
import csv
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPMV = ("k_spmv_sell", "k_spmv_group", "k_spmv_merged")


def child(a):
    sys.path.insert(0, ROOT)
    import pamd
    be = pamd.HIPBackend(devices=[0])
    shape = tuple(int(v) for v in a.shape.split(","))
    parts = be.get_part_ids(shape)
    N = tuple(a.n * s for s in shape)
    partition = pamd.drivers.stencil_partition(parts, N, 27)
    ctx = be.context(1)
    def build(i):
        # --contig "1010": copy i's values in physically contiguous memory
        # when its character is 1 (PA_DIAG_VAL_CONTIGUOUS, read per build)
        if a.contig and a.contig[i % len(a.contig)] == "1":
            os.environ["PA_DIAG_VAL_CONTIGUOUS"] = "1"
        else:
            os.environ.pop("PA_DIAG_VAL_CONTIGUOUS", None)
        return pamd.drivers.stencil_operator(parts, N, 27, np.float64, partition=partition)
    As = [build(i) for i in range(a.k)]
    xs = [pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids), As[0].cols.partition), As[0].cols)
        for _ in range(a.k)]
    y = pamd.PVector.undef(As[0].rows)
    ctx.sync()
    sched = []
    for i in range(a.k):
        for j in range(a.k):
            for _ in range(a.reps):
                pamd.mul_(y, As[i], xs[j])
                sched.append([i, j])
    ctx.sync()
    # and without the profiler's serialisation: HIP-event time per pairing
    ms = {}
    for i in range(a.k):
        for j in range(a.k):
            pamd.mul_(y, As[i], xs[j])
            ctx.sync()
            ctx.span_start()
            for _ in range(a.reps):
                pamd.mul_(y, As[i], xs[j])
            ctx.span_stop()
            ms[f"A{i}x{j}"] = round(ctx.span_ms() / a.reps, 4)
    rebuilt = None
    if a.rebuild:
        # free the first half of the copies, build as many again (the driver
        # hands their physical pages back): if a rebuilt copy runs at the
        # rate of the copy it replaced, the rate belongs to the pages
        import gc
        h = a.k // 2
        freed = {f"A{i}": ms[f"A{i}x0"] for i in range(h)}
        for i in range(h):
            As[i] = None
        gc.collect()
        ctx.sync()
        Bs = [build(i) for i in range(h)]
        ctx.sync()
        rebuilt = {"freed_copies_ms_x0": freed, "rebuilt_ms_x0": {}}
        for i, Bi in enumerate(Bs):
            pamd.mul_(y, Bi, xs[0])
            ctx.sync()
            ctx.span_start()
            for _ in range(a.reps):
                pamd.mul_(y, Bi, xs[0])
            ctx.span_stop()
            rebuilt["rebuilt_ms_x0"][f"B{i}"] = round(ctx.span_ms() / a.reps, 4)
        rebuilt["rebuilt_val"] = [hex(Bi.values.local(1).device_ptrs()["val"]) for Bi in Bs]
        As[:h] = Bs
    ptrs = [{k: hex(v) for k, v in Ai.values.local(1).device_ptrs().items()} for Ai in As]
    # every part's value and column arrays per copy (the
    # bases modulo the interleave granularities a placement effect would
    # follow: 4 KiB pages, 64 KiB, 2 MiB fragments)
    allp = [{str(p): {k: hex(v) for k, v in Ai.values.local(p).device_ptrs().items() if k in ("val", "col", "mask",
                                                                                             "slice_off")}
             for p in parts.part_ids} for Ai in As]
    mods = [{str(p): {f"val_mod_{m}": Ai.values.local(p).device_ptrs()["val"] % m for m in (4096, 65536, 1 << 21)}
             for p in parts.part_ids} for Ai in As]
    print(json.dumps({"tool": "placement_pmc", "k": a.k, "reps": a.reps, "shape": shape, "event_ms": ms,
                      "rebuild": rebuilt, "contig": a.contig,
                      "schedule": sched, "mat_ptrs": ptrs, "all_part_ptrs": allp, "val_base_mods": mods,
                      "x": [hex(x.values.parts[0].device_ptr()) for x in xs],
                      "x_all_parts": [[hex(v.device_ptr()) for v in x.values.parts] for x in xs]}), flush=True)


def _csv(d, suffix):
    for r, _, fs in os.walk(d):
        for f in fs:
            if f.endswith(suffix):
                return list(csv.DictReader(open(os.path.join(r, f))))
    return []


def analyze(dirs):
    out = {}
    sched = None
    for d in dirs:
        log = [json.loads(l) for l in open(d + ".log") if l.startswith("{\"tool\": \"placement_pmc\"")]
        sched = log[0]["schedule"]
        for key, v in log[0].get("event_ms", {}).items():
            out.setdefault(key, {}).setdefault("event_ms", []).append(v)
        trace = [r for r in _csv(d, "kernel_trace.csv") if any(k in r["Kernel_Name"] for k in SPMV)]
        # one mul! = the dispatches of the SpMV kernels; group consecutive dispatches per call
        per_call = len(trace) // len(sched)
        dur = {}
        for c, (i, j) in enumerate(sched):
            rows = trace[c * per_call:(c + 1) * per_call]
            dur.setdefault((i, j), []).append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows))
        ctr = {}
        rows = [r for r in _csv(d, "counter_collection.csv") if any(k in r["Kernel_Name"] for k in SPMV)]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        per_call_c = len(ids) // len(sched)
        by_id = {}
        for r in rows:
            by_id.setdefault(int(r["Dispatch_Id"]), {}).setdefault(r["Counter_Name"], 0.0)
            by_id[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for c, (i, j) in enumerate(sched):
            acc = {}
            for did in ids[c * per_call_c:(c + 1) * per_call_c]:
                for k, v in by_id[did].items():
                    acc[k] = acc.get(k, 0.0) + v
            for k, v in acc.items():
                ctr.setdefault((i, j), {}).setdefault(k, []).append(v)
        for key in dur:
            o = out.setdefault(f"A{key[0]}x{key[1]}", {})
            o.setdefault("kernel_us", []).append(round(float(np.median(dur[key][1:] or dur[key])) / 1e3, 1))
            for k, v in ctr.get(key, {}).items():
                o[k] = float(np.median(v[1:] or v))
    print(json.dumps({"tool": "placement_pmc --analyze", "passes": dirs, "pairings": out}, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--shape", default="1,1,1", help="Cartesian parts of one GPU (n^3 nodes each)")
    ap.add_argument("--analyze", nargs="+")
    ap.add_argument("--contig", default="", help="per copy (cyclic): 1 = values via hipDeviceMallocContiguous")
    ap.add_argument("--rebuild", action="store_true",
                    help="free the first half of the copies, rebuild them, time the new ones against x0")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        child(a)
