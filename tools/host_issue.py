"""Host-issue cost of one mul! (and one device-CG iteration) on the paths a
multi-GPU run takes, measured on one MI355X.

The (2,2,2) partition of a 256³ FE27 operator (8 parts of 128³), every part
on cuda:0:
  * share_streams=False: a stream pair per part and per-part launches, pack,
    transport (pull kernels on the comm streams, cross-stream events),
    interior and boundary phases — the code a process driving 8 GPUs runs;
    issued from the IssuePool's host threads (default) and, for comparison,
    with issue_threads=0 from the calling thread (the HIP-graph replay of
    r05 is gone: 2.7-2.9 ms of device time against 0.94 eager, r06);
  * share_streams=True: the grouped launches of parts sharing one GPU;
  * rccl: HIPBackend(rccl=True), every halo segment through the grouped
    ncclSend/ncclRecv, the transport a one-part-per-GPU process posts.
Host time = wall time of K calls issued back to back with the GPU kept busy
(enqueue only; the GPU finishes later), both through the Python mirror
(pamd.mul_) and through the bare C-ABI call with prebuilt argument arrays
(what a Julia ccall costs).  Prints one JSON object.

    python tools/host_issue.py [--n 256] [--k 40]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402


def measure(be, n, k, label, cg_iters=0):
    parts = be.get_part_ids((2, 2, 2))
    A = pamd.drivers.stencil_operator(parts, (n,) * 3, 27)
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows)
    ctxs = [be.context(p) for p in parts.part_ids]

    def sync():
        for c in ctxs:
            c.sync()
    for _ in range(5):
        pamd.mul_(y, A, x)
    sync()
    # device time per mul! (for the ratio)
    t0 = time.perf_counter()
    for _ in range(k):
        pamd.mul_(y, A, x)
    sync()
    wall = (time.perf_counter() - t0) / k
    # Python-level enqueue
    t0 = time.perf_counter()
    for _ in range(k):
        pamd.mul_(y, A, x)
    host_py = (time.perf_counter() - t0) / k
    sync()
    # bare C-ABI enqueue (argument arrays built once); 7 repetitions of k
    # calls, each after the device drained: the median (and the range) of
    # the per-call host time (host threads make single runs noisy)
    args = pamd.pvector._spmv_args(y, A, x, 1.0, 0.0)
    reps = []
    pamd._lib.issue_stats(reset=True)
    for _ in range(7):
        t0 = time.perf_counter()
        for _ in range(k):
            pamd._lib.call("pa_spmv_all", *args)
        reps.append((time.perf_counter() - t0) / k)
        sync()
    reps.sort()
    host_c = reps[len(reps) // 2]
    out = {"path": label, "parts": 8, "mul_wall_ms": round(1e3 * wall, 4),
           "host_us_per_mul_python": round(1e6 * host_py, 1), "host_us_per_mul_cabi": round(1e6 * host_c, 1),
           "host_us_per_mul_cabi_min_max": [round(1e6 * reps[0], 1), round(1e6 * reps[-1], 1)],
           "host_us_per_part_cabi": round(1e6 * host_c / 8, 1)}
    jmax, jmean, jn = pamd._lib.issue_stats(reset=True)
    if jn:  # threaded issue: one job = one part's share of one phase of a call (pa_issue_stats)
        out.update({"issue_jobs": jn, "issue_job_us_mean": round(jmean, 1), "issue_job_us_max": round(jmax, 1),
                    "issue_jobs_per_call": round(jn / (7 * k), 2),
                    "per_part_issue_us_per_call": round(jmean * jn / (7 * k) / 8, 1)})
    if cg_iters:
        # a tiny operator (8 parts of 8^3): device work is negligible, so the
        # wall time per iteration is the host issue (+ one wait per batch)
        A = pamd.drivers.stencil_operator(parts, (16,) * 3, 27)
        b = pamd.PVector.from_host(pamd.map_parts(
            lambda s: np.random.default_rng(7 + s.part).uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
        xx = pamd.PVector.undef(A.cols).fill_(0)
        pamd.cg_(xx, A, b, reltol=0.0, maxiter=2, device=True, batch=cg_iters)
        sync()
        xx = pamd.PVector.undef(A.cols).fill_(0)
        # batch = the whole run: the host enqueues every iteration, then waits once
        t0 = time.perf_counter()
        pamd.cg_(xx, A, b, reltol=0.0, maxiter=cg_iters, device=True, batch=cg_iters)
        total = time.perf_counter() - t0
        out["cg_host_us_per_iteration_tiny"] = round(1e6 * total / cg_iters, 1)
    del A, x, y
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--k", type=int, default=40)
    args = ap.parse_args()
    res = []
    prev = pamd._lib.tune("issue_threads", 2)  # the default (1) threads only across devices
    res.append(measure(pamd.HIPBackend(devices=[0], share_streams=False), args.n, args.k,
                       "share_streams=False, issue_threads=2 (per-part streams, events and launches, issued from "
                       "host threads)", cg_iters=200))
    pb = pamd._lib.tune("halo_barrier", 2)
    res.append(measure(pamd.HIPBackend(devices=[0], share_streams=False), args.n, args.k,
                       "share_streams=False, issue_threads=2, halo_barrier=2 (the pull on each part's compute "
                       "stream after its interior slices: 6 runtime calls per part instead of 7)"))
    pamd._lib.tune("halo_barrier", 0)
    res.append(measure(pamd.HIPBackend(devices=[0], share_streams=False), args.n, args.k,
                       "share_streams=False, issue_threads=2, halo_barrier=0 (per-neighbour event waits before "
                       "every pack and pull, the r04 issue)"))
    pamd._lib.tune("halo_barrier", pb)
    pamd._lib.tune("issue_threads", prev)
    prev = pamd._lib.tune("issue_threads", 0)
    res.append(measure(pamd.HIPBackend(devices=[0], share_streams=False), args.n, args.k,
                       "share_streams=False, issue_threads=0 (one part after the other on the calling thread)",
                       cg_iters=200))
    pamd._lib.tune("issue_threads", prev)
    res.append(measure(pamd.HIPBackend(devices=[0], share_streams=True), args.n, args.k,
                       "share_streams=True (grouped launches)", cg_iters=200))
    res.append(measure(pamd.HIPBackend(devices=[0], rccl=True), args.n, args.k,
                       "rccl=True (grouped ncclSend/ncclRecv for every halo segment)"))
    print(json.dumps({"tool": "host_issue", "n": args.n, "k": args.k, "results": res}, indent=1))


if __name__ == "__main__":
    main()
