"""bench.py — SpMV+halo throughput of mul!(y, A, x) (Interfaces.jl:2246-2275) on
MI355X: the 27-point FE operator (test_fem_sa.jl's pattern in 3D), 256³ nodes
per GPU, weak scaling over Cartesian parts (1 → (1,1,1), 2 → (2,1,1),
4 → (2,2,1), 8 → (2,2,2)).

A step = one mul! (halo exchange of x + SpMV of every owned row) with A and x
resident in HBM.  value = algorithmic bytes of all parts /
time of K steps (max over ranks) → GB/s.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 256] [--kind 27]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one part per GPU)
    ... --strong    256³ nodes in total split over the N parts (config 3)
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
PART_SHAPES = {1: (1, 1, 1), 2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2)}
DTYPES = {"f64": np.float64, "f32": np.float32, "c128": np.complex128, "c64": np.complex64}


def algorithmic_bytes(nnz, n_own, n_ghost, n_snd, n_rcv, S, I=4):
    """nnz·(S+I) + (n_own+1)·I + (n_own+n_ghost)·S + n_own·S
    + (n_snd+n_rcv)·(I+2S)."""
    return nnz * (S + I) + (n_own + 1) * I + (n_own + n_ghost) * S + n_own * S + (n_snd + n_rcv) * (I + 2 * S)


def host_cores():
    """host cores this process may use, capped at the GPU box's share (16)"""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(kind, seconds=15.0, n=128):
    """oracle/build/spmv_ref: the reference's CSC column loop
    (SparseUtils.jl:157-187) restated in C ("port"), run as MPIBackend would
    run it on this host: one rank per core (--ranks), each with the CSC of
    its block of rows, a barrier per SpMV.  A short 1-core run rides along."""
    exe = os.path.join(ROOT, "oracle", "build", "spmv_ref")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)

    def run(ranks, secs):
        out = subprocess.run([exe, "--kind", str(kind), "--n", str(n), "--seconds", str(secs), "--ranks", str(ranks)],
                             check=True, capture_output=True, text=True).stdout
        return json.loads(out.strip().splitlines()[-1])
    cores = host_cores()
    r = run(cores, 0.7 * seconds)
    r1 = run(1, 0.3 * seconds)
    return {"value": round(r["gbps"], 3), "unit": "GB/s", "cores": cores, "kind": "port",
            "sample": f"{kind}-pt operator {n}^3 nodes ({r['nnz']} nnz), {r['reps']} SpMVs in ~{0.7 * seconds:.0f} s, "
                      f"Int64 CSC column loop (SparseUtils.jl:157-187) in C, {cores} MPIBackend-like ranks "
                      f"(threads, row blocks of PRange(parts, n), barrier per SpMV)",
            "single_core_gbps": round(r1["gbps"], 3)}


def pmc_traffic(args, steps=5):
    """HBM bytes per mul! step from rocprofv3 PMC counters, one counter per
    pass (MI355X_MICROARCH.md §HBM / §rocprofv3): FETCH_SIZE (KB, x2 for the
    gfx950 wide-stream under-count) + WRITE_SIZE (KB), summed over the SpMV
    kernels of the profiled steps / steps.  Runs this script as the profiled
    child (`--child-pmc`)."""
    import csv
    import shutil
    import signal
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not found"
    tot = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="pa_pmc_", dir="/tmp")
        cmd = ["rocprofv3", "--pmc", ctr, "-d", d, "-o", "pmc", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--child-pmc", "--steps", str(steps),
               "--n", str(args.n), "--kind", str(args.kind), "--dtype", args.dtype]
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True,
                             env=dict(os.environ, TMPDIR="/tmp"))
        try:
            p.wait(timeout=240)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            return None, f"rocprofv3 --pmc {ctr} timed out"
        files = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
        if p.returncode != 0 or not files:
            return None, f"rocprofv3 --pmc {ctr} failed (rc {p.returncode})"
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(files[0]))
                if "k_spmv_sell" in r["Kernel_Name"] and r["Counter_Name"] == ctr]
        tot[ctr] = sum(vals) / (steps + 1)  # warmup step + steps
        shutil.rmtree(d, ignore_errors=True)
    traffic = tot["FETCH_SIZE"] * 1024 * 2 + tot["WRITE_SIZE"] * 1024
    return traffic, (f"rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE passes over {steps + 1} mul! steps: "
                     f"FETCH_SIZE {tot['FETCH_SIZE']:.0f} KB x2 (gfx950) + WRITE_SIZE {tot['WRITE_SIZE']:.0f} KB per step")


def box_hbm_gbs(pamd, nbytes, reps=10):
    """Attainable HBM rates of this box (pa_hbm_probe: 16 B non-temporal
    read-only and copy sweeps of an `nbytes` buffer, best of three grid
    sizes).  A calibration beside the roofline, not the metric."""
    try:
        return pamd._lib.hbm_probe(0, nbytes, reps)
    except pamd._lib.PAError:
        return None


def child_pmc(args):
    """the profiled child of pmc_traffic: build the operator, run warmup+steps."""
    import pamd
    be = pamd.HIPBackend(devices=[0])
    parts = be.get_part_ids((1, 1, 1))
    dtype = DTYPES[args.dtype]
    A = pamd.drivers.stencil_operator(parts, (args.n,) * 3, args.kind, dtype)
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(20250114 + s.part).uniform(-1, 1, s.num_lids).astype(dtype),
        A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows, dtype)
    for _ in range(args.steps + 1):
        pamd.mul_(y, A, x)
    be.context(1).sync()


def cg_mode(args, pamd, backend, parts, A, ngpu, world, sync):
    """--cg K: IterativeSolvers.cg! iterations (BASELINE config 4) on the same
    operator: per iteration 1 mul! (+halo), dot, norm, 3 broadcasts.  Prints
    its own JSON line (not the headline metric)."""
    import torch
    import torch.distributed as dist
    cols = A.cols
    dtype = A.dtype
    b = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(7 + s.part).uniform(-1, 1, s.num_lids).astype(dtype), cols.partition), cols)
    out = {}
    variants = {"device": dict(device=True, batch=16), "fused": dict(fused=True), "unfused": dict(fused=False)}
    for name, kw in variants.items():
        x = pamd.PVector.undef(cols, dtype).fill_(0)
        pamd.cg_(x, A, b, reltol=0.0, maxiter=args.warmup, **kw)
        sync()
        if world > 1:
            dist.barrier()
        x = pamd.PVector.undef(cols, dtype).fill_(0)
        t0 = time.perf_counter()
        hist = []
        pamd.cg_(x, A, b, reltol=0.0, maxiter=args.cg, history=hist, **kw)
        sync()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        out[name] = (1e3 * el / max(1, len(hist)), len(hist), hist[-1] if hist else None)
    p0 = parts.part_ids[0]
    info = A.values.local(p0).info()
    S = np.dtype(dtype).itemsize
    n = info["nrows"]
    it_bytes = (info["nnz"] * (S + 4) + (n + 1) * 4 + 2 * n * S) + 12 * n * S  # SpMV + dot 2 + norm 1 + 3 axpy x3
    rows_all = n * ngpu
    line = {"metric": "CG iteration time (weak scaling, BASELINE config 4)",
            "value": round(out["device"][0], 4), "unit": "ms/iteration", "higher_is_better": False,
            "n_gpus": ngpu, "iterations": out["device"][1], "scaling": "weak",
            "dtype": args.dtype, "data": "synthetic (seeded uniform b, x0 = 0)",
            "config": {"workload": f"cg! on the {args.kind}-pt operator, {args.n}^3 nodes per GPU",
                       "dofs": rows_all, "recurrence": "scalars on the device (pa_cg_solve_all, batch 16)",
                       "host_driven_fused_ms_per_iteration": round(out["fused"][0], 4),
                       "host_driven_unfused_ms_per_iteration": round(out["unfused"][0], 4),
                       "algorithmic_bytes_per_iteration_per_gpu": it_bytes,
                       "gbs_per_gpu_device": round(it_bytes / (out["device"][0] * 1e-3) / 1e9, 1),
                       "final_residual": out["device"][2],
                       "same_history_as_host_driven": out["device"][2] == out["fused"][2]}}
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=256, help="nodes per dim per GPU (global with --strong)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling (BASELINE config 3): --n^3 nodes in total, split over the parts")
    ap.add_argument("--kind", type=int, default=27, choices=[7, 27])
    ap.add_argument("--dtype", default="f64", choices=list(DTYPES))
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 HBM-traffic passes")
    ap.add_argument("--child-pmc", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cg", type=int, default=0, help="time K CG iterations instead (own JSON line)")
    args = ap.parse_args()
    if args.child_pmc:
        return child_pmc(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import torch
    import torch.distributed as dist
    import pamd

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
        backend = pamd.HIPDistributedBackend()      # one part per process, halo over RCCL
        ngpu = world
    else:
        ngpu = args.gpus
        backend = pamd.HIPBackend(devices=list(range(ngpu)))  # all parts in this process
    if ngpu not in PART_SHAPES:
        raise SystemExit(f"--gpus must be one of {sorted(PART_SHAPES)}")
    shape = PART_SHAPES[ngpu]
    N = (args.n,) * 3 if args.strong else tuple(args.n * s for s in shape)
    dtype = DTYPES[args.dtype]
    S = np.dtype(dtype).itemsize

    t_setup = time.perf_counter()
    parts = backend.get_part_ids(shape)
    partition = pamd.drivers.stencil_partition(parts, N, args.kind)
    A = pamd.drivers.stencil_operator(parts, N, args.kind, dtype, partition=partition)
    rows, cols = A.rows, A.cols
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(20250114 + s.part).uniform(-1, 1, s.num_lids).astype(dtype),
        cols.partition), cols)
    y = pamd.PVector.undef(rows, dtype)
    ctxs = [backend.context(p) for p in parts.part_ids]

    def sync():
        for c in ctxs:
            c.sync()
    sync()
    t_setup = time.perf_counter() - t_setup

    # algorithmic bytes of the local parts
    ex = cols.exchanger
    B_local, infos = 0, {}
    for p in parts.part_ids:
        info = A.values.local(p).info()
        s = cols.partition.local(p)
        n_snd = len(ex.lids_snd.local(p).data)
        n_rcv = len(ex.lids_rcv.local(p).data)
        infos[p] = (info, s.num_hids)
        B_local += algorithmic_bytes(info["nnz"], info["nrows"], s.num_hids, n_snd, n_rcv, S)
    B_all = B_local
    if world > 1:
        t = torch.tensor([float(B_local)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        B_all = float(t.item())

    def barrier():
        if world > 1:
            dist.barrier()

    if args.cg > 0:
        line = cg_mode(args, pamd, backend, parts, A, ngpu, world, sync)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # Small problems fit the 256 MB MALL (SURVEY.md §7 hard part iv): rotate
    # through copies of (A, x, y) so every step streams from HBM.
    per_gpu = B_local / max(1, len(parts.part_ids))
    ncopies = 1 if per_gpu >= 1.0e9 else int(np.ceil(1.0e9 / per_gpu))
    sets = [(A, x, y)]
    for k in range(1, ncopies):
        Ak = pamd.drivers.stencil_operator(parts, N, args.kind, dtype, partition=partition)
        xk = pamd.PVector.from_host(pamd.map_parts(
            lambda s: np.random.default_rng(20250114 + s.part).uniform(-1, 1, s.num_lids).astype(dtype),
            cols.partition), Ak.cols)
        sets.append((Ak, xk, pamd.PVector.undef(Ak.rows, dtype)))
    sync()

    for i in range(args.warmup):
        Ai, xi, yi = sets[i % ncopies]
        pamd.mul_(yi, Ai, xi)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        Ai, xi, yi = sets[i % ncopies]
        pamd.mul_(yi, Ai, xi)
    sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = B_all / (elapsed / args.steps) / 1e9

    # roofline of the first local part: device time of its SpMV kernels, HIP
    # events on the stream they run on (pa_ctx_last_kernel_ms), mean of K launches
    p0 = parts.part_ids[0]
    info, s_nhids = infos[p0]
    ctx = backend.context(p0)

    def kernel_time(reps):
        ctx.set_timing(True)
        kms = []
        for i in range(reps):
            Ai, xi, yi = sets[i % ncopies]
            pamd.mul_(yi, Ai, xi)
            a_ms, b_ms = ctx.last_kernel_ms()
            kms.append(a_ms + b_ms)
        ctx.set_timing(False)
        sync()
        return float(np.mean(kms))
    reps = max(5, min(args.steps, 50))
    kernel_ms = kernel_time(reps)
    spmv_bytes = info["nnz"] * (S + 4) + (info["nrows"] + 1) * 4 + (info["nrows"] + s_nhids) * S + info["nrows"] * S
    achieved = spmv_bytes / (kernel_ms * 1e-3) / 1e9
    # the same kernels with int32 column ids everywhere (pa_tune spmv_format=0), for reference
    prev = pamd._lib.tune("spmv_format", 0)
    kernel_ms_int32 = kernel_time(reps)
    pamd._lib.tune("spmv_format", prev)
    box = box_hbm_gbs(pamd, spmv_bytes // 2) if world == 1 and ngpu == 1 else None
    traffic, traffic_note = (None, "skipped (--no-pmc)")
    if rank == 0 and ngpu == 1 and not args.no_pmc:
        traffic, traffic_note = pmc_traffic(args)

    line = {
        "metric": "SpMV+halo GB/s (frac of HBM peak), 3D Poisson 27-pt, 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": ngpu,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": {"f64": "f64", "f32": "f32", "c128": "c128", "c64": "c64"}[args.dtype],
        "data": "synthetic (seeded uniform x; operator generated on device)",
        "config": {
            "workload": f"mul!(y,A,x) incl. halo, {args.kind}-pt {'FE (test_fem_sa.jl pattern)' if args.kind == 27 else 'FD (test_fdm.jl)'} "
                        f"operator, {args.n}^3 nodes {'in total' if args.strong else 'per GPU'}, Cartesian parts {shape}",
            "global_nodes": list(N),
            "parts": list(shape),
            "nnz_per_part": info["nnz"],
            "rows_per_part": info["nrows"],
            "ghosts_per_part": s_nhids,
            "process_model": "one part per process (RCCL halo)" if world > 1 else f"{ngpu} part(s) in one process",
            "bytes_per_step_all_parts": B_all,
            "frac_of_hbm_peak": round(value / (HBM_PEAK_GBS * ngpu), 4),
            "setup_s": round(t_setup, 2),
            "operator_copies_rotated": ncopies,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None if traffic is None else int(traffic),
            "traffic_note": traffic_note,
            "kernel": "k_spmv_sell (all SpMV kernels of one mul! step: pattern + side slices)",
            "kernel_ms": round(kernel_ms, 4),
            "algorithmic_bytes_per_launch": spmv_bytes,
            "actual_hbm_gbs": None if traffic is None else round(traffic / (kernel_ms * 1e-3) / 1e9, 1),
            "actual_frac": None if traffic is None else round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "bytes_note": ("achieved/frac count SURVEY.md 8d's format-independent CSR bytes (nnz*(S+4) + ...); "
                           "pattern slices read no column ids for their regular rows, so frac can exceed 1. "
                           "actual_frac = PMC traffic / kernel time / peak is the HBM utilisation."),
            "column_format": (f"pattern slices {info['pattern_slices']}/{info['nslices']}, "
                              f"regular rows {info['regular_rows']}/{info['nrows']}, side rows {info['side_rows']}"),
            "int32_columns_kernel_ms": round(kernel_ms_int32, 4),
            "int32_columns_achieved": round(spmv_bytes / (kernel_ms_int32 * 1e-3) / 1e9, 1),
            "box_read_gbs": None if box is None else round(box[0], 1),
            "box_copy_gbs": None if box is None else round(box[1], 1),
            "actual_vs_box_read": (None if box is None or traffic is None
                                   else round(traffic / (kernel_ms * 1e-3) / 1e9 / box[0], 4)),
            "box_note": ("pa_hbm_probe on the same box and run: best read-only / copy rate of 16 B "
                         "non-temporal sweeps over a buffer of about the SpMV's traffic; the attainable "
                         "rate the kernel's PMC-measured rate compares with (boxes differ by up to ~20 %)"),
        },
    }
    if rank == 0 and ngpu == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.kind, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
