"""bench.py — SpMV+halo throughput of mul!(y, A, x) (Interfaces.jl:2246-2275) on
MI355X: the 27-point FE operator (test_fem_sa.jl's pattern in 3D), 256³ nodes
per GPU, weak scaling over Cartesian parts (1 → (1,1,1), 2 → (2,1,1),
4 → (2,2,1), 8 → (2,2,2)).

A step = one mul! (halo exchange of x + SpMV of every owned row) with A and x
resident in HBM.  value = the bytes one mul! of every part must move in the
layout it runs on (matrix values with padding, column ids and slice metadata
as the kernels load them, pa_mat_traffic; x read once, y written once; pack +
unpack of the halo) / time of K steps (max over ranks) → GB/s.  The format-
independent CSR count of SURVEY.md §8d rides along as csr_equivalent_gbs.

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


def csr_bytes(nnz, n_own, n_ghost, n_snd, n_rcv, S, I=4):
    """SURVEY.md §8d (format-independent CSR count): nnz·(S+I) + (n_own+1)·I
    + (n_own+n_ghost)·S + n_own·S + (n_snd+n_rcv)·(I+2S)."""
    return nnz * (S + I) + (n_own + 1) * I + (n_own + n_ghost) * S + n_own * S + (n_snd + n_rcv) * (I + 2 * S)


def format_bytes(info, n_ghost, n_snd, n_rcv, S, I=4):
    """Bytes one mul! of a part must move in the layout it runs on: the
    matrix streams as its kernels load them (pa_mat_traffic: values incl.
    padding, column ids, slice metadata), x read once (owned + ghost), y
    written once, and the halo (pack: lid + value read + buffer write;
    unpack: lid + buffer read + value write per halo value)."""
    n_own = info["nrows"]
    matrix = info["value_bytes"] + info["index_bytes"] + info["meta_bytes"]
    return matrix + (n_own + n_ghost) * S + n_own * S + (n_snd + n_rcv) * (I + 2 * S)


def host_cores():
    """host cores this process may use, capped at the GPU box's share (16)"""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _spmv_ref(*argv, timeout=900):
    exe = os.path.join(ROOT, "oracle", "build", "spmv_ref")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    out = subprocess.run([exe, *map(str, argv)], check=True, capture_output=True, text=True,
                         timeout=timeout).stdout
    return json.loads(out.strip().splitlines()[-1])


def cpu_baseline(kind, n, seconds=12.0):
    """oracle/build/spmv_ref: the reference's CSC column loop
    (SparseUtils.jl:157-187) restated in C ("port"), run as MPIBackend would
    run it on this host: one rank per core (--ranks), each with the CSC of
    its block of rows of the SAME operator as the GPU line (n^3 nodes), a
    barrier per SpMV.  Reported in the GPU line's CSR-equivalent GB/s
    (SURVEY.md §8d bytes) and ms per SpMV; a 1-rank run on 128^3 rides along."""
    cores = host_cores()
    r = _spmv_ref("--kind", kind, "--n", n, "--seconds", seconds, "--ranks", cores)
    r1 = _spmv_ref("--kind", kind, "--n", 128, "--seconds", 3.0, "--ranks", 1)
    return {"value": round(r["gbps"], 3), "unit": "GB/s (SURVEY.md 8d CSR bytes, like csr_equivalent_gbs)",
            "ms_per_spmv": round(1e3 * r["sec_per_spmv"], 3), "cores": cores, "kind": "port",
            "sample": f"the benched operator ({kind}-pt, {n}^3 nodes, {r['nnz']} nnz), {r['reps']} SpMVs in "
                      f"~{seconds:.0f} s, Int64 CSC column loop (SparseUtils.jl:157-187) in C, {cores} "
                      f"MPIBackend-like ranks (threads, row blocks of PRange(parts, n), barrier per SpMV)",
            "single_core_gbps_128": round(r1["gbps"], 3)}


def cpu_baseline_mpi(kind, dims, shape, seconds=12.0):
    """oracle/build/spmv_ref --mpi: MPIBackend over the SAME Cartesian parts
    as the GPU line (global nodes `dims`, parts `shape`), one rank per part
    on one host core each (mpiexec -n P with one core per rank, SURVEY.md
    §8d), each rank with its local CSC (owned rows over owned then ghost
    columns, Int64), its Exchanger and, in every mul!, the halo exchange of
    x (pack, delivery, unpack) between the owned and the ghost column loops
    (Interfaces.jl:2246-2275, MPIBackend.jl:261-309).  GB/s of SURVEY.md §8d
    CSR bytes summed over the ranks (halo pack/unpack included)."""
    P = int(np.prod(shape))
    r = _spmv_ref("--kind", kind, "--dims", *dims, "--parts", *shape, "--mpi", "--seconds", seconds)
    return {"value": round(r["gbps"], 3), "unit": "GB/s (SURVEY.md 8d CSR bytes incl. halo, all ranks)",
            "ms_per_spmv": round(1e3 * r["sec_per_spmv"], 3), "cores": P, "kind": "port",
            "ranks": P, "halo_values_per_spmv": r["halo_values"],
            "sample": (f"the benched operator ({kind}-pt, {dims[0]}x{dims[1]}x{dims[2]} nodes, {r['nnz']} nnz) on "
                       f"Cartesian parts {tuple(shape)}, {r['reps']} mul! in ~{seconds:.0f} s: {P} MPIBackend-like "
                       f"ranks (one thread each), Int64 CSC column loop (SparseUtils.jl:157-187) over the owned "
                       f"then the ghost columns, halo exchange of x (pack, delivery, unpack) in every mul!, "
                       f"barrier per mul!; build {r['build_s']:.1f} s untimed")}


PROBE_BYTES = 1 << 30


def rccl_run_info(infos, world):
    """The N > 1 line's proof of what ran, from every
    rank's PartContext.comm_info(): the communicator's rank count
    (ncclCommCount, min/max over the ranks: world on every rank), the
    distinct devices (PCI bus ids) the ranks ran on, and the librccl each
    rank resolved.  Fewer distinct devices than ranks is an error, not a
    line."""
    counts = [i["ranks"] for i in infos]
    devices = sorted({i["pci"] for i in infos})
    if len(devices) < world or min(counts) != world or max(counts) != world:
        raise SystemExit(f"{world} ranks: communicator sizes {counts}, distinct devices {devices}")
    return {"rccl_ranks": {"min": min(counts), "max": max(counts)}, "devices": devices,
            "distinct_devices": len(devices), "librccl": sorted({i["librccl"] for i in infos}),
            "rccl_version": sorted({i["rccl_version"] for i in infos})}


# the kernels of one mul! step (SpMV slices, halo pull / pack / unpack)
PMC_KERNELS = ("k_spmv_sell", "k_spmv_group", "k_spmv_merged", "k_pull_", "k_pack", "k_unpack")


def pmc_traffic(args, steps=5, halo=False):
    """HBM bytes per mul! step from rocprofv3 PMC counters, one counter per
    pass (MI355X_MICROARCH.md §HBM / §rocprofv3): FETCH_SIZE (KB) and
    WRITE_SIZE (KB) summed over the kernels of the profiled steps (SpMV
    slices, and with halo=True the halo leg's pulls) / steps.  FETCH_SIZE
    under-counts wide coalesced streaming reads on gfx950
    (MI355X_MICROARCH.md: by 1/2); the factor is calibrated in the same
    profiled process on k_probe_read launches that read a known 1 GiB with
    the SpMV's own 16 B-per-lane non-temporal loads, and applied to the
    SpMV's fetches (its loads are 16 B per lane: values, pattern rows' x
    runs; the side rows' 4-8 B gathers are split out in the note).  Runs
    this script as the profiled child (`--child-pmc`, `--child-halo` for
    the halo leg's (2,2,2) operator)."""
    import csv
    import shutil
    import signal
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not found"
    tot = {}
    # FETCH_SIZE and WRITE_SIZE (one pass each), then the UTCL1 translation
    # counters of the same kernels (address translation beside the bytes:
    # a placement-dependent rate shows here if it is the TLB)
    passes = [("FETCH_SIZE",), ("WRITE_SIZE",),
              ("TCP_UTCL1_REQUEST_sum", "TCP_UTCL1_TRANSLATION_MISS_sum", "TCP_UTCL1_TRANSLATION_HIT_sum")]
    for ctrs in passes:
        ctr = ctrs[0]
        d = tempfile.mkdtemp(prefix="pa_pmc_", dir="/tmp")
        cmd = ["rocprofv3", "--pmc", *ctrs, "-d", d, "-o", "pmc", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--child-pmc", "--steps", str(steps),
               "--n", str(args.n), "--kind", str(args.kind), "--dtype", args.dtype, "--tune", args.tune] + \
            (["--child-halo"] if halo else [])
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True,
                             env=dict(os.environ, TMPDIR="/tmp"))
        try:
            p.wait(timeout=240)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            if ctr.startswith("TCP_"):
                break  # the translation pass is extra: keep the byte counts
            return None, f"rocprofv3 --pmc {ctr} timed out"
        files = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
        if p.returncode != 0 or not files:
            if ctr.startswith("TCP_"):
                break
            return None, f"rocprofv3 --pmc {ctr} failed (rc {p.returncode})"
        rows = list(csv.DictReader(open(files[0])))
        for c in ctrs:
            vals = [float(r["Counter_Value"]) for r in rows
                    if any(k in r["Kernel_Name"] for k in PMC_KERNELS) and r["Counter_Name"] == c]
            tot[c] = sum(vals) / (steps + 1)  # warmup step + steps
        if ctr == "FETCH_SIZE":
            probe = [float(r["Counter_Value"]) for r in rows
                     if "k_probe_read" in r["Kernel_Name"] and r["Counter_Name"] == ctr]
            tot["probe_kb"] = float(np.median(probe)) if probe else None
        shutil.rmtree(d, ignore_errors=True)
    factor = PROBE_BYTES / (tot["probe_kb"] * 1024) if tot.get("probe_kb") else 2.0
    traffic = tot["FETCH_SIZE"] * 1024 * factor + tot["WRITE_SIZE"] * 1024
    tlb = None
    if tot.get("TCP_UTCL1_REQUEST_sum"):
        tlb = {"utcl1_requests": round(tot["TCP_UTCL1_REQUEST_sum"]),
               "utcl1_misses": round(tot["TCP_UTCL1_TRANSLATION_MISS_sum"]),
               "utcl1_hits": round(tot["TCP_UTCL1_TRANSLATION_HIT_sum"]),
               "utcl1_miss_rate": round(tot["TCP_UTCL1_TRANSLATION_MISS_sum"] / tot["TCP_UTCL1_REQUEST_sum"], 5)}
    return traffic, {"fetch_kb": round(tot["FETCH_SIZE"]), "write_kb": round(tot["WRITE_SIZE"]),
                     "fetch_factor": round(factor, 4), "translation_per_step": tlb,
                     "note": (f"rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE passes over {steps + 1} mul! steps; "
                              f"FETCH_SIZE x {factor:.3f}, the factor measured on k_probe_read launches "
                              f"reading a known 1 GiB with 16 B/lane loads in the same process, + WRITE_SIZE")}


def box_hbm_gbs(pamd, nbytes, reps=10):
    """Attainable HBM rates of this box (pa_hbm_probe: 16 B non-temporal
    read-only and copy sweeps of an `nbytes` buffer, best of three grid
    sizes).  A calibration beside the roofline, not the metric."""
    try:
        return pamd._lib.hbm_probe(0, nbytes, reps)
    except pamd._lib.PAError:
        return None


def child_pmc(args):
    """the profiled child of pmc_traffic: build the operator (the headline's
    one part, or with --child-halo the halo leg's (2,2,2) parts of the same
    global operator on the one GPU), run warmup+steps."""
    import pamd
    be = pamd.HIPBackend(devices=[0])
    parts = be.get_part_ids((2, 2, 2) if args.child_halo else (1, 1, 1))
    dtype = DTYPES[args.dtype]
    A = pamd.drivers.stencil_operator(parts, (args.n,) * 3, args.kind, dtype)
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(20250114 + s.part).uniform(-1, 1, s.num_lids).astype(dtype),
        A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows, dtype)
    for _ in range(args.steps + 1):
        pamd.mul_(y, A, x)
    for p in parts.part_ids:
        be.context(p).sync()
    # FETCH_SIZE calibration: read sweeps of a known PROBE_BYTES
    pamd._lib.hbm_probe(0, PROBE_BYTES, 1)


def child_oneproc(args):
    """The one-process-drives-every-GPU leg (SequentialBackend's role, the
    model of julia/HIPBackend.jl): the same weak-scaling
    problem as the N-rank line, its N parts held by ONE process, part p on
    device p-1 with its own stream pair, issued per part from host threads
    behind one pack barrier per call.  Run as a child of rank 0 after the
    rank line is measured (a failure here cannot touch that line).  Prints
    one JSON object: device time per mul!, host issue per mul! (C-ABI, the
    calls enqueued back to back), and a bit-for-bit check of y against the
    per-neighbour-wait issue (halo_barrier 0)."""
    import pamd
    devs = ([int(d) for d in args.oneproc_devices.split(",")] if args.oneproc_devices
            else list(range(args.gpus)))
    ngpu = len(devs)
    shape = PART_SHAPES[ngpu]
    N = tuple(args.n * s for s in shape)
    dtype = DTYPES[args.dtype]
    S = np.dtype(dtype).itemsize
    be = pamd.HIPBackend(devices=devs, share_streams=False)
    parts = be.get_part_ids(shape)
    t0 = time.perf_counter()
    A = pamd.drivers.stencil_operator(parts, N, args.kind, dtype)
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(20250114 + s.part).uniform(-1, 1, s.num_lids).astype(dtype),
        A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows, dtype)
    ctxs = [be.context(p) for p in parts.part_ids]

    def sync():
        for c in ctxs:
            c.sync()
    sync()
    setup = time.perf_counter() - t0
    B = 0
    for p in parts.part_ids:
        s_ = A.cols.partition.local(p)
        B += format_bytes(A.values.local(p).info(), s_.num_hids, len(A.cols.exchanger.lids_snd.local(p).data),
                          len(A.cols.exchanger.lids_rcv.local(p).data), S)
    for _ in range(args.warmup):
        pamd.mul_(y, A, x)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pamd.mul_(y, A, x)
    sync()
    wall = (time.perf_counter() - t0) / args.steps
    cargs = pamd.pvector._spmv_args(y, A, x, 1.0, 0.0)
    host = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pamd._lib.call("pa_spmv_all", *cargs)
        host.append((time.perf_counter() - t0) / args.steps)
        sync()
    host.sort()
    got = [v.copy() for v in y.to_host().parts]
    prev = pamd._lib.tune("halo_barrier", 0)
    try:
        y0 = pamd.PVector.undef(A.rows, dtype)
        pamd.mul_(y0, A, x)
        ref = y0.to_host().parts
    finally:
        pamd._lib.tune("halo_barrier", prev)
    own = [A.rows.partition.local(p).oid_to_lid - 1 for p in parts.part_ids]
    same = all(np.array_equal(a[o], b[o]) for a, b, o in zip(got, ref, own))
    print(json.dumps({
        "process_model": f"{ngpu} parts in one process, part p on device {devs} [p-1], a stream pair each "
                         "(HIPBackend(share_streams=False): SequentialBackend's role, julia/HIPBackend.jl)",
        "devices": devs, "parts": list(shape), "global_nodes": list(N),
        "ms_per_step": round(1e3 * wall, 4), "value": round(B / wall / 1e9, 2), "unit": "GB/s",
        "bytes_per_step_all_parts": int(B), "frac_of_hbm_peak": round(B / wall / 1e9 / (HBM_PEAK_GBS * ngpu), 4),
        "host_issue_us_per_mul": round(1e6 * host[len(host) // 2], 1),
        "host_issue_us_min_max": [round(1e6 * host[0], 1), round(1e6 * host[-1], 1)],
        "y_equals_neighbour_wait_issue": bool(same), "setup_s": round(setup, 2)}), flush=True)
    return 0


def one_process_leg(args):
    """rank 0 of an N-rank run: child_oneproc as a child process (bounded)."""
    cmd = [sys.executable, os.path.abspath(__file__), "--child-oneproc", "--gpus", str(args.gpus), "--n",
           str(args.n), "--kind", str(args.kind), "--dtype", args.dtype, "--steps", str(args.steps), "--warmup",
           str(args.warmup), "--tune", args.tune]
    if args.oneproc_devices:
        cmd += ["--oneproc-devices", args.oneproc_devices]
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
              "TORCHELASTIC_RUN_ID", "MASTER_PORT"):
        env.pop(k, None)
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=420)
    except subprocess.TimeoutExpired:
        return {"note": "one-process leg timed out (420 s)"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"note": f"one-process leg failed (rc {r.returncode})", "stderr_tail": r.stderr[-600:]}
    return json.loads(lines[-1])


def halo_1gpu(args, pamd, dtype, S, reps_phase=20, copies=3):
    """BASELINE config 3 on the one GPU: the SAME global operator as the
    headline (args.n^3 nodes, args.kind points) split into Cartesian parts
    (2,2,2), all eight parts on cuda:0 (HIPBackend, one stream pair).  Every
    mul! exchanges the halo of x between the parts (Interfaces.jl:2258-2272:
    async_exchange!(b) before the owned block, the ghost block after it) and
    is timed exactly like the headline: W untimed calls, then K calls
    bracketed by synchronisation, wall clock / K; the HIP-event span on the
    compute stream gives the kernel time.  Bytes: format_bytes summed over
    the parts (matrix as loaded, x read once incl. ghosts, y written once,
    halo pack + unpack (4+2S) per value on both sides).

    The rate of this shape depends on where a copy's pages land (DESIGN.md
    §4.1: identical copies differ by up to 15 %), so `copies` operators are
    built independently (all alive at once, each with its own x and y) and
    timed one after the other: ms_per_step and frac are the median copy's,
    min / max beside them."""
    be = pamd.HIPBackend(devices=[0])
    shape = (2, 2, 2)
    parts = be.get_part_ids(shape)
    N = (args.n,) * 3
    t_setup = time.perf_counter()
    partition = pamd.drivers.stencil_partition(parts, N, args.kind)
    sets = []
    for k in range(copies):
        A = pamd.drivers.stencil_operator(parts, N, args.kind, dtype, partition=partition)
        x = pamd.PVector.from_host(pamd.map_parts(
            lambda s: np.random.default_rng(20250114 + s.part).uniform(-1, 1, s.num_lids).astype(dtype),
            A.cols.partition), A.cols)
        sets.append((A, x, pamd.PVector.undef(A.rows, dtype)))
    ctxs = [be.context(p) for p in parts.part_ids]

    def sync():
        for c in ctxs:
            c.sync()
    sync()
    t_setup = (time.perf_counter() - t_setup) / copies
    A = sets[0][0]
    ex = A.cols.exchanger
    B = Cb = 0
    ghosts = halo_vals = 0
    for p in parts.part_ids:
        info = A.values.local(p).info()
        s = A.cols.partition.local(p)
        ns, nr = len(ex.lids_snd.local(p).data), len(ex.lids_rcv.local(p).data)
        B += format_bytes(info, s.num_hids, ns, nr, S)
        Cb += csr_bytes(info["nnz"], info["nrows"], s.num_hids, ns, nr, S)
        ghosts += s.num_hids
        halo_vals += nr
    c0 = ctxs[0]
    per_copy = []
    for A, x, y in sets:
        for _ in range(args.warmup):
            pamd.mul_(y, A, x)
        sync()
        t0 = time.perf_counter()
        c0.span_start()
        for _ in range(args.steps):
            pamd.mul_(y, A, x)
        c0.span_stop()
        sync()
        per_copy.append(((time.perf_counter() - t0) / args.steps, c0.span_ms() / args.steps))
    order = sorted(range(copies), key=lambda k: per_copy[k][0])
    med = order[copies // 2]
    el, span = per_copy[med]
    A, x, y = sets[med]
    # per-phase attribution on the median copy (untimed calls; grouped launches report on part 1)
    for c in ctxs:
        c.set_timing(True)
    for _ in range(reps_phase):
        pamd.mul_(y, A, x)
    sync()
    ph = c0.kernel_times()
    for c in ctxs:
        c.set_timing(False)
    # host-issue time of one mul! (the enqueue alone, the GPU kept busy)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pamd.mul_(y, A, x)
    host_us = 1e6 * (time.perf_counter() - t0) / args.steps
    sync()
    out = {
        "workload": (f"mul!(y,A,x), {args.kind}-pt operator, {args.n}^3 nodes in total (BASELINE config 3), "
                     f"Cartesian parts {shape}, all 8 parts on cuda:0; halo exchange of x between the parts "
                     "in every step (direct pull of the ghosts from their owners' x, then the SpMV)"),
        "parts": list(shape),
        "copies": copies,
        "ms_per_step": round(1e3 * el, 4),
        "ms_per_step_min": round(1e3 * per_copy[order[0]][0], 4),
        "ms_per_step_max": round(1e3 * per_copy[order[-1]][0], 4),
        "ms_per_step_copies": [round(1e3 * t, 4) for t, _ in per_copy],
        "copies_note": (f"{copies} operator copies built independently (all alive, own x and y), K steps each "
                        "in build order; ms_per_step, value, frac and kernel_ms are the median copy's"),
        "value": round(B / el / 1e9, 2),
        "unit": "GB/s",
        "frac": round(B / el / 1e9 / HBM_PEAK_GBS, 4),
        "bytes_per_step": int(B),
        "csr_equivalent_gbs": round(Cb / el / 1e9, 2),
        "ghosts_all_parts": int(ghosts),
        "halo_values_per_step": int(halo_vals),
        "kernel_ms": round(span, 4),
        "kernel_ms_copies": [round(sp, 4) for _, sp in per_copy],
        "kernel_frac": round(B / (span * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "kernel_ms_note": "HIP events on the parts' shared compute stream around the K timed steps, / K",
        "per_part_ms": {"interior_ms": round(ph["interior_ms"], 4), "halo_wait_ms": round(ph["halo_wait_ms"], 4),
                        "boundary_ms": round(ph["boundary_ms"], 4), "calls": ph["calls"],
                        "note": ("all 8 parts in each phase (grouped launches, one stream): halo_wait_ms is "
                                 "the direct pull of every ghost from its owner's x; no slice runs before it "
                                 "(interior_ms 0); boundary_ms is every slice in one merged launch")},
        "host_issue_us_per_mul": round(host_us, 1),
        "setup_s": round(t_setup, 2),
    }
    del sets, A, x, y
    return out


def cg_mode(args, pamd, backend, parts, A, ngpu, use_dist, sync):
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
    steady = {}
    variants = {"device_sweep_u": dict(device=True, batch=16), "device_fused_u": dict(device=True, batch=16),
                "fused": dict(fused=True), "unfused": dict(fused=False)}

    def timed(kw, k):
        x = pamd.PVector.undef(cols, dtype).fill_(0)
        sync()
        if use_dist:
            dist.barrier()
        t0 = time.perf_counter()
        hist = []
        pamd.cg_(x, A, b, reltol=0.0, maxiter=k, history=hist, **kw)
        sync()
        el = time.perf_counter() - t0
        if use_dist:
            t = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, hist

    ctxs = [backend.context(p) for p in parts.part_ids]
    for name, kw in variants.items():
        # the device recurrence with u .= r .+ β.*u as its own sweep
        # (cg_fuse 0) or inside the SpMV (cg_fuse 1), set on this run's
        # contexts (pa_ctx_tune; the process default is 2, auto)
        for c in ctxs:
            c.tune("cg_fuse", 1 if name == "device_fused_u" else 0)
        x = pamd.PVector.undef(cols, dtype).fill_(0)
        pamd.cg_(x, A, b, reltol=0.0, maxiter=args.warmup, **kw)
        sync()
        el, hist = timed(kw, args.cg)
        out[name] = (1e3 * el / max(1, len(hist)), len(hist), hist[-1] if hist else None)
        if kw.get("device"):
            # steady state: a cg! of 3K iterations minus one of K (the same
            # setup: cg_iterator!'s SpMV, norms and host syncs) over 2K
            el3, hist3 = timed(kw, 3 * args.cg)
            steady[name] = 1e3 * (el3 - el) / max(1, len(hist3) - len(hist))
        for c in ctxs:
            c.tune("cg_fuse", None)
    best = min(steady, key=steady.get)
    p0 = parts.part_ids[0]
    # the auto mode (cg_fuse 2, the process default): one timed batch of each
    # u update, the times reduced with max over the ranks (RCCL) before the
    # choice, so one part per process chooses too, the same on every rank
    x = pamd.PVector.undef(cols, dtype).fill_(0)
    pamd.cg_(x, A, b, reltol=0.0, maxiter=max(3 * 16, args.cg), device=True, batch=16)
    sync()
    choice = A.values.local(p0).cg_choice()
    auto = {1: "device_fused_u", 0: "device_sweep_u"}.get(choice)
    info = A.values.local(p0).info()
    S = np.dtype(dtype).itemsize
    n = info["nrows"]
    s0 = cols.partition.local(p0)
    ns, nr = len(cols.exchanger.lids_snd.local(p0).data), len(cols.exchanger.lids_rcv.local(p0).data)
    # per iteration of the device recurrence (u update inside the SpMV): mul!
    # (format bytes: matrix, one x read, c written, halo) + the second gathered
    # vector (r and u_old both read) + u_new written + x read+written
    # (deferred x .+= α.*u) + k_cg_xr (r read+written, c read)
    # (the sweep variant: k_cg_xu reads u, x, r and writes u, x: 8 vectors)
    it_bytes = format_bytes(info, s0.num_hids, ns, nr, S) + (8 if best == "device_sweep_u" else 7) * s0.num_lids * S
    rows_all = n * ngpu
    line = {"metric": "CG iteration time (weak scaling, BASELINE config 4)",
            "value": round(steady[best], 4), "unit": "ms/iteration", "higher_is_better": False,
            "n_gpus": ngpu, "iterations": out[best][1], "scaling": "weak",
            "dtype": args.dtype, "data": "synthetic (seeded uniform b, x0 = 0)",
            "config": {"workload": f"cg! on the {args.kind}-pt operator, {args.n}^3 nodes per GPU",
                       "dofs": rows_all, "recurrence": "scalars on the device (pa_cg_solve_all, batch 16)",
                       "value_is": (f"steady-state ms per iteration of the device recurrence ({best}): "
                                    f"(time of cg! with {3 * args.cg} iterations - time with {args.cg}) / "
                                    f"{2 * args.cg}; whole-call times per iteration below include the setup"),
                       "steady_ms_per_iteration": {k: round(v, 4) for k, v in steady.items()},
                       "device_sweep_u_ms_per_iteration_whole_call": round(out["device_sweep_u"][0], 4),
                       "device_fused_u_ms_per_iteration_whole_call": round(out["device_fused_u"][0], 4),
                       "host_driven_fused_ms_per_iteration": round(out["fused"][0], 4),
                       "host_driven_unfused_ms_per_iteration": round(out["unfused"][0], 4),
                       "algorithmic_bytes_per_iteration_per_gpu": it_bytes,
                       "gbs_per_gpu_device": round(it_bytes / (steady[best] * 1e-3) / 1e9, 1),
                       "final_residual": out[best][2],
                       "same_history_as_host_driven": out["device_sweep_u"][2] == out["fused"][2],
                       "same_history_fused_u_as_sweep_u": out["device_fused_u"][2] == out["device_sweep_u"][2],
                       "auto_choice": auto,
                       "auto_choice_note": ("pa_cg_solve_all with cg_fuse 2 (default): the variant its two timed "
                                            "batches chose (times max-reduced over the ranks), as remembered on "
                                            "the matrix")}}
    return line


def launch_ranks(n):
    """Run this script under torch.distributed.run with n ranks (one part and
    one GPU per rank, HIPDistributedBackend) as a child process; rank 0
    prints the JSON line to the inherited stdout."""
    import socket
    with socket.socket() as s:  # a free rendezvous port on the loopback
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


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
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 HBM-traffic passes")
    ap.add_argument("--no-halo-leg", action="store_true",
                    help="skip the halo_1gpu object (config 3 on (2,2,2) parts of the one GPU)")
    ap.add_argument("--child-pmc", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--child-halo", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--child-oneproc", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--oneproc-devices", default="",
                    help="devices of the one-process leg's parts (default 0..N-1; e.g. 0,0 rehearses it on one GPU)")
    ap.add_argument("--no-oneproc", action="store_true",
                    help="skip the one-process leg of N > 1 runs (all N parts driven by one process)")
    ap.add_argument("--cg", type=int, default=0, help="time K CG iterations instead (own JSON line)")
    ap.add_argument("--tune", default="", help="process-default knobs before anything is built (A/B runs): "
                                                 "key=v[,key=v]")
    ap.add_argument("--distributed", action="store_true",
                    help="one part per process (HIPDistributedBackend, RCCL) even for one process: "
                         "rehearses the torchrun path of --gpus N > 1 on a single GPU")
    args = ap.parse_args()
    if args.child_pmc or args.child_oneproc:
        import pamd
        for kv in filter(None, args.tune.split(",")):
            k, v = kv.split("=")
            pamd._lib.tune(k, int(v))
        return child_oneproc(args) if args.child_oneproc else child_pmc(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` (no torchrun around it): start the N
        # one-part-per-GPU ranks ourselves, as the driver's torchrun command
        # does, before this process touches the GPU (no HIP call, no torch
        # import above this line), and pass their exit status on.  One
        # process per GPU keeps every rank's host issue to its own part.
        return launch_ranks(args.gpus)
    # stdout carries exactly one JSON line (rank 0): native libraries print
    # banners to fd 1 during init (RCCL's version block, gloo's connection
    # line), so fd 1 points at stderr until the line is written
    out_fd = os.dup(1)
    os.dup2(2, 1)

    def emit(line):
        os.write(out_fd, (json.dumps(line) + "\n").encode())

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import torch
    import torch.distributed as dist
    import pamd
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        pamd._lib.tune(k, int(v))

    use_dist = world > 1 or args.distributed
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
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

    # bytes of the local parts: in the layout they run on, and SURVEY.md §8d's CSR count
    ex = cols.exchanger
    B_local = C_local = 0
    infos = {}
    for p in parts.part_ids:
        info = A.values.local(p).info()
        s = cols.partition.local(p)
        n_snd = len(ex.lids_snd.local(p).data)
        n_rcv = len(ex.lids_rcv.local(p).data)
        infos[p] = (info, s.num_hids, n_snd, n_rcv)
        B_local += format_bytes(info, s.num_hids, n_snd, n_rcv, S)
        C_local += csr_bytes(info["nnz"], info["nrows"], s.num_hids, n_snd, n_rcv, S)
    B_all, C_all = B_local, C_local
    if use_dist:
        t = torch.tensor([float(B_local), float(C_local)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        B_all, C_all = float(t[0].item()), float(t[1].item())

    def barrier():
        if use_dist:
            dist.barrier()

    if args.cg > 0:
        line = cg_mode(args, pamd, backend, parts, A, ngpu, use_dist, sync)
        if rank == 0:
            emit(line)
        if use_dist:
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
    c0 = ctxs[0]
    comm0 = [c.comm_stats() for c in ctxs] if use_dist else None
    t0 = time.perf_counter()
    c0.span_start()  # HIP events on part 1's compute stream, over the timed region
    for i in range(args.steps):
        Ai, xi, yi = sets[i % ncopies]
        pamd.mul_(yi, Ai, xi)
    c0.span_stop()
    sync()
    t1 = time.perf_counter()
    barrier()
    span_ms = c0.span_ms() / args.steps
    elapsed = t1 - t0
    if use_dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = B_all / (elapsed / args.steps) / 1e9
    rccl = None
    if use_dist:
        # bytes this process posted to RCCL (ncclSend / ncclRecv of the halo
        # segments) over the timed steps, summed over the ranks: the xGMI
        # bytes of SURVEY.md §8d (n_rcv·S per GPU), reported beside `value`
        sent = sum(c.comm_stats()[0] - a[0] for c, a in zip(ctxs, comm0))
        recv = sum(c.comm_stats()[1] - a[1] for c, a in zip(ctxs, comm0))
        t = torch.tensor([float(sent), float(recv)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        rccl = {"bytes_sent_per_step_all_ranks": int(t[0].item()) // args.steps,
                "bytes_recv_per_step_all_ranks": int(t[1].item()) // args.steps,
                "gbs_all_ranks": round(float(t[1].item()) / elapsed / 1e9, 2)}
        # what the communicator ran on: ncclCommCount per
        # rank, the distinct devices of the ranks (PCI bus ids; the backend
        # already refused a run with fewer distinct devices than ranks) and
        # the librccl each rank resolved
        cinfos = [None] * world
        dist.all_gather_object(cinfos, ctxs[0].comm_info())
        rccl.update(rccl_run_info(cinfos, world))

    # attribution (untimed calls): every local part's mul! phases, HIP events
    # on the stream the kernels run on, read after the last call (no
    # synchronisation per call): interior slices, halo completion after them
    # (transport wait + unpack), boundary slices (parts grouped on one stream
    # pair report on their first part)
    reps = max(5, min(args.steps, 50))

    def phase_times():
        for c in ctxs:
            c.set_timing(True)
        for i in range(reps):
            Ai, xi, yi = sets[i % ncopies]
            pamd.mul_(yi, Ai, xi)
        sync()
        return {p: c.kernel_times() for p, c in zip(parts.part_ids, ctxs)}
    phases = phase_times()
    per_part = {p: {k: round(v, 4) if isinstance(v, float) else v for k, v in t.items()} for p, t in phases.items()}
    if use_dist:
        allp = [None] * world
        dist.all_gather_object(allp, per_part)
        per_part = {k: v for d in allp for k, v in d.items()}
    p0 = parts.part_ids[0]
    info, s_nhids, n_snd0, n_rcv0 = infos[p0]
    # the dominant kernels' device time per step: the HIP-event span of the
    # timed region on part 1's compute stream / K; with several parts on one
    # stream pair (grouped launches) the span covers all of them
    grouped_here = (len(ctxs) > 1 and len({c.device for c in ctxs}) == 1
                    and getattr(backend, "share_streams", False))
    kernel_ms = span_ms
    spmv_bytes = B_local if grouped_here else format_bytes(info, s_nhids, n_snd0, n_rcv0, S)
    achieved = spmv_bytes / (kernel_ms * 1e-3) / 1e9
    # the same kernels with int32 column ids everywhere (spmv_format=0 on
    # this run's contexts), for reference
    for c in ctxs:
        c.tune("spmv_format", 0)
    sync()
    c0.span_start()
    for i in range(reps):
        Ai, xi, yi = sets[i % ncopies]
        pamd.mul_(yi, Ai, xi)
    c0.span_stop()
    kernel_ms_int32 = c0.span_ms() / reps
    bytes_int32 = 0
    for p in (parts.part_ids if grouped_here else [p0]):
        inf, nh, ns_, nr_ = infos[p]
        bytes_int32 += format_bytes(dict(inf, **A.values.local(p).traffic()), nh, ns_, nr_, S)
    for c in ctxs:
        c.tune("spmv_format", None)
    # the probe reads as many bytes per launch as the timed loop cycles
    # through (ncopies operator copies when one would fit the 256 MB
    # Infinity Cache), so that neither side is served from it
    box = box_hbm_gbs(pamd, spmv_bytes * ncopies) if world == 1 and ngpu == 1 else None
    # ... and one launch of the operator's own size, rotating over 2 GiB (a
    # short SpMV pays one launch's ramp-up and drain per step; C2's 149 MB)
    box_launch = None
    if box is not None:
        try:
            box_launch = pamd._lib.hbm_probe_launch(0, int(spmv_bytes), max(2 << 30, 8 * int(spmv_bytes)), 40)
        except pamd._lib.PAError:
            box_launch = None
    halo_leg = None
    if world == 1 and ngpu == 1 and not args.strong and not args.no_halo_leg:
        halo_leg = halo_1gpu(args, pamd, dtype, S)
    traffic, tnote = (None, {"note": "skipped (--no-pmc)"})
    if rank == 0 and ngpu == 1 and not args.no_pmc:
        traffic, tnote = pmc_traffic(args)
        if traffic is None:
            tnote = {"note": tnote}
        if halo_leg is not None:
            # the halo leg's HBM bytes from the same counters (all 8 parts'
            # SpMV and pull kernels of a step), beside its format bytes
            ht, hnote = pmc_traffic(args, halo=True)
            hr = halo_leg["roofline"] = {"bound": "hbm", "achieved": halo_leg["value"], "peak": HBM_PEAK_GBS,
                                         "unit": "GB/s", "frac": halo_leg["frac"],
                                         "traffic": None if ht is None else int(ht),
                                         "traffic_detail": hnote if ht is not None else {"note": hnote}}
            if ht is not None:
                k_s = halo_leg["kernel_ms"] * 1e-3
                hr["actual_hbm_gbs"] = round(ht / k_s / 1e9, 1)
                hr["actual_frac"] = round(ht / k_s / 1e9 / HBM_PEAK_GBS, 4)
                hr["traffic_over_bytes"] = round(ht / halo_leg["bytes_per_step"], 4)
                hr["note"] = ("format bytes count x once per part: with the parts' x and y (2 x 134 MB) "
                              "partly held in the 256 MB MALL across steps, HBM traffic can sit below them; "
                              "actual_frac is the counter-based fraction")
                if box is not None and hr["actual_hbm_gbs"] > box[0]:
                    # a counter rate above the box's read
                    # probe is not HBM: FETCH_SIZE (and TCC_EA0_RDREQ_DRAM, which
                    # equals TCC_EA0_RDREQ on gfx950, profiles/r06/f/) counts
                    # Infinity-Cache hits, and no counter separates them
                    hr["actual_exceeds_box_read"] = True
                    hr["actual_frac_hbm_bound"] = round(box[0] / HBM_PEAK_GBS, 4)
                    hr["actual_note"] = ("the counter rate exceeds this box's read probe: it includes Infinity-Cache "
                                         "hits (TCC_EA0_RDREQ_DRAM == TCC_EA0_RDREQ on gfx950), so HBM reads are at "
                                         "most the probe's rate, actual_frac_hbm_bound")
    halo = s_nhids > 0
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
            "workload": (f"mul!(y,A,x), {args.kind}-pt {'FE (test_fem_sa.jl pattern)' if args.kind == 27 else 'FD (test_fdm.jl)'} "
                         f"operator, {args.n}^3 nodes {'in total' if args.strong else 'per GPU'}, Cartesian parts {shape}"
                         + (", halo exchange of x between parts" if halo else ", one part: no halo to exchange")),
            "global_nodes": list(N),
            "parts": list(shape),
            "nnz_per_part": info["nnz"],
            "rows_per_part": info["nrows"],
            "ghosts_per_part": s_nhids,
            "process_model": "one part per process (RCCL halo)" if use_dist else f"{ngpu} part(s) in one process",
            "bytes_per_step_all_parts": int(B_all),
            "bytes_definition": ("per part: matrix streams as loaded (values incl. padding, column ids, slice "
                                 "metadata; pa_mat_traffic) + x read once (owned+ghost) + y written once "
                                 "+ halo pack/unpack (4+2S per value each side)"),
            "frac_of_hbm_peak": round(value / (HBM_PEAK_GBS * ngpu), 4),
            "csr_equivalent_gbs": round(C_all / (elapsed / args.steps) / 1e9, 2),
            "csr_bytes_per_step_all_parts": int(C_all),
            "setup_s": round(t_setup, 2),
            "operator_copies_rotated": ncopies,
            "per_part_ms": per_part,
            "rccl_halo": rccl,
            "tune": args.tune or None,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None if traffic is None else int(traffic),
            "traffic_detail": tnote,
            "kernel": ("k_spmv_sell_group (one part: the pattern slices with the side rows as trailing waves, "
                       "XCD runs; rows <= 7 entries in Float64: k_spmv_group_short7) / k_spmv_merged (parts "
                       "sharing a GPU): all SpMV kernels of one mul! step"
                       + (", halo pack/pull" if halo else "") + ""),
            "kernel_ms": round(kernel_ms, 4),
            "kernel_ms_note": ("HIP events on part %d's compute stream around the K timed steps, / K" % p0
                               + ("; all parts of this process (grouped launches)" if grouped_here else "")),
            "algorithmic_bytes_per_launch": int(spmv_bytes),
            "bytes_split": {"values": info["value_bytes"], "column_ids": info["index_bytes"],
                            "slice_metadata": info["meta_bytes"],
                            "x_y": int((info["nrows"] + s_nhids) * S + info["nrows"] * S)},
            "csr_equivalent_achieved": round((C_local if grouped_here else
                                              csr_bytes(info["nnz"], info["nrows"], s_nhids, n_snd0, n_rcv0, S))
                                             / (kernel_ms * 1e-3) / 1e9, 1),
            "actual_hbm_gbs": None if traffic is None else round(traffic / (kernel_ms * 1e-3) / 1e9, 1),
            "actual_frac": None if traffic is None else round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic_over_bytes": None if traffic is None else round(traffic / spmv_bytes, 4),
            "column_format": (f"pattern slices {info['pattern_slices']}/{info['nslices']}, "
                              f"delta16 slices {info.get('delta16_slices', 0)}, "
                              f"regular rows {info['regular_rows']}/{info['nrows']}, side rows {info['side_rows']}"),
            "int32_columns_kernel_ms": round(kernel_ms_int32, 4),
            "int32_columns_achieved": round(bytes_int32 / (kernel_ms_int32 * 1e-3) / 1e9, 1),
            "box_read_gbs": None if box is None else round(box[0], 1),
            "box_copy_gbs": None if box is None else round(box[1], 1),
            "achieved_vs_box_read": None if box is None else round(achieved / box[0], 4),
            "box_read_gbs_one_launch": None if box_launch is None else round(box_launch, 1),
            "achieved_vs_box_read_one_launch": None if not box_launch else round(achieved / box_launch, 4),
            "box_note": ("pa_hbm_probe on the same box and run: best read-only / copy rate of 16 B "
                         "non-temporal sweeps reading as many bytes per launch as the timed loop cycles "
                         "through (the SpMV's format bytes times the operator copies it rotates); the attainable "
                         "rate next to the 8 TB/s spec (boxes differ by up to ~20 %)"),
        },
    }
    if halo_leg is not None:
        line["halo_1gpu"] = halo_leg
    # N ranks: the same problem with all N parts in ONE process (the Julia
    # binding's model), measured by a child of rank 0 while the other ranks
    # wait (their GPUs idle)
    if use_dist and not args.no_oneproc and (ngpu > 1 or args.oneproc_devices):
        barrier()
        if rank == 0:
            line["one_process"] = one_process_leg(args)
        barrier()
    if rank == 0 and not args.no_cpu_baseline:
        if ngpu == 1:
            line["cpu_baseline"] = cpu_baseline(args.kind, args.n, args.cpu_seconds)
            if halo_leg is not None:
                halo_leg["cpu_baseline"] = cpu_baseline_mpi(args.kind, (args.n,) * 3, (2, 2, 2), args.cpu_seconds)
        else:
            line["cpu_baseline"] = cpu_baseline_mpi(args.kind, N, shape, args.cpu_seconds)
    if rank == 0:
        emit(line)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
