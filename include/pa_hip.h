/*
 * pa_hip.h — C-ABI of the MI355X-native backend for PartitionedArrays.jl's
 * SpMV + halo hot path (libpa_hip.so).
 *
 * This is the drop-in boundary.  A Julia `HIPBackend <: AbstractBackend`
 * binds these symbols with `ccall`; the Python host
 * package in partitionedarrays.jl_amd/ binds them with ctypes and is the
 * stand-in for that shim in this repository (no Julia on this image).
 *
 * Conventions:
 *  - every entry point returns int: 0 = ok, <0 = error; the message of the
 *    last error of the calling thread is in pa_last_error();
 *  - all index inputs are Julia 1-based (Int32 unless a width is passed);
 *    they are converted once, at create time;
 *  - the library copies host inputs and owns all device memory; handles are
 *    opaque and freed by their *_destroy;
 *  - a process holds one or more parts ("local parts"); the *_all entry
 *    points take the arrays of handles of all local parts, in part order,
 *    mirroring `map_parts` over an AbstractPData.  Neighbours held by the
 *    same process are served by device copies, neighbours in other processes
 *    by RCCL point-to-point over xGMI (after pa_comm_init_rank);
 *  - dtype codes: PA_F32, PA_F64, PA_C64 (ComplexF32), PA_C128 (ComplexF64).
 *    Scalars (alpha, beta, results) are passed as pointers to host values of
 *    the vector's element type;
 *  - threading: one host thread drives a set of parts (the reference's
 *    tasks run on the main Julia task too); the library may issue a call's
 *    per-part work from its own threads.  The tuning knobs are resolved per
 *    call (the process defaults of pa_tune under the call's context
 *    overrides, pa_ctx_tune) and never written while a call runs, so calls
 *    on different parts from different host threads each run with their own
 *    context's knobs (pa_knob_selftest).  The per-context caches are not
 *    synchronised: concurrent calls must not share a context.
 *    pa_last_error is per thread.
 */
#ifndef PA_HIP_H
#define PA_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { PA_F32 = 0, PA_F64 = 1, PA_C64 = 2, PA_C128 = 3 };
enum { PA_REPLACE = 0, PA_ADD = 1 };

typedef struct pa_ctx pa_ctx;
typedef struct pa_index pa_index;
typedef struct pa_xchg pa_xchg;
typedef struct pa_vec pa_vec;
typedef struct pa_mat pa_mat;
typedef struct pa_coo pa_coo;

/* ---- errors / library info ------------------------------------------- */
const char* pa_last_error(void);
int pa_version(void);
/* number of visible HIP devices (0 when no GPU). */
int pa_device_count(int* count);
/* Process-wide tuning knobs (performance only, results unchanged); each is
 * an A/B lever kept because a configuration uses it or a test pins it:
 * "spmv_flags"  bit 0: non-temporal value/column streams, bit 1: pattern
 *               and triple-SELL slices read their offset, length and mask /
 *               ghost base as one descriptor load, bit 2: pattern
 *               rows fetch x as 16 B runs, bit 3: the last len % U entries
 *               of a slice as one predicated batch, bit 4: a slice list
 *               covering the whole structure is launched without the list,
 *               bit 5: y written with non-temporal stores, bit 6: launches
 *               whose rows have at most 8 entries use the short-row kernels
 *               (one predicated batch, no loop: fewer registers), bit 7:
 *               the Float64 short-row tail launch of rows <= 7 entries at
 *               7 waves per SIMD (default 223);
 * "spmv_format" 1: pattern slices where the matrix has them (default),
 *               0: int32 column ids everywhere;
 * "long_rows_exact" 1: long rows summed in the reference's order (default),
 *               0: lane-strided partial sums + tree (within 1e-12);
 * "halo_pull"   1: parts of one process read their neighbours' packed
 *               buffers directly (default), 0: staging copies;
 * "spmv_delta16" 1: int32-column slices whose columns fit 16-bit codes
 *               store those (matrices built afterwards; default), 0: off;
 * "spmv_merge"  1: every slice kind of every part of a mul! without a halo
 *               in flight as one launch (default), 0: one launch per kind;
 * "spmv_merge_max" parts with more slices than this run one launch per
 *               kind (default 65536; 0: no limit);
 * "halo_direct" 1: mul! over parts sharing a stream pair reads every ghost
 *               straight from its owner's x on the compute stream (no
 *               pack, no cross-stream event; default), 0: pack + pull on
 *               the comm stream overlapped with the interior slices;
 * "halo_transport" 0 (default): parts of one process exchange by device
 *               reads/copies, except parts whose communicator came from
 *               pa_comm_init_all (RCCL, per context); 1: RCCL send/recv for
 *               every part that has a communicator;
 * "cg_fuse"     0: the device CG's u .= r .+ beta.*u as its own sweep,
 *               1: inside the SpMV (XV kernels), 2 (default, auto): with
 *               all parts in one process and at least three batches, one
 *               batch of each, then the faster (remembered on the matrix);
 *               otherwise the sweep or the matrix's earlier choice;
 * "spmv_group"  1: the parts of one process sharing a stream pair run each
 *               mul! phase as one launch (default), 0: launches per part;
 * "pattern_min_regular" a slice becomes a pattern slice when at least this
 *               percentage of its rows follow its pattern (1-100; 0 = auto,
 *               the default: 70, 50 for Float32's 256-row slices; matrices
 *               built afterwards), the others go to the side SELL;
 * "issue_threads" a mul! over several parts with their own stream pairs is
 *               issued from host threads, one part per thread: 1 when the
 *               parts span several devices (default), 2 always, 0 never
 *               (the calling thread, one part after the other);
 * "halo_barrier" 1: such a mul! (local neighbours) waits for one pack
 *               barrier per call and alternates two send buffers (default),
 *               0: per-neighbour event waits before every pack and pull;
 * "spmv_tri16"  the triple SELL for delta16 slices (see below): 1 for
 *               slices of 1-2 rows per lane (default), 0 never;
 * "spmv_tri_order" 1: its other rows first (default), 0: triple rows first;
 * "spmv_xcd_chunk" -1 (default, auto): one-launch-per-kind calls run their
 *               workgroups in runs of (pattern reach / 8) blocks per XCD,
 *               merged launches round robin; C > 0: runs of C; 0: round robin;
 * "spmv_side_tail" 1: per-kind launches run short side rows as the pattern
 *               launch's trailing waves (default), 0: their own launch;
 * "f32_rows"    Float32 SELL rows per lane (matrices built afterwards):
 *               4 (16 B value packs, 256-row slices), 2 (8 B packs, 128-row
 *               slices: the Float64 geometry, so delta16 rows take the
 *               triple SELL), 0 (default, auto): 4, rebuilt with 2 when
 *               fewer than 80 % of the slices are pattern slices;
 * "spmv_tri_pack" triple-SELL slices of 2 rows per lane (matrices built
 *               afterwards): bit 2 pair slices (every element type,
 *               pa_mat_pair_info), bit 0 their Float32 values as one 16 B
 *               and one 8 B pack per triple and lane (bit 1 unused);
 *               7 (default), 0 none;
 * "spmv_uniform" 1 (default): Float64 pattern slices whose patterns (<= 7
 *               entries) are subsequences of one union U (FD7) also keep
 *               their values at slice * H * |U| in U's order, so the
 *               short-row tail launch issues its loads before the slice's
 *               descriptor arrives (matrices built afterwards); 0 off;
 * "fault_inject" tests only: threaded issue jobs add an invalid launch. */
int pa_tune(const char* key, int value, int* previous);
/* The same knobs for one context: calls led by parts of `c` (their first
 * part's context) run with this value instead of the process default, for
 * the duration of the call; value PA_TUNE_DROP drops the override (a value
 * outside every knob's range: -1 is a valid value, spmv_xcd_chunk's auto).
 * *previous gets the context's former override (PA_TUNE_DROP: none).     */
#define PA_TUNE_DROP (-2147483647 - 1)
int pa_ctx_tune(pa_ctx* c, const char* key, int value, int* previous);
/* Test support (no device needed): `nthreads` host threads resolve calls'
 * knobs with different context overrides, on their own threads and on the
 * library's issue threads, while the process default changes; *mismatches
 * counts resolutions that saw another call's value (0 expected).        */
int pa_knob_selftest(int nthreads, int iters, int* mismatches);
/* HBM calibration of `device` (not the hot path): best read-only and copy
 * rates (GB/s, read+write bytes for the copy; best of 4/8 loads in flight
 * per lane and four grid sizes) over `reps` sweeps of a
 * `bytes` buffer with the SpMV's 16 B non-temporal loads.  bench.py reports
 * the SpMV's PMC-measured rate against it, since boxes differ.           */
int pa_hbm_probe(int device, int64_t bytes, int reps, double* read_gbs, double* copy_gbs);
/* The same read sweep at the size of ONE launch: every launch reads
 * `bytes_per_launch` (one operator's bytes), the launches rotating over
 * `span` bytes (>= 1 GiB: from HBM, not the 256 MB Infinity Cache), so the
 * rate includes one launch's ramp-up and drain; best of the grid sizes.  A
 * short SpMV (C2's 149 MB) is compared with this, not with the sweep of a
 * large buffer.                                                           */
int pa_hbm_probe_launch(int device, int64_t bytes_per_launch, int64_t span, int reps, double* read_gbs);

/* ---- part context ------------------------------------------------------
 * One context per part: its device, its streams, its scratch.
 * Replaces the part slot of `get_part_ids(b::AbstractBackend, nparts)`
 * (Interfaces.jl:24) — part is 1-based, 1 <= part <= nparts.          */
int pa_ctx_create(int device, int part, int nparts, pa_ctx** out);
/* A context for another part on `with`'s device that shares its stream
 * pair: several parts of one process on one GPU then form a single
 * in-order chain (no cross-stream events between them).                 */
int pa_ctx_create_shared(int part, int nparts, pa_ctx* with, pa_ctx** out);
int pa_ctx_destroy(pa_ctx* ctx);
int pa_ctx_sync(pa_ctx* ctx);

/* RCCL bootstrap for the one-part-per-process mode (the MPIBackend role,
 * MPIBackend.jl:9-36): rank 0 makes the id, the host broadcasts it (MPI
 * Bcast / torch.distributed), every rank calls pa_comm_init_rank with
 * rank = part-1 and nranks = nparts.                                    */
int pa_comm_unique_id(unsigned char id[128]);
int pa_comm_init_rank(pa_ctx* ctx, const unsigned char id[128]);
/* RCCL between the parts of one process (ncclCommInitAll over the distinct
 * devices of ctx[0..n-1] = parts 1..nparts, in order: one rank per device,
 * in order of first appearance; parts of one device share its rank, and
 * must share their stream pair, so a segment between them is a send to
 * self).  Every halo segment of these contexts then moves by the same
 * grouped ncclSend/ncclRecv as across processes (MPIBackend.jl:261-309),
 * posted in (sender part, receiver part) order; contexts without it (or
 * not from pa_comm_init_all) read each other's buffers.                  */
int pa_comm_init_all(int n, pa_ctx* const ctx[]);
/* Halo bytes this part has posted to RCCL sends / receives so far (what the
 * grouped ncclSend/ncclRecv carried for it; 0 when every segment moved by
 * device reads).                                                          */
int pa_comm_stats(pa_ctx* ctx, int64_t* bytes_sent, int64_t* bytes_recv);
/* What this part's communicator runs on, so that a multi-process run can
 * show it (the reference asserts Comm_size == prod(nparts),
 * MPIBackend.jl:11,17,61): *ranks = ncclCommCount (0: no communicator),
 * *rank = ncclCommUserRank, the context's device ordinal and its PCI bus id
 * (pci, >= 16 bytes: distinct GPUs of a node have distinct ids), the RCCL
 * version (ncclGetVersion) and the path of the librccl the process resolved
 * it from (lib, lib_len bytes; dladdr on ncclGetVersion: a host that loads
 * another RCCL first, e.g. torch's bundled one, shows it here).          */
/* Host time of the library's issue jobs (one part's share of a call issued
 * from an IssuePool thread: its runtime calls and launches) since the last
 * reset: the largest and the mean job, and their count.  The per-thread
 * issue time of one process driving several GPUs.         */
int pa_issue_stats(int reset, double* max_job_us, double* mean_job_us, int64_t* jobs);
int pa_comm_info(pa_ctx* ctx, int* ranks, int* rank, int* device, char* pci, int pci_len, int* version,
                 char* lib, int lib_len);

/* ---- index sets --------------------------------------------------------
 * Device copy of an AbstractIndexSet's oid_to_lid / hid_to_lid
 * (IndexSets.jl:215-265, 343-421).  1-based Int32 inputs.  Contiguous
 * layouts (oid_to_lid == 1:noids, hid_to_lid == noids+1:nlids) are detected
 * and kept as ranges (no device table).                                  */
int pa_index_create(pa_ctx* ctx, int64_t nlids,
                    int64_t noids, const int32_t* oid_to_lid,
                    int64_t nhids, const int32_t* hid_to_lid,
                    pa_index** out);
int pa_index_destroy(pa_index* idx);

/* ---- exchanger (halo plan) ----------------------------------------------
 * `Exchanger{parts_rcv,parts_snd,lids_rcv,lids_snd}` (Interfaces.jl:698-713)
 * verbatim: parts_* are 1-based part ids, ptrs_* are the 1-based Table ptrs
 * (length n+1), lids_* the 1-based Table data.                            */
int pa_xchg_create(pa_ctx* ctx,
                   int32_t n_rcv, const int32_t* parts_rcv,
                   const int32_t* ptrs_rcv, const int32_t* lids_rcv,
                   int32_t n_snd, const int32_t* parts_snd,
                   const int32_t* ptrs_snd, const int32_t* lids_snd,
                   pa_xchg** out);
int pa_xchg_destroy(pa_xchg* xg);

/* Global ids on the device.
 * pa_index_set_gids: attach lid_to_gid (num_lids 1-based gids) to the
 * index set; the library keeps a sorted gid → lid table on the device.
 * pa_add_gids: add_gids!(a, gids) (Interfaces.jl:579-603, 618-627) — the
 * n gids that are not local ids of the set, each once, in first-touch order,
 * into new_gids (capacity cap; *n_new is set even when it exceeds cap, and
 * the call then fails so the caller can retry).  The host appends them as
 * ghosts with their owners (gid_to_part) and builds the Exchanger.       */
int pa_index_set_gids(pa_index* idx, const int64_t* lid_to_gid);
int pa_add_gids(pa_index* idx, int64_t n, const int64_t* gids, int64_t cap,
                int64_t* new_gids, int64_t* n_new);
/* to_lids!(ids, a) (Interfaces.jl:1541-1543, IndexSets.jl gid_to_lid): the
 * n 1-based gids in ids become 1-based lids, in place, through the device
 * gid table; a gid that is not a local id fails (KeyError).  Exchanger
 * (Interfaces.jl:723-786) uses it for lids_snd of the gids its receivers
 * asked for.                                                              */
int pa_index_to_lids(pa_index* idx, int64_t n, int64_t* ids);

/* ---- vectors (the values of one part of a PVector) --------------------- */
int pa_vec_create(pa_ctx* ctx, int dtype, int64_t n, pa_vec** out);
int pa_vec_destroy(pa_vec* v);
int pa_vec_upload(pa_vec* v, const void* host, int64_t n);
int pa_vec_download(const pa_vec* v, void* host, int64_t n);
/* the device address of v's values (lid 1 at offset 0; valid until
 * pa_vec_destroy): zero-copy interop, e.g. Julia's unsafe_wrap of a
 * ROCArray over a part's values, and placement diagnostics              */
int pa_vec_device_ptr(const pa_vec* v, void** out);
/* fill!(v, s) (Interfaces.jl:1966-1971), all lids */
int pa_vec_fill(pa_vec* v, const void* s);
/* copyto!(dst, src): all lids when same_layout, owned values otherwise
 * (Interfaces.jl:1659-1667).  idx_* describe each vector's partition.    */
int pa_vec_copy(pa_vec* dst, const pa_index* idx_dst,
                const pa_vec* src, const pa_index* idx_src, int same_layout);
/* Fused broadcast kernels for the CG recurrence (Interfaces.jl:1710-1737),
 * evaluated exactly as Julia's scalar loop (no FMA contraction):
 *   mode 0: y[i] = x[i] + a*y[i]     (u .= r .+ β.*u)
 *   mode 1: y[i] = y[i] + a*x[i]     (x .+= α.*u)
 *   mode 2: y[i] = y[i] - a*x[i]     (r .-= α.*c)
 *   mode 3: y[i] = y[i] - x[i]       (r .-= c)
 *   mode 4: y[i] = a*y[i]            (rmul!, Interfaces.jl:1675)
 * over all lids when all_lids != 0 (same partition: ghosts too), else over
 * the owned values through idx (which must describe both vectors).
 * The scalar a is of the element type, or — mode | PA_BCAST_F64 — a
 * Float64 (double), or — mode | PA_BCAST_C128 — a ComplexF64 (complex
 * vectors only): then each element is evaluated in Float64 / ComplexF64
 * (Real * Complex componentwise) and rounded to the element type once,
 * Julia's promotion for e.g. IterativeSolvers' Float64 α, β with Float32
 * vectors.                                                                */
#define PA_BCAST_F64 8
#define PA_BCAST_C128 16
int pa_vec_axpby(pa_vec* y, const pa_vec* x, const pa_index* idx,
                 const void* a, int mode, int all_lids);

/* ---- matrices (one part of a PSparseMatrix) ----------------------------
 * From the reference's local SparseMatrixCSC (1-based colptr/rowval with
 * index_bytes = 4 or 8, nzval of dtype), with the matrix's rows/cols index
 * sets.  Builds the owned-row split SELL layout once:
 * own-column entries in oid order, then ghost-column entries in hid order,
 * i.e. the summation order of SparseUtils.jl:176-185 applied to the
 * owned_owned and owned_ghost blocks (Interfaces.jl:2142-2156, 2261-2272).
 * Stored entries of ghost rows are dropped (the `i>0` filter).            */
int pa_mat_from_csc(pa_ctx* ctx, int dtype, int index_bytes,
                    int64_t nrows_lids, int64_t ncols_lids,
                    const void* colptr, const void* rowval, const void* nzval,
                    const pa_index* rows, const pa_index* cols,
                    pa_mat** out);
/* From the local SparseMatrixCSR{Bi} of one part (SparseUtils.jl:189-252;
 * PSparseMatrix(sparsecsr, I, J, V, rows, cols; ids), Interfaces.jl:
 * 2194-2215 with a CSR init): rowptr (nrows_lids+1) and colval hold
 * Bi-based indices (Bi = 0 or 1, index_bytes 4 or 8), nzval in storage
 * order.  Same SELL layout as pa_mat_from_csc; each owned row keeps its
 * owned-column entries in storage order, then its ghost-column entries in
 * storage order (the owned_owned then owned_ghost passes of
 * SparseUtils.jl:242-250), and mul! with α != 1 scales each product,
 * (v*x)*α, as SparseUtils.jl:247 does (a CSC parent scales x, :177).
 * pa_mat_set_values / pa_mat_get_values / pa_mat_xchg_create index the CSR
 * nonzeros.                                                             */
int pa_mat_from_csr(pa_ctx* ctx, int dtype, int index_bytes, int Bi,
                    int64_t nrows_lids, int64_t ncols_lids,
                    const void* rowptr, const void* colval, const void* nzval,
                    const pa_index* rows, const pa_index* cols,
                    pa_mat** out);
/* From COO triplets: PSparseMatrix(I, J, V, rows, cols; ids=:local)
 * (Interfaces.jl:2194-2244) → sparse(I, J, V, m, n, +) (SparseUtils.jl:
 * 80-94) on the device (stable radix sort, duplicates summed in input
 * order), then the same SELL layout as pa_mat_from_csc.  I, J: 1-based
 * local ids (index_bytes 4 or 8), ncoo entries each; an index out of range
 * is an error (BoundsError).  ids_global = 1 (ids=:global): I, J are Int64
 * global ids, mapped by to_lids! on the device through the gid tables of
 * rows and cols (pa_index_set_gids; an unknown gid is a KeyError).  *csc_nnz = nnz of the combined CSC; when
 * colptr_out (ncols_lids+1) / rowval_out (>= ncoo) are non-NULL the CSC
 * pattern is written there, 1-based, for host setup that needs it
 * (matrix_exchanger, Interfaces.jl:2300-2372).  The nonzeros' CSC order is
 * what pa_mat_set_values / pa_mat_get_values / pa_mat_xchg_create use.   */
int pa_mat_from_coo(pa_ctx* ctx, int dtype, int index_bytes, int ids_global,
                    int64_t nrows_lids, int64_t ncols_lids, int64_t ncoo,
                    const void* I, const void* J, const void* V,
                    const pa_index* rows, const pa_index* cols,
                    int64_t* csc_nnz, int64_t* colptr_out,
                    int64_t* rowval_out, pa_mat** out);
/* PSparseMatrix(sparsecsr, I, J, V, rows, cols; ids) with the compress on
 * the device: pa_mat_from_coo / pa_mat_from_dcoo with a SparseMatrixCSR{Bi}
 * parent — sparsecsr(Val(Bi), I, J, V, m, n, +) (SparseUtils.jl:193-208:
 * duplicates combined with + in input order, columns ascending in each
 * row), the matrix's nonzeros in CSR order and mul! with α applied to each
 * product (SparseUtils.jl:247), as pa_mat_from_csr.  *nnz = nonzeros;
 * rowptr_out (nrows_lids+1) / colval_out (>= ncoo), when non-NULL, receive
 * the CSR pattern in base Bi.  Needs ascending oid_to_lid / hid_to_lid in
 * cols (every PRange the reference builds).                              */
int pa_mat_from_coo_csr(pa_ctx* ctx, int dtype, int index_bytes, int ids_global, int Bi,
                        int64_t nrows_lids, int64_t ncols_lids, int64_t ncoo,
                        const void* I, const void* J, const void* V,
                        const pa_index* rows, const pa_index* cols, int64_t* nnz,
                        int64_t* rowptr_out, int64_t* colval_out, pa_mat** out);
int pa_mat_from_dcoo_csr(const pa_coo* coo, int ids_global, int Bi, int64_t nrows_lids,
                         int64_t ncols_lids, const pa_index* rows, const pa_index* cols,
                         int64_t* nnz, int64_t* rowptr_out, int64_t* colval_out,
                         pa_mat** out);
/* COO triplets of one part on the device: I, J global ids (Int64, 1-based),
 * V of dtype — the (I, J, V) of PSparseMatrix(I, J, V, rows, cols;
 * ids=:global), test_fem_sa.jl:60-131.                                  */
int pa_coo_create(pa_ctx* ctx, int dtype, int64_t n, const int64_t* I,
                  const int64_t* J, const void* V, pa_coo** out);
int pa_coo_destroy(pa_coo* coo);
int pa_coo_size(const pa_coo* coo, int64_t* n);
int pa_coo_download(const pa_coo* coo, int64_t* I, int64_t* J, void* V);
/* async_assemble!(I, J, V, rows) + wait (Interfaces.jl:2406-2492) over the
 * n parts of this process: each triplet whose row (a gid of rows, which
 * needs pa_index_set_gids) is owned by another part is sent to that owner —
 * segments in rows.exchanger.parts_rcv order, input order inside — and its
 * local value becomes zero (the entry stays); every part appends what it
 * receives in parts_snd order.  I and J stay global.  Parts of this process
 * exchange by device copies, other processes' parts by RCCL (counts first,
 * then I, J, V per segment).  A row gid that is not a local id of rows is
 * a KeyError (to_lids!, Interfaces.jl:2420).                              */
int pa_coo_assemble_all(int n, pa_coo* const coo[], const pa_index* const rows[],
                        pa_xchg* const rows_xchg[]);
/* pa_mat_from_coo over a device COO (index_bytes 8): ids_global = 1 maps
 * I, J through rows' and cols' gid tables; the COO is left unchanged.    */
int pa_mat_from_dcoo(const pa_coo* coo, int ids_global, int64_t nrows_lids,
                     int64_t ncols_lids, const pa_index* rows,
                     const pa_index* cols, int64_t* csc_nnz,
                     int64_t* colptr_out, int64_t* rowval_out, pa_mat** out);
/* Replace the stored values keeping the pattern (same CSC nz order),
 * e.g. after fillstored!/re-assembly (Interfaces.jl:2127-2132).          */
int pa_mat_set_values(pa_mat* A, const void* nzval);
/* fillstored!(A, v) (Interfaces.jl:2127-2132): every stored value of the
 * part (ghost rows included) becomes the scalar *v of the matrix's dtype,
 * on the device, stream-ordered with the part's other work.              */
int pa_mat_fillstored(pa_mat* A, const void* v);
/* nonzeros(A) in CSC nz order, ghost rows included (the device keeps the
 * ghost rows' values beside the SELL slots for exchange!/assemble!(A)).  */
int pa_mat_get_values(const pa_mat* A, void* nzval);
/* matrix_exchanger(values, rows, cols) (Interfaces.jl:2300-2372): the
 * Exchanger whose lids are CSC nz positions k (1-based, Int64 as Julia's
 * Table{Int}): k_rcv = nonzeros of ghost rows grouped by owner, k_snd = the
 * owner's nonzeros at the same (gi, gj).  Usable with pa_mat_exchange_all. */
int pa_mat_xchg_create(pa_mat* A, int32_t n_rcv, const int32_t* parts_rcv,
                       const int32_t* ptrs_rcv, const int64_t* k_rcv,
                       int32_t n_snd, const int32_t* parts_snd,
                       const int32_t* ptrs_snd, const int64_t* k_snd,
                       pa_xchg** out);
/* exchange!(A) (Interfaces.jl:2375-2381: op PA_REPLACE, reverse 0) and
 * assemble!(A) (2383-2404: op PA_ADD, reverse 1, zero_sent 1 — the ghost
 * rows' values are zeroed after sending) over nonzeros(A), n local parts.
 * Contributions to one nonzero are combined in the reference's order.     */
int pa_mat_exchange_all(int n, pa_mat* const A[], pa_xchg* const xg[],
                        int op, int reverse, int zero_sent);
int pa_mat_destroy(pa_mat* A);
/* nnz stored on device (padding included) and owned-row nnz. */
int pa_mat_info(const pa_mat* A, int64_t* nrows_owned, int64_t* nnz_owned,
                int64_t* slots, int64_t* nslices, int64_t* nslices_interior);
/* Column encoding chosen at build time: slices whose rows
 * mostly follow one offset pattern store no column ids ("pattern slices");
 * their other rows live in a side SELL.                                   */
int pa_mat_format_info(const pa_mat* A, int64_t* pattern_slices,
                       int64_t* regular_rows, int64_t* side_rows,
                       int64_t* side_slots);
/* delta16 slices (pa_tune "spmv_delta16", default on): int32-column slices
 * whose columns all fit 16-bit codes — an owned column as the row + a
 * signed 15-bit delta, a ghost column as the slice's smallest ghost column
 * + 15 bits — stream 2 B of column id per slot instead of 4.              */
int pa_mat_delta16_info(const pa_mat* A, int64_t* delta16_slices);
/* The triple SELL (pa_tune "spmv_tri16" 1, the default: Float64,
 * ComplexF32, ComplexF64 and Float32 with 2 rows per lane): the delta16 slices'
 * rows re-sliced — rows whose columns are consecutive triples (c, c+1, c+2)
 * first — so that most slices keep one 16-bit code per triple and read a
 * triple's x as one run.  Its slices and rows, and how many of them are
 * triple slices (tri_slices, their rows tri_rows).                       */
int pa_mat_triple_info(const pa_mat* A, int64_t* t_slices, int64_t* t_rows, int64_t* tri_slices,
                       int64_t* tri_rows);
/* The triple SELL's pair slices (pa_tune "spmv_tri_pack" bit 2, default on;
 * 2 rows per lane): each lane holds rows a and a + 1 whose columns differ
 * by one, entry for entry, and reads one code and one x run per triple for
 * both.  Its pair slices (counted in tri_slices too) and their rows.     */
int pa_mat_pair_info(const pa_mat* A, int64_t* pair_slices, int64_t* pair_rows);

/* device addresses of the matrix's main arrays, for placement diagnostics:
 * out[0..7] = values, int32 columns, slice offsets, slice lengths (pattern),
 * patterns, masks, side values, side columns (0 where absent)           */
int pa_mat_device_ptrs(const pa_mat* A, uint64_t out[8]);

/* Bytes one mul! streams from this matrix in its current encoding
 * (pa_tune("spmv_format")), as its kernels load them: values (padding
 * included), column ids (int32 slices, side rows, long rows) and slice
 * metadata (offsets, lengths, lists, patterns, masks, row maps).  The
 * bench's roofline adds x (read once), y and the halo to these.          */
int pa_mat_traffic(const pa_mat* A, int64_t* value_bytes, int64_t* index_bytes,
                   int64_t* meta_bytes);

/* Long rows (row-length histogram): rows with more than max(256, 8 × the
 * 90th-percentile row length) entries leave the SELL and run one wave per
 * row over their own CSR (in the reference's summation order unless
 * pa_tune("long_rows_exact", 0)).  Number of such rows and their nonzeros. */
int pa_mat_long_rows(const pa_mat* A, int64_t* n_long, int64_t* n_long_nnz);

/* ---- hot path -----------------------------------------------------------
 * mul!(c, a, b, α, β) (Interfaces.jl:2246-2275) for the n local parts:
 * starts the halo exchange of x (pack → P2P → unpack into x's ghost lids,
 * i.e. exchange!(b)), runs the interior slices meanwhile, then the slices
 * that read ghost values.  y_idx / x_idx are the partitions of c and b
 * (c.rows / b.rows); x_idx must have the matrix's column layout.
 * Asynchronous with respect to the host (stream-ordered per part).       */
int pa_spmv_all(int n, pa_mat* const A[], pa_vec* const y[],
                const pa_index* const y_idx[],
                pa_vec* const x[], const pa_index* const x_idx[],
                pa_xchg* const xg[], const void* alpha, const void* beta);

/* CG fusions (the caller of the hot path, IterativeSolvers.cg! at
 * test_fdm.jl:115 / test_fem_sa.jl:135):
 * pa_spmv_dot_all = mul!(c, A, u) followed by dot(u, c), the dot being
 * accumulated by the SpMV kernel over the owned rows it writes (u = x must
 * have contiguous owned lids); pa_cg_update_all = x .+= α.*u; r .-= α.*c
 * (all lids; the four vectors share one partition) and returns norm(r).
 * alpha is a Float64 (double) for real vectors, a ComplexF64 for complex
 * ones — IterativeSolvers' α = residual²/dot with a Float64 residual — and
 * each element is evaluated in that type and rounded once (PA_BCAST_*).
 * Reductions (dot, sum, norm) round each part's value to the element type
 * and add the parts in that type, as Julia's reduce over the parts' T
 * values does; norm's ^(1/2) is Float64.                                  */
int pa_spmv_dot_all(int n, pa_mat* const A[], pa_vec* const y[],
                    const pa_index* const y_idx[],
                    pa_vec* const x[], const pa_index* const x_idx[],
                    pa_xchg* const xg[], const void* alpha, const void* beta,
                    void* dot_result);
int pa_cg_update_all(int n, pa_vec* const x[], pa_vec* const r[],
                     const pa_vec* const u[], const pa_vec* const c[],
                     const pa_index* const idx[], const void* alpha,
                     double* rnorm);

/* IterativeSolvers.cg!(x, A, b; reltol, abstol, maxiter) (v0.9, not
 * vendored; called at test_fdm.jl:115, test_fem_sa.jl:135, recurrence in
 * SURVEY.md §3.5) with the scalar recurrence on the device (SURVEY.md §8f
 * item 3): u, r, c are the caller's work vectors (CGStateVariables), all
 * five vectors on a.cols' partition with contiguous owned lids.  Setup as
 * cg_iterator!: u = 0, r = b - A*x, tolerance = max(reltol*norm(b), abstol).
 * Then per iteration β = res²/prev², u .= r .+ β.*u, mul!(c,A,u) with
 * dot(u,c) fused, α = res²/dot, x .+= α.*u, r .-= α.*c, res = norm(r) — the
 * same arithmetic as the host-driven loop over pa_spmv_dot_all /
 * pa_cg_update_all, bit for bit.  The host enqueues `batch` iterations
 * between reads of the device's done flag (iterations after convergence
 * are no-ops); every rank enqueues the same number, so RCCL calls match.
 * history (optional, maxiter doubles): the residual after each iteration. */
int pa_cg_solve_all(int n, pa_mat* const A[], pa_vec* const x[],
                    const pa_vec* const b[], pa_vec* const u[],
                    pa_vec* const r[], pa_vec* const c[],
                    const pa_index* const idx[], pa_xchg* const xg[],
                    double reltol, double abstol, int64_t maxiter, int batch,
                    int64_t* iterations, double* residual, double* history);

/* The u-update variant choice of pa_cg_solve_all's auto mode (pa_tune
 * "cg_fuse" 2): the first timed batch runs the sweep, the second the fused
 * update; with one part per process (RCCL) every rank reduces the two
 * batch times with max over the ranks before choosing, so all ranks keep
 * the same variant.  pa_cg_variant_agree runs that decision on local_ms
 * (ms per iteration of the sweep and of the fused batch) with `fn` as the
 * all-reduce (max, in place on n floats; null: none), *choice = 1 fused,
 * 0 sweep, -1 no valid measurement.  pa_mat_cg_choice: the variant the
 * matrix remembers (-1: none yet).                                        */
typedef int (*pa_allreduce_max_fn)(float* v, int n, void* user);
int pa_cg_variant_agree(const float local_ms[2], pa_allreduce_max_fn fn, void* user, int* choice);
/* Whether the fused u update may run at all: only if every rank's part can
 * (no long rows, no triple SELL: their kernels gather x directly), or the
 * ranks would run different variants, whose halos carry different vectors
 * (ADVICE r05).  pa_cg_solve_all max-reduces "cannot fuse" over the ranks
 * (RCCL); this runs the same decision with fn as the all-reduce.  *agreed
 * = 1 when every rank's local_can_fuse is 1.                             */
int pa_cg_fuse_agree(int local_can_fuse, pa_allreduce_max_fn fn, void* user, int* agreed);
int pa_mat_cg_choice(const pa_mat* A, int* choice);

/* exchange!(combine, values, exchanger) (Interfaces.jl:846-889) for the n
 * local parts; reverse != 0 uses reverse(exchanger) (Interfaces.jl:796).
 * With reverse=1, op=PA_ADD and zero_ghosts=1 this is assemble!(v)
 * (Interfaces.jl:2084-2106).  Contributions to one lid are combined in the
 * receive-buffer order of the reference (bit-exact).                      */
int pa_exchange_all(int n, pa_vec* const v[], pa_xchg* const xg[],
                    const pa_index* const idx[], int op, int reverse,
                    int zero_ghosts);

/* dot(a,b) (Interfaces.jl:1985-1992) → sum over parts, folded in part
 * order as reduce(+, …; init=0) (Interfaces.jl:221-238).  result: host
 * scalar of the vectors' dtype (complex: conj(a)·b).                      */
int pa_dot_all(int n, const pa_vec* const a[], const pa_index* const ia[],
               const pa_vec* const b[], const pa_index* const ib[],
               void* result);
/* norm(a, 2) (Interfaces.jl:1767-1772); result: host double (the
 * reference's `(…)^(1/p)` promotes Float32 partials to Float64).          */
int pa_norm2_all(int n, const pa_vec* const a[], const pa_index* const ia[],
                 void* result);
/* sum(a) = reduce(+, a; init=0) over owned values (Interfaces.jl:1973-1983) */
int pa_sum_all(int n, const pa_vec* const a[], const pa_index* const ia[],
               void* result);

/* ---- synthetic operators (benchmark driver, not a reference entry point) --
 * One Cartesian part box [box_lo, box_lo+box_n) of a gdims[0]×gdims[1]×
 * gdims[2] node grid (0-based coordinates, x fastest), built directly on the
 * device in the layout pa_mat_from_csc would produce for the CSC that the
 * drivers assemble: kind 7 = test_fdm.jl's FD Poisson operator (coeffs =
 * {diag, offdiag}), kind 27 = Q1-hex FE operator of test_fem_sa.jl's
 * pattern (coeffs = Ke, 8×8 row-major).  Owned lids are the box's nodes in
 * x-fastest order; shell_lid[(ez*(ny+2)+ey)*(nx+2)+ex] is the 0-based lid of
 * the node at box-local (ex-1,ey-1,ez-1) of the one-node shell (ghosts), or
 * -1; NULL when the part has no ghosts.  nlids_cols = noids + nhids.      */
int pa_mat_stencil(pa_ctx* ctx, int dtype, int kind, const int64_t gdims[3],
                   const int64_t box_lo[3], const int64_t box_n[3],
                   int64_t nlids_cols, const int32_t* shell_lid,
                   const double* coeffs, int ncoeffs, pa_mat** out);

/* ---- timing (PTimer analogue, PTimers.jl) -------------------------------
 * pa_ctx_set_timing(ctx, 1) starts recording the mul! calls of this context
 * with HIP events on the stream they run on (no synchronisation inside the
 * calls).  pa_ctx_kernel_times returns the means over the recorded calls of
 * the interior slices, the halo completion seen by the compute stream (wait
 * for the transport + unpack, after the interior slices) and the boundary
 * slices (+ long rows, fused-dot fold), and the number of calls; it clears
 * the record.  With the direct pull (parts sharing a stream pair,
 * halo_direct) no slice runs before the halo is complete: interior is 0,
 * halo is the pull kernel, boundary is every slice.
 * pa_ctx_last_kernel_ms: the interior and boundary means.                  */
int pa_ctx_set_timing(pa_ctx* ctx, int enable);
int pa_ctx_kernel_times(pa_ctx* ctx, float* interior_ms, float* halo_ms,
                        float* boundary_ms, int* count);
int pa_ctx_last_kernel_ms(pa_ctx* ctx, float* spmv_interior_ms,
                          float* spmv_boundary_ms);
/* Device time of a region on the compute stream: pa_ctx_span(ctx, 0) before
 * it, pa_ctx_span(ctx, 1) after it (event records, no synchronisation);
 * pa_ctx_span_ms waits for the end and returns the elapsed ms.  Parts whose
 * mul! runs grouped (shared stream pair) record their phase times on the
 * first part of the call only (pa_ctx_kernel_times: count 0 for the rest). */
int pa_ctx_span(pa_ctx* ctx, int stop);
int pa_ctx_span_ms(pa_ctx* ctx, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* PA_HIP_H */
