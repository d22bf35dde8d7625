// pa_internal.h — shared types of libpa_hip.so (host API + kernels).
//
// Element types follow Julia's arithmetic exactly (no FMA contraction: the
// whole library is compiled with -ffp-contract=off).  Complex products are
// Julia's `*(z::Complex, w::Complex)` = (zr*wr - zi*wi, zr*wi + zi*wr)
// (base/complex.jl), sums are componentwise.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/pa_hip.h"

namespace pa {

struct alignas(8) c64 {
  float re, im;
};
struct alignas(16) c128 {
  double re, im;
};

__host__ __device__ inline c64 operator+(c64 a, c64 b) { return {a.re + b.re, a.im + b.im}; }
__host__ __device__ inline c64 operator-(c64 a, c64 b) { return {a.re - b.re, a.im - b.im}; }
__host__ __device__ inline c64 operator*(c64 a, c64 b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__host__ __device__ inline c128 operator+(c128 a, c128 b) { return {a.re + b.re, a.im + b.im}; }
__host__ __device__ inline c128 operator-(c128 a, c128 b) { return {a.re - b.re, a.im - b.im}; }
__host__ __device__ inline c128 operator*(c128 a, c128 b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

template <typename T> struct real_of { using type = T; };
template <> struct real_of<c64> { using type = float; };
template <> struct real_of<c128> { using type = double; };

// The wide type of Julia's mixed broadcasts with a Float64 / ComplexF64
// scalar (IterativeSolvers' α, β are Float64 even for Float32 vectors: norm
// of a PVector returns Float64, Interfaces.jl:1771): `r .+ β.*u` evaluates
// in W and rounds to T once on the store.
template <typename T> struct wide_of { using type = T; };
template <> struct wide_of<float> { using type = double; };
template <> struct wide_of<c64> { using type = c128; };
__host__ __device__ inline double widen(float v) { return (double)v; }
__host__ __device__ inline double widen(double v) { return v; }
__host__ __device__ inline c128 widen(c64 v) { return c128{(double)v.re, (double)v.im}; }
__host__ __device__ inline c128 widen(c128 v) { return v; }
template <typename T> __host__ __device__ inline T narrow(typename wide_of<T>::type v) { return (T)v; }
template <> __host__ __device__ inline c64 narrow<c64>(c128 v) { return c64{(float)v.re, (float)v.im}; }
template <> __host__ __device__ inline c128 narrow<c128>(c128 v) { return v; }
// Real * Complex is componentwise in Julia (base/complex.jl: x*real(z), x*imag(z))
__host__ __device__ inline double rscale(double a, double x) { return a * x; }
__host__ __device__ inline c128 rscale(double a, c128 z) { return c128{a * z.re, a * z.im}; }

template <typename T> __host__ __device__ inline T zero_of() { return T(0); }
template <> __host__ __device__ inline c64 zero_of<c64>() { return {0.f, 0.f}; }
template <> __host__ __device__ inline c128 zero_of<c128>() { return {0.0, 0.0}; }

// conj(a)*b, Julia's dot kernel for one element (LinearAlgebra: dot(x,y) = Σ dot(x_i,y_i))
__host__ __device__ inline float cdot(float a, float b) { return a * b; }
__host__ __device__ inline double cdot(double a, double b) { return a * b; }
__host__ __device__ inline c64 cdot(c64 a, c64 b) { return c64{a.re, -a.im} * b; }
__host__ __device__ inline c128 cdot(c128 a, c128 b) { return c128{a.re, -a.im} * b; }
// abs2
__host__ __device__ inline float abs2(float a) { return a * a; }
__host__ __device__ inline double abs2(double a) { return a * a; }
__host__ __device__ inline float abs2(c64 a) { return a.re * a.re + a.im * a.im; }
__host__ __device__ inline double abs2(c128 a) { return a.re * a.re + a.im * a.im; }

// ---- deterministic block reductions (shared by the .hip files) -----------
template <typename A>
__device__ inline A shfl_down64(A v, int d) {
  return __shfl_down(v, d, 64);
}
template <>
__device__ inline c128 shfl_down64<c128>(c128 v, int d) {
  return c128{__shfl_down(v.re, d, 64), __shfl_down(v.im, d, 64)};
}

// 256-thread block sum in a fixed order (wave tree, then waves 0..3); the
// result is valid on thread 0
template <typename A>
__device__ inline A block_reduce(A v) {
  __shared__ A sm[4];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = v + shfl_down64(v, d);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sm[w] = v;
  __syncthreads();
  A r = zero_of<A>();
  if (threadIdx.x == 0) {
    r = sm[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = r + sm[i];
  }
  return r;
}

// In-launch hand-off of one value per block (cdna_hip_programming.md §6
// Guideline 16, R1 with a ticket counter): lane 0 stores its value
// write-through (sc1), drains, then takes a ticket; the block whose ticket
// is the last one reads every value with sc1 loads.  The ticket is zeroed at
// allocation and reset by the last block, so it is 0 between launches.
typedef __attribute__((address_space(1))) unsigned long long pa_gu64;
typedef __attribute__((address_space(1))) unsigned int pa_gu32;

__device__ inline void st_wt(double* p, double v) {
  __hip_atomic_store((pa_gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_wt(c128* p, c128 v) {
  st_wt(reinterpret_cast<double*>(p), v.re);
  st_wt(reinterpret_cast<double*>(p) + 1, v.im);
}
__device__ inline double ld_wt(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((pa_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ inline c128 ld_wt(const c128* p) {
  const double* q = reinterpret_cast<const double*>(p);
  return c128{ld_wt(q), ld_wt(q + 1)};
}

// every thread of the block gets: did this block arrive last?
template <typename A>
__device__ inline bool publish_arrive(A* slots, A v, unsigned* ticket) {
  __shared__ int last;
  if (threadIdx.x == 0) {
    st_wt(&slots[blockIdx.x], v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add((pa_gu32*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x - 1;
    if (last) __hip_atomic_store((pa_gu32*)ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return last != 0;
}

struct NoTail {
  __device__ void operator()(const void*) const {}
};

constexpr int kFoldBlocks = 256;  // first-level blocks of a long fold (scratch: kFoldBlocks accumulators)

// Fold nb partials into out[0] in ONE launch, in the order of the two-level
// fold it replaces (k_fold_chunks + k_reduce_final): with g > 1 blocks,
// block b sums chunk [b*chunk, (b+1)*chunk) and hands it over; the last
// block sums the g chunk sums in block order.  tail(out) then runs on
// thread 0 of the finishing block (e.g. the CG scalar update).
template <typename A, typename Tail>
__global__ __launch_bounds__(256) void k_fold(int nb, int chunk, const A* __restrict__ in, A* scratch,
                                              A* __restrict__ out, unsigned* ticket, Tail tail) {
  const bool one = gridDim.x == 1;
  const int lo = one ? 0 : (int)blockIdx.x * chunk;
  const int hi = one ? nb : min(nb, lo + chunk);
  A s = zero_of<A>();
  for (int i = lo + (int)threadIdx.x; i < hi; i += blockDim.x) s = s + in[i];
  A r = block_reduce(s);
  if (!one) {
    if (!publish_arrive(scratch, r, ticket)) return;
    A s2 = zero_of<A>();
    for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) s2 = s2 + ld_wt(&scratch[i]);
    r = block_reduce(s2);
  }
  if (threadIdx.x == 0) {
    out[0] = r;
    tail(out);
  }
}

template <typename A, typename Tail>
inline void fold_launch(int nb, const A* in, A* scratch, A* out, unsigned* ticket, Tail tail, hipStream_t st) {
  int g = 1, chunk = nb;
  if (nb > 2 * kFoldBlocks && scratch) {  // one block over 10^5 partials is ~150 us
    chunk = (nb + kFoldBlocks - 1) / kFoldBlocks;
    g = (nb + chunk - 1) / chunk;
  }
  hipLaunchKernelGGL((k_fold<A, Tail>), dim3(g), dim3(256), 0, st, nb, chunk, in, scratch, out, ticket, tail);
}

inline size_t dtype_size(int dt) {
  switch (dt) {
    case PA_F32: return 4;
    case PA_F64: return 8;
    case PA_C64: return 8;
    case PA_C128: return 16;
  }
  return 0;
}

// Rows per lane of the SELL layout so that one lane's value load is 16 B
// (Float32: pa_tune "f32_rows" 2 gives 8 B loads in 128-row slices, the
// Float64 geometry, so its delta16 rows can take the triple SELL).
int f32_rows_knob();
// finalize_pattern's answer for a Float32 matrix built with 4 rows per lane
// under f32_rows 0 (auto) that is better off with 2: the caller rebuilds it
constexpr int kPreferR2 = 2;
inline int sell_rows_per_lane(int dt) {
  switch (dt) {
    case PA_F32: return f32_rows_knob();
    case PA_F64: return 2;
    case PA_C64: return 2;
    case PA_C128: return 1;
  }
  return 1;
}

void set_error(const std::string& msg);

// Device-resident scalars of the device-driven CG (pa_cg_solve_all): the
// IterativeSolvers 0.9 recurrence state, one copy per part (every part
// folds the same gathered partials in part order, so all copies agree).
struct CGState {
  double res;        // it.residual = norm(r)
  double prev;       // it.prev_residual
  double tol;        // max(reltol*norm(b), abstol)
  int64_t it;        // iterations done
  int64_t maxiter;
  int32_t done;      // it >= maxiter || res <= tol
  int32_t pad;
  c128 alpha;        // α in the wide type: Float64 (.re) for real T, ComplexF64 for complex T
  int64_t xit;       // iterations whose x .+= α.*u is applied (deferred into the next u update)
};

// Grouped launches (parts of one process sharing a stream pair): one launch
// per phase covers up to PA_GROUP_MAX parts (kernel-argument tables).
constexpr int PA_GROUP_MAX = 8;
constexpr int32_t kTriSlice = 1 << 30;  // pa_mat::d_t_len: a triple slice
constexpr int32_t kTriPair = 1 << 29;   // pa_mat::d_t_len: a pair slice (lane l: rows a_l, a_l + 1; build_triple_sell)
constexpr int32_t kTriLen = kTriPair - 1;  // pa_mat::d_t_len: the entries per row
struct SpmvPart {
  int64_t nwork;          // slices of this part in the launch
  const int32_t* list;    // slice ids (null: 0..nwork-1)
  const pa_mat* A;
  const void* x;
  void* y;
  const int32_t* ymap;
  void* dotp;
  // the device CG's fused u update (pa_cg_solve_all; null cg: a plain SpMV):
  // x is r, the SpMV multiplies u_new = r .+ β.*xu, writes u_new of the owned
  // rows to un and applies the deferred x .+= α.*xu to xacc
  const void* xu = nullptr;
  void* un = nullptr;
  void* xacc = nullptr;
  const CGState* cg = nullptr;
  // a side-row entry (kind 2) trailing the pattern entries of one grouped
  // launch (which 6: spmv_grouped's side tail)
  bool side = false;
};

struct PackGroup {
  int np;
  int64_t n[PA_GROUP_MAX];
  const int32_t* lids[PA_GROUP_MAX];
  const void* v[PA_GROUP_MAX];
  void* buf[PA_GROUP_MAX];
};
struct PullGroup {
  int np;
  int64_t n[PA_GROUP_MAX];
  const int32_t* lids[PA_GROUP_MAX];
  const int32_t* bid[PA_GROUP_MAX];
  const int64_t* elem[PA_GROUP_MAX];
  const void* const* bases[PA_GROUP_MAX];
  void* v[PA_GROUP_MAX];
};

// Cartesian part box of a synthetic stencil operator (pa_mat_stencil).
struct StencilGeom {
  int64_t N[3];   // global nodes per dim
  int64_t lo[3];  // box origin (0-based global coords)
  int64_t n[3];   // box extent
  int kind;       // 7 (test_fdm.jl FD) or 27 (Q1 FE, test_fem_sa.jl pattern)
};

}  // namespace pa

// ---------------------------------------------------------------------------
// Opaque handle definitions.
struct pa_ctx {
  // parts of one process on the same device may share one stream pair
  // (pa_ctx_create_shared): their work then forms one in-order chain
  struct StreamRefs { int n = 1; };
  StreamRefs* stream_refs = nullptr;
  int device = 0;
  int part = 1;    // 1-based
  int nparts = 1;
  hipStream_t s_main = nullptr;   // compute stream
  hipStream_t s_comm = nullptr;   // halo transport stream (high priority)
  void* comm = nullptr;           // ncclComm_t (null: no remote transport)
  bool halo_rccl = false;         // pa_comm_init_all: halo segments between parts of this process over RCCL too
  // the communicator is destroyed with the last part using it; parts of one
  // device share their device's rank (pa_comm_init_all), so the peer of a
  // halo segment from/to part q is rank_of_part[q-1] (null: rank = q-1)
  std::shared_ptr<void> comm_owner;
  std::shared_ptr<const std::vector<int>> rank_of_part;
  int peer_rank(int q) const { return rank_of_part ? (*rank_of_part)[q - 1] : q - 1; }
  int64_t rccl_bytes_sent = 0, rccl_bytes_recv = 0;  // halo bytes this part posted to RCCL (pa_comm_stats)
  // reduction scratch
  void* d_partials = nullptr;     // per-block partials (max 16 B each)
  void* d_fold = nullptr;         // 256*16 B first-level fold of long partial lists
  void* d_result = nullptr;       // 16 B final per-part value
  void* d_gather = nullptr;       // nparts*16 B gathered partials (RCCL mode)
  unsigned* d_ticket = nullptr;   // arrival counter of the one-launch folds (0 between launches)
  void* h_pinned = nullptr;       // pinned host staging (>= nparts*16 B)
  // timing (pa_ctx_set_timing): four events per recorded mul! — before the
  // interior slices, after them, after the halo wait (+unpack), after the
  // boundary slices — read back only by pa_ctx_kernel_times (no sync per call)
  bool timing = false;
  std::vector<hipEvent_t> tev;
  int tn = 0;                     // mul! calls recorded since timing was enabled
  hipEvent_t span_ev[2] = {nullptr, nullptr};  // pa_ctx_span: start / end of a region
  // events for the exchange pipeline
  hipEvent_t ev_packed = nullptr;
  hipEvent_t ev_recvd = nullptr;
  // the pack barrier of stream-pair mul! calls this part leads (spmv_impl's
  // barrier issue): recorded on its s_comm once every part of the call packed
  hipEvent_t ev_barrier = nullptr;
  // device arrays of the x pointers of grouped mul! calls led by this part
  // (the direct pull's bases), most recent first
  std::vector<std::pair<std::vector<void*>, void**>> bases_cache;
  // device copies of the merged-launch tables of calls led by this part
  std::vector<std::pair<std::vector<char>, void*>> merged_cache;
  // pa_ctx_tune: this context's knob values over the process defaults,
  // applied to the calls it leads (TuneScope)
  static constexpr int kMaxKnobs = 24;
  bool has_over[kMaxKnobs] = {};
  int64_t over[kMaxKnobs] = {};
};

// The tuning knobs of one call (performance only, results unchanged; the
// table with their meaning is kKnobs in pa_api.cpp).  A call resolves them
// once — the process defaults (pa_tune) under its first part's context
// overrides (pa_ctx_tune) — into its own Knobs, which the launchers and the
// IssuePool jobs of that call read through pa::knobs(): no process-global
// knob is written while a call runs, so concurrent calls from several host
// threads each see their own context's values.
namespace pa {
struct Knobs {
  int spmv_flags;        // SPMV_* bits of pa_spmv.hip
  int long_exact;
  int halo_pull;
  int spmv_delta16;
  int spmv_merge;
  int64_t spmv_merge_max;
  int cg_fuse;
  int halo_direct;
  int halo_transport;
  int spmv_group;
  int spmv_format;
  int pattern_min_pct;
  int issue_threads;
  int fault_inject;      // tests only: the IssuePool jobs issue an invalid launch
  int spmv_xcd_chunk;    // XCD-chunked block order of the SpMV launches (pa_spmv.hip xcd_block), 0 off, -1 auto
  int spmv_tri16;        // delta16 slices re-sliced into the triple SELL (pa_mat::d_t_*): 0 never, 1 R <= 2
  int halo_barrier;      // stream-pair mul!: one pack barrier + double-buffered sends (spmv_impl)
  int tri_order;         // triple SELL row order: 0 triple rows first, 1 the other rows first (build_triple_sell)
  int side_tail;         // per-kind launches: the side rows as the trailing waves of the pattern launch
  int f32_rows;          // Float32 SELL rows per lane (matrices built afterwards): 4 (16 B packs), 2 (8 B), 0 auto
  int tri_pack;          // triple SELL: bit 2 pair slices, bit 0 their Float32 per-triple value packs
  int spmv_uniform;      // Float64 short pattern rows: the uniform layout (build_uniform)
};
// the knobs of the call running on this thread (outside a call: a snapshot
// of the process defaults)
const Knobs& knobs();
// this thread runs work of a call whose knobs are *k (IssuePool workers)
struct KnobBind {
  explicit KnobBind(const Knobs* k);
  ~KnobBind();
  const Knobs* prev;
};
}  // namespace pa

// the knobs of a call's (first part's) context for the call's duration
struct TuneScope {
  explicit TuneScope(const pa_ctx* c);
  ~TuneScope();
  TuneScope(const TuneScope&) = delete;
  TuneScope& operator=(const TuneScope&) = delete;
  pa::Knobs k;
  const pa::Knobs* prev;
};

struct pa_index {
  pa_ctx* ctx = nullptr;
  int64_t nlids = 0, noids = 0, nhids = 0;
  bool own_contig = true;    // oid_to_lid == 0..noids-1 (0-based)
  bool ghost_contig = true;  // hid_to_lid == noids..nlids-1
  int32_t* d_oid_to_lid = nullptr;  // 0-based, null when own_contig
  int32_t* d_hid_to_lid = nullptr;  // 0-based, null when ghost_contig
  std::vector<int32_t> h_oid_to_lid;  // 0-based host copies
  std::vector<int32_t> h_hid_to_lid;
  std::vector<int32_t> h_lid_to_ohid;  // reference's lid_to_ohid (1-based ±)
  // gid → lid table (pa_index_set_gids): gids sorted ascending, their lids
  uint64_t* d_sgid = nullptr;
  int64_t* d_slid = nullptr;
  bool has_gids = false;
};

// Ordered combine plan: for each distinct target lid, the buffer positions
// that land on it, ascending (= the reference's unpack loop order).
struct pa_combine_plan {
  int64_t ntargets = 0;
  bool unique = true;                // every lid at most once → plain scatter
  int32_t* d_target = nullptr;       // distinct target lids (0-based)
  int32_t* d_ptr = nullptr;          // ntargets+1
  int32_t* d_pos = nullptr;          // buffer positions
};

// Pull table of one exchange direction (parts of one process): receive slot
// p of this part reads bases[bid[p]][elem[p]] — a sender's send buffer, or
// this part's own receive buffer for segments that came over RCCL.
struct pa_pull {
  bool built = false;
  bool ok = false;                   // false: peers not reachable, use staging copies
  std::vector<const void*> key;      // the local senders (exchanger ids) and buffers the table was built for
  int32_t* d_bid = nullptr;
  int64_t* d_elem = nullptr;
  void** d_bases = nullptr;
  // host copies: a graph capture gives the graph its own device copies
  // (the cached tables may be rebuilt while the graph still replays)
  std::vector<int32_t> h_bid;
  std::vector<int64_t> h_elem;
  std::vector<void*> h_bases;
};

struct pa_xchg {
  pa_ctx* ctx = nullptr;
  uint64_t id = 0;                             // unique per exchanger of the process (cache keys)
  pa_pull pull[2];                             // [0] forward, [1] reverse
  // direct pull of mul! over parts sharing one stream pair (spmv_grouped):
  // receive slot p reads x of the call's part bid[p] at lid elem[p] (the
  // sender's lids_snd entry), no pack, no send buffer, no cross-stream event
  pa_pull direct;
  std::vector<int32_t> h_lids_snd;             // 0-based host copy (vector exchangers)
  std::vector<int32_t> parts_rcv, parts_snd;   // 1-based
  std::vector<int64_t> ptrs_rcv, ptrs_snd;     // 0-based offsets, size n+1
  int64_t n_rcv_data = 0, n_snd_data = 0;
  int64_t max_lid = -1;                        // 0-based, over both lists
  int32_t* d_lids_rcv = nullptr;               // 0-based
  int32_t* d_lids_snd = nullptr;
  void* d_buf_rcv = nullptr;                   // 16 B per slot
  void* d_buf_snd = nullptr;
  // the barrier issue of stream-pair mul! (spmv_impl): a second forward send
  // buffer, used every other call, and the pull table against the senders'
  // second buffers; the last barrier call these exchangers took part in
  // (key of its exchanger set, its sequence number, the buffer it packed)
  void* d_buf_snd2 = nullptr;
  pa_pull pull_alt;
  uint64_t fast_key = 0, fast_seq = 0;
  int fast_parity = 0;
  pa_combine_plan plan_fwd;   // unpack targets = lids_rcv
  pa_combine_plan plan_rev;   // unpack targets = lids_snd (reverse/assemble)
};

constexpr size_t kVecPad = 64;  // bytes before and after a vector's values (pa_vec_create)

// COO triplets of one part on the device (global row/column ids, Int64),
// the input of async_assemble!(I, J, V, rows) and PSparseMatrix(I, J, V, …)
struct pa_coo {
  pa_ctx* ctx = nullptr;
  int dtype = PA_F64;
  int64_t n = 0;
  int64_t* d_I = nullptr;
  int64_t* d_J = nullptr;
  void* d_V = nullptr;
};

struct pa_vec {
  pa_ctx* ctx = nullptr;
  int dtype = PA_F64;
  int64_t n = 0;
  void* d = nullptr;      // the values (base + kVecPad)
  void* base = nullptr;   // the allocation (owned; null for views)
};

// int32 words of a pattern slice's descriptor (dedup_patterns, SPMV_DESC):
// 4 header words + the slice's H/64 64-bit mask words, a power of two
constexpr int desc_words(int R) { return R <= 2 ? 8 : 16; }

struct pa_mat {
  pa_ctx* ctx = nullptr;
  int dtype = PA_F64;
  int cg_fuse_choice = -1;   // device CG with cg_fuse 2 (auto): the faster u-update variant measured on this matrix
  int R = 2;                 // rows per lane
  int H = 128;               // rows per slice = 64*R
  int64_t nrows = 0;         // owned rows
  int64_t ncols_lids = 0;    // x length expected
  int64_t nnz = 0;           // owned-row nonzeros
  int64_t slots = 0;         // SELL slots incl. padding
  int64_t nslices = 0;
  int64_t nslices_int = 0;   // slices without ghost-column entries
  bool csr = false;          // built from a SparseMatrixCSR: α scales each product, (v*x)*α (SparseUtils.jl:247)
  std::vector<int32_t> h_slen;      // host copies for pa_mat_traffic: int32-layout slice lengths,
  std::vector<int32_t> h_kind;      // pattern-layout slice kinds (0 int32, 1 pattern, 3 delta16)
  std::vector<int32_t> h_plen;      // and entries per row of each pattern-layout slice
  // longest row of each launch kind (SH kernels when <= 8): pattern slices,
  // int32 slices (of the current encoding), side SELL
  int maxlen_all = INT32_MAX, maxlen_pm_int = INT32_MAX, maxlen_pat = INT32_MAX, maxlen_side = INT32_MAX;
  int64_t* d_slice_off = nullptr;   // nslices (slot offset of each slice)
  int32_t* d_slice_len = nullptr;   // nslices (entries per row, max over slice)
  int32_t* d_int_list = nullptr;    // interior slice ids (null: all interior 0..n-1)
  int32_t* d_bnd_list = nullptr;    // boundary slice ids
  int32_t* d_col = nullptr;         // slots, x lid (0-based) or -1 padding
  void* d_val = nullptr;            // slots, then n_gnz ghost-row values
  // CSC nz p → its value: main slot (>= 0) or ghost-row value g (-(g+1)).
  // The ghost rows' nonzeros (stored by FE assembly, never multiplied) sit
  // after the SELL slots in d_val: the nz exchange/assemble (matrix
  // exchanger, Interfaces.jl:2312-2404) addresses both through one index.
  // Built by pa_mat_from_coo, the map stays on the device (d_nz_slot) until
  // a call that needs it on the host (set/get values, matrix exchanger).
  std::vector<int64_t> h_nz_slot;
  int64_t* d_nz_slot = nullptr;
  bool nz_map = false;              // built from a CSC pattern
  int64_t csc_nnz = 0;
  int64_t n_gnz = 0;
  // long rows (row-length histogram): their own CSR, values in d_val at
  // long_off = slots + n_gnz; CSC nz of a long row: h_nz_slot = -(n_gnz+t+1)
  int64_t n_long = 0, n_lnz = 0, long_off = 0;
  int32_t* d_long_row = nullptr;     // oids, ascending
  int64_t* d_long_ptr = nullptr;     // n_long+1
  int32_t* d_long_col = nullptr;     // x lids, reference order per row
  int32_t* d_sflags = nullptr;       // per slice: 1 if it holds long rows (int32 path skips them)
  uint64_t* d_lmask = nullptr;       // nslices*(H/64) bits: long rows
  std::vector<int32_t> h_long_rows;  // sorted oids (excluded from the side SELL)
  // chunks of the long rows (long_rows_exact = 0): chunk c covers long-CSR
  // entries [lchunk_start[c], lchunk_start[c+1]); row i owns chunks
  // [lrow_chunk[i], lrow_chunk[i+1]); one partial per chunk in d_lpart
  int64_t n_lchunks = 0;
  int64_t* d_lchunk_start = nullptr;
  int64_t* d_lrow_chunk = nullptr;
  void* d_lpart = nullptr;

  // Pattern slices (implied columns): in a pattern slice the
  // rows whose column sequence is `row + pat[k]` (k < plen) are "regular"
  // (mask bit set) and need no column ids; the other rows of the slice are
  // computed from the side SELL below.  Values keep their int32-SELL slots.
  bool has_pat = false;
  int kmax = 0;                      // pattern stride per slice
  int32_t* d_kind = nullptr;         // per slice: 1 pattern, 0 int32 columns
  int32_t* d_pdesc = nullptr;        // per slice desc_words(R) int32: {offset / H, d_plen, 0, 0, mask words} (SPMV_DESC)
  int32_t* d_plen = nullptr;         // per slice: entries per row (int32 len; pattern slices: len (bits 0-7) | tri flag (bit 8) | pattern id << 9)
  int32_t* d_pat = nullptr;          // npatterns*kmax offsets: the distinct patterns (dedup_patterns)
  int64_t npatterns = 0;
  // XCD run length of this matrix's per-kind launches in spmv_xcd_chunk's
  // auto mode (dedup_patterns: the pattern's reach in blocks / 8), 0 = none
  int xcd_auto = 0;
  uint64_t* d_mask = nullptr;        // nslices*(H/64) regular-row bits
  int32_t* d_pint_list = nullptr;    // pattern mode: pattern slices without ghost reads
  int32_t* d_pbnd_list = nullptr;    // pattern mode: pattern slices reading ghosts
  int64_t np_int = 0, np_bnd = 0;
  int32_t* d_xint_list = nullptr;    // pattern mode: int32-column slices without ghost columns
  int32_t* d_xbnd_list = nullptr;    // pattern mode: int32-column slices with ghost columns
  int64_t nx_int = 0, nx_bnd = 0;
  int64_t npattern_slices = 0, nregular_rows = 0;
  // delta16 slices (kind 3): int32-column slices whose columns all fit a
  // 16-bit code (pa_tune "spmv_delta16"): an owned column c of row r as
  // c - r in 15 signed bits, a ghost column as the slice's ghost base +
  // 15 unsigned bits (bit 15 set), 0xFFFF padding — 2 B per slot instead of 4
  uint16_t* d_col16 = nullptr;       // slots (codes of the delta16 slices)
  int32_t* d_gbase = nullptr;        // per slice: smallest ghost column
  int32_t* d_dint_list = nullptr;    // delta16 slices without ghost columns
  int32_t* d_dbnd_list = nullptr;    // delta16 slices with ghost columns
  int64_t nd_int = 0, nd_bnd = 0;
  int maxlen_d16 = INT32_MAX;
  // side SELL: the irregular rows of pattern slices (row map → oid)
  int64_t s_nrows = 0, s_nslices = 0, s_slots = 0;
  int64_t* d_s_off = nullptr;
  int32_t* d_s_len = nullptr;
  int32_t* d_s_col = nullptr;
  void* d_s_val = nullptr;
  int32_t* d_s_rowmap = nullptr;
  int32_t* d_s_rowlen = nullptr;
  // Triple SELL (pa_tune "spmv_tri16"): the rows of the
  // delta16 slices, re-sliced by class — rows whose column list is
  // consecutive triples (c, c+1, c+2) first, then the other rows, each class
  // by length (descending) and oid — with a row map.  A "tri" slice (every
  // row regular, length % 3 == 0) keeps one 16-bit code per triple and its
  // lane reads a triple's x as one run; the other slices keep one code per
  // entry.  Rows of a slice are interleaved (row i at lane i % 64, position
  // i / 64).  Values are copies of the main slots (refreshed with the side
  // SELL); the main delta16 slices are not launched then (host kind 5).
  int64_t t_nrows = 0, t_nslices = 0, t_slots = 0, t_tri_slices = 0, t_tri_rows = 0, t_code_slots = 0;
  int64_t* d_t_off = nullptr;        // slot offset per slice
  int32_t* d_t_len = nullptr;        // entries per row (max over the slice), bit 30: tri slice (kTriSlice), bit 29: pair slice
  uint16_t* d_t_col16 = nullptr;     // codes (tri slices: one per triple, slot groups 0..len/3-1)
  void* d_t_val = nullptr;           // values (lane-major packs of R, like the main SELL; t_pack: tri slices per triple)
  int t_pack = 0;                    // slices of 2 rows per lane (spmv_tri_pack): bit 2 pair slices; bit 0 (Float32)
                                     // a pair slice's triple t as {entries 0,1 × R rows} 16 B + {entry 2} 8 B per lane
  int64_t t_pair_slices = 0, t_pair_rows = 0;  // pair slices and the rows they hold
  // the uniform layout of short pattern rows (build_uniform): K = |U| <= 7
  // entries per row at slice * H * K, U's offsets, pattern id -> U position
  void* d_uval = nullptr;
  int32_t* d_uemap = nullptr;
  int uK = 0;
  int32_t upat[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int32_t* d_t_gbase = nullptr;      // per slice: smallest ghost column
  int32_t* d_t_desc = nullptr;       // per slice {offset / H, d_t_len, d_t_gbase, 0} (SPMV_DESC)
  int32_t* d_t_rowmap = nullptr;     // structure row → oid
  int64_t* d_t_src = nullptr;        // structure row → its main-layout slot of entry 0 (entry k: + k*64*R)
  int32_t* d_t_rowlen = nullptr;     // structure row → its entries
  int32_t* d_t_int_list = nullptr;   // slices without ghost reads
  int32_t* d_t_bnd_list = nullptr;   // slices reading ghosts
  int64_t nt_int = 0, nt_bnd = 0;
  int maxlen_t = INT32_MAX;
  std::vector<int32_t> h_t_len;      // host copies for pa_mat_traffic
  void* d_dotp = nullptr;            // fused dot: one partial per (main + side + triple) slice and long row
};
