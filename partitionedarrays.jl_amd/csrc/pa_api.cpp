// pa_api.cpp — host side of libpa_hip.so: the C-ABI declared in
// include/pa_hip.h.  Contexts, index sets, the halo plan, the one-time
// CSC → SELL conversion, the halo transport (device copies between parts of
// one process, RCCL send/recv between processes) and the reductions' fold.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <unordered_map>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "pa_internal.h"

namespace pa {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// kernels (pa_spmv.hip, pa_kernels.hip)
void launch_spmv_part(int which, int64_t nwork, const int32_t* list, const pa_mat* A, const void* x,
                      void* y, const int32_t* ymap, bool has_alpha, int bmode, const void* alpha,
                      const void* beta, void* dotp, hipStream_t st,
                      const SpmvPart* cgp = nullptr);
void launch_delta16(pa_mat* A, int64_t noids, const int32_t* kind, int32_t* ok, hipStream_t st);
void launch_pattern_detect(pa_mat* A, int64_t noids, int min_pct, int32_t* kind, int32_t* plen, int32_t* pat,
                           uint64_t* mask, int32_t* pghost, int32_t* nirreg, hipStream_t st);
void launch_side_len(pa_mat* A, int64_t n, const int32_t* rows, int32_t* len, int64_t noids,
                     int32_t* sghost, hipStream_t st);
void launch_side_fill(pa_mat* A, const int32_t* rows, const int32_t* len, hipStream_t st);
void launch_fold(int cplx, int nb, const void* in, void* scratch, void* out, unsigned* ticket, hipStream_t st);
void launch_fold_cg_alpha(int dtype, int nb, const void* in, void* scratch, void* out, unsigned* ticket,
                          CGState* cst, hipStream_t st);
void launch_fold_cg_step(int dtype, int nb, const void* in, void* scratch, void* out, unsigned* ticket,
                         CGState* cst, double* history, hipStream_t st);
void launch_cg_xr(int dtype, int64_t n, int64_t noids, const int32_t* own, void* x, void* r, const void* u,
                  const void* c, const void* alpha, const CGState* cst, double* part, int nb, hipStream_t st);
void launch_cg_xu(int dtype, int64_t n, void* x, void* u, const void* r, const CGState* cst, hipStream_t st);
void launch_cg_ghost(int dtype, int64_t lo, int64_t hi, const void* r, const void* uo, void* un, void* x,
                     const CGState* cst, hipStream_t st);
void launch_cg_alpha(int dtype, int P, const void* gathered, CGState* cst, hipStream_t st);
void launch_cg_step(int dtype, int P, const double* gathered, CGState* cst, double* history, hipStream_t st);
void launch_gather_ptrs(int P, const void* const* srcs, int accsz, void* out, hipStream_t st);
void launch_gather_scatter(int P, const void* const* srcs, int accsz, int nd, void* const* dsts, hipStream_t st);
// Process defaults of the tuning knobs (pa_tune; the per-call Knobs of
// pa_internal.h).  Why each default:
//  * halo_pull 1: pull-unpack between parts of one process;
//  * spmv_group 1: one launch per phase for the parts sharing a stream pair;
//  * spmv_delta16 1: int32-column slices with 16-bit column codes where they fit;
//  * spmv_merge 1: one launch for every slice kind of every part when no halo is in flight;
//  * spmv_merge_max 65536: ... unless one part alone has more slices than
//    this: such a part fills the GPU many times over, and one launch per kind
//    (the kind's own kernel, fewer registers) is faster — FE27 256³ F64 −1.0 %,
//    F32 −2.8 %; C2 (16 k slices) and C5 stay merged (−10 % / −15 %).
//    profiles/r02/open/ab_merge.jsonl; r04 again: F64 −0.6 %, F32 ±0
//    (profiles/r04/an/).  0: no limit;
//  * pattern_min_regular 0 (auto): % of a slice's rows that must follow its
//    pattern for a pattern slice (the others become side rows); auto = 70 %
//    for slices of 128 rows, 50 % for Float32's 256-row slices.  A/B on C5
//    (profiles/r04/y/, copies per variant): F64 50 % 0.1195 ms, 70 % 0.1131,
//    90 % 0.1124 (the side SELL's duplicate values and ids gone: 621 -> 589 MB
//    per mul!); F32 0.0737 / 0.0725 / 0.0742 (within noise); 30 % +11 % / +6 %.
//    A 256-row Float32 slice of a structured grid at 128³ spans two x-lines,
//    one of them on a domain face (its own pattern): 50 % keeps it a pattern
//    slice (FD7 128³: all 8192 slices).  FE27 / FD7 slices of one x-line and
//    Cartesian parts are >= 99 % regular either way;
//  * issue_threads 1: 1 auto (several devices), 2 always, 0 never;
//  * halo_direct 1: grouped mul! pulls ghosts straight from the owners' x;
//  * halo_transport 0: parts of this process by device reads, 1 RCCL for all;
//  * cg_fuse 2: the device CG's u update inside the SpMV (XV kernels) or its
//    own sweep.  Steady-state iteration on FE27 256³, sweep vs fused, on four
//    boxes: 0.958 / 1.080, 0.947 / 0.973, 0.917 / 0.882, whole call 1.043 /
//    1.075 ms (profiles/r03/s, final, f, d) — the fused SpMV gathers two
//    vectors (r and u_old) per x value — so 2 = measure one batch of each on
//    this box and keep the faster (pa_cg_solve_all);
//  * spmv_flags 223, spmv_format 1, long_rows_exact 1: pa_spmv.hip.
const Knobs kDefaults = {
    /*spmv_flags*/ 223, /*long_exact*/ 1, /*halo_pull*/ 1, /*spmv_delta16*/ 1, /*spmv_merge*/ 1,
    /*spmv_merge_max*/ 65536, /*cg_fuse*/ 2, /*halo_direct*/ 1, /*halo_transport*/ 0, /*spmv_group*/ 1,
    /*spmv_format*/ 1, /*pattern_min_pct*/ 0, /*issue_threads*/ 1, /*fault_inject*/ 0, /*spmv_xcd_chunk*/ -1, /*spmv_tri16*/ 1,
    /*halo_barrier*/ 1, /*tri_order*/ 1, /*side_tail*/ 1, /*f32_rows*/ 0, /*tri_pack*/ 7, /*uniform*/ 1};
// COO → CSC → SELL on the device (pa_coo.hip)
int coo_compress(int dtype, int index_bytes, int64_t m, int64_t ncols, int64_t n, const void* dI, const void* dJ,
                 const void* dV, int csr, int64_t* nu_out, int32_t** crow, int32_t** ccol, void** cval,
                 int64_t** colptr, hipStream_t st, hipError_t* err_out);
int coo_row_order(int64_t nu, const int32_t* crow, const int32_t* ccol, const int32_t* rl2o, const int32_t* cl2o,
                  int64_t nrows, int64_t noids_c, int64_t ncols, int H, uint64_t** key2, int64_t** idx2,
                  int64_t** rowptr, int64_t** gflag, int64_t** grank, int32_t** slen, int32_t** sghost,
                  int64_t* nnz_out, int64_t* ngh_out, hipStream_t st, hipError_t* err_out);
void coo_slices(int64_t ns, int64_t nrows, int H, const int64_t* rowptr, const uint64_t* key2, int64_t ncols,
                int64_t noids_c, const int32_t* lidx, int32_t* slen, int32_t* sghost, hipStream_t st);
void coo_fill(int dtype, int64_t nnz, int64_t nu, const uint64_t* key2, const int64_t* idx2, const int64_t* rowptr,
              const int64_t* soff, int H, int R, int64_t ncols, const int32_t* ccol, const void* cval,
              const int64_t* gflag, const int64_t* grank, int64_t slots, int32_t* col, void* val, int64_t* nz_slot,
              const int32_t* lidx, const int64_t* lptr, int32_t* lcol, int64_t long_off, hipStream_t st);
void launch_fill_i32(int64_t n, int32_t* a, int32_t v, hipStream_t st);
void launch_spmv_long(const pa_mat* A, const void* x, void* y, const int32_t* ymap, bool has_alpha, int bmode,
                      const void* alpha, const void* beta, void* dotp, int64_t dot_base, hipStream_t st);
int gid_table(int64_t n, const int64_t* d_lid_to_gid, uint64_t** sgid, int64_t** slid, hipStream_t st);
int gids_to_lids(int64_t n, int64_t* ids, const uint64_t* sgid, const int64_t* slid, int64_t nl, hipStream_t st);
int coo_assemble_pack(int dtype, int64_t n, const int64_t* I, const int64_t* J, void* V, const uint64_t* sgid,
                      const int64_t* slid, int64_t nl, const std::vector<int32_t>& lid_to_ohid, int nseg,
                      const int32_t* d_lids_rcv, const std::vector<int64_t>& ptrs_rcv, int64_t** sI, int64_t** sJ,
                      void** sV, std::vector<int64_t>* cnt, hipStream_t st);
int gids_first_touch(int64_t n, const int64_t* gids, const uint64_t* sgid, const int64_t* slid, int64_t nl,
                     int64_t** out, int64_t* m_out, hipStream_t st);
// ev (optional): recorded on st when the kernel completes (one runtime call)
void launch_pack(int dtype, int64_t n, const int32_t* lids, const void* v, void* buf,
                 hipStream_t st, hipEvent_t ev = nullptr);
void launch_unpack(int dtype, int64_t n, const int32_t* lids, const pa_combine_plan& plan, int op,
                   const void* buf, void* v, hipStream_t st);
void launch_pull(int dtype, int64_t n, const int32_t* lids, const pa_combine_plan& plan, int op, const int32_t* bid,
                 const int64_t* elem, const void* const* bases, void* v, hipStream_t st, hipEvent_t ev = nullptr);
void launch_fill(int dtype, int64_t n, int64_t base, const int32_t* map, void* v, const void* s,
                 hipStream_t st);
int launch_spmv_merged(int n, const int* which, const SpmvPart* parts, bool has_alpha, int bmode,
                       const void* alpha, const void* beta, pa_ctx* owner,
                       hipStream_t st);
void launch_spmv_group(int which, int np, const SpmvPart* parts, bool has_alpha, int bmode, const void* alpha,
                       const void* beta, hipStream_t st);
void launch_pack_group(int dtype, const PackGroup& g, hipStream_t st);
void launch_pull_group(int dtype, const PullGroup& g, hipStream_t st);
void launch_copy(int dtype, int64_t n, const int32_t* dmap, void* d, const int32_t* smap,
                 const void* s, hipStream_t st);
void launch_axpby(int dtype, int64_t n, const int32_t* map, void* y, const void* x, const void* a,
                  int mode, hipStream_t st, int sk = 0);
void launch_reduce(int dtype, int kind, int64_t n, const int32_t* ma, const void* a,
                   const int32_t* mb, const void* b, void* partials, void* result,
                   unsigned* ticket, hipStream_t st);
void launch_stencil_count(const StencilGeom& g, const int32_t* shell, const double* coef,
                          int64_t nrows, int noids, int H, int32_t* slen, int32_t* sghost,
                          int32_t* err, hipStream_t st);
void launch_stencil_fill(const StencilGeom& g, const int32_t* shell, const double* coef,
                         int64_t nrows, int noids, pa_mat* A, int32_t* err, hipStream_t st);
void launch_probe(int copy, int unroll, int64_t n16, const void* a, void* b, int blocks, hipStream_t st);
void launch_invalid_config();
void launch_t_rowinfo(const pa_mat* A, int64_t n, const int32_t* rows, int64_t noids, int32_t* info, hipStream_t st);
void launch_t_pairinfo(const pa_mat* A, int64_t n, const int32_t* rows, int32_t* pairable, hipStream_t st);
void launch_u_fill(const pa_mat* A, hipStream_t st);
void launch_t_gbase(const pa_mat* A, int64_t noids, int32_t* ok, hipStream_t st);
void launch_t_fill(const pa_mat* A, int64_t noids, bool codes, hipStream_t st);
void launch_t_check(const pa_mat* A, unsigned* bad, hipStream_t st);

}  // namespace pa

using namespace pa;

#define PA_FAIL(msg)             \
  do {                           \
    pa::set_error(msg);          \
    return -1;                   \
  } while (0)

#define HIPC(expr)                                                                       \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      pa::set_error(std::string(#expr) + " failed: " + hipGetErrorString(e_));           \
      return -1;                                                                         \
    }                                                                                    \
  } while (0)

#define NCCLC(expr)                                                                      \
  do {                                                                                   \
    ncclResult_t r_ = (expr);                                                            \
    if (r_ != ncclSuccess) {                                                             \
      pa::set_error(std::string(#expr) + " failed: " + ncclGetErrorString(r_));          \
      return -1;                                                                         \
    }                                                                                    \
  } while (0)

#define CHECK_ARG(cond, msg) \
  do {                       \
    if (!(cond)) PA_FAIL(msg); \
  } while (0)

namespace {

template <typename T>
int dev_upload(T** dptr, const std::vector<T>& h) {
  *dptr = nullptr;
  if (h.empty()) return 0;
  HIPC(hipMalloc((void**)dptr, h.size() * sizeof(T)));
  HIPC(hipMemcpy(*dptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

void dev_free(void* p) {
  if (p) (void)hipFree(p);
}

bool valid_dtype(int dt) { return dt == PA_F32 || dt == PA_F64 || dt == PA_C64 || dt == PA_C128; }

// scalar helpers on host values of a dtype
bool scalar_is(int dt, const void* s, double re) {
  switch (dt) {
    case PA_F32: return *(const float*)s == (float)re;
    case PA_F64: return *(const double*)s == re;
    case PA_C64: { const float* f = (const float*)s; return f[0] == (float)re && f[1] == 0.f; }
    case PA_C128: { const double* d = (const double*)s; return d[0] == re && d[1] == 0.0; }
  }
  return false;
}

// Build an ordered combine plan for unpack targets `lids` (0-based, buffer order).
int build_plan(const std::vector<int32_t>& lids, pa_combine_plan* plan) {
  const int64_t n = (int64_t)lids.size();
  std::vector<int32_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return lids[a] < lids[b]; });
  std::vector<int32_t> target, ptr{0}, pos;
  pos.reserve(n);
  for (int64_t i = 0; i < n; ++i) {
    const int32_t l = lids[order[i]];
    if (target.empty() || target.back() != l) {
      if (!target.empty()) ptr.push_back((int32_t)pos.size());
      target.push_back(l);
    }
    pos.push_back(order[i]);
  }
  if (!target.empty()) ptr.push_back((int32_t)pos.size());
  plan->ntargets = (int64_t)target.size();
  plan->unique = plan->ntargets == n;
  if (!plan->unique) {
    if (dev_upload(&plan->d_target, target)) return -1;
    if (dev_upload(&plan->d_ptr, ptr)) return -1;
    if (dev_upload(&plan->d_pos, pos)) return -1;
  }
  return 0;
}

void free_plan(pa_combine_plan& p) {
  dev_free(p.d_target);
  dev_free(p.d_ptr);
  dev_free(p.d_pos);
  p = pa_combine_plan{};
}

// Row-length histogram → long rows: a row is long when it has more than
// max(kLongMin, 8 × the 90th-percentile length) entries.  Such rows would pad
// every row of their SELL slice to their length; they run in k_spmv_long.
constexpr int32_t kLongMin = 256;
int32_t long_threshold(const std::vector<int32_t>& len) {
  if (len.empty()) return INT32_MAX;
  std::vector<int32_t> t(len);
  const size_t k = (t.size() * 9) / 10;
  std::nth_element(t.begin(), t.begin() + k, t.end());
  const int64_t thr = std::max<int64_t>(kLongMin, 8 * (int64_t)t[k]);
  return (int32_t)std::min<int64_t>(thr, INT32_MAX);
}

// device arrays of the long rows (rows ascending, CSR pointers) and the
// per-slice skip mask of the int32 kernel
int upload_long(pa_mat* A, const std::vector<int32_t>& lrows, const std::vector<int64_t>& lptr,
                const std::vector<int32_t>& lcol) {
  A->n_long = (int64_t)lrows.size();
  A->h_long_rows = lrows;
  if (A->n_long == 0) return 0;
  const int64_t ns = (A->nrows + A->H - 1) / A->H, W = A->H / 64;
  std::vector<int32_t> sflags(ns, 0);
  std::vector<uint64_t> lmask(ns * W, 0);
  for (int32_t r : lrows) {
    const int64_t s = r / A->H, i = r - s * A->H;
    sflags[s] = 1;
    lmask[s * W + i / 64] |= 1ull << (i & 63);
  }
  if (dev_upload(&A->d_long_row, lrows) || dev_upload(&A->d_long_ptr, lptr) || dev_upload(&A->d_sflags, sflags) ||
      dev_upload(&A->d_lmask, lmask))
    return -1;
  // chunks for the parallel (non-exact) mode: consecutive kLongChunk
  // entries; chunk c ends where chunk c+1 starts (the last at lptr.back())
  constexpr int64_t kLongChunk = 4096;
  std::vector<int64_t> cstart, rchunk{0};
  for (size_t i = 0; i < lrows.size(); ++i) {
    for (int64_t b = lptr[i]; b < lptr[i + 1]; b += kLongChunk) cstart.push_back(b);
    rchunk.push_back((int64_t)cstart.size());
  }
  A->n_lchunks = (int64_t)cstart.size();
  cstart.push_back(lptr.back());
  if (dev_upload(&A->d_lchunk_start, cstart) || dev_upload(&A->d_lrow_chunk, rchunk)) return -1;
  HIPC(hipMalloc(&A->d_lpart, std::max<int64_t>(A->n_lchunks, 1) * 16));
  if (!lcol.empty() && dev_upload(&A->d_long_col, lcol)) return -1;
  return 0;
}

inline bool is_long_row(const pa_mat* A, int64_t r) {
  return A->n_long > 0 && std::binary_search(A->h_long_rows.begin(), A->h_long_rows.end(), (int32_t)r);
}

inline int64_t nvals(const pa_mat* A) { return A->slots + A->n_gnz + A->n_lnz; }

int finish_sell_layout(pa_mat* A, const std::vector<int32_t>& slen, const std::vector<char>& sghost,
                       std::vector<int64_t>* soff_out) {
  const int64_t ns = (int64_t)slen.size();
  std::vector<int64_t> soff(ns);
  int64_t acc = 0;
  for (int64_t s = 0; s < ns; ++s) {
    soff[s] = acc;
    acc += (int64_t)slen[s] * A->H;
  }
  A->slots = acc;
  A->nslices = ns;
  A->h_slen = slen;
  A->maxlen_all = 0;
  for (int32_t l : slen) A->maxlen_all = std::max(A->maxlen_all, (int)l);
  std::vector<int32_t> ilist, blist;
  for (int64_t s = 0; s < ns; ++s) (sghost[s] ? blist : ilist).push_back((int32_t)s);
  A->nslices_int = (int64_t)ilist.size();
  if (dev_upload(&A->d_slice_off, soff)) return -1;
  if (dev_upload(&A->d_slice_len, slen)) return -1;
  if (!blist.empty()) {
    if (dev_upload(&A->d_int_list, ilist)) return -1;
    if (dev_upload(&A->d_bnd_list, blist)) return -1;
  }
  if (soff_out) *soff_out = std::move(soff);
  return 0;
}

// The pattern slices' offset lists as a table of the distinct ones (a
// Cartesian part has a handful: interior rows, the boundary planes' Dirichlet
// rows): d_pat becomes that table and d_plen[s] of a pattern slice packs
// its entries per row (bits 0-7, <= 255 by detection), the triple flag
// (bit 8: every entry group is a consecutive column triple) and its table
// row (bits 9-30).  A wave's pattern load then hits a small hot table instead of
// one cold row per slice, and the slice metadata shrinks by kmax*4 B each.
// A/B (one row per slice vs the table, profiles/r04/g/ab_pattern_dedup.jsonl):
// FE27 256³ 0.6539 -> 0.6407 ms, FD7 128³ 0.02865 -> 0.02833 ms.
// The uniform layout of short pattern rows (pa_tune "spmv_uniform", Float64
// with 2 rows per lane and patterns of at most 7 entries: FD7, C2): the
// union U of the distinct patterns' offsets (K <= 7 entries, ascending;
// every pattern is a subsequence of it), and the pattern slices' values
// again at slice s * H * K, entry k of the slice's pattern at U's position
// e(k) (the others 0, never multiplied).  A wave of the short-row tail
// launch then knows its values' and x runs' addresses from its slice index
// and U alone and issues them before its descriptor arrives; the
// descriptor's word 2 (emask: which of U's entries the slice's pattern
// holds) and mask only select the terms (rows_pattern_u).
void free_uniform(pa_mat* A) {
  dev_free(A->d_uval);
  dev_free(A->d_uemap);
  A->d_uval = nullptr;
  A->d_uemap = nullptr;
  A->uK = 0;
}

int build_uniform(pa_mat* A, const std::vector<int32_t>& kind, const std::vector<int32_t>& table,
                  const std::vector<int32_t>& packed, std::vector<int32_t>& desc) {
  free_uniform(A);
  if (!knobs().spmv_uniform || A->dtype != PA_F64 || A->R != 2 || A->npatterns == 0) return 0;
  const int64_t ns = A->nslices, K0 = A->kmax, np = A->npatterns;
  std::vector<int32_t> plen(np, 0);
  for (int64_t s = 0; s < ns; ++s)
    if (kind[s] == 1) plen[packed[s] >> 9] = packed[s] & 0xff;
  std::vector<int32_t> U;
  for (int64_t p = 0; p < np; ++p)
    for (int32_t k = 0; k < plen[p]; ++k) U.push_back(table[p * K0 + k]);
  std::sort(U.begin(), U.end());
  U.erase(std::unique(U.begin(), U.end()), U.end());
  if (U.size() > 7 || U.empty()) return 0;
  const int K = (int)U.size();
  std::vector<int32_t> emap(np * 8, 0), emask(np, 0);
  for (int64_t p = 0; p < np; ++p)
    for (int32_t k = 0; k < plen[p]; ++k) {
      const int e = (int)(std::lower_bound(U.begin(), U.end(), table[p * K0 + k]) - U.begin());
      CHECK_ARG(k == 0 || e > emap[p * 8 + k - 1], "uniform layout: a pattern out of column order (internal error)");
      emap[p * 8 + k] = e;
      emask[p] |= 1 << e;
    }
  const int DW = desc_words(A->R);
  for (int64_t s = 0; s < ns; ++s)
    if (kind[s] == 1) desc[DW * s + 2] = emask[packed[s] >> 9];
  hipStream_t st = A->ctx->s_main;
  const size_t S = dtype_size(A->dtype);
  if (dev_upload(&A->d_uemap, emap)) return -1;
  HIPC(hipMalloc(&A->d_uval, (size_t)ns * A->H * K * S));
  HIPC(hipMemsetAsync(A->d_uval, 0, (size_t)ns * A->H * K * S, st));
  A->uK = K;
  for (int e = 0; e < 8; ++e) A->upat[e] = e < K ? U[e] : 0;
  launch_u_fill(A, st);
  HIPC(hipGetLastError());
  return 0;
}

int dedup_patterns(pa_mat* A, const std::vector<int32_t>& kind) {
  const int64_t ns = A->nslices, K = A->kmax;
  hipStream_t st = A->ctx->s_main;
  std::vector<int32_t> pat(ns * K);
  HIPC(hipMemcpyAsync(pat.data(), A->d_pat, ns * K * 4, hipMemcpyDeviceToHost, st));
  HIPC(hipStreamSynchronize(st));
  std::vector<int32_t> table, packed(A->h_plen);
  std::unordered_map<std::string, int32_t> ids;
  int64_t reach = 0;  // largest |column - row| of the pattern slices' patterns
  for (int64_t s = 0; s < ns; ++s) {
    if (kind[s] != 1) continue;
    const int32_t len = A->h_plen[s];
    CHECK_ARG(len >= 1 && len <= 255, "pattern slice with more than 255 entries per row");
    std::string key(reinterpret_cast<const char*>(&pat[s * K]), (size_t)len * 4);
    auto it = ids.find(key);
    int32_t id;
    if (it == ids.end()) {
      id = (int32_t)ids.size();
      CHECK_ARG(id < (1 << 22), "more than 2^22 distinct slice patterns");
      ids.emplace(std::move(key), id);
      table.insert(table.end(), pat.begin() + s * K, pat.begin() + (s + 1) * K);
      for (int32_t k = 0; k < len; ++k) reach = std::max<int64_t>(reach, std::llabs((long long)pat[s * K + k]));
    } else {
      id = it->second;
    }
    // tri: the pattern is consecutive column triples (o, o+1, o+2) — every
    // FE27 interior row — so a lane reads the three x runs of a triple with
    // two 16 B loads (rows_pattern_tri)
    bool tri = len % 3 == 0;
    for (int32_t k = 0; tri && k < len; k += 3)
      tri = pat[s * K + k + 1] == pat[s * K + k] + 1 && pat[s * K + k + 2] == pat[s * K + k] + 2;
    packed[s] = len | ((tri ? 1 : 0) << 8) | (id << 9);
  }
  A->npatterns = (int64_t)ids.size();
  // spmv_xcd_chunk auto: the pattern's reach (largest |column - row|) in
  // 4-slice blocks; runs of reach/8 blocks per XCD put a block's farthest
  // neighbour plane (FE27: the z-neighbour, N² rows away) one run-group
  // later on the same XCD, whose L2 still holds those x lines
  A->xcd_auto = (int)std::min<int64_t>(64, reach / (4 * A->H) / 8);
  dev_free(A->d_pat);
  A->d_pat = nullptr;
  if (table.empty()) table.assign(K, 0);
  if (dev_upload(&A->d_pat, table)) return -1;
  HIPC(hipMemcpyAsync(A->d_plen, packed.data(), ns * 4, hipMemcpyHostToDevice, st));
  {
    // the pattern slices' descriptors (SPMV_DESC): offset / H, the length
    // word and the mask words in one aligned record per slice, so a wave
    // reads its slice's metadata with one scalar load (FD7 128^3: 0.0287 ->
    // 0.0277 ms, profiles/r06/p/)
    std::vector<int64_t> soff(ns);
    HIPC(hipMemcpyAsync(soff.data(), A->d_slice_off, ns * 8, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    const int W = A->H / 64, DW = desc_words(A->R);
    std::vector<uint64_t> mask(ns * W);
    HIPC(hipMemcpyAsync(mask.data(), A->d_mask, ns * W * 8, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    std::vector<int32_t> desc(DW * ns, 0);
    for (int64_t s = 0; s < ns; ++s) {
      CHECK_ARG(soff[s] % A->H == 0 && soff[s] / A->H <= INT32_MAX, "slice offset outside the descriptor's range");
      desc[DW * s] = (int32_t)(soff[s] / A->H);
      desc[DW * s + 1] = packed[s];
      std::memcpy(&desc[DW * s + 4], &mask[s * W], W * 8);
    }
    if (build_uniform(A, kind, table, packed, desc)) return -1;
    dev_free(A->d_pdesc);
    A->d_pdesc = nullptr;
    if (dev_upload(&A->d_pdesc, desc)) return -1;
  }
  HIPC(hipStreamSynchronize(st));
  return 0;
}

// Pattern slices + side SELL from the int32 layout (device detection, host
// bookkeeping).  noids: owned columns (x lids >= noids are ghosts).
// The CSC nz → slot map (pa_mat_from_csc / _coo) after k_delta16 moved the
// delta16 slices' values to the interleaved layout: a slot of such a slice
// at (k, lane, r) held row w = lane*R + r, which now sits at (k, w % 64,
// w / 64).  The map moves to the host here (as load_nz_map does).
int remap_nz_interleaved(pa_mat* A, const std::vector<int32_t>& kind, hipStream_t st) {
  HIPC(hipStreamSynchronize(st));
  if (A->d_nz_slot) {
    A->h_nz_slot.resize(A->csc_nnz);
    HIPC(hipMemcpy(A->h_nz_slot.data(), A->d_nz_slot, A->csc_nnz * 8, hipMemcpyDeviceToHost));
    dev_free(A->d_nz_slot);
    A->d_nz_slot = nullptr;
  }
  const int64_t ns = A->nslices, R = A->R, H = A->H;
  std::vector<int64_t> soff(ns);
  HIPC(hipMemcpy(soff.data(), A->d_slice_off, ns * 8, hipMemcpyDeviceToHost));
  for (int64_t& slot : A->h_nz_slot) {
    if (slot < 0) continue;
    const int64_t s = (int64_t)(std::upper_bound(soff.begin(), soff.end(), slot) - soff.begin()) - 1;
    if (kind[s] != 3) continue;
    const int64_t t = slot - soff[s], k = t / H, w = t % H;  // w = lane*R + r before the move
    slot = soff[s] + (k * 64 + w % 64) * R + w / 64;
  }
  return 0;
}

void free_triple_sell(pa_mat* A) {
  for (void* p : {(void*)A->d_t_off, (void*)A->d_t_len, (void*)A->d_t_col16, A->d_t_val, (void*)A->d_t_gbase,
                  (void*)A->d_t_rowmap, (void*)A->d_t_src, (void*)A->d_t_rowlen, (void*)A->d_t_int_list,
                  (void*)A->d_t_bnd_list, (void*)A->d_t_desc})
    dev_free(p);
  A->d_t_off = nullptr;
  A->d_t_desc = nullptr;
  A->d_t_len = A->d_t_gbase = A->d_t_rowmap = A->d_t_rowlen = A->d_t_int_list = A->d_t_bnd_list = nullptr;
  A->d_t_col16 = nullptr;
  A->d_t_val = nullptr;
  A->d_t_src = nullptr;
  A->t_pack = 0;
  A->t_nrows = A->t_nslices = A->t_slots = A->t_tri_slices = A->t_tri_rows = A->t_code_slots = 0;
  A->t_pair_slices = A->t_pair_rows = 0;
  A->nt_int = A->nt_bnd = 0;
  A->h_t_len.clear();
}

// The triple SELL: the rows of the delta16 slices (kind 3),
// re-sliced — the rows whose columns are not all consecutive triples, then
// the triple rows (spmv_tri_order), each class by length (descending) and
// oid — so that most slices
// hold only triple rows and keep one 16-bit code per triple (their lanes
// read a triple's x as one run), and no row's values stream twice (unlike
// the side SELL of pattern slices).  The main delta16 slices become kind 5
// (not launched in pattern mode; spmv_format 0 still runs them as int32).
// Returns 0 without building when a slice's ghost codes would not fit.
int build_triple_sell(pa_mat* A, std::vector<int32_t>& kind, int64_t noids) {
  hipStream_t st = A->ctx->s_main;
  const int64_t ns = A->nslices, H = A->H, R = A->R;
  std::vector<int32_t> rows;
  for (int64_t s = 0; s < ns; ++s)
    if (kind[s] == 3)
      for (int64_t i = s * H; i < std::min<int64_t>(A->nrows, s * H + H); ++i) rows.push_back((int32_t)i);
  const int64_t n = (int64_t)rows.size();
  if (n == 0) return 0;
  int32_t *d_rows = nullptr, *d_info = nullptr;
  if (dev_upload(&d_rows, rows)) return -1;
  HIPC(hipMalloc((void**)&d_info, n * 4));
  launch_t_rowinfo(A, n, d_rows, noids, d_info, st);
  HIPC(hipGetLastError());
  std::vector<int32_t> info(n);
  std::vector<int64_t> soff(ns);
  HIPC(hipMemcpyAsync(info.data(), d_info, n * 4, hipMemcpyDeviceToHost, st));
  HIPC(hipMemcpyAsync(soff.data(), A->d_slice_off, ns * 8, hipMemcpyDeviceToHost, st));
  HIPC(hipStreamSynchronize(st));
  dev_free(d_rows);
  dev_free(d_info);
  constexpr int32_t kLen = (1 << 28) - 1, kReg = 1 << 28, kGhost = 1 << 29, kBad = 1 << 30;
  for (int32_t v : info)
    if (v & kBad) return 0;
  // spmv_tri_pack: 2 rows per lane only; the value packs Float32 only
  const int tpack = R == 2 ? (A->dtype == PA_F32 ? knobs().tri_pack & 5 : knobs().tri_pack & 4) : 0;
  // pair slices (spmv_tri_pack bit 2): candidate i and i + 1 (rows a, a + 1,
  // both regular, one length) pair up when row a + 1's columns are row a's
  // plus one, entry for entry (k_t_pairinfo); pairs are taken greedily in
  // oid order
  std::vector<int64_t> pairs;  // candidate index of each pair's row a
  std::vector<char> paired(n, 0);
  if (tpack & 4) {
    int32_t *d_rows2 = nullptr, *d_pair = nullptr;
    if (dev_upload(&d_rows2, rows)) return -1;
    HIPC(hipMalloc((void**)&d_pair, n * 4));
    launch_t_pairinfo(A, n, d_rows2, d_pair, st);
    HIPC(hipGetLastError());
    std::vector<int32_t> pairable(n);
    HIPC(hipMemcpyAsync(pairable.data(), d_pair, n * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    dev_free(d_rows2);
    dev_free(d_pair);
    for (int64_t i = 0; i + 1 < n; ++i)
      if (pairable[i] && !paired[i] && (info[i] & kReg) && (info[i + 1] & kReg) &&
          (info[i] & kLen) == (info[i + 1] & kLen)) {
        pairs.push_back(i);
        paired[i] = paired[i + 1] = 1;
      }
  }
  // order: the other rows, then the regular (triple) rows (spmv_tri_order 1;
  // 0: regular first); each by length (descending), then oid; then, from a
  // slice boundary, the pairs by length (descending), then oid (lane p of a
  // pair slice: row a at position p, row a + 1 at 64 + p; padding
  // positions: row map -1)
  std::vector<int64_t> ord;
  for (int64_t i = 0; i < n; ++i)
    if (!paired[i]) ord.push_back(i);
  const bool others_first = knobs().tri_order == 1;
  std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) {
    const bool ra = (info[a] & kReg) != 0, rb = (info[b] & kReg) != 0;
    if (ra != rb) return others_first ? rb : ra;
    return (info[a] & kLen) > (info[b] & kLen);
  });
  std::stable_sort(pairs.begin(), pairs.end(), [&](int64_t a, int64_t b) { return (info[a] & kLen) > (info[b] & kLen); });
  const int64_t nsingle = (int64_t)ord.size(), npairs = (int64_t)pairs.size();
  const int64_t pstart = npairs ? (nsingle + H - 1) / H * H : nsingle;  // first position of the pair slices
  const int64_t npos = npairs ? pstart + (npairs + 63) / 64 * H : nsingle;
  std::vector<int64_t> at(npos, -1);  // position -> candidate index (-1: padding)
  for (int64_t i = 0; i < nsingle; ++i) at[i] = ord[i];
  for (int64_t q = 0; q < npairs; ++q) {
    const int64_t b = pstart + q / 64 * H + q % 64;
    at[b] = pairs[q];
    at[b + 64] = pairs[q] + 1;
  }
  const int64_t tns = (npos + H - 1) / H;
  std::vector<int32_t> rowmap(npos, -1), rowlen(npos, 0), tlen(tns, 0), tint, tbnd;
  std::vector<int64_t> src(npos, 0), toff(tns), nreal(tns, 0);
  std::vector<char> tri(tns, 1), ghost(tns, 0);
  for (int64_t i = 0; i < npos; ++i) {
    if (at[i] < 0) continue;
    const int32_t v = info[at[i]], row = rows[at[i]];
    const int64_t ts = i / H, s = row / H;
    const int w = (int)(row - s * H);
    rowmap[i] = row;
    rowlen[i] = v & kLen;
    // entry 0 of the row in the main layout (as k_delta16 left it, main_slot0)
    src[i] = R == 4 ? soff[s] + (int64_t)(w & 63) * R + (w >> 6) : soff[s] + (int64_t)(w / R) * R + (w % R);
    tlen[ts] = std::max(tlen[ts], rowlen[i]);
    ++nreal[ts];
    if (!(v & kReg)) tri[ts] = 0;
    if (v & kGhost) ghost[ts] = 1;
  }
  int64_t nreg = 0;
  for (int32_t v : info) nreg += (v & kReg) ? 1 : 0;
  if (4 * nreg < n) return 0;  // mostly rows without triples (e.g. FD7): the delta16 slices stay
  int64_t acc = 0, codes = 0;
  A->maxlen_t = 0;
  for (int64_t ts = 0; ts < tns; ++ts) {
    toff[ts] = acc;
    acc += (int64_t)tlen[ts] * H;
    A->maxlen_t = std::max(A->maxlen_t, (int)tlen[ts]);
    if (ts * H >= pstart && npairs) {  // pair slices (regular rows: length % 3 == 0)
      ++A->t_tri_slices;
      ++A->t_pair_slices;
      A->t_tri_rows += nreal[ts];
      A->t_pair_rows += nreal[ts];
      codes += (int64_t)tlen[ts] / 3 * 64;
      tlen[ts] |= kTriSlice | kTriPair;
    } else if (tri[ts] && tlen[ts] % 3 == 0) {
      ++A->t_tri_slices;
      A->t_tri_rows += nreal[ts];
      codes += (int64_t)tlen[ts] / 3 * H;
      tlen[ts] |= kTriSlice;
    } else {
      codes += (int64_t)tlen[ts] * H;
    }
    (ghost[ts] ? tbnd : tint).push_back((int32_t)ts);
  }
  A->t_nrows = npos;
  A->t_nslices = tns;
  A->t_pack = tpack;
  A->t_slots = acc;
  A->t_code_slots = codes;
  A->h_t_len = tlen;
  const size_t S = dtype_size(A->dtype);
  if (dev_upload(&A->d_t_off, toff) || dev_upload(&A->d_t_len, tlen) || dev_upload(&A->d_t_rowmap, rowmap) ||
      dev_upload(&A->d_t_rowlen, rowlen) || dev_upload(&A->d_t_src, src) || dev_upload(&A->d_t_int_list, tint) ||
      dev_upload(&A->d_t_bnd_list, tbnd))
    return -1;
  A->nt_int = (int64_t)tint.size();
  A->nt_bnd = (int64_t)tbnd.size();
  HIPC(hipMalloc((void**)&A->d_t_col16, std::max<int64_t>(acc, 1) * 2));
  HIPC(hipMalloc(&A->d_t_val, std::max<int64_t>(acc, 1) * S));
  // the positions past the last row of the last slice (and code groups no
  // row writes) are padding: codes 0xFFFF (column -1, never gathered), values 0
  HIPC(hipMemsetAsync(A->d_t_col16, 0xFF, std::max<int64_t>(acc, 1) * 2, st));
  HIPC(hipMemsetAsync(A->d_t_val, 0, std::max<int64_t>(acc, 1) * S, st));
  HIPC(hipMalloc((void**)&A->d_t_gbase, tns * 4));
  int32_t* d_ok = nullptr;
  HIPC(hipMalloc((void**)&d_ok, tns * 4));
  launch_t_gbase(A, noids, d_ok, st);
  HIPC(hipGetLastError());
  std::vector<int32_t> ok(tns);
  HIPC(hipMemcpyAsync(ok.data(), d_ok, tns * 4, hipMemcpyDeviceToHost, st));
  HIPC(hipStreamSynchronize(st));
  dev_free(d_ok);
  for (int32_t v : ok)
    if (!v) {  // a slice's ghost columns span more than 15 bits: keep the delta16 slices
      free_triple_sell(A);
      return 0;
    }
  {  // one 16 B descriptor per slice (SPMV_DESC): offset / H, length word, ghost base
    std::vector<int32_t> gbase(tns), desc(4 * tns, 0);
    HIPC(hipMemcpyAsync(gbase.data(), A->d_t_gbase, tns * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    for (int64_t ts = 0; ts < tns; ++ts) {
      CHECK_ARG(toff[ts] / H <= INT32_MAX, "slice offset outside the descriptor's range");
      desc[4 * ts] = (int32_t)(toff[ts] / H);
      desc[4 * ts + 1] = tlen[ts];
      desc[4 * ts + 2] = gbase[ts];
    }
    if (dev_upload(&A->d_t_desc, desc)) return -1;
  }
  launch_t_fill(A, noids, true, st);
  HIPC(hipGetLastError());
  unsigned* d_bad = nullptr;
  unsigned bad = 0;
  HIPC(hipMalloc((void**)&d_bad, 4));
  HIPC(hipMemsetAsync(d_bad, 0, 4, st));
  launch_t_check(A, d_bad, st);
  HIPC(hipGetLastError());
  HIPC(hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, st));
  HIPC(hipStreamSynchronize(st));
  dev_free(d_bad);
  CHECK_ARG(bad == 0, "triple SELL build: a column code decodes outside x (internal error)");
  for (int64_t s = 0; s < ns; ++s)
    if (kind[s] == 3) kind[s] = 5;
  return 0;
}

int finalize_pattern(pa_mat* A, int kmax, int64_t noids, bool retry_r2) {
  A->kmax = std::max(kmax, 1);
  const int64_t ns = A->nslices;
  if (ns == 0) return 0;
  hipStream_t st = A->ctx->s_main;
  const int W = A->H / 64;
  int32_t *d_pghost = nullptr, *d_nirreg = nullptr;
  HIPC(hipMalloc((void**)&A->d_kind, ns * 4));
  HIPC(hipMalloc((void**)&A->d_plen, ns * 4));
  HIPC(hipMalloc((void**)&A->d_pat, ns * A->kmax * 4));
  HIPC(hipMalloc((void**)&A->d_mask, ns * W * 8));
  HIPC(hipMalloc((void**)&d_pghost, ns * 4));
  HIPC(hipMalloc((void**)&d_nirreg, ns * 4));
  HIPC(hipMemsetAsync(A->d_mask, 0, ns * W * 8, st));
  const int min_pct = knobs().pattern_min_pct ? knobs().pattern_min_pct : (A->R == 4 ? 50 : 70);
  launch_pattern_detect(A, noids, min_pct, A->d_kind, A->d_plen, A->d_pat, A->d_mask, d_pghost, d_nirreg, st);
  HIPC(hipGetLastError());
  std::vector<int32_t> kind(ns), pghost(ns), nirreg(ns);
  std::vector<uint64_t> mask(ns * W);
  A->h_plen.resize(ns);
  HIPC(hipMemcpyAsync(A->h_plen.data(), A->d_plen, ns * 4, hipMemcpyDeviceToHost, st));
  HIPC(hipMemcpyAsync(kind.data(), A->d_kind, ns * 4, hipMemcpyDeviceToHost, st));
  HIPC(hipMemcpyAsync(pghost.data(), d_pghost, ns * 4, hipMemcpyDeviceToHost, st));
  HIPC(hipMemcpyAsync(nirreg.data(), d_nirreg, ns * 4, hipMemcpyDeviceToHost, st));
  HIPC(hipMemcpyAsync(mask.data(), A->d_mask, ns * W * 8, hipMemcpyDeviceToHost, st));
  HIPC(hipStreamSynchronize(st));
  dev_free(d_pghost);
  dev_free(d_nirreg);
  if (retry_r2 && A->dtype == PA_F32 && A->R == 4 && knobs().f32_rows == 0) {
    // f32_rows auto: a Float32 matrix with int32/delta16 slices (irregular
    // parts, C5) streams faster as 128-row slices of 8 B packs, whose delta16
    // rows take the triple SELL (C5 F32 0.0736 -> 0.0683 ms, 345 -> 289 MB);
    // a matrix of pattern slices keeps 256-row slices (FE27 256^3 F32 0.328
    // -> 0.374 ms with 128: profiles/r05/af/).  C5's parts hold 6-62 %
    // pattern slices, a stencil's parts ~100 %: the cut is 80 %
    int64_t np = 0;
    for (int64_t s = 0; s < ns; ++s) np += kind[s] == 1;
    if (5 * np < 4 * ns) return kPreferR2;
  }
  if (dedup_patterns(A, kind)) return -1;
  if (knobs().spmv_delta16) {  // int32-column slices whose columns fit 16-bit codes (kind 3)
    int32_t* d_ok = nullptr;
    HIPC(hipMalloc((void**)&A->d_col16, std::max<int64_t>(A->slots, 1) * 2));
    HIPC(hipMalloc((void**)&A->d_gbase, ns * 4));
    HIPC(hipMalloc((void**)&d_ok, ns * 4));
    launch_delta16(A, noids, A->d_kind, d_ok, st);
    HIPC(hipGetLastError());
    std::vector<int32_t> ok(ns);
    HIPC(hipMemcpyAsync(ok.data(), d_ok, ns * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    dev_free(d_ok);
    int64_t nd = 0;
    for (int64_t s = 0; s < ns; ++s)
      if (ok[s]) { kind[s] = 3; ++nd; }
    if (nd == 0) {
      dev_free(A->d_col16);
      dev_free(A->d_gbase);
      A->d_col16 = nullptr;
      A->d_gbase = nullptr;
    } else {
      // Float32 delta16 slices' rows are interleaved now (k_delta16): the
      // int32 kernel of spmv_format 0 reads the layout per slice from d_kind
      // (3), and the CSC nz → slot map follows the moved values
      HIPC(hipMemcpyAsync(A->d_kind, kind.data(), ns * 4, hipMemcpyHostToDevice, st));
      if (A->nz_map && A->R == 4 && remap_nz_interleaved(A, kind, st)) return -1;
      // the device keeps kind 3 (the int32 kernel of spmv_format 0 reads
      // the interleaved layout from it); the host marks moved slices 5
      // spmv_tri16 1: slices of R <= 2 rows per lane (Float64, complex,
      // Float32 with 2 rows per lane); Float32's 4-row interleaved delta16
      // slices already gather compactly (the triple SELL with R = 4: C5 F32
      // +3 %, F64 -10 %, profiles/r05/d/; removed r06)
      if (knobs().spmv_tri16 && A->R <= 2 && build_triple_sell(A, kind, noids)) return -1;
    }
  }
  std::vector<int32_t> pint, pbnd, xint, xbnd, dint, dbnd, side;
  for (int64_t s = 0; s < ns; ++s) {
    if (kind[s] == 1) (pghost[s] ? pbnd : pint).push_back((int32_t)s);
    else if (kind[s] == 3) (pghost[s] ? dbnd : dint).push_back((int32_t)s);
    else if (kind[s] == 0) (pghost[s] ? xbnd : xint).push_back((int32_t)s);  // (5: in the triple SELL)
    if (kind[s] == 1) {
      ++A->npattern_slices;
      const int64_t nvalid = std::min<int64_t>(A->H, A->nrows - s * A->H);
      for (int64_t i = 0; i < nvalid; ++i) {
        if ((mask[s * W + i / 64] >> (i & 63)) & 1ull) ++A->nregular_rows;
        else if (!is_long_row(A, s * A->H + i)) side.push_back((int32_t)(s * A->H + i));
      }
    }
  }
  A->h_kind = kind;
  A->maxlen_pat = A->maxlen_pm_int = A->maxlen_d16 = 0;
  for (int64_t s = 0; s < ns; ++s) {
    if (kind[s] == 1) A->maxlen_pat = std::max(A->maxlen_pat, (int)A->h_plen[s]);
    else if (kind[s] == 0) A->maxlen_pm_int = std::max(A->maxlen_pm_int, (int)A->h_slen[s]);
    else if (kind[s] == 3) A->maxlen_d16 = std::max(A->maxlen_d16, (int)A->h_slen[s]);
  }
  A->np_int = (int64_t)pint.size();
  A->np_bnd = (int64_t)pbnd.size();
  A->nx_int = (int64_t)xint.size();
  A->nx_bnd = (int64_t)xbnd.size();
  A->nd_int = (int64_t)dint.size();
  A->nd_bnd = (int64_t)dbnd.size();
  if (dev_upload(&A->d_pint_list, pint) || dev_upload(&A->d_pbnd_list, pbnd) ||
      dev_upload(&A->d_xint_list, xint) || dev_upload(&A->d_xbnd_list, xbnd) ||
      dev_upload(&A->d_dint_list, dint) || dev_upload(&A->d_dbnd_list, dbnd))
    return -1;
  // side SELL
  A->s_nrows = (int64_t)side.size();
  std::vector<int32_t> rl;  // entries per side row
  if (A->s_nrows > 0) {
    // the side rows (oids = structure rows) through d_s_rowmap
    if (dev_upload(&A->d_s_rowmap, side)) return -1;
    int32_t* srow = A->d_s_rowmap;
    int32_t* d_dummy = nullptr;
    A->s_nslices = (A->s_nrows + A->H - 1) / A->H;
    HIPC(hipMalloc((void**)&A->d_s_rowlen, A->s_nrows * 4));
    HIPC(hipMalloc((void**)&d_dummy, A->s_nslices * 4));
    HIPC(hipMemsetAsync(d_dummy, 0, A->s_nslices * 4, st));
    launch_side_len(A, A->s_nrows, srow, A->d_s_rowlen, noids, d_dummy, st);
    HIPC(hipGetLastError());
    rl.resize(A->s_nrows);
    HIPC(hipMemcpyAsync(rl.data(), A->d_s_rowlen, A->s_nrows * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    dev_free(d_dummy);
  }
  if (A->s_nrows > 0) {
    int32_t* srow = A->d_s_rowmap;
    std::vector<int32_t> slen(A->s_nslices, 0);
    std::vector<int64_t> soff(A->s_nslices);
    for (int64_t i = 0; i < A->s_nrows; ++i) slen[i / A->H] = std::max(slen[i / A->H], rl[i]);
    A->maxlen_side = 0;
    for (int32_t l : slen) A->maxlen_side = std::max(A->maxlen_side, (int)l);
    int64_t acc = 0;
    for (int64_t s = 0; s < A->s_nslices; ++s) { soff[s] = acc; acc += (int64_t)slen[s] * A->H; }
    A->s_slots = acc;
    if (dev_upload(&A->d_s_off, soff) || dev_upload(&A->d_s_len, slen)) return -1;
    const size_t S = dtype_size(A->dtype);
    HIPC(hipMalloc((void**)&A->d_s_col, std::max<int64_t>(acc, 1) * 4));
    HIPC(hipMalloc(&A->d_s_val, std::max<int64_t>(acc, 1) * S));
    launch_side_fill(A, srow, A->d_s_rowlen, st);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(st));
  }
  A->has_pat = true;
  return 0;
}

// The parts of this call, by part id → position.
struct LocalSet {
  std::vector<int> pos_of_part;  // index part (1-based) → position or -1
  int find(int part) const {
    return (part >= 1 && part < (int)pos_of_part.size()) ? pos_of_part[part] : -1;
  }
};

// The parts whose halo segments move by device copies / pull reads in this
// call.  When every part's communicator came from pa_comm_init_all (one rank
// per device of this process: HIPBackend(rccl=True)), or with
// pa_tune("halo_transport", 1) and a communicator on every part, none: every
// segment goes through the grouped ncclSend/ncclRecv, as across processes.
template <typename H>
LocalSet local_set(int n, H* const* hs) {
  LocalSet L;
  int maxp = 0;
  bool all_comm = true;
  for (int i = 0; i < n; ++i) {
    const pa_ctx* c = hs[i]->ctx;
    maxp = std::max(maxp, c->nparts);
    all_comm = all_comm && c->comm != nullptr && (c->halo_rccl || knobs().halo_transport == 1);
  }
  L.pos_of_part.assign(maxp + 1, -1);
  if (all_comm) return L;
  for (int i = 0; i < n; ++i) L.pos_of_part[hs[i]->ctx->part] = i;
  return L;
}

uint64_t g_xchg_next_id = 1;

// Pull table of receiver i for direction dir (see pa_pull): built once per
// set of local senders; ok = false when a sender's device is not reachable
// by peer access (then the staging copies below are used).  alt: the
// forward table against the senders' second send buffers (d_buf_snd2, the
// barrier issue of spmv_impl).
int build_pull(int i, int n, pa_xchg* const xg[], const LocalSet& L, int dtype, int dir, bool alt = false) {
  pa_xchg* X = xg[i];
  pa_ctx* c = X->ctx;
  pa_pull& P = alt ? X->pull_alt : X->pull[dir];
  auto sender_buf = [&](const pa_xchg* Q) -> void* {
    return alt ? Q->d_buf_snd2 : (dir == 0 ? Q->d_buf_snd : Q->d_buf_rcv);
  };
  const auto& prcv = dir == 0 ? X->parts_rcv : X->parts_snd;
  const auto& orcv = dir == 0 ? X->ptrs_rcv : X->ptrs_snd;
  void* own = dir == 0 ? X->d_buf_rcv : X->d_buf_snd;
  std::vector<const void*> key;
  key.push_back((const void*)(intptr_t)dtype_size(dtype));
  for (int32_t q : prcv) {
    const int j = L.find(q);
    key.push_back(j >= 0 ? (const void*)(uintptr_t)xg[j]->id : nullptr);
    key.push_back(j >= 0 ? sender_buf(xg[j]) : own);
  }
  if (P.built && P.key == key) return 0;
  dev_free(P.d_bid);
  dev_free(P.d_elem);
  dev_free(P.d_bases);
  P = pa_pull{};
  P.built = true;
  P.key = key;
  HIPC(hipSetDevice(c->device));
  std::vector<void*> bases;
  auto base_id = [&](void* b) {
    for (size_t t = 0; t < bases.size(); ++t)
      if (bases[t] == b) return (int32_t)t;
    bases.push_back(b);
    return (int32_t)(bases.size() - 1);
  };
  const int64_t nslots = orcv.empty() ? 0 : orcv.back();
  std::vector<int32_t> bid(nslots);
  std::vector<int64_t> elem(nslots);
  for (size_t k = 0; k < prcv.size(); ++k) {
    const int j = L.find(prcv[k]);
    const int64_t cnt = orcv[k + 1] - orcv[k];
    if (j < 0) {  // remote sender: RCCL delivers into this part's own buffer
      const int32_t b = base_id(own);
      for (int64_t t = 0; t < cnt; ++t) { bid[orcv[k] + t] = b; elem[orcv[k] + t] = orcv[k] + t; }
      continue;
    }
    pa_xchg* Q = xg[j];
    const auto& qsnd = dir == 0 ? Q->parts_snd : Q->parts_rcv;
    const auto& qo = dir == 0 ? Q->ptrs_snd : Q->ptrs_rcv;
    int m = -1;
    for (size_t t = 0; t < qsnd.size(); ++t)
      if (qsnd[t] == c->part) { m = (int)t; break; }
    CHECK_ARG(m >= 0, "exchanger mismatch: a receiver lists a sender that does not send to it");
    CHECK_ARG(cnt == qo[m + 1] - qo[m], "exchanger mismatch: segment lengths differ (SequentialBackend.jl:187)");
    const int qdev = Q->ctx->device;
    if (qdev != c->device) {
      int can = 0;
      HIPC(hipDeviceCanAccessPeer(&can, c->device, qdev));
      if (!can) return 0;  // P.ok stays false
      hipError_t e = hipDeviceEnablePeerAccess(qdev, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPC(e);
      (void)hipGetLastError();
    }
    const int32_t b = base_id(sender_buf(Q));
    for (int64_t t = 0; t < cnt; ++t) { bid[orcv[k] + t] = b; elem[orcv[k] + t] = qo[m] + t; }
  }
  if (dev_upload(&P.d_bid, bid) || dev_upload(&P.d_elem, elem) || dev_upload(&P.d_bases, bases)) return -1;
  P.h_bid = std::move(bid);
  P.h_elem = std::move(elem);
  P.h_bases = std::move(bases);
  P.ok = true;
  return 0;
}

// Direct pull table of receiver i for a grouped mul! over the n parts of
// the call (all local, one device): receive slot p of segment k (sender q at
// call position j) reads x_j at the lid q lists for this part in its
// lids_snd.  ok = false when a sender is not in the call.
int build_direct(int i, int n, pa_xchg* const xg[], const LocalSet& L) {
  pa_xchg* X = xg[i];
  pa_pull& P = X->direct;
  std::vector<const void*> key(n);
  for (int j = 0; j < n; ++j) key[j] = (const void*)(uintptr_t)xg[j]->id;
  if (P.built && P.key == key) return 0;
  dev_free(P.d_bid);
  dev_free(P.d_elem);
  dev_free(P.d_bases);
  P = pa_pull{};
  P.built = true;
  P.key = key;
  const int64_t nslots = X->n_rcv_data;
  std::vector<int32_t> bid(nslots);
  std::vector<int64_t> elem(nslots);
  for (size_t k = 0; k < X->parts_rcv.size(); ++k) {
    const int j = L.find(X->parts_rcv[k]);
    if (j < 0) return 0;
    const pa_xchg* Q = xg[j];
    if ((int64_t)Q->h_lids_snd.size() != Q->n_snd_data) return 0;
    int m = -1;
    for (size_t t = 0; t < Q->parts_snd.size(); ++t)
      if (Q->parts_snd[t] == X->ctx->part) { m = (int)t; break; }
    CHECK_ARG(m >= 0, "exchanger mismatch: a receiver lists a sender that does not send to it");
    const int64_t cnt = X->ptrs_rcv[k + 1] - X->ptrs_rcv[k];
    CHECK_ARG(cnt == Q->ptrs_snd[m + 1] - Q->ptrs_snd[m],
              "exchanger mismatch: segment lengths differ (SequentialBackend.jl:187)");
    for (int64_t t = 0; t < cnt; ++t) {
      bid[X->ptrs_rcv[k] + t] = j;
      elem[X->ptrs_rcv[k] + t] = Q->h_lids_snd[Q->ptrs_snd[m] + t];
    }
  }
  HIPC(hipSetDevice(X->ctx->device));
  if (dev_upload(&P.d_bid, bid) || dev_upload(&P.d_elem, elem)) return -1;
  P.h_bid = std::move(bid);
  P.h_elem = std::move(elem);
  P.ok = true;
  return 0;
}

// device array of the call's x pointers (the direct pull's bases), cached on
// the leading context; a new set of vectors uploads once
void** direct_bases(pa_ctx* c0, int n, pa_vec* const x[]) {
  std::vector<void*> key(n);
  for (int i = 0; i < n; ++i) key[i] = x[i]->d;
  auto& C = c0->bases_cache;
  for (size_t k = 0; k < C.size(); ++k)
    if (C[k].first == key) {
      if (k) std::swap(C[k], C[0]);
      return C[0].second;
    }
  void** d = nullptr;
  if (dev_upload(&d, key)) return nullptr;
  if (C.size() >= 16) {
    (void)hipStreamSynchronize(c0->s_main);  // the evicted array may still be read
    dev_free(C.back().second);
    C.pop_back();
  }
  C.insert(C.begin(), {key, d});
  return d;
}

// One RCCL group of point-to-point byte transfers (segment src part → dst
// part).  Sends to one peer rank are matched with that rank's receives in
// posting order, and a rank may hold several parts (pa_comm_init_all: the
// parts of a device; a segment between two of them is a send to self), so
// every rank posts in (sender part, receiver part) order; transfers of one
// pair keep the order they were listed in.
struct P2P {
  int src, dst;
  bool send;
  char* buf;
  size_t cnt;
  int peer;
  ncclComm_t comm;
  hipStream_t s;
};

int rccl_group(std::vector<P2P>& ops) {
  std::stable_sort(ops.begin(), ops.end(), [](const P2P& a, const P2P& b) {
    return a.src != b.src ? a.src < b.src : a.dst < b.dst;
  });
  NCCLC(ncclGroupStart());
  for (const P2P& o : ops) {
    ncclResult_t r = o.send ? ncclSend(o.buf, o.cnt, ncclUint8, o.peer, o.comm, o.s)
                            : ncclRecv(o.buf, o.cnt, ncclUint8, o.peer, o.comm, o.s);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      PA_FAIL(std::string(o.send ? "ncclSend: " : "ncclRecv: ") + ncclGetErrorString(r));
    }
  }
  NCCLC(ncclGroupEnd());
  return 0;
}

// Halo transport for n local parts.  dir 0 (forward): send A-layout buffers
// (ptrs_snd) to parts_snd, receive B-layout (ptrs_rcv) from parts_rcv;
// dir 1 (reverse): the opposite.  Each part's s_comm first waits for the
// packs of every sender it reads from (ev_packed), then ev_recvd is recorded
// on it.  Senders in other processes: RCCL into the receive buffer.
// Senders in this process: when every part's pull table is usable and the
// target vectors v are given, s_comm runs one pull-unpack kernel per part
// that combines (op) the values straight from the senders' buffers into
// v[i] (*unpacked = true; the caller must not unpack again); otherwise
// device-to-device copies into the receive buffer.
// The transport of one call, planned once (pull tables, RCCL or not), then
// issued per part: transport_part(i) is what part i's streams get (the
// waits for its senders' packs, the pull or the staging copies, ev_recvd),
// so the parts can be issued from several host threads (IssuePool).
struct TransportPlan {
  LocalSet L;
  bool remote = false;
  bool pull = false;
  bool alt = false;  // the pull reads the senders' second buffers (pull_alt)
  bool on_main = false;  // the pull kernel on the receiver's compute stream (halo_barrier 2)
  size_t S = 0;
  int dtype = 0, dir = 0, op = 0;
};

int transport_plan(int n, pa_xchg* const xg[], int dtype, int dir, int op, pa_vec* const v[], TransportPlan* T) {
  T->S = dtype_size(dtype);
  T->dtype = dtype;
  T->dir = dir;
  T->op = op;
  T->L = local_set(n, xg);
  T->pull = v != nullptr && knobs().halo_pull;
  for (int i = 0; i < n && T->pull; ++i) {
    if (build_pull(i, n, xg, T->L, dtype, dir)) return -1;
    T->pull = xg[i]->pull[dir].ok;
  }
  T->remote = false;
  for (int i = 0; i < n; ++i) {
    const pa_xchg* X = xg[i];
    for (const auto* lst : {&X->parts_rcv, &X->parts_snd})
      for (int32_t q : *lst)
        if (T->L.find(q) < 0) T->remote = true;
  }
  return 0;
}

// part i's s_comm waits for the packs of every sender it reads from (and its own)
int transport_wait(int i, pa_xchg* const xg[], const TransportPlan& T) {
  pa_xchg* X = xg[i];
  pa_ctx* c = X->ctx;
  HIPC(hipSetDevice(c->device));
  HIPC(hipStreamWaitEvent(c->s_comm, c->ev_packed, 0));
  const auto& prcv = T.dir == 0 ? X->parts_rcv : X->parts_snd;
  for (int32_t q : prcv) {
    const int j = T.L.find(q);
    if (j >= 0 && xg[j]->ctx->ev_packed != c->ev_packed) HIPC(hipStreamWaitEvent(c->s_comm, xg[j]->ctx->ev_packed, 0));
  }
  return 0;
}

// part i's local segments (pull kernel or staging copies), then ev_recvd
int transport_local(int i, pa_xchg* const xg[], pa_vec* const v[], const TransportPlan& T) {
  pa_xchg* X = xg[i];
  pa_ctx* c = X->ctx;
  const int dir = T.dir;
  const size_t S = T.S;
  HIPC(hipSetDevice(c->device));
  if (T.pull) {
    const pa_pull& P = T.alt ? X->pull_alt : X->pull[dir];
    const int32_t* bid = P.d_bid;
    const int64_t* elem = P.d_elem;
    void* const* bases = P.d_bases;
    // the pull's completion is ev_recvd (recorded with the launch)
    hipEvent_t ev = c->ev_recvd;
    hipStream_t st = T.on_main ? c->s_main : c->s_comm;
    if (dir == 0)
      launch_pull(T.dtype, X->n_rcv_data, X->d_lids_rcv, X->plan_fwd, T.op, bid, elem, (const void* const*)bases,
                  v[i]->d, st, ev);
    else
      launch_pull(T.dtype, X->n_snd_data, X->d_lids_snd, X->plan_rev, T.op, bid, elem, (const void* const*)bases,
                  v[i]->d, st, ev);
    return 0;
  } else {
    // staging copies: receiver r, segment k from sender q (local), which
    // holds the matching segment at the position of r in its send list
    const auto& prcv = dir == 0 ? X->parts_rcv : X->parts_snd;
    const auto& orcv = dir == 0 ? X->ptrs_rcv : X->ptrs_snd;
    char* brcv = (char*)(dir == 0 ? X->d_buf_rcv : X->d_buf_snd);
    for (size_t k = 0; k < prcv.size(); ++k) {
      const int j = T.L.find(prcv[k]);
      if (j < 0) continue;
      pa_xchg* Q = xg[j];
      const auto& qsnd = dir == 0 ? Q->parts_snd : Q->parts_rcv;
      const auto& qo = dir == 0 ? Q->ptrs_snd : Q->ptrs_rcv;
      const char* bq = (const char*)(dir == 0 ? Q->d_buf_snd : Q->d_buf_rcv);
      int m = -1;
      for (size_t t = 0; t < qsnd.size(); ++t)
        if (qsnd[t] == c->part) { m = (int)t; break; }
      CHECK_ARG(m >= 0, "exchanger mismatch: a receiver lists a sender that does not send to it");
      const int64_t cnt = orcv[k + 1] - orcv[k];
      CHECK_ARG(cnt == qo[m + 1] - qo[m], "exchanger mismatch: segment lengths differ (SequentialBackend.jl:187)");
      if (cnt > 0)
        HIPC(hipMemcpyAsync(brcv + orcv[k] * S, bq + qo[m] * S, (size_t)cnt * S, hipMemcpyDefault, c->s_comm));
    }
  }
  HIPC(hipEventRecord(c->ev_recvd, c->s_comm));
  return 0;
}

// every (sender part, receiver part) segment with a part of another process
// through one RCCL group
int transport_remote(int n, pa_xchg* const xg[], const TransportPlan& T) {
  const int dir = T.dir;
  const size_t S = T.S;
  for (int i = 0; i < n; ++i)
    CHECK_ARG(xg[i]->ctx->comm, "halo neighbour is not held by this process and no RCCL communicator was initialised (pa_comm_init_rank)");
  std::vector<P2P> ops;
  for (int i = 0; i < n; ++i) {
    pa_xchg* X = xg[i];
    pa_ctx* c = X->ctx;
    ncclComm_t comm = (ncclComm_t)c->comm;
    const auto& psnd = dir == 0 ? X->parts_snd : X->parts_rcv;
    const auto& osnd = dir == 0 ? X->ptrs_snd : X->ptrs_rcv;
    char* bsnd = (char*)(dir == 0 ? X->d_buf_snd : X->d_buf_rcv);
    const auto& prcv = dir == 0 ? X->parts_rcv : X->parts_snd;
    const auto& orcv = dir == 0 ? X->ptrs_rcv : X->ptrs_snd;
    char* brcv = (char*)(dir == 0 ? X->d_buf_rcv : X->d_buf_snd);
    for (size_t k = 0; k < psnd.size(); ++k) {
      const size_t cnt = (size_t)(osnd[k + 1] - osnd[k]) * S;
      // an empty segment: the peer's matching one is empty too (SequentialBackend.jl:187)
      if (T.L.find(psnd[k]) >= 0 || cnt == 0) continue;
      ops.push_back({c->part, psnd[k], true, bsnd + osnd[k] * S, cnt, c->peer_rank(psnd[k]), comm, c->s_comm});
    }
    for (size_t k = 0; k < prcv.size(); ++k) {
      const size_t cnt = (size_t)(orcv[k + 1] - orcv[k]) * S;
      if (T.L.find(prcv[k]) >= 0 || cnt == 0) continue;
      ops.push_back({prcv[k], c->part, false, brcv + orcv[k] * S, cnt, c->peer_rank(prcv[k]), comm, c->s_comm});
    }
  }
  for (int i = 0; i < n; ++i) {
    pa_ctx* c = xg[i]->ctx;
    for (const P2P& o : ops) {
      if (o.send && o.src == c->part) c->rccl_bytes_sent += (int64_t)o.cnt;
      if (!o.send && o.dst == c->part) c->rccl_bytes_recv += (int64_t)o.cnt;
    }
  }
  return rccl_group(ops);
}

// Halo transport for n local parts.  dir 0 (forward): send A-layout buffers
// (ptrs_snd) to parts_snd, receive B-layout (ptrs_rcv) from parts_rcv;
// dir 1 (reverse): the opposite.  Each part's s_comm first waits for the
// packs of every sender it reads from (ev_packed), then ev_recvd is recorded
// on it.  Senders in other processes: RCCL into the receive buffer.
// Senders in this process: when every part's pull table is usable and the
// target vectors v are given, s_comm runs one pull-unpack kernel per part
// that combines (op) the values straight from the senders' buffers into
// v[i] (*unpacked = true; the caller must not unpack again); otherwise
// device-to-device copies into the receive buffer.
int transport(int n, pa_xchg* const xg[], int dtype, int dir, int op, pa_vec* const v[], bool* unpacked) {
  TransportPlan T;
  *unpacked = false;
  if (transport_plan(n, xg, dtype, dir, op, v, &T)) return -1;
  for (int i = 0; i < n; ++i)
    if (transport_wait(i, xg, T)) return -1;
  if (T.remote && transport_remote(n, xg, T)) return -1;
  for (int i = 0; i < n; ++i)
    if (transport_local(i, xg, v, T)) return -1;
  HIPC(hipGetLastError());
  *unpacked = T.pull;
  return 0;
}

int check_lids(const pa_xchg* X, const pa_vec* v) {
  CHECK_ARG(X->max_lid < v->n, "exchanger lids exceed the vector length (BoundsError)");
  return 0;
}

// Before packing into the send buffers again, wait for the copies that read
// them in the previous exchange (local receivers record ev_recvd after their
// copies; for RCCL sends the part's own ev_recvd covers them).
// before part i packs into its send buffer: the previous exchange's reads
// of it (its own unpack and its receivers' pulls) are done
int pre_pack_wait_part(int i, pa_xchg* const xg[], const LocalSet& L) {
  xg[i]->fast_key = 0;  // the next barrier call of these exchangers waits too (spmv_impl)
  pa_ctx* c = xg[i]->ctx;
  HIPC(hipSetDevice(c->device));
  HIPC(hipStreamWaitEvent(c->s_main, c->ev_recvd, 0));
  std::vector<hipEvent_t> seen{c->ev_recvd};
  for (const auto* lst : {&xg[i]->parts_snd, &xg[i]->parts_rcv})
    for (int32_t q : *lst) {
      const int j = L.find(q);
      if (j < 0 || j == i) continue;
      const hipEvent_t e = xg[j]->ctx->ev_recvd;
      if (std::find(seen.begin(), seen.end(), e) != seen.end()) continue;  // parts_snd and parts_rcv overlap
      seen.push_back(e);
      HIPC(hipStreamWaitEvent(c->s_main, e, 0));
    }
  return 0;
}

int pre_pack_wait(int n, pa_xchg* const xg[]) {
  LocalSet L = local_set(n, xg);
  for (int i = 0; i < n; ++i)
    if (pre_pack_wait_part(i, xg, L)) return -1;
  return 0;
}

// Host threads that issue the per-part work of one call in parallel (parts
// with their own stream pairs, typically one per GPU: one thread driving 8
// GPUs issues them one after the other, SURVEY.md §8(b)'s model).  run(n, f)
// calls f(i) for i in [0, n) on the pool and the caller, returns the first
// failure (its error text is carried over to the caller's thread).  Workers
// spin briefly between calls, then sleep.
class IssuePool {
 public:
  // host time of the jobs (one part's issue each) since the last reset
  // (pa_issue_stats: the per-thread issue time of the one-process-per-node
  // model)
  std::atomic<uint64_t> job_ns_sum{0}, job_ns_max{0}, jobs{0};
  static IssuePool& get() {
    static IssuePool* p = new IssuePool();  // never destroyed: workers may outlive static destruction
    return *p;
  }
  // The call returns once its n items are done and no worker is inside it;
  // a worker joins a call by reading the job under the lock, so the caller
  // never waits for workers that are asleep, and a late one joins whichever
  // call is current (or none).
  int run(int n, const std::function<int(int)>& f) {
    std::lock_guard<std::mutex> call_lock(call_mu_);
    ensure_workers(std::min(n - 1, kMaxWorkers));
    {
      std::lock_guard<std::mutex> g(mu_);
      f_ = &f;
      kn_ = &knobs();  // the calling thread's call: its jobs run with its knobs
      n_ = n;
      next_.store(0);
      finished_.store(0);
      failed_.store(false);
      err_.clear();
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    work(&f, n);
    while (finished_.load(std::memory_order_acquire) < n) std::this_thread::yield();
    {  // no worker joins after this; those that joined find no item left
      std::lock_guard<std::mutex> g(mu_);
      f_ = nullptr;
      n_ = 0;
    }
    while (busy_.load(std::memory_order_acquire) > 0) std::this_thread::yield();
    if (failed_.load()) {
      pa::set_error(err_);
      return -1;
    }
    return 0;
  }

 private:
  static constexpr int kMaxWorkers = 15;
  // A job's kernel launches report their errors to the thread that made
  // them (HIP keeps the last error per thread): each job ends with this
  // thread's hipGetLastError, so a launch that failed on a worker fails the
  // call instead of being lost there.
  void work(const std::function<int(int)>* f, int n) {
    for (int i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) {
      const auto t0 = std::chrono::steady_clock::now();
      int rc = (*f)(i);
      const uint64_t ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now() - t0).count();
      job_ns_sum.fetch_add(ns, std::memory_order_relaxed);
      jobs.fetch_add(1, std::memory_order_relaxed);
      for (uint64_t m = job_ns_max.load(); ns > m && !job_ns_max.compare_exchange_weak(m, ns);) {
      }
      if (rc == 0 && knobs().fault_inject) launch_invalid_config();
      const hipError_t e = hipGetLastError();
      if (rc == 0 && e != hipSuccess) {
        pa::set_error(std::string("kernel launch of an issue job failed: ") + hipGetErrorString(e));
        rc = -1;
      }
      if (rc != 0 && !failed_.exchange(true)) {
        std::lock_guard<std::mutex> g(mu_);
        err_ = pa_last_error();
      }
      finished_.fetch_add(1, std::memory_order_release);
    }
  }
  void ensure_workers(int k) {
    while ((int)workers_.size() < k) {
      workers_.emplace_back([this]() {
        uint64_t seen = 0;
        for (;;) {
          for (int spin = 0; gen_.load(std::memory_order_acquire) == seen; ++spin) {
            if (spin < 20000) continue;  // ~tens of µs busy, then sleep
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [&] { return gen_.load() != seen; });
          }
          const std::function<int(int)>* f;
          const Knobs* kn;
          int n;
          {
            std::lock_guard<std::mutex> g(mu_);
            seen = gen_.load();
            f = f_;
            kn = kn_;
            n = n_;
            if (f) busy_.fetch_add(1);
          }
          if (!f) continue;  // woke after the call ended: wait for the next
          {
            KnobBind kb(kn);
            work(f, n);
          }
          busy_.fetch_sub(1, std::memory_order_release);
        }
      });
      workers_.back().detach();
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> next_{0}, finished_{0}, busy_{0};
  std::atomic<bool> failed_{false};
  std::string err_;
  const std::function<int(int)>* f_ = nullptr;  // the current call's job (under mu_)
  const Knobs* kn_ = nullptr;                    // ... and its knobs
  int n_ = 0;
  std::vector<std::thread> workers_;
};

}  // namespace

// ===========================================================================
// the communicator of a part, destroyed with the last part holding it
static std::shared_ptr<void> own_comm(ncclComm_t comm) {
  return std::shared_ptr<void>((void*)comm, [](void* p) { (void)ncclCommDestroy((ncclComm_t)p); });
}

extern "C" {

const char* pa_last_error(void) { return g_err.c_str(); }
int pa_version(void) { return 1; }

// The tuning knobs (performance only, results unchanged): the process
// defaults (pa_tune) and per-context overrides (pa_ctx_tune).  A call
// resolves the overrides of its first part's context over the defaults into
// its own Knobs (TuneScope), so parts of one stream group always run with
// one setting and no global is written while a call runs.
}  // extern "C"
namespace {
struct Knob {
  const char* key;
  int Knobs::*slot;        // int knobs
  int64_t Knobs::*slot64;  // ... or 64-bit
  int64_t lo, hi;          // valid range
  int64_t mask;            // spmv_flags: allowed bits (0: range only)
  const char* help;
};
const Knob kKnobs[] = {
    {"spmv_flags", &Knobs::spmv_flags, nullptr, 0, 0xff, 0xff,
     "spmv_flags: bit 0 = non-temporal streams, bit 1 = pattern and triple-SELL slices' one-load descriptor, "
     "bit 2 = 16 B x runs (pattern rows), bit 3 = masked tail batch, bit 4 = identity slice lists dropped, "
     "bit 5 = non-temporal y stores, bit 6 = short-row kernels (launches whose rows have <= 8 entries), "
     "bit 7 = the Float64 short-row tail launch at 7 entries and 7 waves per SIMD (rows <= 7 entries)"},
    {"long_rows_exact", &Knobs::long_exact, nullptr, 0, 1, 0,
     "long_rows_exact: 1 = reference summation order, 0 = lane-strided tree (1e-12)"},
    {"halo_pull", &Knobs::halo_pull, nullptr, 0, 1, 0,
     "halo_pull: 1 = receivers read the senders' buffers (one kernel), 0 = staging copies"},
    {"spmv_delta16", &Knobs::spmv_delta16, nullptr, 0, 1, 0,
     "spmv_delta16: 1 = int32-column slices whose columns fit 16-bit codes store those (matrices built "
     "afterwards; default), 0 = int32 column ids"},
    {"spmv_merge", &Knobs::spmv_merge, nullptr, 0, 1, 0,
     "spmv_merge: 1 = mul! without a halo in flight (one part, or parts of one stream pair with the direct "
     "pull) runs every slice kind of every part as one launch (default), 0 = one launch per kind"},
    {"spmv_merge_max", nullptr, &Knobs::spmv_merge_max, 0, INT32_MAX, 0,
     "spmv_merge_max: one part with more slices than this runs one launch per kind (0: always merge)"},
    {"cg_fuse", &Knobs::cg_fuse, nullptr, 0, 2, 0,
     "cg_fuse: 1 = the device CG computes u = r .+ beta.*u inside the SpMV, 0 = a separate sweep, "
     "2 = auto (default: one batch of each, then the faster; all parts in one process, else the sweep)"},
    {"halo_direct", &Knobs::halo_direct, nullptr, 0, 1, 0,
     "halo_direct: 1 = mul! over parts sharing a stream pair reads the ghosts straight from the owners' x "
     "on the compute stream (default), 0 = pack + pull on the comm stream"},
    {"halo_transport", &Knobs::halo_transport, nullptr, 0, 1, 0,
     "halo_transport: 0 = parts of this process by device reads/copies, 1 = RCCL send/recv for every part "
     "with a communicator (pa_comm_init_all)"},
    {"spmv_group", &Knobs::spmv_group, nullptr, 0, 1, 0,
     "spmv_group: 1 = one launch per phase for parts sharing a stream pair, 0 = per part"},
    {"spmv_format", &Knobs::spmv_format, nullptr, 0, 1, 0, "spmv_format: 0 = int32 columns, 1 = pattern slices"},
    {"pattern_min_regular", &Knobs::pattern_min_pct, nullptr, 0, 100, 0,
     "pattern_min_regular: a slice becomes a pattern slice when at least this % of its rows follow its pattern "
     "(matrices built afterwards); 0 = auto (default): 70 for 128-row slices, 50 for Float32's 256-row slices"},
    {"issue_threads", &Knobs::issue_threads, nullptr, 0, 2, 0,
     "issue_threads: a call over parts with their own stream pairs is issued from host threads, one part "
     "per thread: 1 = when the parts span several devices (default), 2 = always, 0 = never (the calling "
     "thread, one part after the other)"},
    {"spmv_tri16", &Knobs::spmv_tri16, nullptr, 0, 1, 0,
     "spmv_tri16: the delta16 slices' rows re-sliced into the triple SELL (rows of consecutive column triples "
     "keep one 16-bit code per triple; matrices built afterwards): 1 = slices of 1-2 rows per lane (Float64, "
     "ComplexF32, ComplexF64, Float32 with f32_rows 2; default), 0 = never"},
    {"f32_rows", &Knobs::f32_rows, nullptr, 0, 4, 6,
     "f32_rows: Float32 SELL rows per lane (matrices built afterwards): 4 = 16 B value packs in 256-row "
     "slices, 2 = 8 B packs in 128-row slices (the Float64 geometry; delta16 rows then take the triple "
     "SELL), 0 = auto (default): 4, rebuilt with 2 when fewer than 80 % of the slices are pattern slices "
     "(C5 F32 -7 %, FE27 256^3 F32 +14 % with 2, profiles/r05/af/)"},
    {"spmv_tri_pack", &Knobs::tri_pack, nullptr, 0, 7, 0,
     "spmv_tri_pack: triple-SELL slices of 2 rows per lane (matrices built afterwards): bit 2 = pair slices "
     "(all element types): rows a, a + 1 whose columns differ by one, entry for entry, share one lane, one "
     "code and one x run per triple (C5 F32 -2.4 %, F64 -1 %, profiles/r06/u/); bit 0 = Float32 pair slices: "
     "a triple's values as one 16 B pack (entries 0 and 1 of both rows) and one 8 B pack (entry 2) per lane "
     "(two loads instead of three); bit 1: unused since r06/aa (the Float32 tri slices' code packs); 7 = "
     "default, 0 = none"},
    {"spmv_uniform", &Knobs::spmv_uniform, nullptr, 0, 1, 0,
     "spmv_uniform: Float64 pattern slices whose patterns (<= 7 entries) fit one union U (FD7; matrices built "
     "afterwards): 1 = a copy of their values at slice * H * |U| in U's entry order, so the short-row tail "
     "launch issues its value and x loads before the slice descriptor arrives (default), 0 = off"},
    {"spmv_side_tail", &Knobs::side_tail, nullptr, 0, 1, 0,
     "spmv_side_tail: per-kind launches without a halo in flight (big single parts): 1 = the side rows (<= 8 "
     "entries) run as the trailing waves of the pattern launch (default: FE27 256^3 -0.4 %, profiles/r05/o/), "
     "0 = a launch of their own after it"},
    {"spmv_tri_order", &Knobs::tri_order, nullptr, 0, 1, 0,
     "spmv_tri_order: the triple SELL's row order (matrices built afterwards): 1 = the other rows first "
     "(their slower waves start early, the launch ends on uniform triple slices; default: C5 F64 -1 %, "
     "Float32 triples -4..-7 %, profiles/r05/n/), 0 = rows of column triples first"},
    {"halo_barrier", &Knobs::halo_barrier, nullptr, 0, 2, 0,
     "halo_barrier: mul! over parts with their own stream pairs and local neighbours (one process driving "
     "several GPUs): 1 = one pack barrier event per call and double-buffered send buffers (default), 2 = the "
     "same with each part's pull on its compute stream after its interior slices (one runtime call less per "
     "part), 0 = per-neighbour event waits before every pack and every pull"},
    {"spmv_xcd_chunk", &Knobs::spmv_xcd_chunk, nullptr, -1, 64, 0,
     "spmv_xcd_chunk: the SpMV launches' workgroups in runs of C consecutive blocks per XCD (C > 0; the x lines "
     "of neighbouring slices shared in one L2), 0 = the hardware's round robin, -1 = auto (default): per-kind "
     "launches (big single parts) take C = the pattern's reach in blocks / 8, so that a block's z-neighbour "
     "plane runs on its XCD (FE27 256^3 F64: C = 16, -1.0..-1.2 %, profiles/r05/q,r/), merged launches keep "
     "the round robin (C2: C = 4 +1.4 %, r05/k/)"},
    {"fault_inject", &Knobs::fault_inject, nullptr, 0, 1, 0,
     "fault_inject: 1 = every job of a threaded issue (IssuePool) also issues an invalid kernel launch (tests "
     "of the error path; test_exception.jl's role), 0 = off (default)"},
};
constexpr int kNumKnobs = (int)(sizeof(kKnobs) / sizeof(kKnobs[0]));
static_assert(kNumKnobs <= pa_ctx::kMaxKnobs, "pa_ctx::over too small");

// the process defaults: written by pa_tune, copied by every call's
// TuneScope, both under g_knob_mu
std::mutex g_knob_mu;
Knobs g_knob_defaults = kDefaults;
thread_local const Knobs* t_knobs = nullptr;   // the running call's knobs on this thread
thread_local Knobs t_knob_snapshot;            // knobs() outside a call

// the knob's index (-1: unknown key), value checked (-2: out of range)
int knob_find(const char* key) {
  for (int i = 0; i < kNumKnobs; ++i)
    if (!std::strcmp(key, kKnobs[i].key)) return i;
  pa::set_error(std::string("pa_tune: unknown key ") + key);
  return -1;
}
int knob_index(const char* key, int64_t value) {
  const int i = knob_find(key);
  if (i < 0) return -1;
  const Knob& k = kKnobs[i];
  if (value < k.lo || value > k.hi || (k.mask != 0 && (value & ~k.mask) != 0)) {
    pa::set_error(k.help);
    return -2;
  }
  return i;
}
int64_t knob_get(const Knobs& K, int i) { return kKnobs[i].slot ? (int64_t)(K.*kKnobs[i].slot) : K.*kKnobs[i].slot64; }
void knob_set(Knobs& K, int i, int64_t v) {
  if (kKnobs[i].slot) K.*kKnobs[i].slot = (int)v;
  else K.*kKnobs[i].slot64 = v;
}
}  // namespace

namespace pa {
const Knobs& knobs() {
  if (t_knobs) return *t_knobs;
  std::lock_guard<std::mutex> g(g_knob_mu);
  t_knob_snapshot = g_knob_defaults;
  return t_knob_snapshot;
}
KnobBind::KnobBind(const Knobs* k) : prev(t_knobs) { t_knobs = k; }
KnobBind::~KnobBind() { t_knobs = prev; }
// a rebuild of a Float32 matrix with 2 rows per lane (f32_rows auto) in progress on this thread
thread_local int t_force_f32_rows = 0;
int f32_rows_knob() { return t_force_f32_rows ? t_force_f32_rows : (knobs().f32_rows == 2 ? 2 : 4); }
struct ForceF32Rows {
  int prev;
  explicit ForceF32Rows(int r) : prev(t_force_f32_rows) { t_force_f32_rows = r; }
  ~ForceF32Rows() { t_force_f32_rows = prev; }
};
}  // namespace pa

// For the duration of a call: the knobs of the call's context (its
// overrides over the process defaults) in the scope's own Knobs, current on
// this thread (and on the IssuePool workers the call's jobs run on).  A call
// nested in another (a library entry point calling another) keeps the outer
// call's knobs.
TuneScope::TuneScope(const pa_ctx* c) : prev(t_knobs) {
  if (prev) {
    k = *prev;
  } else {
    std::lock_guard<std::mutex> g(g_knob_mu);
    k = g_knob_defaults;
  }
  if (c && !prev)
    for (int i = 0; i < kNumKnobs; ++i)
      if (c->has_over[i]) knob_set(k, i, c->over[i]);
  t_knobs = &k;
}
TuneScope::~TuneScope() { t_knobs = prev; }

extern "C" {

int pa_tune(const char* key, int value, int* previous) {
  CHECK_ARG(key, "null key");
  const int i = knob_index(key, value);
  if (i < 0) return -1;
  std::lock_guard<std::mutex> g(g_knob_mu);
  if (previous) *previous = (int)std::min<int64_t>(knob_get(g_knob_defaults, i), INT32_MAX);
  knob_set(g_knob_defaults, i, value);
  return 0;
}

int pa_ctx_tune(pa_ctx* c, const char* key, int value, int* previous) {
  CHECK_ARG(c && key, "null argument");
  // PA_TUNE_DROP (outside every knob's range: spmv_xcd_chunk's auto is -1)
  // drops the override
  const int i = value == PA_TUNE_DROP ? knob_find(key) : knob_index(key, value);
  if (i < 0) return -1;
  if (previous) *previous = c->has_over[i] ? (int)c->over[i] : PA_TUNE_DROP;
  c->has_over[i] = value != PA_TUNE_DROP;
  c->over[i] = value;
  return 0;
}

// Test support, no device needed: `nthreads` host threads, each with its
// own context whose override of "spmv_merge_max" is 1000 + t, resolve a
// call's knobs `iters` times (TuneScope) and read them on the calling thread
// and in IssuePool jobs, while the process default of the same knob changes
// underneath; *mismatches counts the resolutions that saw a value other than
// their own context's (0: the knobs of concurrent calls are independent).
int pa_knob_selftest(int nthreads, int iters, int* mismatches) {
  CHECK_ARG(nthreads >= 1 && nthreads <= 64 && iters >= 0 && mismatches, "bad arguments");
  const int ki = knob_find("spmv_merge_max");
  std::vector<std::unique_ptr<pa_ctx>> cs;
  for (int t = 0; t < nthreads; ++t) {
    cs.emplace_back(new pa_ctx());
    cs.back()->has_over[ki] = true;
    cs.back()->over[ki] = 1000 + t;
  }
  std::atomic<int> bad{0};
  std::atomic<bool> stop{false};
  std::thread tuner([&]() {  // the process default moves while the calls run
    for (int v = 0; !stop.load(); v = (v + 1) % 997) (void)pa_tune("spmv_merge_max", v, nullptr);
  });
  std::vector<std::thread> ths;
  for (int t = 0; t < nthreads; ++t)
    ths.emplace_back([&, t]() {
      for (int it = 0; it < iters; ++it) {
        TuneScope ts(cs[t].get());
        if (knobs().spmv_merge_max != 1000 + t) bad.fetch_add(1);
        if (it % 16 == 0) {  // jobs on the pool's threads see the caller's knobs
          (void)IssuePool::get().run(2, [&](int) -> int {
            if (knobs().spmv_merge_max != 1000 + t) bad.fetch_add(1);
            return 0;
          });
        }
      }
    });
  for (auto& th : ths) th.join();
  stop.store(true);
  tuner.join();
  (void)pa_tune("spmv_merge_max", (int)kDefaults.spmv_merge_max, nullptr);
  *mismatches = bad.load();
  return 0;
}

int pa_device_count(int* count) {
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  *count = c;
  return 0;
}

int pa_hbm_probe(int device, int64_t bytes, int reps, double* read_gbs, double* copy_gbs) {
  CHECK_ARG(bytes >= (1 << 20) && reps > 0 && read_gbs && copy_gbs, "pa_hbm_probe: bytes >= 1 MiB, reps > 0");
  HIPC(hipSetDevice(device));
  const int64_t n16 = bytes / 16;
  void *a = nullptr, *b = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  auto cleanup = [&]() {
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
  };
#define PROBE_CALL(expr) do { if ((expr) != hipSuccess) { cleanup(); PA_FAIL(std::string("pa_hbm_probe: ") + #expr); } } while (0)
  PROBE_CALL(hipMalloc(&a, (size_t)n16 * 16));
  PROBE_CALL(hipMalloc(&b, (size_t)n16 * 16));
  PROBE_CALL(hipMemset(a, 0x5a, (size_t)n16 * 16));
  PROBE_CALL(hipStreamCreate(&st));
  PROBE_CALL(hipEventCreate(&e0));
  PROBE_CALL(hipEventCreate(&e1));
  double best[2] = {0.0, 0.0};
  for (int copy = 0; copy < 2; ++copy)
    for (int unroll : {4, 8})
    for (int blocks : {2048, 4096, 8192, 16384}) {
      launch_probe(copy, unroll, n16, a, b, blocks, st);  // warm
      PROBE_CALL(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) launch_probe(copy, unroll, n16, a, b, blocks, st);
      PROBE_CALL(hipEventRecord(e1, st));
      PROBE_CALL(hipEventSynchronize(e1));
      float ms = 0.f;
      PROBE_CALL(hipEventElapsedTime(&ms, e0, e1));
      const double gbs = (double)n16 * 16 * (copy ? 2 : 1) * reps / (ms * 1e-3) / 1e9;
      best[copy] = std::max(best[copy], gbs);
    }
#undef PROBE_CALL
  cleanup();
  *read_gbs = best[0];
  *copy_gbs = best[1];
  return 0;
}

int pa_hbm_probe_launch(int device, int64_t bytes_per_launch, int64_t span, int reps, double* read_gbs) {
  CHECK_ARG(bytes_per_launch >= (1 << 20) && span >= bytes_per_launch && reps > 0 && read_gbs,
            "pa_hbm_probe_launch: 1 MiB <= bytes_per_launch <= span, reps > 0");
  HIPC(hipSetDevice(device));
  const int64_t n16 = bytes_per_launch / 16, seg = n16 * 16;
  const int64_t nseg = std::max<int64_t>(1, span / seg);
  void *a = nullptr, *b = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  auto cleanup = [&]() {
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
  };
#define PROBE_CALL(expr) do { if ((expr) != hipSuccess) { cleanup(); PA_FAIL(std::string("pa_hbm_probe_launch: ") + #expr); } } while (0)
  PROBE_CALL(hipMalloc(&a, (size_t)(nseg * seg)));
  PROBE_CALL(hipMalloc(&b, 4096));
  PROBE_CALL(hipMemset(a, 0x5a, (size_t)(nseg * seg)));
  PROBE_CALL(hipStreamCreate(&st));
  PROBE_CALL(hipEventCreate(&e0));
  PROBE_CALL(hipEventCreate(&e1));
  double best = 0.0;
  for (int unroll : {4, 8})
    for (int blocks : {2048, 4096, 8192, 16384}) {
      launch_probe(0, unroll, n16, a, b, blocks, st);  // warm
      PROBE_CALL(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) launch_probe(0, unroll, n16, (const char*)a + (r % nseg) * seg, b, blocks, st);
      PROBE_CALL(hipEventRecord(e1, st));
      PROBE_CALL(hipEventSynchronize(e1));
      float ms = 0.f;
      PROBE_CALL(hipEventElapsedTime(&ms, e0, e1));
      best = std::max(best, (double)seg * reps / (ms * 1e-3) / 1e9);
    }
#undef PROBE_CALL
  cleanup();
  *read_gbs = best;
  return 0;
}

static int ctx_scratch(pa_ctx* c, const pa_ctx* share_events = nullptr) {
  HIPC(hipMalloc(&c->d_partials, 8192 * 16));  // block partials (reductions, CG update)
  HIPC(hipMalloc(&c->d_fold, 256 * 16));
  HIPC(hipMalloc(&c->d_result, 16));
  HIPC(hipMalloc(&c->d_gather, (size_t)c->nparts * 16));
  HIPC(hipMalloc((void**)&c->d_ticket, 16));
  HIPC(hipMemset(c->d_ticket, 0, 16));
  HIPC(hipDeviceSynchronize());  // (the null-stream memset done before any stream of the context uses it)
  HIPC(hipHostMalloc(&c->h_pinned, std::max<size_t>((size_t)(c->nparts + 1) * 16, 256)));  // gathered partials / CG state
  if (share_events) {  // one stream pair, one pair of pipeline events
    c->ev_packed = share_events->ev_packed;
    c->ev_recvd = share_events->ev_recvd;
    return 0;
  }
  HIPC(hipEventCreateWithFlags(&c->ev_packed, hipEventDisableTiming));
  HIPC(hipEventCreateWithFlags(&c->ev_recvd, hipEventDisableTiming));
  return 0;
}

int pa_ctx_create(int device, int part, int nparts, pa_ctx** out) {
  CHECK_ARG(out, "null out");
  CHECK_ARG(nparts >= 1 && part >= 1 && part <= nparts, "part must satisfy 1 <= part <= nparts");
  int ndev = 0;
  HIPC(hipGetDeviceCount(&ndev));
  CHECK_ARG(device >= 0 && device < ndev, "invalid device ordinal");
  HIPC(hipSetDevice(device));
  pa_ctx* c = new pa_ctx();
  c->device = device;
  c->part = part;
  c->nparts = nparts;
  int least = 0, greatest = 0;
  HIPC(hipDeviceGetStreamPriorityRange(&least, &greatest));
  HIPC(hipStreamCreateWithFlags(&c->s_main, hipStreamNonBlocking));
  HIPC(hipStreamCreateWithPriority(&c->s_comm, hipStreamNonBlocking, greatest));
  c->stream_refs = new pa_ctx::StreamRefs();
  if (ctx_scratch(c)) return -1;
  *out = c;
  return 0;
}

int pa_ctx_create_shared(int part, int nparts, pa_ctx* with, pa_ctx** out) {
  CHECK_ARG(out && with, "null argument");
  CHECK_ARG(nparts == with->nparts && part >= 1 && part <= nparts, "part must satisfy 1 <= part <= nparts");
  HIPC(hipSetDevice(with->device));
  pa_ctx* c = new pa_ctx();
  c->device = with->device;
  c->part = part;
  c->nparts = nparts;
  c->s_main = with->s_main;
  c->s_comm = with->s_comm;
  c->stream_refs = with->stream_refs;
  ++c->stream_refs->n;
  if (ctx_scratch(c, with)) return -1;
  *out = c;
  return 0;
}

int pa_ctx_destroy(pa_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->s_main);
  (void)hipStreamSynchronize(c->s_comm);
  c->comm = nullptr;
  c->comm_owner.reset();  // ncclCommDestroy with the last part of the communicator
  dev_free(c->d_partials);
  dev_free(c->d_fold);
  dev_free(c->d_result);
  dev_free(c->d_gather);
  dev_free(c->d_ticket);
  for (auto& b : c->bases_cache) dev_free(b.second);
  for (auto& b : c->merged_cache) dev_free(b.second);
  if (c->h_pinned) (void)hipHostFree(c->h_pinned);
  for (auto& e : c->tev) (void)hipEventDestroy(e);
  for (auto& e : c->span_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->ev_barrier) (void)hipEventDestroy(c->ev_barrier);
  if (c->stream_refs && --c->stream_refs->n == 0) {  // the last context of a shared stream pair
    (void)hipEventDestroy(c->ev_packed);
    (void)hipEventDestroy(c->ev_recvd);
    (void)hipStreamDestroy(c->s_main);
    (void)hipStreamDestroy(c->s_comm);
    delete c->stream_refs;
  }
  delete c;
  return 0;
}

int pa_ctx_sync(pa_ctx* c) {
  CHECK_ARG(c, "null ctx");
  HIPC(hipSetDevice(c->device));
  HIPC(hipStreamSynchronize(c->s_comm));
  HIPC(hipStreamSynchronize(c->s_main));
  return 0;
}

int pa_comm_unique_id(unsigned char id[128]) {
  ncclUniqueId u;
  NCCLC(ncclGetUniqueId(&u));
  static_assert(sizeof(u) == 128, "ncclUniqueId size");
  std::memcpy(id, &u, 128);
  return 0;
}

int pa_comm_init_rank(pa_ctx* c, const unsigned char id[128]) {
  CHECK_ARG(c, "null ctx");
  HIPC(hipSetDevice(c->device));
  ncclUniqueId u;
  std::memcpy(&u, id, 128);
  CHECK_ARG(!c->comm, "pa_comm_init_rank: a communicator is already attached");
  ncclComm_t comm;
  NCCLC(ncclCommInitRank(&comm, c->nparts, u, c->part - 1));
  c->comm = comm;
  c->comm_owner = own_comm(comm);
  c->rank_of_part = nullptr;  // rank = part - 1
  return 0;
}

// RCCL for the parts of ONE process (ncclCommInitAll): one rank per distinct
// device, in order of first appearance among parts 1..nparts; the parts of a
// device share its communicator and their stream pair (pa_ctx_create_shared),
// so a segment between two parts of one device is an RCCL send to self.  The
// MPIBackend transport (MPIBackend.jl:261-309) without processes; used for
// every halo segment with pa_tune("halo_transport", 1).
int pa_comm_init_all(int n, pa_ctx* const ctx[]) {
  CHECK_ARG(n >= 1 && ctx, "null argument");
  std::vector<int> devs, first;  // rank -> device, rank -> position of its first part
  auto rank_of = std::make_shared<std::vector<int>>(n);
  for (int i = 0; i < n; ++i) {
    CHECK_ARG(ctx[i], "null ctx");
    CHECK_ARG(ctx[i]->part == i + 1 && ctx[i]->nparts == n, "pa_comm_init_all: pass the contexts of parts 1..nparts in order");
    CHECK_ARG(!ctx[i]->comm, "pa_comm_init_all: a communicator is already attached");
    int r = (int)(std::find(devs.begin(), devs.end(), ctx[i]->device) - devs.begin());
    if (r == (int)devs.size()) {
      devs.push_back(ctx[i]->device);
      first.push_back(i);
    } else {
      CHECK_ARG(ctx[i]->s_comm == ctx[first[r]]->s_comm,
                "pa_comm_init_all: parts of one device must share their stream pair (pa_ctx_create_shared)");
    }
    (*rank_of)[i] = r;
  }
  std::vector<ncclComm_t> comms(devs.size());
  NCCLC(ncclCommInitAll(comms.data(), (int)devs.size(), devs.data()));
  std::vector<std::shared_ptr<void>> owners;
  for (ncclComm_t cm : comms) owners.push_back(own_comm(cm));
  for (int i = 0; i < n; ++i) {
    const int r = (*rank_of)[i];
    ctx[i]->comm = comms[r];
    ctx[i]->comm_owner = owners[r];
    ctx[i]->rank_of_part = rank_of;
    ctx[i]->halo_rccl = true;  // these parts exchange their halos over RCCL (per context, not a global knob)
  }
  return 0;
}

int pa_comm_stats(pa_ctx* c, int64_t* bytes_sent, int64_t* bytes_recv) {
  CHECK_ARG(c && bytes_sent && bytes_recv, "null argument");
  *bytes_sent = c->rccl_bytes_sent;
  *bytes_recv = c->rccl_bytes_recv;
  return 0;
}

int pa_comm_info(pa_ctx* c, int* ranks, int* rank, int* device, char* pci, int pci_len, int* version,
                 char* lib, int lib_len) {
  CHECK_ARG(c && ranks && rank && device && version, "null argument");
  *ranks = 0;
  *rank = -1;
  if (c->comm) {
    NCCLC(ncclCommCount((ncclComm_t)c->comm, ranks));
    NCCLC(ncclCommUserRank((ncclComm_t)c->comm, rank));
  }
  *device = c->device;
  if (pci && pci_len > 0) {
    pci[0] = 0;
    HIPC(hipDeviceGetPCIBusId(pci, pci_len, c->device));
  }
  NCCLC(ncclGetVersion(version));
  if (lib && lib_len > 0) {
    lib[0] = 0;
    Dl_info di{};
    if (dladdr(reinterpret_cast<void*>(&ncclGetVersion), &di) && di.dli_fname)
      std::snprintf(lib, (size_t)lib_len, "%s", di.dli_fname);
  }
  return 0;
}

int pa_issue_stats(int reset, double* max_job_us, double* mean_job_us, int64_t* jobs) {
  IssuePool& P = IssuePool::get();
  const uint64_t n = P.jobs.load();
  if (max_job_us) *max_job_us = 1e-3 * (double)P.job_ns_max.load();
  if (mean_job_us) *mean_job_us = n ? 1e-3 * (double)P.job_ns_sum.load() / (double)n : 0.0;
  if (jobs) *jobs = (int64_t)n;
  if (reset) {
    P.job_ns_sum.store(0);
    P.job_ns_max.store(0);
    P.jobs.store(0);
  }
  return 0;
}

int pa_ctx_set_timing(pa_ctx* c, int enable) {
  CHECK_ARG(c, "null ctx");
  c->timing = enable != 0;
  c->tn = 0;
  return 0;
}

// Means over the mul! calls recorded since timing was enabled (events read
// after the last one completes: no synchronisation inside the timed calls);
// the record is then cleared.
int pa_ctx_kernel_times(pa_ctx* c, float* int_ms, float* halo_ms, float* bnd_ms, int* count) {
  CHECK_ARG(c, "null ctx");
  float a = 0.f, h = 0.f, b = 0.f;
  const int n = c->tn;
  if (n > 0) {
    HIPC(hipSetDevice(c->device));
    HIPC(hipEventSynchronize(c->tev[4 * (n - 1) + 3]));
    for (int k = 0; k < n; ++k) {
      float t01 = 0.f, t12 = 0.f, t23 = 0.f;
      HIPC(hipEventElapsedTime(&t01, c->tev[4 * k], c->tev[4 * k + 1]));
      HIPC(hipEventElapsedTime(&t12, c->tev[4 * k + 1], c->tev[4 * k + 2]));
      HIPC(hipEventElapsedTime(&t23, c->tev[4 * k + 2], c->tev[4 * k + 3]));
      a += t01; h += t12; b += t23;
    }
    a /= n; h /= n; b /= n;
  }
  if (int_ms) *int_ms = a;
  if (halo_ms) *halo_ms = h;
  if (bnd_ms) *bnd_ms = b;
  if (count) *count = n;
  c->tn = 0;
  return 0;
}

// Device time of a region of work on the compute stream: stop = 0 records
// the start, stop = 1 the end (no synchronisation); pa_ctx_span_ms waits for
// the end and returns the elapsed time.
int pa_ctx_span(pa_ctx* c, int stop) {
  CHECK_ARG(c && (stop == 0 || stop == 1), "pa_ctx_span: stop is 0 or 1");
  HIPC(hipSetDevice(c->device));
  if (!c->span_ev[stop]) HIPC(hipEventCreate(&c->span_ev[stop]));
  HIPC(hipEventRecord(c->span_ev[stop], c->s_main));
  return 0;
}

int pa_ctx_span_ms(pa_ctx* c, float* ms) {
  CHECK_ARG(c && ms && c->span_ev[0] && c->span_ev[1], "pa_ctx_span_ms: record a start and an end first");
  HIPC(hipSetDevice(c->device));
  HIPC(hipEventSynchronize(c->span_ev[1]));
  HIPC(hipEventElapsedTime(ms, c->span_ev[0], c->span_ev[1]));
  return 0;
}

int pa_ctx_last_kernel_ms(pa_ctx* c, float* int_ms, float* bnd_ms) {
  return pa_ctx_kernel_times(c, int_ms, nullptr, bnd_ms, nullptr);
}

// ---------------------------------------------------------------------------
int pa_index_create(pa_ctx* c, int64_t nlids, int64_t noids, const int32_t* oid_to_lid,
                    int64_t nhids, const int32_t* hid_to_lid, pa_index** out) {
  CHECK_ARG(c && out, "null argument");
  CHECK_ARG(nlids >= 0 && noids >= 0 && nhids >= 0 && noids + nhids == nlids,
            "index set: noids + nhids must equal nlids");
  CHECK_ARG(nlids < (int64_t)INT32_MAX, "index set larger than Int32 lids");
  HIPC(hipSetDevice(c->device));
  pa_index* I = new pa_index();
  I->ctx = c;
  I->nlids = nlids;
  I->noids = noids;
  I->nhids = nhids;
  I->h_oid_to_lid.resize(noids);
  I->h_hid_to_lid.resize(nhids);
  I->h_lid_to_ohid.assign(nlids, 0);
  for (int64_t i = 0; i < noids; ++i) {
    const int32_t l = oid_to_lid[i];
    if (l < 1 || l > nlids || I->h_lid_to_ohid[l - 1] != 0) { delete I; PA_FAIL("index set: invalid or repeated oid_to_lid entry"); }
    I->h_oid_to_lid[i] = l - 1;
    I->h_lid_to_ohid[l - 1] = (int32_t)(i + 1);
    if (l - 1 != i) I->own_contig = false;
  }
  for (int64_t i = 0; i < nhids; ++i) {
    const int32_t l = hid_to_lid[i];
    if (l < 1 || l > nlids || I->h_lid_to_ohid[l - 1] != 0) { delete I; PA_FAIL("index set: invalid or repeated hid_to_lid entry"); }
    I->h_hid_to_lid[i] = l - 1;
    I->h_lid_to_ohid[l - 1] = (int32_t)(-(i + 1));
    if (l - 1 != noids + i) I->ghost_contig = false;
  }
  if (!I->own_contig && dev_upload(&I->d_oid_to_lid, I->h_oid_to_lid)) { delete I; return -1; }
  if (!I->ghost_contig && dev_upload(&I->d_hid_to_lid, I->h_hid_to_lid)) { delete I; return -1; }
  *out = I;
  return 0;
}

int pa_index_destroy(pa_index* I) {
  if (!I) return 0;
  (void)hipSetDevice(I->ctx->device);
  dev_free(I->d_oid_to_lid);
  dev_free(I->d_hid_to_lid);
  dev_free(I->d_sgid);
  dev_free(I->d_slid);
  delete I;
  return 0;
}

// gid → lid table of the index set (lid_to_gid: nlids 1-based gids), sorted
// on the device; used by pa_add_gids and pa_mat_from_coo(ids_global=1).
int pa_index_set_gids(pa_index* I, const int64_t* lid_to_gid) {
  CHECK_ARG(I && (lid_to_gid || I->nlids == 0), "null argument");
  pa_ctx* c = I->ctx;
  HIPC(hipSetDevice(c->device));
  dev_free(I->d_sgid);
  dev_free(I->d_slid);
  I->d_sgid = nullptr;
  I->d_slid = nullptr;
  int64_t* d = nullptr;
  if (I->nlids > 0) {
    std::vector<int64_t> h(lid_to_gid, lid_to_gid + I->nlids);
    for (int64_t g : h) CHECK_ARG(g >= 1, "lid_to_gid: gids are 1-based");
    if (dev_upload(&d, h)) return -1;
    const int rc = gid_table(I->nlids, d, &I->d_sgid, &I->d_slid, c->s_main);
    dev_free(d);
    CHECK_ARG(rc == 0, "pa_index_set_gids: device sort failed");
  }
  I->has_gids = true;
  return 0;
}

// add_gids!(a, gids) (Interfaces.jl:579-603, 618-627): the gids that are not
// local ids of the index set, each once, in first-touch order → new_gids
// (cap entries available; *n_new is set even when it exceeds cap, which is
// then an error so the caller can retry with a larger buffer).
int pa_add_gids(pa_index* I, int64_t n, const int64_t* gids, int64_t cap, int64_t* new_gids, int64_t* n_new) {
  CHECK_ARG(I && n_new && (n == 0 || gids), "null argument");
  CHECK_ARG(I->has_gids, "pa_add_gids: call pa_index_set_gids first");
  pa_ctx* c = I->ctx;
  HIPC(hipSetDevice(c->device));
  *n_new = 0;
  if (n == 0) return 0;
  int64_t* d = nullptr;
  HIPC(hipMalloc((void**)&d, n * 8));
  hipError_t e = hipMemcpy(d, gids, n * 8, hipMemcpyHostToDevice);
  if (e != hipSuccess) { dev_free(d); HIPC(e); }
  int64_t* out = nullptr;
  int64_t m = 0;
  const int rc = gids_first_touch(n, d, I->d_sgid, I->d_slid, I->nlids, &out, &m, c->s_main);
  dev_free(d);
  CHECK_ARG(rc == 0, "pa_add_gids: device pass failed");
  *n_new = m;
  if (m > cap || (m > 0 && !new_gids)) { dev_free(out); PA_FAIL("pa_add_gids: new_gids buffer too small (see *n_new)"); }
  if (m > 0) {
    e = hipStreamSynchronize(c->s_main);  // (hipMemcpy runs on the null stream)
    if (e == hipSuccess) e = hipMemcpy(new_gids, out, m * 8, hipMemcpyDeviceToHost);
    dev_free(out);
    HIPC(e);
  }
  return 0;
}

int pa_index_to_lids(pa_index* I, int64_t n, int64_t* ids) {
  CHECK_ARG(I && (n == 0 || ids), "null argument");
  CHECK_ARG(I->has_gids, "pa_index_to_lids: call pa_index_set_gids first");
  pa_ctx* c = I->ctx;
  HIPC(hipSetDevice(c->device));
  if (n == 0) return 0;
  int64_t* d = nullptr;
  HIPC(hipMalloc((void**)&d, n * 8));
  hipError_t e = hipMemcpy(d, ids, n * 8, hipMemcpyHostToDevice);
  const int rc = e == hipSuccess ? gids_to_lids(n, d, I->d_sgid, I->d_slid, I->nlids, c->s_main) : -1;
  if (rc == 0) e = hipStreamSynchronize(c->s_main);  // (hipMemcpy runs on the null stream)
  if (rc == 0 && e == hipSuccess) e = hipMemcpy(ids, d, n * 8, hipMemcpyDeviceToHost);
  dev_free(d);
  HIPC(e);
  CHECK_ARG(rc >= 0, "pa_index_to_lids: device pass failed");
  CHECK_ARG(rc == 0, "to_lids!: a global id is not a local id of the part (KeyError)");
  return 0;
}

// ---------------------------------------------------------------------------
int pa_xchg_create(pa_ctx* c, int32_t n_rcv, const int32_t* parts_rcv, const int32_t* ptrs_rcv,
                   const int32_t* lids_rcv, int32_t n_snd, const int32_t* parts_snd,
                   const int32_t* ptrs_snd, const int32_t* lids_snd, pa_xchg** out) {
  CHECK_ARG(c && out, "null argument");
  CHECK_ARG(n_rcv >= 0 && n_snd >= 0, "negative neighbour count");
  HIPC(hipSetDevice(c->device));
  pa_xchg* X = new pa_xchg();
  X->ctx = c;
  X->id = g_xchg_next_id++;
  auto take = [&](int32_t n, const int32_t* parts, const int32_t* ptrs, const int32_t* lids,
                  std::vector<int32_t>& P, std::vector<int64_t>& O, std::vector<int32_t>& Lh) -> int {
    P.assign(parts, parts + n);
    O.resize(n + 1);
    for (int32_t i = 0; i <= n; ++i) O[i] = (int64_t)(n == 0 && i == 0 ? 1 : ptrs[i]) - 1;
    for (int32_t i = 0; i < n; ++i) {
      if (P[i] < 1 || P[i] > c->nparts) PA_FAIL("exchanger: part id out of range");
      if (O[i + 1] < O[i]) PA_FAIL("exchanger: ptrs not non-decreasing");
    }
    if (O[0] != 0) PA_FAIL("exchanger: ptrs[1] must be 1");
    Lh.resize(O[n]);
    for (int64_t p = 0; p < O[n]; ++p) {
      if (lids[p] < 1) PA_FAIL("exchanger: lids must be >= 1");
      Lh[p] = lids[p] - 1;
    }
    return 0;
  };
  std::vector<int32_t> hr, hs;
  if (take(n_rcv, parts_rcv, ptrs_rcv, lids_rcv, X->parts_rcv, X->ptrs_rcv, hr) ||
      take(n_snd, parts_snd, ptrs_snd, lids_snd, X->parts_snd, X->ptrs_snd, hs)) {
    delete X;
    return -1;
  }
  for (int32_t l : hr) X->max_lid = std::max<int64_t>(X->max_lid, l);
  for (int32_t l : hs) X->max_lid = std::max<int64_t>(X->max_lid, l);
  X->n_rcv_data = (int64_t)hr.size();
  X->n_snd_data = (int64_t)hs.size();
  if (dev_upload(&X->d_lids_rcv, hr) || dev_upload(&X->d_lids_snd, hs)) { delete X; return -1; }
  X->h_lids_snd = hs;
  if (X->n_rcv_data) HIPC(hipMalloc(&X->d_buf_rcv, X->n_rcv_data * 16));
  if (X->n_snd_data) HIPC(hipMalloc(&X->d_buf_snd, X->n_snd_data * 16));
  if (build_plan(hr, &X->plan_fwd) || build_plan(hs, &X->plan_rev)) { delete X; return -1; }
  *out = X;
  return 0;
}

int pa_xchg_destroy(pa_xchg* X) {
  if (!X) return 0;
  (void)hipSetDevice(X->ctx->device);
  dev_free(X->d_lids_rcv);
  dev_free(X->d_lids_snd);
  dev_free(X->d_buf_rcv);
  dev_free(X->d_buf_snd);
  dev_free(X->d_buf_snd2);
  free_plan(X->plan_fwd);
  free_plan(X->plan_rev);
  for (pa_pull* t : {&X->pull[0], &X->pull[1], &X->direct, &X->pull_alt}) {
    dev_free(t->d_bid);
    dev_free(t->d_elem);
    dev_free(t->d_bases);
  }
  delete X;
  return 0;
}

// ---------------------------------------------------------------------------
int pa_vec_create(pa_ctx* c, int dtype, int64_t n, pa_vec** out) {
  CHECK_ARG(c && out, "null argument");
  CHECK_ARG(valid_dtype(dtype), "invalid dtype");
  CHECK_ARG(n >= 0, "negative length");
  HIPC(hipSetDevice(c->device));
  pa_vec* v = new pa_vec();
  v->ctx = c;
  v->dtype = dtype;
  v->n = n;
  if (n) {
    // kVecPad bytes on both sides: the SpMV's 16 B x runs may start up to
    // 3 elements before lid 0 or end up to 3 after the last lid
    const size_t bytes = (size_t)n * dtype_size(dtype) + 2 * kVecPad;
    hipError_t e = hipMalloc(&v->base, bytes);
    if (e != hipSuccess) { delete v; PA_FAIL(std::string("hipMalloc(vector) failed: ") + hipGetErrorString(e)); }
    v->d = (char*)v->base + kVecPad;
    HIPC(hipMemsetAsync(v->base, 0, bytes, c->s_main));
  }
  *out = v;
  return 0;
}

int pa_vec_destroy(pa_vec* v) {
  if (!v) return 0;
  (void)hipSetDevice(v->ctx->device);
  (void)hipStreamSynchronize(v->ctx->s_main);
  dev_free(v->base);
  delete v;
  return 0;
}

int pa_vec_upload(pa_vec* v, const void* host, int64_t n) {
  CHECK_ARG(v && (host || n == 0), "null argument");
  CHECK_ARG(n == v->n, "upload length differs from vector length");
  HIPC(hipSetDevice(v->ctx->device));
  if (n) {
    HIPC(hipMemcpyAsync(v->d, host, (size_t)n * dtype_size(v->dtype), hipMemcpyHostToDevice, v->ctx->s_main));
    HIPC(hipStreamSynchronize(v->ctx->s_main));
  }
  return 0;
}

int pa_vec_download(const pa_vec* v, void* host, int64_t n) {
  CHECK_ARG(v && (host || n == 0), "null argument");
  CHECK_ARG(n == v->n, "download length differs from vector length");
  HIPC(hipSetDevice(v->ctx->device));
  if (n) {
    HIPC(hipStreamSynchronize(v->ctx->s_comm));
    HIPC(hipMemcpyAsync(host, v->d, (size_t)n * dtype_size(v->dtype), hipMemcpyDeviceToHost, v->ctx->s_main));
    HIPC(hipStreamSynchronize(v->ctx->s_main));
  }
  return 0;
}

int pa_vec_device_ptr(const pa_vec* v, void** out) {
  CHECK_ARG(v && out, "null argument");
  *out = v->d;
  return 0;
}

int pa_vec_fill(pa_vec* v, const void* s) {
  CHECK_ARG(v && s, "null argument");
  HIPC(hipSetDevice(v->ctx->device));
  launch_fill(v->dtype, v->n, 0, nullptr, v->d, s, v->ctx->s_main);
  HIPC(hipGetLastError());
  return 0;
}

int pa_vec_copy(pa_vec* d, const pa_index* id, const pa_vec* s, const pa_index* is, int same_layout) {
  CHECK_ARG(d && s, "null argument");
  CHECK_ARG(d->dtype == s->dtype, "copyto!: element types differ");
  CHECK_ARG(d->ctx == s->ctx, "copyto!: vectors of different parts");
  HIPC(hipSetDevice(d->ctx->device));
  if (same_layout) {
    CHECK_ARG(d->n == s->n, "copyto!: lengths differ");
    if (d->n) HIPC(hipMemcpyAsync(d->d, s->d, (size_t)d->n * dtype_size(d->dtype), hipMemcpyDeviceToDevice, d->ctx->s_main));
    return 0;
  }
  CHECK_ARG(id && is, "copyto! across partitions needs both index sets");
  CHECK_ARG(id->noids == is->noids, "copyto!: owned counts differ (oids_are_equal)");
  launch_copy(d->dtype, id->noids, id->d_oid_to_lid, d->d, is->d_oid_to_lid, s->d, d->ctx->s_main);
  HIPC(hipGetLastError());
  return 0;
}

int pa_vec_axpby(pa_vec* y, const pa_vec* x, const pa_index* idx, const void* a, int mode, int all_lids) {
  CHECK_ARG(y && a, "null argument");
  const int sk = (mode & PA_BCAST_F64) ? 1 : (mode & PA_BCAST_C128) ? 2 : 0;
  CHECK_ARG(!((mode & PA_BCAST_F64) && (mode & PA_BCAST_C128)), "axpby: one scalar kind");
  CHECK_ARG(sk != 2 || y->dtype == PA_C64 || y->dtype == PA_C128,
            "axpby: a ComplexF64 scalar into a real vector (InexactError)");
  mode &= ~(PA_BCAST_F64 | PA_BCAST_C128);
  CHECK_ARG(mode >= 0 && mode <= 4, "invalid axpby mode");
  CHECK_ARG(mode == 4 || (x && x->dtype == y->dtype && x->n == y->n), "axpby: x must match y");
  HIPC(hipSetDevice(y->ctx->device));
  if (all_lids) {
    launch_axpby(y->dtype, y->n, nullptr, y->d, x ? x->d : nullptr, a, mode, y->ctx->s_main, sk);
  } else {
    CHECK_ARG(idx && idx->nlids == y->n, "axpby over owned values needs the vector's index set");
    launch_axpby(y->dtype, idx->noids, idx->d_oid_to_lid, y->d, x ? x->d : nullptr, a, mode, y->ctx->s_main, sk);
  }
  HIPC(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// Local matrix → owned-row SELL (one time, host side).  `visit(f)` calls
// f(row oid (0-based), x lid (0-based), input nz position, ghost column?)
// for every owned-row entry, each row's entries in the reference's
// summation order (owned columns, then ghost columns; SparseUtils.jl:176-185
// for a CSC parent, 242-250 for a CSR parent), and returns -1 on an index
// out of range.  The input's other nonzeros (stored ghost rows) are kept
// after the slots for exchange!/assemble!(A); nz positions index nzval.
extern "C++" {
namespace {
template <class Visit>
int mat_from_visit(pa_ctx* c, int dtype, int64_t nrows_lids, int64_t ncols_lids, int64_t in_nnz,
                   const void* nzval, const pa_index* rows, const pa_index* cols, Visit&& visit,
                   const char* range_error, bool csr, pa_mat** out) {
  const size_t S = dtype_size(dtype);
  pa_mat* A = new pa_mat();
  A->csr = csr;
  A->ctx = c;
  A->dtype = dtype;
  A->R = sell_rows_per_lane(dtype);
  A->H = 64 * A->R;
  A->nrows = rows->noids;
  A->ncols_lids = ncols_lids;
  A->csc_nnz = in_nnz;
  const int64_t nr = A->nrows;
  std::vector<int32_t> len(nr, 0);
  std::vector<char> has_ghost(nr, 0);
  if (visit([&](int64_t r, int64_t, int64_t, bool g) { ++len[r]; if (g) has_ghost[r] = 1; })) {
    delete A;
    PA_FAIL(range_error);
  }
  const int64_t ns = (nr + A->H - 1) / A->H;
  // long rows (row-length histogram) leave the SELL
  const int32_t thr = long_threshold(len);
  std::vector<int32_t> lidx(nr, -1), lrows;
  std::vector<int64_t> lptr{0};
  for (int64_t r = 0; r < nr; ++r)
    if (len[r] > thr) {
      lidx[r] = (int32_t)lrows.size();
      lrows.push_back((int32_t)r);
      lptr.push_back(lptr.back() + len[r]);
    }
  A->n_lnz = lptr.back();
  std::vector<int32_t> slen(ns, 0);
  std::vector<char> sghost(ns, 0);
  int64_t nnz = 0;
  for (int64_t r = 0; r < nr; ++r) {
    nnz += len[r];
    if (lidx[r] >= 0) continue;
    slen[r / A->H] = std::max(slen[r / A->H], len[r]);
    if (has_ghost[r]) sghost[r / A->H] = 1;
  }
  A->nnz = nnz;
  std::vector<int64_t> soff;
  if (finish_sell_layout(A, slen, sghost, &soff)) { pa_mat_destroy(A); return -1; }
  std::vector<int32_t> hcol(A->slots, -1);
  std::vector<unsigned char> hval(A->slots * S, 0);
  std::vector<int32_t> lcol(A->n_lnz);
  std::vector<unsigned char> lval(A->n_lnz * S);
  std::vector<int64_t> lpos(in_nnz, -1);  // input nz → position in the long CSR
  A->h_nz_slot.assign(in_nnz, -1);
  A->nz_map = true;
  std::vector<int32_t> cur(nr, 0);
  const int R = A->R;
  visit([&](int64_t r, int64_t J, int64_t p, bool) {
    if (lidx[r] >= 0) {  // long row: its CSR, in the same (reference) order
      const int64_t t = lptr[lidx[r]] + cur[r]++;
      lcol[t] = (int32_t)J;
      std::memcpy(&lval[t * S], (const unsigned char*)nzval + p * S, S);
      lpos[p] = t;
      return;
    }
    const int64_t s = r / A->H;
    const int64_t w = r - s * A->H;
    const int64_t lane = w / R, rr = w % R;
    const int64_t slot = soff[s] + ((int64_t)cur[r] * 64 + lane) * R + rr;
    ++cur[r];
    hcol[slot] = (int32_t)J;
    std::memcpy(&hval[slot * S], (const unsigned char*)nzval + p * S, S);
    A->h_nz_slot[p] = slot;
  });
  // ghost-row nonzeros (dropped by the SpMV, kept for exchange!/assemble!(A)),
  // then the long rows' values: both after the SELL slots in d_val
  for (int64_t p = 0; p < in_nnz; ++p)
    if (A->h_nz_slot[p] < 0 && lpos[p] < 0) A->h_nz_slot[p] = -(++A->n_gnz);
  A->long_off = A->slots + A->n_gnz;
  for (int64_t p = 0; p < in_nnz; ++p)
    if (lpos[p] >= 0) A->h_nz_slot[p] = -(A->n_gnz + lpos[p] + 1);
  hval.resize(nvals(A) * S);
  for (int64_t p = 0; p < in_nnz; ++p)
    if (A->h_nz_slot[p] < 0 && lpos[p] < 0)
      std::memcpy(&hval[(A->slots - A->h_nz_slot[p] - 1) * S], (const unsigned char*)nzval + p * S, S);
  if (A->n_lnz) std::memcpy(&hval[A->long_off * S], lval.data(), A->n_lnz * S);
  if (dev_upload(&A->d_col, hcol)) { pa_mat_destroy(A); return -1; }
  if (nvals(A)) {
    HIPC(hipMalloc(&A->d_val, nvals(A) * S));
    HIPC(hipMemcpy(A->d_val, hval.data(), nvals(A) * S, hipMemcpyHostToDevice));
  }
  if (upload_long(A, lrows, lptr, lcol)) { pa_mat_destroy(A); return -1; }
  // pattern slices need "x lid >= noids ⇔ ghost column" (contiguous layout)
  if (cols->own_contig && cols->ghost_contig) {
    int kmax = 0;
    for (int32_t l : slen) kmax = std::max(kmax, l);
    const int rc = finalize_pattern(A, kmax, cols->noids, true);
    if (rc == kPreferR2) {
      pa_mat_destroy(A);
      ForceF32Rows f(2);
      return mat_from_visit(c, dtype, nrows_lids, ncols_lids, in_nnz, nzval, rows, cols, visit, range_error, csr,
                            out);
    }
    if (rc) { pa_mat_destroy(A); return -1; }
  }
  *out = A;
  return 0;
}

}  // namespace
}  // extern "C++"

// CSC parent: columns in oid order, then in hid order; each row's entries
// are appended in that order.
int pa_mat_from_csc(pa_ctx* c, int dtype, int index_bytes, int64_t nrows_lids, int64_t ncols_lids,
                    const void* colptr, const void* rowval, const void* nzval, const pa_index* rows,
                    const pa_index* cols, pa_mat** out) {
  CHECK_ARG(c && out && rows && cols, "null argument");
  TuneScope ts(c);
  CHECK_ARG(valid_dtype(dtype), "invalid dtype");
  CHECK_ARG(index_bytes == 4 || index_bytes == 8, "index_bytes must be 4 or 8");
  CHECK_ARG(rows->nlids == nrows_lids && cols->nlids == ncols_lids,
            "matrix size must be num_lids(rows) x num_lids(cols) (DimensionMismatch)");
  HIPC(hipSetDevice(c->device));
  auto cp = [&](int64_t j) -> int64_t {
    return index_bytes == 8 ? ((const int64_t*)colptr)[j] : ((const int32_t*)colptr)[j];
  };
  auto rv = [&](int64_t p) -> int64_t {
    return index_bytes == 8 ? ((const int64_t*)rowval)[p] : ((const int32_t*)rowval)[p];
  };
  const int64_t csc_nnz = ncols_lids > 0 ? cp(ncols_lids) - 1 : 0;
  CHECK_ARG(csc_nnz >= 0, "colptr[end] must be >= 1");
  auto visit = [&](auto&& f) -> int {
    for (int64_t j = 0; j < cols->noids; ++j) {
      const int64_t J = cols->h_oid_to_lid[j];
      for (int64_t p = cp(J) - 1; p < cp(J + 1) - 1; ++p) {
        const int64_t I = rv(p) - 1;
        if (I < 0 || I >= nrows_lids) return -1;
        const int32_t o = rows->h_lid_to_ohid[I];
        if (o > 0) f(o - 1, J, p, false);
      }
    }
    for (int64_t h = 0; h < cols->nhids; ++h) {
      const int64_t J = cols->h_hid_to_lid[h];
      for (int64_t p = cp(J) - 1; p < cp(J + 1) - 1; ++p) {
        const int64_t I = rv(p) - 1;
        if (I < 0 || I >= nrows_lids) return -1;
        const int32_t o = rows->h_lid_to_ohid[I];
        if (o > 0) f(o - 1, J, p, true);
      }
    }
    return 0;
  };
  return mat_from_visit(c, dtype, nrows_lids, ncols_lids, csc_nnz, nzval, rows, cols, visit,
                        "CSC rowval out of range", false, out);
}

// CSR parent (SparseMatrixCSR{Bi}): rows in oid order; each row's owned
// columns in storage order, then its ghost columns in storage order
// (SparseUtils.jl:242-250 over owned_owned, then owned_ghost).
int pa_mat_from_csr(pa_ctx* c, int dtype, int index_bytes, int Bi, int64_t nrows_lids, int64_t ncols_lids,
                    const void* rowptr, const void* colval, const void* nzval, const pa_index* rows,
                    const pa_index* cols, pa_mat** out) {
  CHECK_ARG(c && out && rows && cols, "null argument");
  TuneScope ts(c);
  CHECK_ARG(valid_dtype(dtype), "invalid dtype");
  CHECK_ARG(index_bytes == 4 || index_bytes == 8, "index_bytes must be 4 or 8");
  CHECK_ARG(Bi == 0 || Bi == 1, "Bi (index base) must be 0 or 1");
  CHECK_ARG(rows->nlids == nrows_lids && cols->nlids == ncols_lids,
            "matrix size must be num_lids(rows) x num_lids(cols) (DimensionMismatch)");
  HIPC(hipSetDevice(c->device));
  auto rp = [&](int64_t i) -> int64_t {
    return (index_bytes == 8 ? ((const int64_t*)rowptr)[i] : ((const int32_t*)rowptr)[i]) - Bi;
  };
  auto cv = [&](int64_t p) -> int64_t {
    return (index_bytes == 8 ? ((const int64_t*)colval)[p] : ((const int32_t*)colval)[p]) - Bi;
  };
  CHECK_ARG(nrows_lids == 0 || rp(0) == 0, "rowptr[1] must equal Bi");
  const int64_t csr_nnz = nrows_lids > 0 ? rp(nrows_lids) : 0;
  CHECK_ARG(csr_nnz >= 0, "rowptr[end] must be >= Bi");
  for (int64_t i = 0; i < nrows_lids; ++i)
    CHECK_ARG(rp(i) <= rp(i + 1), "rowptr must be nondecreasing");
  auto visit = [&](auto&& f) -> int {
    for (int pass = 0; pass < 2; ++pass)
      for (int64_t o = 0; o < rows->noids; ++o) {
        const int64_t I = rows->h_oid_to_lid[o];
        for (int64_t p = rp(I); p < rp(I + 1); ++p) {
          const int64_t J = cv(p);
          if (J < 0 || J >= ncols_lids) return -1;
          const int32_t oh = cols->h_lid_to_ohid[J];
          if (pass == 0 ? oh > 0 : oh < 0) f(o, J, p, pass == 1);
        }
      }
    return 0;
  };
  return mat_from_visit(c, dtype, nrows_lids, ncols_lids, csr_nnz, nzval, rows, cols, visit,
                        "CSR colval out of range", true, out);
}

// sparse(I, J, V, m, n, +) (SparseUtils.jl:80-94) and the SELL build on the
// device (pa_coo.hip); same layout and nz_slot map as pa_mat_from_csc.
namespace {
// PA_TRACE_SETUP=1: phase times of the device matrix build on stderr (each
// mark synchronises the stream, so the phases are attributed, not overlapped)
struct SetupTrace {
  bool on = std::getenv("PA_TRACE_SETUP") != nullptr;
  hipStream_t st;
  std::chrono::steady_clock::time_point t;
  explicit SetupTrace(hipStream_t s) : st(s), t(std::chrono::steady_clock::now()) {}
  void mark(const char* what) {
    if (!on) return;
    (void)hipStreamSynchronize(st);
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[pa setup] %-28s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};
struct DevBufs {
  std::vector<void*> p;
  ~DevBufs() { for (void* q : p) dev_free(q); }
  void add(void* q) { p.push_back(q); }
};
}  // namespace

namespace {
// I, J, V: host arrays (kind H2D) or device arrays (D2D, pa_mat_from_dcoo);
// either way they are copied first (to_lids! works in place).
// csr_bi: -1 = sparse (CSC parent); 0 / 1 = sparsecsr with index base Bi
// (the pattern returned is then rowptr / colval in base Bi)
int mat_from_coo_impl(pa_ctx* c, int dtype, int index_bytes, int ids_global, int64_t nrows_lids,
                      int64_t ncols_lids, int64_t ncoo, const void* I, const void* J, const void* V,
                      hipMemcpyKind kind, const pa_index* rows, const pa_index* cols, int csr_bi, int64_t* csc_nnz,
                      int64_t* colptr_out, int64_t* rowval_out, pa_mat** out);
}  // namespace

int pa_mat_from_coo(pa_ctx* c, int dtype, int index_bytes, int ids_global, int64_t nrows_lids, int64_t ncols_lids,
                    int64_t ncoo, const void* I, const void* J, const void* V, const pa_index* rows,
                    const pa_index* cols, int64_t* csc_nnz, int64_t* colptr_out, int64_t* rowval_out, pa_mat** out) {
  return mat_from_coo_impl(c, dtype, index_bytes, ids_global, nrows_lids, ncols_lids, ncoo, I, J, V,
                           hipMemcpyHostToDevice, rows, cols, -1, csc_nnz, colptr_out, rowval_out, out);
}

int pa_mat_from_dcoo(const pa_coo* coo, int ids_global, int64_t nrows_lids, int64_t ncols_lids, const pa_index* rows,
                     const pa_index* cols, int64_t* csc_nnz, int64_t* colptr_out, int64_t* rowval_out, pa_mat** out) {
  CHECK_ARG(coo, "null argument");
  CHECK_ARG(rows && rows->ctx == coo->ctx && cols && cols->ctx == coo->ctx, "COO and index sets of different parts");
  return mat_from_coo_impl(coo->ctx, coo->dtype, 8, ids_global, nrows_lids, ncols_lids, coo->n, coo->d_I, coo->d_J,
                           coo->d_V, hipMemcpyDeviceToDevice, rows, cols, -1, csc_nnz, colptr_out, rowval_out, out);
}

int pa_mat_from_coo_csr(pa_ctx* c, int dtype, int index_bytes, int ids_global, int Bi, int64_t nrows_lids,
                        int64_t ncols_lids, int64_t ncoo, const void* I, const void* J, const void* V,
                        const pa_index* rows, const pa_index* cols, int64_t* nnz, int64_t* rowptr_out,
                        int64_t* colval_out, pa_mat** out) {
  CHECK_ARG(Bi == 0 || Bi == 1, "Bi (index base) must be 0 or 1");
  return mat_from_coo_impl(c, dtype, index_bytes, ids_global, nrows_lids, ncols_lids, ncoo, I, J, V,
                           hipMemcpyHostToDevice, rows, cols, Bi, nnz, rowptr_out, colval_out, out);
}

int pa_mat_from_dcoo_csr(const pa_coo* coo, int ids_global, int Bi, int64_t nrows_lids, int64_t ncols_lids,
                         const pa_index* rows, const pa_index* cols, int64_t* nnz, int64_t* rowptr_out,
                         int64_t* colval_out, pa_mat** out) {
  CHECK_ARG(coo, "null argument");
  CHECK_ARG(Bi == 0 || Bi == 1, "Bi (index base) must be 0 or 1");
  CHECK_ARG(rows && rows->ctx == coo->ctx && cols && cols->ctx == coo->ctx, "COO and index sets of different parts");
  return mat_from_coo_impl(coo->ctx, coo->dtype, 8, ids_global, nrows_lids, ncols_lids, coo->n, coo->d_I, coo->d_J,
                           coo->d_V, hipMemcpyDeviceToDevice, rows, cols, Bi, nnz, rowptr_out, colval_out, out);
}

}  // extern "C"

namespace {
int mat_from_coo_impl(pa_ctx* c, int dtype, int index_bytes, int ids_global, int64_t nrows_lids,
                      int64_t ncols_lids, int64_t ncoo, const void* I, const void* J, const void* V,
                      hipMemcpyKind kind, const pa_index* rows, const pa_index* cols, int csr_bi, int64_t* csc_nnz,
                      int64_t* colptr_out, int64_t* rowval_out, pa_mat** out) {
  CHECK_ARG(c && out && rows && cols && csc_nnz, "null argument");
  TuneScope ts(c);
  const bool csr = csr_bi >= 0;
  if (csr) {  // the row order below (owned columns by oid, ghosts by hid) is the CSR storage order
    bool inc = true;  // when oid_to_lid and hid_to_lid ascend (every PRange / IndexSet the reference builds)
    for (size_t k = 1; inc && k < cols->h_oid_to_lid.size(); ++k) inc = cols->h_oid_to_lid[k] > cols->h_oid_to_lid[k - 1];
    for (size_t k = 1; inc && k < cols->h_hid_to_lid.size(); ++k) inc = cols->h_hid_to_lid[k] > cols->h_hid_to_lid[k - 1];
    CHECK_ARG(inc, "sparsecsr on the device needs ascending oid_to_lid / hid_to_lid of cols (use pa_mat_from_csr)");
  }
  CHECK_ARG(!ids_global || (index_bytes == 8 && rows->has_gids && cols->has_gids),
            "ids=:global needs Int64 ids and pa_index_set_gids on rows and cols");
  CHECK_ARG(ncoo >= 0 && (ncoo == 0 || (I && J && V)), "null COO arrays");
  CHECK_ARG(valid_dtype(dtype), "invalid dtype");
  CHECK_ARG(index_bytes == 4 || index_bytes == 8, "index_bytes must be 4 or 8");
  CHECK_ARG(rows->nlids == nrows_lids && cols->nlids == ncols_lids,
            "matrix size must be num_lids(rows) x num_lids(cols) (DimensionMismatch)");
  HIPC(hipSetDevice(c->device));
  hipStream_t st = c->s_main;
  const size_t S = dtype_size(dtype);
  SetupTrace tr(st);
  DevBufs tmp, inp;
  void *dI = nullptr, *dJ = nullptr, *dV = nullptr;
  if (ncoo > 0) {
    HIPC(hipMalloc(&dI, ncoo * index_bytes));
    inp.add(dI);
    HIPC(hipMalloc(&dJ, ncoo * index_bytes));
    inp.add(dJ);
    HIPC(hipMalloc(&dV, ncoo * S));
    inp.add(dV);
    HIPC(hipMemcpy(dI, I, ncoo * index_bytes, kind));
    HIPC(hipMemcpy(dJ, J, ncoo * index_bytes, kind));
    HIPC(hipMemcpy(dV, V, ncoo * S, kind));
    if (ids_global) {  // to_lids!(I, rows); to_lids!(J, cols) (Interfaces.jl:2206-2209, 1541-1543)
      const int r1 = gids_to_lids(ncoo, (int64_t*)dI, rows->d_sgid, rows->d_slid, rows->nlids, st);
      const int r2 = r1 ? r1 : gids_to_lids(ncoo, (int64_t*)dJ, cols->d_sgid, cols->d_slid, cols->nlids, st);
      tr.mark("upload + to_lids!");
      CHECK_ARG(r1 >= 0 && r2 >= 0, "to_lids!: device pass failed");
      CHECK_ARG(r1 == 0 && r2 == 0, "to_lids!: a global id is not a local id of the part (KeyError)");
    }
  }
  tr.mark("upload / to_lids!");
  int64_t nu = 0;
  int32_t *crow = nullptr, *ccol = nullptr;
  void* cval = nullptr;
  int64_t* dcolptr = nullptr;
  hipError_t e = hipSuccess;
  const int rc = coo_compress(dtype, index_bytes, nrows_lids, ncols_lids, ncoo, dI, dJ, dV, csr ? 1 : 0, &nu, &crow,
                              &ccol, &cval, &dcolptr, st, &e);
  if (rc < 0) HIPC(e);
  CHECK_ARG(rc == 0, "sparse: COO index out of range (BoundsError)");
  tmp.add(crow); tmp.add(ccol); tmp.add(cval); tmp.add(dcolptr);
  for (void*& q : inp.p) { dev_free(q); q = nullptr; }  // the COO input is no longer needed
  tr.mark("sparse (sort, combine)");
  *csc_nnz = nu;
  const int64_t nptr = csr ? nrows_lids : ncols_lids;
  const int64_t base = csr ? csr_bi : 1;
  if (colptr_out) {  // colptr (CSC, 1-based) or rowptr (CSR, base Bi)
    HIPC(hipStreamSynchronize(st));  // (hipMemcpy runs on the null stream)
    HIPC(hipMemcpy(colptr_out, dcolptr, (nptr + 1) * 8, hipMemcpyDeviceToHost));
    for (int64_t j = 0; j <= nptr; ++j) colptr_out[j] += base;
  }
  if (rowval_out && nu > 0) {  // rowval (CSC) or colval (CSR)
    std::vector<int32_t> rv(nu);
    HIPC(hipMemcpy(rv.data(), csr ? ccol : crow, nu * 4, hipMemcpyDeviceToHost));
    for (int64_t p = 0; p < nu; ++p) rowval_out[p] = (int64_t)rv[p] + base;
  }
  tr.mark("CSC pattern to host");
  int32_t *rl2o = nullptr, *cl2o = nullptr;
  if (dev_upload(&rl2o, rows->h_lid_to_ohid) || dev_upload(&cl2o, cols->h_lid_to_ohid)) return -1;
  tmp.add(rl2o); tmp.add(cl2o);

  pa_mat* A = new pa_mat();
  A->ctx = c;
  A->dtype = dtype;
  A->csr = csr;
  A->R = sell_rows_per_lane(dtype);
  A->H = 64 * A->R;
  A->nrows = rows->noids;
  A->ncols_lids = ncols_lids;
  A->csc_nnz = nu;
  uint64_t* key2 = nullptr;
  int64_t *idx2 = nullptr, *rowptr = nullptr, *gflag = nullptr, *grank = nullptr, *nzs = nullptr;
  int32_t *slen_d = nullptr, *sghost_d = nullptr;
  int64_t nnz = 0, ngh = 0;
  if (coo_row_order(nu, crow, ccol, rl2o, cl2o, A->nrows, cols->noids, ncols_lids, A->H, &key2, &idx2, &rowptr,
                    &gflag, &grank, &slen_d, &sghost_d, &nnz, &ngh, st, &e)) {
    delete A;
    HIPC(e);
  }
  tmp.add(key2); tmp.add(idx2); tmp.add(rowptr); tmp.add(gflag); tmp.add(grank); tmp.add(slen_d); tmp.add(sghost_d);
  tr.mark("row order");
  A->nnz = nnz;
  const int64_t ns = (A->nrows + A->H - 1) / A->H;
  // row-length histogram → long rows (they leave the SELL, see long_threshold)
  std::vector<int32_t> lrows;
  std::vector<int64_t> lptr{0};
  int32_t *lidx_d = nullptr, *lcol_d = nullptr;
  int64_t* lptr_d = nullptr;
  if (A->nrows > 0) {
    std::vector<int64_t> rp(A->nrows + 1);
    HIPC(hipStreamSynchronize(st));  // (hipMemcpy runs on the null stream)
    HIPC(hipMemcpy(rp.data(), rowptr, (A->nrows + 1) * 8, hipMemcpyDeviceToHost));
    std::vector<int32_t> len(A->nrows);
    for (int64_t r = 0; r < A->nrows; ++r) len[r] = (int32_t)(rp[r + 1] - rp[r]);
    const int32_t thr = long_threshold(len);
    std::vector<int32_t> lidx(A->nrows, -1);
    for (int64_t r = 0; r < A->nrows; ++r)
      if (len[r] > thr) {
        lidx[r] = (int32_t)lrows.size();
        lrows.push_back((int32_t)r);
        lptr.push_back(lptr.back() + len[r]);
      }
    if (!lrows.empty()) {
      if (dev_upload(&lidx_d, lidx) || dev_upload(&lptr_d, lptr)) return -1;
      tmp.add(lidx_d);
      tmp.add(lptr_d);
      HIPC(hipMalloc((void**)&lcol_d, lptr.back() * 4));
    }
  }
  A->n_lnz = lptr.back();
  coo_slices(ns, A->nrows, A->H, rowptr, key2, ncols_lids, cols->noids, lidx_d, slen_d, sghost_d, st);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(st));  // the copies below run on the null stream
  std::vector<int32_t> slen(ns), sg(ns);
  std::vector<char> sghost(ns);
  if (ns > 0) {
    HIPC(hipMemcpy(slen.data(), slen_d, ns * 4, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(sg.data(), sghost_d, ns * 4, hipMemcpyDeviceToHost));
  }
  for (int64_t s = 0; s < ns; ++s) sghost[s] = sg[s] ? 1 : 0;
  if (finish_sell_layout(A, slen, sghost, nullptr)) { pa_mat_destroy(A); return -1; }
  if (A->slots > 0) {
    HIPC(hipMalloc((void**)&A->d_col, A->slots * 4));
    launch_fill_i32(A->slots, A->d_col, -1, st);
  }
  A->n_gnz = ngh;
  A->long_off = A->slots + ngh;
  if (nvals(A) > 0) {
    HIPC(hipMalloc(&A->d_val, nvals(A) * S));
    HIPC(hipMemsetAsync(A->d_val, 0, nvals(A) * S, st));
  }
  if (nu > 0) HIPC(hipMalloc((void**)&nzs, nu * 8));
  A->d_nz_slot = nzs;  // downloaded on first use (load_nz_map)
  A->nz_map = true;
  tr.mark("slices");
  coo_fill(dtype, nnz, nu, key2, idx2, rowptr, A->d_slice_off, A->H, A->R, ncols_lids, ccol, cval, gflag, grank,
           A->slots, A->d_col, A->d_val, nzs, lidx_d, lptr_d, lcol_d, A->long_off, st);
  HIPC(hipGetLastError());
  tr.mark("SELL fill");
  if (upload_long(A, lrows, lptr, {})) { pa_mat_destroy(A); return -1; }
  A->d_long_col = lcol_d;
  HIPC(hipStreamSynchronize(st));
  tr.mark("long rows");
  if (cols->own_contig && cols->ghost_contig) {
    int kmax = 0;
    for (int32_t l : slen) kmax = std::max(kmax, l);
    const int rc = finalize_pattern(A, kmax, cols->noids, true);
    if (rc == kPreferR2) {
      pa_mat_destroy(A);
      ForceF32Rows f(2);
      return mat_from_coo_impl(c, dtype, index_bytes, ids_global, nrows_lids, ncols_lids, ncoo, I, J, V, kind, rows,
                               cols, csr_bi, csc_nnz, colptr_out, rowval_out, out);
    }
    if (rc) { pa_mat_destroy(A); return -1; }
  }
  tr.mark("pattern slices");
  *out = A;
  return 0;
}
}  // namespace

extern "C" {

// ---------------------------------------------------------------------------
// COO triplets on the device and async_assemble!(I, J, V, rows)
// (Interfaces.jl:2406-2492)

int pa_coo_create(pa_ctx* c, int dtype, int64_t n, const int64_t* I, const int64_t* J, const void* V, pa_coo** out) {
  CHECK_ARG(c && out, "null argument");
  CHECK_ARG(valid_dtype(dtype), "invalid dtype");
  CHECK_ARG(n >= 0 && (n == 0 || (I && J && V)), "null COO arrays");
  HIPC(hipSetDevice(c->device));
  auto C = std::make_unique<pa_coo>();
  C->ctx = c;
  C->dtype = dtype;
  C->n = n;
  if (n > 0) {
    const size_t S = dtype_size(dtype);
    hipError_t e = hipMalloc((void**)&C->d_I, n * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&C->d_J, n * 8);
    if (e == hipSuccess) e = hipMalloc(&C->d_V, n * S);
    if (e == hipSuccess) e = hipMemcpy(C->d_I, I, n * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(C->d_J, J, n * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(C->d_V, V, n * S, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      pa_coo_destroy(C.release());
      HIPC(e);
    }
  }
  *out = C.release();
  return 0;
}

int pa_coo_destroy(pa_coo* C) {
  if (!C) return 0;
  (void)hipSetDevice(C->ctx->device);
  (void)hipStreamSynchronize(C->ctx->s_main);
  dev_free(C->d_I);
  dev_free(C->d_J);
  dev_free(C->d_V);
  delete C;
  return 0;
}

int pa_coo_size(const pa_coo* C, int64_t* n) {
  CHECK_ARG(C && n, "null argument");
  *n = C->n;
  return 0;
}

int pa_coo_download(const pa_coo* C, int64_t* I, int64_t* J, void* V) {
  CHECK_ARG(C && (C->n == 0 || (I && J && V)), "null argument");
  if (C->n == 0) return 0;
  HIPC(hipSetDevice(C->ctx->device));
  HIPC(hipStreamSynchronize(C->ctx->s_main));
  HIPC(hipMemcpy(I, C->d_I, C->n * 8, hipMemcpyDeviceToHost));
  HIPC(hipMemcpy(J, C->d_J, C->n * 8, hipMemcpyDeviceToHost));
  HIPC(hipMemcpy(V, C->d_V, C->n * dtype_size(C->dtype), hipMemcpyDeviceToHost));
  return 0;
}

int pa_coo_assemble_all(int n, pa_coo* const coo[], const pa_index* const rows[], pa_xchg* const xg[]) {
  CHECK_ARG(n >= 1 && coo && rows && xg && coo[0], "null argument");
  TuneScope ts(coo[0]->ctx);
  const int dt = coo[0]->dtype;
  const size_t S = dtype_size(dt);
  for (int i = 0; i < n; ++i) {
    CHECK_ARG(coo[i] && rows[i] && xg[i], "null handle");
    CHECK_ARG(coo[i]->dtype == dt, "assemble!: element types differ across parts");
    CHECK_ARG(coo[i]->ctx == rows[i]->ctx && xg[i]->ctx == rows[i]->ctx, "assemble!: COO, rows and exchanger of different parts");
    CHECK_ARG(rows[i]->has_gids, "assemble!(I,J,V,rows): rows needs its global ids on the device (pa_index_set_gids)");
    CHECK_ARG(xg[i]->max_lid < rows[i]->nlids, "assemble!: the exchanger's lids exceed rows' local ids");
  }
  // per part: the sent triplets (segments in parts_rcv order), counts and
  // offsets; the received counts (parts_snd order); the new arrays
  struct Side {
    int64_t *sI = nullptr, *sJ = nullptr;
    void* sV = nullptr;
    std::vector<int64_t> cnt, off, rcnt, roff;
    int64_t *nI = nullptr, *nJ = nullptr;
    void* nV = nullptr;
    int64_t nn = 0;
  };
  std::vector<Side> sd(n);
  auto free_all = [&]() {
    for (int i = 0; i < n; ++i) {
      (void)hipSetDevice(coo[i]->ctx->device);
      for (void* p : {(void*)sd[i].sI, (void*)sd[i].sJ, sd[i].sV, (void*)sd[i].nI, (void*)sd[i].nJ, sd[i].nV})
        if (p) (void)hipFree(p);
      sd[i] = Side{};
    }
  };
  // 1. group the triplets of rows owned elsewhere by owner, zero them locally
  for (int i = 0; i < n; ++i) {
    pa_coo* C = coo[i];
    pa_xchg* X = xg[i];
    const pa_index* R = rows[i];
    HIPC(hipSetDevice(C->ctx->device));
    const int rc = coo_assemble_pack(dt, C->n, C->d_I, C->d_J, C->d_V, R->d_sgid, R->d_slid, R->nlids,
                                     R->h_lid_to_ohid, (int)X->parts_rcv.size(), X->d_lids_rcv, X->ptrs_rcv,
                                     &sd[i].sI, &sd[i].sJ, &sd[i].sV, &sd[i].cnt, C->ctx->s_main);
    if (rc) {
      free_all();
      if (rc < 0) PA_FAIL("assemble!(I,J,V,rows): device pass failed");
      if (rc == 2) PA_FAIL("assemble!(I,J,V,rows): a ghost row's owner is not in the exchanger's parts_rcv (KeyError)");
      PA_FAIL("to_lids!: a row global id is not a local id of rows (KeyError)");
    }
    sd[i].off.assign(sd[i].cnt.size() + 1, 0);
    for (size_t k = 0; k < sd[i].cnt.size(); ++k) sd[i].off[k + 1] = sd[i].off[k] + sd[i].cnt[k];
  }
  // 2. the counts each part receives, per entry of its parts_snd
  LocalSet L = local_set(n, xg);
  bool remote = false;
  for (int i = 0; i < n; ++i) {
    pa_xchg* X = xg[i];
    sd[i].rcnt.assign(X->parts_snd.size(), 0);
    for (size_t j = 0; j < X->parts_snd.size(); ++j) {
      const int jj = L.find(X->parts_snd[j]);
      if (jj < 0) { remote = true; continue; }
      const auto& q = xg[jj]->parts_rcv;
      const auto it = std::find(q.begin(), q.end(), X->ctx->part);
      if (it == q.end()) { free_all(); PA_FAIL("assemble!: exchanger mismatch (a part in parts_snd does not list this part in parts_rcv)"); }
      sd[i].rcnt[j] = sd[jj].cnt[it - q.begin()];
    }
    for (int32_t q : X->parts_rcv)
      if (L.find(q) < 0) remote = true;
  }
  if (remote) {  // counts of the other processes' parts: one RCCL group of 8 B messages
    std::vector<int64_t*> dsc(n, nullptr), drc(n, nullptr);
    auto free_cnt = [&]() {
      for (int i = 0; i < n; ++i) { (void)hipSetDevice(coo[i]->ctx->device); dev_free(dsc[i]); dev_free(drc[i]); }
    };
    std::vector<P2P> ops;
    for (int i = 0; i < n; ++i) {
      pa_xchg* X = xg[i];
      pa_ctx* c = X->ctx;
      if (!c->comm) { free_cnt(); free_all(); PA_FAIL("assemble!: a neighbour is not held by this process and no RCCL communicator was initialised"); }
      HIPC(hipSetDevice(c->device));
      if (dev_upload(&dsc[i], sd[i].cnt)) { free_cnt(); free_all(); return -1; }
      if (!X->parts_snd.empty()) HIPC(hipMalloc((void**)&drc[i], X->parts_snd.size() * 8));
      for (size_t k = 0; k < X->parts_rcv.size(); ++k)
        if (L.find(X->parts_rcv[k]) < 0)
          ops.push_back({c->part, X->parts_rcv[k], true, (char*)(dsc[i] + k), 8, c->peer_rank(X->parts_rcv[k]),
                         (ncclComm_t)c->comm, c->s_main});
      for (size_t j = 0; j < X->parts_snd.size(); ++j)
        if (L.find(X->parts_snd[j]) < 0)
          ops.push_back({X->parts_snd[j], c->part, false, (char*)(drc[i] + j), 8, c->peer_rank(X->parts_snd[j]),
                         (ncclComm_t)c->comm, c->s_main});
    }
    if (rccl_group(ops)) { free_cnt(); free_all(); return -1; }
    for (int i = 0; i < n; ++i) {
      pa_xchg* X = xg[i];
      HIPC(hipSetDevice(X->ctx->device));
      HIPC(hipStreamSynchronize(X->ctx->s_main));
      std::vector<int64_t> got(X->parts_snd.size());
      if (!got.empty()) HIPC(hipMemcpy(got.data(), drc[i], got.size() * 8, hipMemcpyDeviceToHost));
      for (size_t j = 0; j < X->parts_snd.size(); ++j)
        if (L.find(X->parts_snd[j]) < 0) sd[i].rcnt[j] = got[j];
    }
    free_cnt();
  }
  // 3. the new lists: the local triplets (sent ones now zero), then the
  // received segments in parts_snd order (Interfaces.jl:2470-2486)
  for (int i = 0; i < n; ++i) {
    pa_coo* C = coo[i];
    Side& d = sd[i];
    d.roff.assign(d.rcnt.size() + 1, 0);
    for (size_t j = 0; j < d.rcnt.size(); ++j) d.roff[j + 1] = d.roff[j] + d.rcnt[j];
    d.nn = C->n + d.roff.back();
    HIPC(hipSetDevice(C->ctx->device));
    if (d.nn > 0) {
      hipError_t e = hipMalloc((void**)&d.nI, d.nn * 8);
      if (e == hipSuccess) e = hipMalloc((void**)&d.nJ, d.nn * 8);
      if (e == hipSuccess) e = hipMalloc(&d.nV, d.nn * S);
      if (e != hipSuccess) { free_all(); HIPC(e); }
    }
    if (C->n > 0) {
      hipStream_t st = C->ctx->s_main;
      HIPC(hipMemcpyAsync(d.nI, C->d_I, C->n * 8, hipMemcpyDeviceToDevice, st));
      HIPC(hipMemcpyAsync(d.nJ, C->d_J, C->n * 8, hipMemcpyDeviceToDevice, st));
      HIPC(hipMemcpyAsync(d.nV, C->d_V, C->n * S, hipMemcpyDeviceToDevice, st));
    }
  }
  for (int i = 0; i < n; ++i) {  // every pack has finished before any part reads it
    HIPC(hipSetDevice(coo[i]->ctx->device));
    HIPC(hipStreamSynchronize(coo[i]->ctx->s_main));
  }
  // 4. the segments: device copies between the parts of this process, one
  // RCCL group (I, J, V per segment) for the others
  std::vector<P2P> ops;
  for (int i = 0; i < n; ++i) {
    pa_xchg* X = xg[i];
    pa_ctx* c = X->ctx;
    Side& d = sd[i];
    HIPC(hipSetDevice(c->device));
    for (size_t j = 0; j < X->parts_snd.size(); ++j) {
      const int64_t m = d.rcnt[j];
      if (m == 0) continue;
      const int64_t at = coo[i]->n + d.roff[j];
      const int jj = L.find(X->parts_snd[j]);
      if (jj < 0) {
        const int q = X->parts_snd[j], pr = c->peer_rank(q);
        ncclComm_t cm = (ncclComm_t)c->comm;
        ops.push_back({q, c->part, false, (char*)(d.nI + at), (size_t)m * 8, pr, cm, c->s_main});
        ops.push_back({q, c->part, false, (char*)(d.nJ + at), (size_t)m * 8, pr, cm, c->s_main});
        ops.push_back({q, c->part, false, (char*)d.nV + at * S, (size_t)m * S, pr, cm, c->s_main});
        continue;
      }
      const auto& qr = xg[jj]->parts_rcv;
      const int64_t k = std::find(qr.begin(), qr.end(), c->part) - qr.begin();
      const Side& src = sd[jj];
      const int64_t from = src.off[k];
      const int sdev = xg[jj]->ctx->device;
      if (sdev == c->device) {
        HIPC(hipMemcpyAsync(d.nI + at, src.sI + from, m * 8, hipMemcpyDeviceToDevice, c->s_main));
        HIPC(hipMemcpyAsync(d.nJ + at, src.sJ + from, m * 8, hipMemcpyDeviceToDevice, c->s_main));
        HIPC(hipMemcpyAsync((char*)d.nV + at * S, (const char*)src.sV + from * S, m * S, hipMemcpyDeviceToDevice,
                            c->s_main));
      } else {
        HIPC(hipMemcpyPeerAsync(d.nI + at, c->device, src.sI + from, sdev, m * 8, c->s_main));
        HIPC(hipMemcpyPeerAsync(d.nJ + at, c->device, src.sJ + from, sdev, m * 8, c->s_main));
        HIPC(hipMemcpyPeerAsync((char*)d.nV + at * S, c->device, (const char*)src.sV + from * S, sdev, m * S,
                                c->s_main));
      }
    }
    for (size_t k = 0; k < X->parts_rcv.size(); ++k) {
      const int64_t m = d.cnt[k];
      const int q = X->parts_rcv[k];
      if (m == 0 || L.find(q) >= 0) continue;
      const int pr = c->peer_rank(q);
      ncclComm_t cm = (ncclComm_t)c->comm;
      ops.push_back({c->part, q, true, (char*)(d.sI + d.off[k]), (size_t)m * 8, pr, cm, c->s_main});
      ops.push_back({c->part, q, true, (char*)(d.sJ + d.off[k]), (size_t)m * 8, pr, cm, c->s_main});
      ops.push_back({c->part, q, true, (char*)d.sV + d.off[k] * S, (size_t)m * S, pr, cm, c->s_main});
    }
  }
  if (!ops.empty() && rccl_group(ops)) { free_all(); return -1; }
  for (int i = 0; i < n; ++i) {
    HIPC(hipSetDevice(coo[i]->ctx->device));
    HIPC(hipStreamSynchronize(coo[i]->ctx->s_main));
  }
  // 5. swap in the new lists
  for (int i = 0; i < n; ++i) {
    pa_coo* C = coo[i];
    Side& d = sd[i];
    HIPC(hipSetDevice(C->ctx->device));
    dev_free(C->d_I);
    dev_free(C->d_J);
    dev_free(C->d_V);
    C->d_I = d.nI;
    C->d_J = d.nJ;
    C->d_V = d.nV;
    C->n = d.nn;
    d.nI = nullptr;
    d.nJ = nullptr;
    d.nV = nullptr;
  }
  free_all();
  return 0;
}

// the CSC nz → value map on the host (built on the device by pa_mat_from_coo)
static int load_nz_map(const pa_mat* cA) {
  CHECK_ARG(cA->nz_map, "matrix was not built from a CSC pattern");
  pa_mat* A = const_cast<pa_mat*>(cA);
  if (A->d_nz_slot) {
    HIPC(hipSetDevice(A->ctx->device));
    HIPC(hipStreamSynchronize(A->ctx->s_main));
    A->h_nz_slot.resize(A->csc_nnz);
    HIPC(hipMemcpy(A->h_nz_slot.data(), A->d_nz_slot, A->csc_nnz * 8, hipMemcpyDeviceToHost));
    dev_free(A->d_nz_slot);
    A->d_nz_slot = nullptr;
  }
  return 0;
}

// value index of CSC nz p in d_val (main slot, or ghost-row value after the slots)
static inline int64_t nz_index(const pa_mat* A, int64_t p) {
  const int64_t s = A->h_nz_slot[p];
  return s >= 0 ? s : A->slots - s - 1;
}

// refresh the side SELL's copies of the irregular rows' values
static int refresh_side(pa_mat* A, hipStream_t st) {
  if (A->s_nrows > 0) {
    launch_side_fill(A, A->d_s_rowmap, A->d_s_rowlen, st);
    HIPC(hipGetLastError());
  }
  if (A->t_nrows > 0) {  // and the triple SELL's (values only: the columns are unchanged)
    launch_t_fill(A, 0, false, st);
    HIPC(hipGetLastError());
  }
  if (A->d_uval) {  // and the uniform layout's (build_uniform)
    launch_u_fill(A, st);
    HIPC(hipGetLastError());
  }
  return 0;
}

int pa_mat_set_values(pa_mat* A, const void* nzval) {
  CHECK_ARG(A && nzval, "null argument");
  if (load_nz_map(A)) return -1;
  HIPC(hipSetDevice(A->ctx->device));
  const size_t S = dtype_size(A->dtype);
  const int64_t nv = nvals(A);
  std::vector<unsigned char> hval(nv * S, 0);
  for (int64_t p = 0; p < A->csc_nnz; ++p)
    std::memcpy(&hval[nz_index(A, p) * S], (const unsigned char*)nzval + p * S, S);
  HIPC(hipStreamSynchronize(A->ctx->s_main));
  if (nv) HIPC(hipMemcpy(A->d_val, hval.data(), nv * S, hipMemcpyHostToDevice));
  if (refresh_side(A, A->ctx->s_main)) return -1;
  HIPC(hipStreamSynchronize(A->ctx->s_main));
  return 0;
}

// fillstored!(A, v) (Interfaces.jl:2127-2132 → SparseArrays.fillstored!):
// every stored value of the part becomes v, on the device.  The padding
// slots take v too (never multiplied: masked or column -1 / 0xFFFF).
int pa_mat_fillstored(pa_mat* A, const void* v) {
  CHECK_ARG(A && v, "null argument");
  HIPC(hipSetDevice(A->ctx->device));
  const int64_t nv = nvals(A);
  if (nv) launch_fill(A->dtype, nv, 0, nullptr, A->d_val, v, A->ctx->s_main);
  HIPC(hipGetLastError());
  if (refresh_side(A, A->ctx->s_main)) return -1;
  return 0;
}

int pa_mat_get_values(const pa_mat* A, void* nzval) {
  CHECK_ARG(A && nzval, "null argument");
  if (load_nz_map(A)) return -1;
  HIPC(hipSetDevice(A->ctx->device));
  const size_t S = dtype_size(A->dtype);
  const int64_t nv = nvals(A);
  std::vector<unsigned char> hval(nv * S, 0);
  HIPC(hipStreamSynchronize(A->ctx->s_comm));
  HIPC(hipStreamSynchronize(A->ctx->s_main));
  if (nv) HIPC(hipMemcpy(hval.data(), A->d_val, nv * S, hipMemcpyDeviceToHost));
  for (int64_t p = 0; p < A->csc_nnz; ++p)
    std::memcpy((unsigned char*)nzval + p * S, &hval[nz_index(A, p) * S], S);
  return 0;
}

// Matrix exchanger (Interfaces.jl:2312-2372): lids are CSC nz positions k
// (1-based); they become value indices of d_val.
int pa_mat_xchg_create(pa_mat* A, int32_t n_rcv, const int32_t* parts_rcv, const int32_t* ptrs_rcv,
                       const int64_t* k_rcv, int32_t n_snd, const int32_t* parts_snd, const int32_t* ptrs_snd,
                       const int64_t* k_snd, pa_xchg** out) {
  CHECK_ARG(A && out, "null argument");
  if (load_nz_map(A)) return -1;
  CHECK_ARG(nvals(A) < ((int64_t)1 << 31), "matrix exchanger: value index exceeds int32");
  CHECK_ARG(n_rcv >= 0 && n_snd >= 0, "negative neighbour count");
  auto conv = [&](int32_t n, const int32_t* ptrs, const int64_t* k, std::vector<int32_t>& o) -> int {
    const int64_t m = n > 0 ? (int64_t)ptrs[n] - 1 : 0;
    CHECK_ARG(m >= 0, "matrix exchanger: bad ptrs");
    o.resize(m);
    for (int64_t i = 0; i < m; ++i) {
      CHECK_ARG(k[i] >= 1 && k[i] <= A->csc_nnz, "matrix exchanger: nz index out of range");
      o[i] = (int32_t)(nz_index(A, k[i] - 1) + 1);
    }
    return 0;
  };
  std::vector<int32_t> lr, ls;
  if (conv(n_rcv, ptrs_rcv, k_rcv, lr) || conv(n_snd, ptrs_snd, k_snd, ls)) return -1;
  return pa_xchg_create(A->ctx, n_rcv, parts_rcv, ptrs_rcv, lr.data(), n_snd, parts_snd, ptrs_snd, ls.data(),
                        out);
}

// exchange!(A) / assemble!(A) (Interfaces.jl:2375-2404) for n local parts:
// the vector exchange over nonzeros(A); assemble zeroes the sent ghost-row
// values afterwards (2398) and refreshes the side SELL copies.
int pa_mat_exchange_all(int n, pa_mat* const A[], pa_xchg* const xg[], int op, int reverse, int zero_sent) {
  CHECK_ARG(n >= 1 && A && xg && A[0], "null argument");
  TuneScope ts(A[0]->ctx);
  std::vector<pa_vec> vs(n);
  std::vector<pa_vec*> vp(n);
  for (int i = 0; i < n; ++i) {
    CHECK_ARG(A[i] && xg[i] && A[i]->ctx == xg[i]->ctx, "exchange!(A): matrix and exchanger of different parts");
    vs[i].ctx = A[i]->ctx;
    vs[i].dtype = A[i]->dtype;
    vs[i].n = nvals(A[i]);
    vs[i].d = A[i]->d_val;
    vp[i] = &vs[i];
  }
  if (pa_exchange_all(n, vp.data(), xg, nullptr, op, reverse, 0)) return -1;
  for (int i = 0; i < n; ++i) {
    pa_ctx* c = A[i]->ctx;
    HIPC(hipSetDevice(c->device));
    if (zero_sent) {
      unsigned char z[16] = {0};
      if (reverse) launch_fill(A[i]->dtype, xg[i]->n_rcv_data, 0, xg[i]->d_lids_rcv, A[i]->d_val, z, c->s_main);
      else launch_fill(A[i]->dtype, xg[i]->n_snd_data, 0, xg[i]->d_lids_snd, A[i]->d_val, z, c->s_main);
    }
    if (refresh_side(A[i], c->s_main)) return -1;
  }
  HIPC(hipGetLastError());
  return 0;
}

int pa_mat_destroy(pa_mat* A) {
  if (!A) return 0;
  (void)hipSetDevice(A->ctx->device);
  (void)hipStreamSynchronize(A->ctx->s_main);
  dev_free(A->d_slice_off);
  dev_free(A->d_slice_len);
  dev_free(A->d_int_list);
  dev_free(A->d_bnd_list);
  dev_free(A->d_col);
  dev_free(A->d_val);
  dev_free(A->d_nz_slot);
  for (void* p : {(void*)A->d_kind, (void*)A->d_plen, (void*)A->d_pdesc, (void*)A->d_pat, (void*)A->d_mask,
                  (void*)A->d_pint_list, (void*)A->d_pbnd_list, (void*)A->d_xint_list,
                  (void*)A->d_xbnd_list, (void*)A->d_s_off, (void*)A->d_s_len,
                  (void*)A->d_s_col, A->d_s_val, (void*)A->d_s_rowmap, (void*)A->d_s_rowlen, A->d_dotp,
                  (void*)A->d_long_row, (void*)A->d_long_ptr, (void*)A->d_long_col, (void*)A->d_sflags,
                  (void*)A->d_lmask, (void*)A->d_lchunk_start, (void*)A->d_lrow_chunk, A->d_lpart,
                  (void*)A->d_col16, (void*)A->d_gbase, (void*)A->d_dint_list, (void*)A->d_dbnd_list})
    dev_free(p);
  free_triple_sell(A);
  free_uniform(A);
  delete A;
  return 0;
}

int pa_mat_format_info(const pa_mat* A, int64_t* pattern_slices, int64_t* regular_rows,
                       int64_t* side_rows, int64_t* side_slots) {
  CHECK_ARG(A, "null matrix");
  if (pattern_slices) *pattern_slices = A->npattern_slices;
  if (regular_rows) *regular_rows = A->nregular_rows;
  if (side_rows) *side_rows = A->s_nrows;
  if (side_slots) *side_slots = A->s_slots;
  return 0;
}

int pa_mat_delta16_info(const pa_mat* A, int64_t* delta16_slices) {
  CHECK_ARG(A, "null matrix");
  if (delta16_slices) *delta16_slices = A->nd_int + A->nd_bnd;
  return 0;
}

int pa_mat_pair_info(const pa_mat* A, int64_t* pair_slices, int64_t* pair_rows) {
  CHECK_ARG(A, "null matrix");
  if (pair_slices) *pair_slices = A->t_pair_slices;
  if (pair_rows) *pair_rows = A->t_pair_rows;
  return 0;
}

int pa_mat_triple_info(const pa_mat* A, int64_t* t_slices, int64_t* t_rows, int64_t* tri_slices,
                       int64_t* tri_rows) {
  CHECK_ARG(A, "null matrix");
  if (t_slices) *t_slices = A->t_nslices;
  if (t_rows) *t_rows = A->t_nrows;
  if (tri_slices) *tri_slices = A->t_tri_slices;
  if (tri_rows) *tri_rows = A->t_tri_rows;
  return 0;
}

int pa_mat_long_rows(const pa_mat* A, int64_t* n_long, int64_t* n_long_nnz) {
  CHECK_ARG(A, "null matrix");
  if (n_long) *n_long = A->n_long;
  if (n_long_nnz) *n_long_nnz = A->n_lnz;
  return 0;
}

// Bytes one mul! streams from the matrix in its current encoding (the
// kernels' own loads, padding included): values, column ids, and the slice
// metadata (offsets, lengths, lists, patterns, masks, side-row maps).
int pa_mat_device_ptrs(const pa_mat* A, uint64_t out[8]) {
  CHECK_ARG(A && out, "null argument");
  const void* p[8] = {A->d_val, A->d_col, A->d_slice_off, A->d_plen, A->d_pat, A->d_mask, A->d_s_val, A->d_s_col};
  for (int i = 0; i < 8; ++i) out[i] = (uint64_t)(uintptr_t)p[i];
  return 0;
}

int pa_mat_traffic(const pa_mat* A, int64_t* value_bytes, int64_t* index_bytes, int64_t* meta_bytes) {
  CHECK_ARG(A, "null matrix");
  TuneScope ts(A->ctx);
  const int64_t S = (int64_t)dtype_size(A->dtype), H = A->H, W = H / 64;
  const bool pat = knobs().spmv_format == 1 && A->has_pat;
  const bool split = A->d_bnd_list != nullptr;
  int64_t v = 0, ix = 0, m = 0;
  for (int64_t s = 0; s < A->nslices; ++s) {
    const int kd = pat ? A->h_kind[s] : 0;
    if (kd == 1) {
      // (the uniform layout: the short-row tail launch reads K entries)
      v += (int64_t)(A->d_uval ? A->uK : A->h_plen[s]) * H * S;
      // mask, offset, length | pattern id, list entry; with SPMV_DESC the
      // descriptor instead (desc_words): counted as the larger
      m += std::max<int64_t>(W * 8 + 8 + 4, 4 * desc_words(A->R)) + 4;
    } else if (kd == 3) {
      v += (int64_t)A->h_slen[s] * H * S;
      ix += (int64_t)A->h_slen[s] * H * 2;
      m += 8 + 4 + 4 + 4;  // offset, length, list entry, ghost base
    } else if (kd == 5) {
      // rows in the triple SELL (below)
    } else {
      v += (int64_t)A->h_slen[s] * H * S;
      ix += (int64_t)A->h_slen[s] * H * 4;
      m += 8 + 4 + ((pat || split) ? 4 : 0);
    }
  }
  if (pat) {
    m += A->npatterns * A->kmax * 4;  // the distinct patterns (read once; hot thereafter)
    v += A->s_slots * S;
    ix += A->s_slots * 4 + A->s_nrows * 4;  // column ids, row map
    m += A->s_nslices * 12;
    v += A->t_slots * S;              // triple SELL: values (padding included)
    ix += A->t_code_slots * 2 + A->t_nrows * 4;  // codes (one per triple in tri slices), row map
    m += A->t_nslices * (8 + 4 + 4 + 4);  // offset, length, ghost base, list entry (the 16 B descriptor + list entry)
  }
  v += A->n_lnz * S;
  ix += A->n_lnz * 4;
  m += A->n_long * 16;
  if (value_bytes) *value_bytes = v;
  if (index_bytes) *index_bytes = ix;
  if (meta_bytes) *meta_bytes = m;
  return 0;
}

int pa_mat_info(const pa_mat* A, int64_t* nrows, int64_t* nnz, int64_t* slots, int64_t* nslices,
                int64_t* nslices_int) {
  CHECK_ARG(A, "null matrix");
  if (nrows) *nrows = A->nrows;
  if (nnz) *nnz = A->nnz;
  if (slots) *slots = A->slots;
  if (nslices) *nslices = A->nslices;
  if (nslices_int) *nslices_int = A->nslices_int;
  return 0;
}

// ---------------------------------------------------------------------------
// mul! for the n local parts; with want_dot each part's dot(x, y) over its
// owned rows is accumulated by the SpMV kernel itself (per-slice partials in
// A->d_dotp, folded by fold_dot) — the CG's `dot(u, c)` after `mul!(c, A, u)`.
constexpr int kMaxTimed = 1024;  // mul! calls recorded per context between reads

// The device CG's fused u update of one mul!(c, A, u) (pa_cg_solve_all): the
// call's x is r; per part the old u, the buffer for the new u, x (for the
// deferred x .+= α.*u) and the CG state.  The SpMV kernels (XV) compute
// u_new = r .+ β.*u_old on the fly; the ghost lids (after the halo of r)
// get u_new and the x update from k_cg_ghost.
struct CGFuse {
  std::vector<const void*> u_old;
  std::vector<void*> u_new, xacc;
  std::vector<CGState*> st;
};

// u_new and the deferred x update of part i's ghost lids (owned lids are
// 0..noids-1: the device CG needs contiguous owned lids), after the halo and
// before the dot fold (whose α step marks the x update as applied)
static void cg_ghosts(const CGFuse* fz, int i, const pa_mat* A, const pa_vec* r, hipStream_t st) {
  if (!fz || r->n <= A->nrows) return;
  launch_cg_ghost(A->dtype, A->nrows, r->n, r->d, fz->u_old[i], fz->u_new[i], fz->xacc[i], fz->st[i], st);
}

// The grouped path applies when every part of the call shares one stream
// pair (pa_ctx_create_shared: same device, one in-order chain) and every
// halo neighbour is a part of this call served by the pull-unpack.
// Returns 0 (per-part launches), 1 (grouped: pack + pull on the comm
// stream, overlapped with the interior slices) or 2 (grouped, direct pull:
// the ghosts read straight from the owners' x on the compute stream, one
// in-order chain without cross-stream events, pa_tune("halo_direct")).
static int group_ok(int n, pa_mat* const A[], pa_xchg* const xg[], bool any_x, int dt) {
  if (!knobs().spmv_group || (n < 2 && any_x)) return 0;  // one part without a halo: the merged launch
  const pa_ctx* c0 = A[0]->ctx;
  for (int i = 0; i < n; ++i)
    if (A[i]->ctx->s_main != c0->s_main || A[i]->ctx->s_comm != c0->s_comm) return 0;
  if (!any_x) return 1;
  if (!knobs().halo_pull) return 0;
  LocalSet L = local_set(n, xg);
  for (int i = 0; i < n; ++i)
    for (const auto* lst : {&xg[i]->parts_snd, &xg[i]->parts_rcv})
      for (int32_t q : *lst)
        if (L.find(q) < 0) return 0;
  for (int i = 0; i < n; ++i)
    if (!xg[i]->plan_fwd.unique) return 0;
  if (knobs().halo_direct) {
    bool ok = true;
    for (int i = 0; i < n && ok; ++i) {
      if (build_direct(i, n, xg, L)) return 0;
      ok = xg[i]->direct.ok;
    }
    if (ok) return 2;
  }
  for (int i = 0; i < n; ++i) {
    if (build_pull(i, n, xg, L, dt, 0)) return 0;
    if (!xg[i]->pull[0].ok) return 0;
  }
  return 1;
}

// mul! over parts sharing a stream pair: one pack, one pull-unpack and one
// launch per slice kind and phase for all parts (kernel-argument tables),
// instead of the same sequence per part.  Every slice is computed by the
// same wave code as in the per-part launches: results are identical.
static int spmv_grouped(int n, pa_mat* const A[], pa_vec* const y[], const pa_index* const y_idx[],
                        pa_vec* const x[], pa_xchg* const xg[], bool any_x, bool has_alpha, int bmode,
                        const void* alpha, const void* beta, const std::vector<void*>& dotp, bool want_dot,
                        CGState* const* dot_tail, const std::vector<hipEvent_t*>& tslot, int dt, bool direct,
                        const CGFuse* fz) {
  pa_ctx* c0 = A[0]->ctx;
  HIPC(hipSetDevice(c0->device));
  const hipStream_t sm = c0->s_main, sc = c0->s_comm;
  auto mark = [&](int k) -> int {
    for (int i = 0; i < n; ++i)
      if (tslot[i]) HIPC(hipEventRecord(tslot[i][k], sm));
    return 0;
  };
  // timing marks of the direct pull: no slice runs before the halo is
  // complete, so interior = 0, halo = the pull, boundary = every slice
  const bool dmark = any_x && direct;
  if (dmark && (mark(0) || mark(1))) return -1;
  if (any_x && direct) {
    // every ghost of x straight from its owner's x, in stream order before
    // the slices (owned values are only read, ghosts only written)
    void** bases = direct_bases(c0, n, x);
    if (!bases) return -1;
    PullGroup qg{};
    for (int i0 = 0; i0 < n; i0 += PA_GROUP_MAX) {
      qg.np = 0;
      for (int i = i0; i < n && i < i0 + PA_GROUP_MAX; ++i) {
        pa_xchg* X = xg[i];
        const int k = qg.np++;
        qg.n[k] = X->n_rcv_data;
        qg.lids[k] = X->d_lids_rcv;
        qg.bid[k] = X->direct.d_bid;
        qg.elem[k] = X->direct.d_elem;
        qg.bases[k] = (const void* const*)bases;
        qg.v[k] = x[i]->d;
      }
      launch_pull_group(dt, qg, sm);
    }
  } else if (any_x) {
    // the previous exchange's pulls read the send buffers: pack after them
    HIPC(hipStreamWaitEvent(c0->s_main, c0->ev_recvd, 0));
    for (int i = 0; i < n; ++i) xg[i]->fast_key = 0;
    PackGroup pg{};
    PullGroup qg{};
    for (int i0 = 0; i0 < n; i0 += PA_GROUP_MAX) {
      pg.np = qg.np = 0;
      for (int i = i0; i < n && i < i0 + PA_GROUP_MAX; ++i) {
        pa_xchg* X = xg[i];
        const int k = pg.np++;
        pg.n[k] = X->n_snd_data;
        pg.lids[k] = X->d_lids_snd;
        pg.v[k] = x[i]->d;
        pg.buf[k] = X->d_buf_snd;
      }
      launch_pack_group(dt, pg, sm);
    }
    HIPC(hipEventRecord(c0->ev_packed, sm));
    HIPC(hipStreamWaitEvent(sc, c0->ev_packed, 0));
    for (int i0 = 0; i0 < n; i0 += PA_GROUP_MAX) {
      qg.np = 0;
      for (int i = i0; i < n && i < i0 + PA_GROUP_MAX; ++i) {
        pa_xchg* X = xg[i];
        const pa_pull& P = X->pull[0];
        const int k = qg.np++;
        qg.n[k] = X->n_rcv_data;
        qg.lids[k] = X->d_lids_rcv;
        qg.bid[k] = P.d_bid;
        qg.elem[k] = P.d_elem;
        qg.bases[k] = (const void* const*)P.d_bases;
        qg.v[k] = x[i]->d;
      }
      launch_pull_group(dt, qg, sc);
    }
    HIPC(hipEventRecord(c0->ev_recvd, sc));
  }
  HIPC(hipGetLastError());
  std::vector<SpmvPart> P0, P1, P4, P5;
  auto part = [&](int i, int64_t nwork, const int32_t* list) {
    const int32_t* ymap = y_idx[i]->own_contig ? nullptr : y_idx[i]->d_oid_to_lid;
    SpmvPart q{nwork, list, A[i], x[i]->d, y[i]->d, ymap, dotp[i]};
    if (fz) {
      q.xu = fz->u_old[i];
      q.un = fz->u_new[i];
      q.xacc = fz->xacc[i];
      q.cg = fz->st[i];
    }
    return q;
  };
  auto launch_all = [&](int which, const std::vector<SpmvPart>& v, hipStream_t st = nullptr) {
    if (!v.empty()) launch_spmv_group(which, (int)v.size(), v.data(), has_alpha, bmode, alpha, beta, st ? st : sm);
  };
  if (dmark ? mark(2) : mark(0)) return -1;
  // no halo in flight (none, or pulled already on this stream): every slice
  // kind of every part in one launch — side rows and int32 slices first, so
  // their few long waves start early, then delta16, multi-pattern, pattern
  int merged = 1;
  bool big_part = false;  // one part alone fills the GPU many times: per-kind launches (knobs().spmv_merge_max)
  if (knobs().spmv_merge_max > 0 && n == 1) big_part = A[0]->nslices > knobs().spmv_merge_max;
  // parts of pattern slices and short side rows only, no halo: the per-kind
  // path's side tail is ONE launch too, through the group kernel (its
  // arguments in the kernel's argument segment, no table search per wave):
  // C2 FD7 128³ 0.0285-0.0286 -> 0.0281 ms, FE27 128³ one part 0.0843 ->
  // 0.0817 (profiles/r05/y,z/); not for Float32's 256-row slices (C2 F32
  // 0.0195 -> 0.0216 ms, z/)
  bool tail_only = knobs().side_tail && !any_x && !fz && 2 * n <= PA_GROUP_MAX && A[0]->R <= 2;
  for (int i = 0; i < n && tail_only; ++i) {
    const pa_mat* M = A[i];
    tail_only = knobs().spmv_format == 1 && M->has_pat && M->np_bnd == 0 && M->nx_int + M->nx_bnd == 0 &&
                M->nd_int + M->nd_bnd == 0 && M->t_nslices == 0 && M->n_long == 0 &&
                (M->s_nslices == 0 || M->maxlen_side <= 8);
  }
  if (knobs().spmv_merge && !big_part && !tail_only && (!any_x || direct)) {
    std::vector<SpmvPart> E;
    std::vector<int> W;
    auto add = [&](int which, int i, int64_t nwork, const int32_t* list) {
      if (nwork <= 0) return;
      E.push_back(part(i, nwork, list));
      W.push_back(which);
    };
    // (side rows first also when they are short: FD7's Dirichlet rows last
    // made C2 0.7 % slower, 0.0285 -> 0.0287 ms, profiles/r05/o/)
    for (int i = 0; i < n; ++i)
      if (knobs().spmv_format == 1 && A[i]->has_pat) add(2, i, A[i]->s_nslices, nullptr);
    for (int i = 0; i < n; ++i) {
      if (knobs().spmv_format == 1 && A[i]->has_pat) {
        add(1, i, A[i]->nx_int, A[i]->d_xint_list);
        add(1, i, A[i]->nx_bnd, A[i]->d_xbnd_list);
      } else if (A[i]->d_bnd_list) {
        add(1, i, A[i]->nslices_int, A[i]->d_int_list);
        add(1, i, A[i]->nslices - A[i]->nslices_int, A[i]->d_bnd_list);
      } else {
        add(1, i, A[i]->nslices, nullptr);
      }
    }
    for (int i = 0; i < n; ++i)
      if (knobs().spmv_format == 1 && A[i]->has_pat) {
        add(4, i, A[i]->nd_int, A[i]->d_dint_list);
        add(4, i, A[i]->nd_bnd, A[i]->d_dbnd_list);
        add(5, i, A[i]->t_nslices, nullptr);
      }
    for (int i = 0; i < n; ++i)
      if (knobs().spmv_format == 1 && A[i]->has_pat) {
        add(0, i, A[i]->np_int, A[i]->d_pint_list);
        add(0, i, A[i]->np_bnd, A[i]->d_pbnd_list);
      }
    merged = launch_spmv_merged((int)E.size(), W.data(), E.data(), has_alpha, bmode, alpha, beta, c0,
                                sm);
    if (merged < 0) PA_FAIL("mul!: merged launch table (device allocation or copy) failed");
    if (merged == 0 && !dmark && (mark(1) || mark(2))) return -1;
  }
  if (merged) {
  // interior slices (no ghost column): overlap with the pulls on the comm stream
  for (int i = 0; i < n; ++i) {
    if (knobs().spmv_format == 1 && A[i]->has_pat) {
      P0.push_back(part(i, A[i]->np_int, A[i]->d_pint_list));
      P1.push_back(part(i, A[i]->nx_int, A[i]->d_xint_list));
      P4.push_back(part(i, A[i]->nd_int, A[i]->d_dint_list));
      P5.push_back(part(i, A[i]->nt_int, A[i]->d_t_int_list));
    } else if (A[i]->d_bnd_list) {
      P1.push_back(part(i, A[i]->nslices_int, A[i]->d_int_list));
    } else {
      P1.push_back(part(i, A[i]->nslices, nullptr));
    }
  }
  // the side rows as the pattern launch's trailing waves (spmv_side_tail):
  // no halo in flight, the side rows short, pattern and side entries within
  // one group launch, no fused CG update
  bool side_tailed = false;
  if (knobs().side_tail && (!any_x || direct) && !fz && 2 * n <= PA_GROUP_MAX) {
    bool ok = false;
    for (int i = 0; i < n; ++i) {
      const bool pat = knobs().spmv_format == 1 && A[i]->has_pat;
      if (!pat) { ok = false; break; }
      if (A[i]->s_nslices > 0) {
        if (A[i]->maxlen_side > 8) { ok = false; break; }
        ok = true;
      }
    }
    if (ok) {
      std::vector<SpmvPart> PT = P0;
      for (int i = 0; i < n; ++i)
        if (A[i]->s_nslices > 0) {
          SpmvPart q = part(i, A[i]->s_nslices, nullptr);
          q.side = true;
          PT.push_back(q);
        }
      launch_all(6, PT);
      side_tailed = true;
    }
  }
  if (!side_tailed) launch_all(0, P0);
  launch_all(5, P5);
  launch_all(4, P4);
  launch_all(1, P1);
  if (!dmark && mark(1)) return -1;
  if (any_x && !direct) HIPC(hipStreamWaitEvent(sm, c0->ev_recvd, 0));
  if (!dmark && mark(2)) return -1;
  P0.clear(); P1.clear(); P4.clear(); P5.clear();
  std::vector<SpmvPart> P2;
  for (int i = 0; i < n; ++i) {
    if (knobs().spmv_format == 1 && A[i]->has_pat) {
      P0.push_back(part(i, A[i]->np_bnd, A[i]->d_pbnd_list));
      P4.push_back(part(i, A[i]->nd_bnd, A[i]->d_dbnd_list));
      P5.push_back(part(i, A[i]->nt_bnd, A[i]->d_t_bnd_list));
      P1.push_back(part(i, A[i]->nx_bnd, A[i]->d_xbnd_list));
      if (!side_tailed) P2.push_back(part(i, A[i]->s_nslices, nullptr));
    } else if (A[i]->d_bnd_list) {
      P1.push_back(part(i, A[i]->nslices - A[i]->nslices_int, A[i]->d_bnd_list));
    }
  }
  launch_all(0, P0);
  launch_all(5, P5);
  launch_all(4, P4);
  launch_all(1, P1);
  launch_all(2, P2);
  }  // per-kind launches
  for (int i = 0; i < n; ++i) {
    const int32_t* ymap = y_idx[i]->own_contig ? nullptr : y_idx[i]->d_oid_to_lid;
    const bool pat = knobs().spmv_format == 1 && A[i]->has_pat;
    const int64_t long_base = A[i]->nslices + (pat ? A[i]->s_nslices + A[i]->t_nslices : 0);
    cg_ghosts(fz, i, A[i], x[i], sm);
    launch_spmv_long(A[i], x[i]->d, y[i]->d, ymap, has_alpha, bmode, alpha, beta, dotp[i], long_base, sm);
    if (want_dot) {
      pa_ctx* c = A[i]->ctx;
      const bool cplx = dt == PA_C64 || dt == PA_C128;
      const int nbp = (int)(long_base + A[i]->n_long);
      if (dot_tail)
        launch_fold_cg_alpha(dt, nbp, A[i]->d_dotp, c->d_fold, c->d_result, c->d_ticket, dot_tail[i], sm);
      else
        launch_fold(cplx, nbp, A[i]->d_dotp, c->d_fold, c->d_result, c->d_ticket, sm);
    }
  }
  if (mark(3)) return -1;
  HIPC(hipGetLastError());
  for (int i = 0; i < n; ++i)
    if (tslot[i]) ++A[i]->ctx->tn;
  return 0;
}

// One phase of one part's slices (0: interior, before the halo; 1: boundary
// slices and side rows, after it): one merged launch (pa_tune spmv_merge)
// or one launch per slice kind.
static int launch_phase(int phase, pa_mat* A, const void* x, void* y, const int32_t* ymap, bool has_alpha,
                        int bmode, const void* alpha, const void* beta, void* dotp, hipStream_t st,
                        const CGFuse* fz = nullptr, int fi = 0) {
  std::vector<SpmvPart> E;
  std::vector<int> W;
  auto add = [&](int which, int64_t nwork, const int32_t* list) {
    if (nwork <= 0) return;
    SpmvPart q{nwork, list, A, x, y, ymap, dotp};
    if (fz) {
      q.xu = fz->u_old[fi];
      q.un = fz->u_new[fi];
      q.xacc = fz->xacc[fi];
      q.cg = fz->st[fi];
    }
    E.push_back(q);
    W.push_back(which);
  };
  if (knobs().spmv_format == 1 && A->has_pat) {
    if (phase == 0) {
      add(1, A->nx_int, A->d_xint_list);
      add(4, A->nd_int, A->d_dint_list);
      add(5, A->nt_int, A->d_t_int_list);
      add(0, A->np_int, A->d_pint_list);
    } else {
      add(2, A->s_nslices, nullptr);
      add(1, A->nx_bnd, A->d_xbnd_list);
      add(4, A->nd_bnd, A->d_dbnd_list);
      add(5, A->nt_bnd, A->d_t_bnd_list);
      add(0, A->np_bnd, A->d_pbnd_list);
    }
  } else if (A->d_bnd_list) {  // split layout (the interior list may be empty)
    if (phase == 0) add(1, A->nslices_int, A->d_int_list);
    else add(1, A->nslices - A->nslices_int, A->d_bnd_list);
  } else if (phase == 0) {
    add(1, A->nslices, nullptr);
  }
  if (E.empty()) return 0;
  if (E.size() > 1 && knobs().spmv_merge && !(knobs().spmv_merge_max > 0 && A->nslices > knobs().spmv_merge_max)) {
    const int rc = launch_spmv_merged((int)E.size(), W.data(), E.data(), has_alpha, bmode, alpha, beta, A->ctx,
                                      st);
    if (rc < 0) PA_FAIL("mul!: merged launch table (device allocation or copy) failed");
    if (rc == 0) return 0;
  }
  for (size_t k = 0; k < E.size(); ++k)
    launch_spmv_part(W[k], E[k].nwork, E[k].list, A, x, y, ymap, has_alpha, bmode, alpha, beta, dotp, st, &E[k]);
  return 0;
}

// Barrier issue of a mul! over parts with their own stream pairs and local
// neighbours (pa_tune "halo_barrier"; the model of one process driving
// several GPUs, SequentialBackend.jl:52-58's map_parts over every part):
//   A  per part: pack into send buffer b, record ev_packed, interior slices
//      (the first call of a chain first waits for the previous exchange's
//      reads of the send buffers, pre_pack_wait_part);
//   B  the leading part's s_comm waits for every part's pack and records
//      ev_barrier — one wait per part instead of one per neighbour and part;
//   C  per part: s_comm waits ev_barrier, pulls its ghosts from the senders'
//      buffers b and records ev_recvd; s_main waits ev_recvd, boundary slices
//      (halo_barrier 2: s_main waits ev_barrier and pulls itself, after its
//      interior slices, then the boundary slices: one runtime call less per
//      part, the pull no longer beside the interior).
// b alternates between d_buf_snd and d_buf_snd2 from one call to the next,
// so a pack does not wait for the readers of the previous call's buffer: the
// last reads of b before pack(k+2) are the pulls of call k, and every part
// issued its pack(k+1) after its boundary(k), i.e. after its pull(k); pack(k+2)
// follows barrier(k+1) on the part's own chain (s_comm → ev_recvd → s_main).
// That holds while consecutive calls cover the same exchanger set
// (pa_xchg::fast_key / fast_seq); any other use of the send buffers
// (pre_pack_wait_part, the grouped path) restarts the chain with the waits.
// About 8 HIP calls per part and call instead of ≈24.
static int spmv_barrier_issue(int n, pa_vec* const x[], pa_xchg* const xg[], int dt, const TransportPlan& T,
                              bool threads, const std::function<int(int)>& interior,
                              const std::function<int(int)>& boundary, bool pull_on_main) {
  uint64_t key = 1469598103934665603ull ^ (uint64_t)n;
  for (int i = 0; i < n; ++i) key = (key ^ xg[i]->id) * 1099511628211ull;
  bool chain = true;
  for (int i = 0; i < n; ++i) chain = chain && xg[i]->fast_key == key && xg[i]->fast_seq == xg[0]->fast_seq;
  const int parity = chain ? (xg[0]->fast_parity ^ 1) : 0;
  for (int i = 0; i < n; ++i) xg[i]->fast_key = 0;  // set again once the call is issued
  TransportPlan TB = T;
  TB.alt = parity == 1;
  TB.on_main = pull_on_main;
  if (TB.alt) {  // the second send buffers and the pull tables reading them
    for (int i = 0; i < n; ++i)
      if (!xg[i]->d_buf_snd2 && xg[i]->n_snd_data) {
        HIPC(hipSetDevice(xg[i]->ctx->device));
        HIPC(hipMalloc(&xg[i]->d_buf_snd2, xg[i]->n_snd_data * 16));
      }
    for (int i = 0; i < n; ++i) {
      if (build_pull(i, n, xg, T.L, dt, 0, true)) return -1;
      CHECK_ARG(xg[i]->pull_alt.ok, "mul!: pull table of the second send buffers (internal error)");
    }
  }
  pa_ctx* c0 = xg[0]->ctx;
  if (!c0->ev_barrier) {
    HIPC(hipSetDevice(c0->device));
    HIPC(hipEventCreateWithFlags(&c0->ev_barrier, hipEventDisableTiming));
  }
  const LocalSet& L = T.L;
  auto stepA = [&](int i) -> int {
    pa_xchg* X = xg[i];
    pa_ctx* c = X->ctx;
    if (!chain && pre_pack_wait_part(i, xg, L)) return -1;
    HIPC(hipSetDevice(c->device));
    launch_pack(dt, X->n_snd_data, X->d_lids_snd, x[i]->d, TB.alt ? X->d_buf_snd2 : X->d_buf_snd, c->s_main,
                c->ev_packed);
    // the barrier stream's wait for this pack, from this part's thread (the
    // record of ev_barrier follows once every part's job is done)
    HIPC(hipStreamWaitEvent(c0->s_comm, c->ev_packed, 0));
    return interior(i);
  };
  auto stepC = [&](int i) -> int {
    pa_ctx* c = xg[i]->ctx;
    HIPC(hipSetDevice(c->device));
    if (pull_on_main) HIPC(hipStreamWaitEvent(c->s_main, c0->ev_barrier, 0));
    else if (i) HIPC(hipStreamWaitEvent(c->s_comm, c0->ev_barrier, 0));
    if (transport_local(i, xg, x, TB)) return -1;
    return boundary(i);
  };
  if (threads) {
    if (IssuePool::get().run(n, stepA)) return -1;
  } else {
    for (int i = 0; i < n; ++i)
      if (stepA(i)) return -1;
  }
  HIPC(hipSetDevice(c0->device));
  HIPC(hipEventRecord(c0->ev_barrier, c0->s_comm));
  if (threads) {
    if (IssuePool::get().run(n, stepC)) return -1;
  } else {
    for (int i = 0; i < n; ++i)
      if (stepC(i)) return -1;
  }
  static std::atomic<uint64_t> seq_next{1};
  const uint64_t seq = seq_next.fetch_add(1);
  for (int i = 0; i < n; ++i) {
    xg[i]->fast_key = key;
    xg[i]->fast_seq = seq;
    xg[i]->fast_parity = parity;
  }
  return 0;
}

static int spmv_impl(int n, pa_mat* const A[], pa_vec* const y[], const pa_index* const y_idx[],
                     pa_vec* const x[], const pa_index* const x_idx[], pa_xchg* const xg[],
                     const void* alpha, const void* beta, bool want_dot, CGState* const* dot_tail = nullptr,
                     const CGFuse* fz = nullptr) {
  CHECK_ARG(n >= 1 && A && y && x && alpha && beta, "null argument");
  const int dt = A[0]->dtype;
  bool any_x = false;
  std::vector<void*> dotp(n, nullptr);
  if (want_dot) {
    for (int i = 0; i < n; ++i) {
      CHECK_ARG(x_idx && x_idx[i] && x_idx[i]->own_contig, "fused dot needs b with contiguous owned lids");
      if (!A[i]->d_dotp) {
        HIPC(hipSetDevice(A[i]->ctx->device));
        // one partial per main, side and triple-SELL slice and long row;
        // zeroed once: the slices a call does not launch (moved to the
        // triple SELL) add 0 to the fold
        const int64_t nbp = std::max<int64_t>(A[i]->nslices + A[i]->s_nslices + A[i]->t_nslices + A[i]->n_long, 1);
        HIPC(hipMalloc(&A[i]->d_dotp, nbp * 16));
        HIPC(hipMemset(A[i]->d_dotp, 0, nbp * 16));
      }
      dotp[i] = A[i]->d_dotp;
    }
  }
  for (int i = 0; i < n; ++i) {
    CHECK_ARG(A[i] && y[i] && x[i], "null handle");
    CHECK_ARG(A[i]->dtype == dt && y[i]->dtype == dt && x[i]->dtype == dt, "mul!: element types differ");
    CHECK_ARG(x[i]->n == A[i]->ncols_lids, "mul!: length(b.values) != num_lids(a.cols) (DimensionMismatch)");
    const pa_index* yi = y_idx ? y_idx[i] : nullptr;
    CHECK_ARG(yi && yi->noids == A[i]->nrows && yi->nlids == y[i]->n,
              "mul!: c.rows owned ids differ from a.rows (oids_are_equal)");
    if (x_idx && x_idx[i]) {
      const pa_index* xi = x_idx[i];
      CHECK_ARG(xi->nlids == A[i]->ncols_lids, "mul!: b.rows differs from a.cols");
    }
    if (xg && xg[i]) any_x = true;
  }
  const bool has_alpha = !scalar_is(dt, alpha, 1.0);
  const int bmode = scalar_is(dt, beta, 0.0) ? 0 : (scalar_is(dt, beta, 1.0) ? 1 : 2);
  bool pulled = false;
  bool pulled_on_main = false;  // the pull ran on s_main itself (halo_barrier 2): no ev_recvd wait
  // timing: the events of this call (slot tn of each timed context); the
  // grouped path brackets all parts with the same launches: part 1 of the
  // call records them once
  if (any_x)  // before group_ok, which reads every exchanger
    for (int i = 0; i < n; ++i) {
      CHECK_ARG(xg[i] && xg[i]->ctx == x[i]->ctx, "mul!: exchanger missing for some parts");
      if (check_lids(xg[i], x[i])) return -1;
    }
  const int gmode = group_ok(n, A, xg, any_x, dt);
  const bool grouped = gmode != 0;
  std::vector<hipEvent_t*> tslot(n, nullptr);
  for (int i = 0; i < n; ++i) {
    pa_ctx* c = A[i]->ctx;
    if (!c->timing || c->tn >= kMaxTimed || (grouped && i > 0)) continue;
    if ((int)c->tev.size() < 4 * (c->tn + 1)) {
      HIPC(hipSetDevice(c->device));
      for (int k = 0; k < 4; ++k) {
        hipEvent_t e;
        HIPC(hipEventCreate(&e));
        c->tev.push_back(e);
      }
    }
    tslot[i] = &c->tev[4 * c->tn];
  }
  if (grouped) {
    return spmv_grouped(n, A, y, y_idx, x, xg, any_x, has_alpha, bmode, alpha, beta, dotp, want_dot, dot_tail,
                        tslot, dt, gmode == 2, fz);
  }

  auto pack = [&](int i) -> int {
    pa_ctx* c = xg[i]->ctx;
    HIPC(hipSetDevice(c->device));
    launch_pack(dt, xg[i]->n_snd_data, xg[i]->d_lids_snd, x[i]->d, xg[i]->d_buf_snd, c->s_main);
    HIPC(hipEventRecord(c->ev_packed, c->s_main));
    return 0;
  };
  auto interior = [&](int i) -> int {
    pa_ctx* c = A[i]->ctx;
    HIPC(hipSetDevice(c->device));
    const int32_t* ymap = y_idx[i]->own_contig ? nullptr : y_idx[i]->d_oid_to_lid;
    if (tslot[i]) HIPC(hipEventRecord(tslot[i][0], c->s_main));
    // interior slices (no ghost column): overlap with the halo transport
    if (launch_phase(0, A[i], x[i]->d, y[i]->d, ymap, has_alpha, bmode, alpha, beta, dotp[i], c->s_main, fz, i)) return -1;
    if (tslot[i]) HIPC(hipEventRecord(tslot[i][1], c->s_main));
    return 0;
  };
  auto boundary = [&](int i) -> int {
    pa_ctx* c = A[i]->ctx;
    HIPC(hipSetDevice(c->device));
    if (any_x) {
      if (!pulled_on_main) HIPC(hipStreamWaitEvent(c->s_main, c->ev_recvd, 0));
      if (!pulled)
        launch_unpack(dt, xg[i]->n_rcv_data, xg[i]->d_lids_rcv, xg[i]->plan_fwd, PA_REPLACE,
                      xg[i]->d_buf_rcv, x[i]->d, c->s_main);
    }
    if (tslot[i]) HIPC(hipEventRecord(tslot[i][2], c->s_main));
    const int32_t* ymap = y_idx[i]->own_contig ? nullptr : y_idx[i]->d_oid_to_lid;
    // slices reading ghosts and the side rows (after the halo)
    if (launch_phase(1, A[i], x[i]->d, y[i]->d, ymap, has_alpha, bmode, alpha, beta, dotp[i], c->s_main, fz, i)) return -1;
    cg_ghosts(fz, i, A[i], x[i], c->s_main);
    // long rows (after the halo: they may read ghost columns)
    const bool pat = knobs().spmv_format == 1 && A[i]->has_pat;
    const int64_t long_base = A[i]->nslices + (pat ? A[i]->s_nslices + A[i]->t_nslices : 0);
    launch_spmv_long(A[i], x[i]->d, y[i]->d, ymap, has_alpha, bmode, alpha, beta, dotp[i], long_base, c->s_main);
    if (want_dot) {  // fold the partials (main slices, side slices, long rows) in order
      const bool cplx = dt == PA_C64 || dt == PA_C128;
      const int nbp = (int)(long_base + A[i]->n_long);
      if (dot_tail)  // one part per process: the fold ends in the CG's α
        launch_fold_cg_alpha(dt, nbp, A[i]->d_dotp, c->d_fold, c->d_result, c->d_ticket, dot_tail[i], c->s_main);
      else
        launch_fold(cplx, nbp, A[i]->d_dotp, c->d_fold, c->d_result, c->d_ticket, c->s_main);
    }
    if (tslot[i]) HIPC(hipEventRecord(tslot[i][3], c->s_main));
    return 0;
  };
  // several parts, each with its own stream pair (one per GPU when one
  // process drives several GPUs): the parts are issued from the IssuePool's
  // host threads in three rounds — pre-pack waits + packs (every part's
  // ev_packed recorded before any receiver waits on it), per part its
  // transport (waits, pull) and interior phase, then the boundary phases;
  // with an RCCL transport (parts in other processes) the call stays on
  // this thread
  // issue_threads 1 (auto): only when the parts span several devices; on
  // one device the parts' streams share its hardware queues and the serial
  // order keeps the device time lower (1.44 vs 1.70 ms for 8 parts of the
  // 256³ (2,2,2) problem, profiles/r04/k/host_issue_3round.json); 2: always
  bool distinct = n >= 2;  // every part its own stream pair
  bool multi_dev = false;
  for (int i = 0; distinct && i < n; ++i) {
    multi_dev = multi_dev || A[i]->ctx->device != A[0]->ctx->device;
    for (int j = 0; j < i; ++j)
      if (A[i]->ctx->s_main == A[j]->ctx->s_main || A[i]->ctx->s_comm == A[j]->ctx->s_comm) distinct = false;
  }
  bool threads = knobs().issue_threads && distinct;
  if (knobs().issue_threads == 1 && !multi_dev) threads = false;
  TransportPlan T;
  if (any_x && transport_plan(n, xg, dt, 0, PA_REPLACE, x, &T)) return -1;
  if (any_x && distinct && knobs().halo_barrier && T.pull && !T.remote) {
    pulled = true;
    pulled_on_main = knobs().halo_barrier == 2;
    if (spmv_barrier_issue(n, x, xg, dt, T, threads, interior, boundary, pulled_on_main)) return -1;
  } else if (threads && !(any_x && T.remote)) {
    if (any_x) {
      const LocalSet L = local_set(n, xg);
      if (IssuePool::get().run(n, [&](int i) -> int { return pre_pack_wait_part(i, xg, L) || pack(i); })) return -1;
    }
    pulled = any_x && T.pull;
    if (IssuePool::get().run(n, [&](int i) -> int {
          if (any_x && (transport_wait(i, xg, T) || transport_local(i, xg, x, T))) return -1;
          return interior(i);
        }))
      return -1;
    // every interior enqueued before any boundary's wait for its halo: with
    // several parts' streams sharing a hardware queue (one GPU), a wait
    // enqueued early would hold back the other parts' interiors behind it
    if (IssuePool::get().run(n, boundary)) return -1;
  } else {
    if (any_x) {
      if (pre_pack_wait(n, xg)) return -1;
      for (int i = 0; i < n; ++i)
        if (pack(i)) return -1;
      for (int i = 0; i < n; ++i)
        if (transport_wait(i, xg, T)) return -1;
      if (T.remote && transport_remote(n, xg, T)) return -1;
      for (int i = 0; i < n; ++i)
        if (transport_local(i, xg, x, T)) return -1;
      pulled = T.pull;
    }
    for (int i = 0; i < n; ++i)
      if (interior(i)) return -1;
    HIPC(hipGetLastError());
    for (int i = 0; i < n; ++i)
      if (boundary(i)) return -1;
  }
  HIPC(hipGetLastError());
  for (int i = 0; i < n; ++i)
    if (tslot[i]) ++A[i]->ctx->tn;
  return 0;
}

int pa_exchange_all(int n, pa_vec* const v[], pa_xchg* const xg[], const pa_index* const idx[], int op,
                    int reverse, int zero_ghosts) {
  CHECK_ARG(n >= 1 && v && xg && v[0], "null argument");
  CHECK_ARG(op == PA_REPLACE || op == PA_ADD, "invalid combine op");
  TuneScope ts(v[0]->ctx);
  const int dt = v[0]->dtype;
  for (int i = 0; i < n; ++i) {
    CHECK_ARG(v[i] && xg[i], "null handle");
    CHECK_ARG(v[i]->dtype == dt, "exchange!: element types differ across parts");
    CHECK_ARG(v[i]->ctx == xg[i]->ctx, "exchange!: vector and exchanger of different parts");
    if (check_lids(xg[i], v[i])) return -1;
  }
  if (pre_pack_wait(n, xg)) return -1;
  for (int i = 0; i < n; ++i) {
    pa_xchg* X = xg[i];
    pa_ctx* c = X->ctx;
    HIPC(hipSetDevice(c->device));
    if (!reverse)
      launch_pack(dt, X->n_snd_data, X->d_lids_snd, v[i]->d, X->d_buf_snd, c->s_main);
    else
      launch_pack(dt, X->n_rcv_data, X->d_lids_rcv, v[i]->d, X->d_buf_rcv, c->s_main);
    HIPC(hipEventRecord(c->ev_packed, c->s_main));
  }
  HIPC(hipGetLastError());
  bool pulled = false;
  if (transport(n, xg, dt, reverse ? 1 : 0, op, v, &pulled)) return -1;
  for (int i = 0; i < n; ++i) {
    pa_xchg* X = xg[i];
    pa_ctx* c = X->ctx;
    HIPC(hipSetDevice(c->device));
    HIPC(hipStreamWaitEvent(c->s_main, c->ev_recvd, 0));
    if (pulled) {
    } else if (!reverse) {
      launch_unpack(dt, X->n_rcv_data, X->d_lids_rcv, X->plan_fwd, op, X->d_buf_rcv, v[i]->d, c->s_main);
    } else {
      launch_unpack(dt, X->n_snd_data, X->d_lids_snd, X->plan_rev, op, X->d_buf_snd, v[i]->d, c->s_main);
    }
    if (zero_ghosts) {
      CHECK_ARG(idx && idx[i] && idx[i]->nlids == v[i]->n, "assemble!: index set of the vector required");
      unsigned char z[16] = {0};
      launch_fill(dt, idx[i]->nhids, idx[i]->noids, idx[i]->d_hid_to_lid, v[i]->d, z, c->s_main);
    }
  }
  HIPC(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
namespace {

// Each local part's d_result (double / c128 accumulator) → host, one entry
// per part id 1..P (RCCL all-gather when parts live in other processes).
int gather_results(int n, pa_ctx* const* ctxs, bool cplx, std::vector<c128>* vals) {
  const int P = ctxs[0]->nparts;
  vals->assign(P, c128{0.0, 0.0});
  std::vector<char> have(P, 0);
  // one part per process (pa_comm_init_rank): the part values of every rank
  // come by RCCL all-gather (with one process too: a one-rank gather)
  const bool remote_mode = ctxs[0]->comm && !ctxs[0]->rank_of_part && n == 1;
  const size_t accsz = cplx ? 16 : 8;
  if (remote_mode) {
    pa_ctx* c = ctxs[0];
    HIPC(hipSetDevice(c->device));
    NCCLC(ncclAllGather(c->d_result, c->d_gather, accsz, ncclUint8, (ncclComm_t)c->comm, c->s_main));
    HIPC(hipMemcpyAsync(c->h_pinned, c->d_gather, accsz * P, hipMemcpyDeviceToHost, c->s_main));
    HIPC(hipStreamSynchronize(c->s_main));
    for (int p = 0; p < P; ++p) {
      const char* src = (const char*)c->h_pinned + accsz * p;
      if (cplx) std::memcpy(&(*vals)[p], src, 16);
      else std::memcpy(&(*vals)[p].re, src, 8);
      have[p] = 1;
    }
  } else {
    for (int i = 0; i < n; ++i) {
      pa_ctx* c = ctxs[i];
      HIPC(hipSetDevice(c->device));
      HIPC(hipMemcpyAsync(c->h_pinned, c->d_result, accsz, hipMemcpyDeviceToHost, c->s_main));
      HIPC(hipStreamSynchronize(c->s_main));
      const int p = c->part - 1;
      if (cplx) std::memcpy(&(*vals)[p], c->h_pinned, 16);
      else std::memcpy(&(*vals)[p].re, c->h_pinned, 8);
      have[p] = 1;
    }
  }
  for (int p = 0; p < P; ++p)
    CHECK_ARG(have[p], "reduction over a subset of the parts: pass every part held by this process, or use one part per process with RCCL");
  return 0;
}

// kind 0: dot, 1: sum |a|^2, 2: sum a.  Leaves each part's accumulator
// (double / c128) in host memory `vals` (one per part id 1..P, folded in
// part order by the caller), covering remote parts through RCCL all-gather.
int reduce_all(int n, const pa_vec* const a[], const pa_index* const ia[], const pa_vec* const b[],
               const pa_index* const ib[], int kind, std::vector<c128>* vals) {
  CHECK_ARG(n >= 1 && a && ia, "null argument");
  const int dt = a[0]->dtype;
  const bool cplx = dt == PA_C64 || dt == PA_C128;
  for (int i = 0; i < n; ++i) {
    CHECK_ARG(a[i] && ia[i], "null handle");
    CHECK_ARG(a[i]->dtype == dt, "element types differ across parts");
    CHECK_ARG(ia[i]->nlids == a[i]->n, "index set does not describe the vector");
    if (kind == 0) {
      CHECK_ARG(b && b[i] && ib && ib[i] && b[i]->dtype == dt && ib[i]->nlids == b[i]->n, "dot: second vector");
      CHECK_ARG(ia[i]->noids == ib[i]->noids, "dot: owned counts differ");
    }
    pa_ctx* c = a[i]->ctx;
    HIPC(hipSetDevice(c->device));
    launch_reduce(dt, kind, ia[i]->noids, ia[i]->d_oid_to_lid, a[i]->d,
                  kind == 0 ? ib[i]->d_oid_to_lid : nullptr, kind == 0 ? b[i]->d : nullptr,
                  c->d_partials, c->d_result, c->d_ticket, c->s_main);
  }
  HIPC(hipGetLastError());
  std::vector<pa_ctx*> ctxs(n);
  for (int i = 0; i < n; ++i) ctxs[i] = a[i]->ctx;
  return gather_results(n, ctxs.data(), cplx, vals);
}

// reduce(+, c; init=zero(T)) over the part values in part order
// (Interfaces.jl:221-238), in T: each part's value is rounded to T first
// (Julia's local dot / sum / norm^2 return T), Float32 parts add in Float32
c128 fold_parts(int dt, const std::vector<c128>& vals, bool real_only) {
  if (dt == PA_F32 || dt == PA_C64) {
    float re = 0.f, im = 0.f;
    for (const auto& v : vals) {
      re = re + (float)v.re;
      if (!real_only) im = im + (float)v.im;
    }
    return c128{(double)re, (double)im};
  }
  c128 s{0.0, 0.0};
  for (const auto& v : vals) s = s + (real_only ? c128{v.re, 0.0} : v);
  return s;
}

void store_scalar(int dt, c128 s, void* result) {
  switch (dt) {
    case PA_F32: *(float*)result = (float)s.re; break;
    case PA_F64: *(double*)result = s.re; break;
    case PA_C64: ((float*)result)[0] = (float)s.re; ((float*)result)[1] = (float)s.im; break;
    case PA_C128: ((double*)result)[0] = s.re; ((double*)result)[1] = s.im; break;
  }
}

}  // namespace

int pa_spmv_all(int n, pa_mat* const A[], pa_vec* const y[], const pa_index* const y_idx[],
                pa_vec* const x[], const pa_index* const x_idx[], pa_xchg* const xg[],
                const void* alpha, const void* beta) {
  CHECK_ARG(n >= 1 && A && A[0], "null argument");
  TuneScope ts(A[0]->ctx);
  return spmv_impl(n, A, y, y_idx, x, x_idx, xg, alpha, beta, false);
}

int pa_spmv_dot_all(int n, pa_mat* const A[], pa_vec* const y[], const pa_index* const y_idx[],
                    pa_vec* const x[], const pa_index* const x_idx[], pa_xchg* const xg[],
                    const void* alpha, const void* beta, void* dot_result) {
  CHECK_ARG(dot_result && n >= 1 && A && A[0], "null argument");
  TuneScope ts(A[0]->ctx);
  if (spmv_impl(n, A, y, y_idx, x, x_idx, xg, alpha, beta, true)) return -1;
  std::vector<pa_ctx*> ctxs(n);
  for (int i = 0; i < n; ++i) ctxs[i] = A[i]->ctx;
  const int dt = A[0]->dtype;
  std::vector<c128> vals;
  if (gather_results(n, ctxs.data(), dt == PA_C64 || dt == PA_C128, &vals)) return -1;
  store_scalar(dt, fold_parts(dt, vals, false), dot_result);
  return 0;
}

int pa_cg_update_all(int n, pa_vec* const x[], pa_vec* const r[], const pa_vec* const u[],
                     const pa_vec* const c[], const pa_index* const idx[], const void* alpha,
                     double* rnorm) {
  CHECK_ARG(n >= 1 && x && r && u && c && idx && alpha && rnorm, "null argument");
  const int dt = x[0]->dtype;
  std::vector<pa_ctx*> ctxs(n);
  for (int i = 0; i < n; ++i) {
    CHECK_ARG(x[i] && r[i] && u[i] && c[i] && idx[i], "null handle");
    const int64_t m = x[i]->n;
    CHECK_ARG(r[i]->n == m && u[i]->n == m && c[i]->n == m && idx[i]->nlids == m,
              "cg update: vectors must share the partition");
    CHECK_ARG(r[i]->dtype == dt && u[i]->dtype == dt && c[i]->dtype == dt, "cg update: element types differ");
    pa_ctx* cx = x[i]->ctx;
    ctxs[i] = cx;
    HIPC(hipSetDevice(cx->device));
    if (idx[i]->own_contig) {
      const int nb = (int)std::min<int64_t>(8192, std::max<int64_t>(1, (m + 255) / 256));
      launch_cg_xr(dt, m, idx[i]->noids, nullptr, x[i]->d, r[i]->d, u[i]->d, c[i]->d, alpha, nullptr,
                   (double*)cx->d_partials, nb, cx->s_main);
      launch_fold(0, nb, cx->d_partials, cx->d_fold, cx->d_result, cx->d_ticket, cx->s_main);
    } else {  // unfused: two broadcasts and the norm reduction
      const int sk = (dt == PA_C64 || dt == PA_C128) ? 2 : 1;  // α: Float64 / ComplexF64
      launch_axpby(dt, m, nullptr, x[i]->d, u[i]->d, alpha, 1, cx->s_main, sk);
      launch_axpby(dt, m, nullptr, r[i]->d, c[i]->d, alpha, 2, cx->s_main, sk);
      launch_reduce(dt, 1, idx[i]->noids, idx[i]->d_oid_to_lid, r[i]->d, nullptr, nullptr, cx->d_partials,
                    cx->d_result, cx->d_ticket, cx->s_main);
    }
  }
  HIPC(hipGetLastError());
  std::vector<c128> vals;
  if (gather_results(n, ctxs.data(), false, &vals)) return -1;
  *rnorm = std::sqrt(fold_parts(dt, vals, true).re);  // (…)^(1/2) in Float64, correctly rounded
  return 0;
}

// ---------------------------------------------------------------------------
// Device-driven CG (IterativeSolvers 0.9 cg!): the
// scalar recurrence lives on the device (CGState per part), so the host
// enqueues iterations in batches and only reads the done flag between
// batches.  Each reduction ends in a device all-gather of the part values
// (RCCL across processes; a gather kernel over the local parts' results in
// one process), then every part folds them in part order.
namespace {

struct CGRun {
  int n = 0, P = 0;
  bool remote = false;
  std::vector<pa_ctx*> ctxs;
  std::vector<CGState*> st;
  std::vector<double*> hist;
  std::vector<void**> ptrs;         // local mode: per part, device table of the parts' d_result
  void** dsts = nullptr;            // local mode: the local parts' d_gather (device table on part 1's device)
  std::vector<hipEvent_t> ev_red;   // local mode: part value ready
  std::vector<hipEvent_t> ev_gat;   // local mode: [0] the values gathered into every part
  ~CGRun() {
    for (int i = 0; i < n; ++i) {
      if (i < (int)ctxs.size()) (void)hipSetDevice(ctxs[i]->device);
      if (i < (int)st.size()) dev_free(st[i]);
      if (i < (int)hist.size()) dev_free(hist[i]);
      if (i < (int)ptrs.size()) dev_free(ptrs[i]);
      if (i < (int)ev_red.size() && ev_red[i]) (void)hipEventDestroy(ev_red[i]);
      if (i < (int)ev_gat.size() && ev_gat[i]) (void)hipEventDestroy(ev_gat[i]);
    }
    if (dsts) {
      (void)hipSetDevice(ctxs[0]->device);
      dev_free(dsts);
    }
  }
};

// every part's d_result (accsz bytes) → d_gather[part-1] of every part.
// Local mode (all parts in this process): part 1's stream waits for every
// part's value, one kernel copies the P values into every part's d_gather
// (peer stores), and every other part waits for that kernel — 3n runtime
// calls; the previous form (a gather kernel per part behind n-1 waits each,
// then n-1 more waits each before any d_result is reused) took 2n² + 2n,
// which at 8 stream-pair parts filled the queues with cross-stream waits
// (tools/host_issue.py cg_host_us_per_iteration_tiny, profiles/r05/h/).
// The kernel's reads of the d_result precede ev_gat[0], which every part
// waits for before it writes its d_result again.
int cg_gather(CGRun& R, size_t accsz) {
  if (R.remote) {
    pa_ctx* c = R.ctxs[0];
    HIPC(hipSetDevice(c->device));
    NCCLC(ncclAllGather(c->d_result, c->d_gather, accsz, ncclUint8, (ncclComm_t)c->comm, c->s_main));
    return 0;
  }
  pa_ctx* c0 = R.ctxs[0];
  for (int i = 1; i < R.n; ++i) {
    HIPC(hipSetDevice(R.ctxs[i]->device));
    HIPC(hipEventRecord(R.ev_red[i], R.ctxs[i]->s_main));
  }
  HIPC(hipSetDevice(c0->device));
  for (int i = 1; i < R.n; ++i) HIPC(hipStreamWaitEvent(c0->s_main, R.ev_red[i], 0));
  launch_gather_scatter(R.P, (const void* const*)R.ptrs[0], (int)accsz, R.n, R.dsts, c0->s_main);
  HIPC(hipEventRecord(R.ev_gat[0], c0->s_main));
  for (int i = 1; i < R.n; ++i) {
    HIPC(hipSetDevice(R.ctxs[i]->device));
    HIPC(hipStreamWaitEvent(R.ctxs[i]->s_main, R.ev_gat[0], 0));
  }
  return 0;
}

// The u-update variant of the device CG's auto mode (cg_fuse 2) from the
// two timed batches (ms[0] the sweep, ms[1] the fused update): with one
// part per process every rank measures its own batches, so the times are
// first reduced with max over the ranks (the slowest rank sets the
// iteration time), and every rank makes the same choice.  -1: no valid
// measurement.
int cg_agree_choice(float ms[2], const std::function<int(float*)>& allreduce_max) {
  if (allreduce_max && allreduce_max(ms)) return -2;
  if (!(ms[0] > 0.f) || !(ms[1] > 0.f)) return -1;
  return ms[1] < ms[0] ? 1 : 0;
}

// Whether the fused u update may run: every rank must be able
// to, since a rank that cannot runs the sweep, whose halo carries u while
// the fused variant's carries r, and the ranks' collectives would no longer
// pair.  "cannot fuse" is max-reduced over the ranks.  -2: reduction failed.
int cg_agree_fuse(bool local_can_fuse, const std::function<int(float*)>& allreduce_max) {
  float v[2] = {local_can_fuse ? 0.f : 1.f, 0.f};
  if (allreduce_max && allreduce_max(v)) return -2;
  return v[0] > 0.f ? 0 : 1;
}

void scalar_one(int dt, unsigned char out[16], double v) {
  std::memset(out, 0, 16);
  switch (dt) {
    case PA_F32: case PA_C64: { const float f = (float)v; std::memcpy(out, &f, 4); } break;
    default: std::memcpy(out, &v, 8); break;
  }
}

}  // namespace

int pa_cg_solve_all(int n, pa_mat* const A[], pa_vec* const x[], const pa_vec* const b[],
                    pa_vec* const u[], pa_vec* const r[], pa_vec* const c[],
                    const pa_index* const idx[], pa_xchg* const xg[], double reltol, double abstol,
                    int64_t maxiter, int batch, int64_t* iterations, double* residual, double* history) {
  CHECK_ARG(n >= 1 && A && A[0] && x && b && u && r && c && idx && iterations && residual, "null argument");
  CHECK_ARG(batch >= 1, "batch must be >= 1");
  TuneScope ts(A[0]->ctx);
  const int dt = A[0]->dtype;
  const bool cplx = dt == PA_C64 || dt == PA_C128;
  CGRun R;
  R.n = n;
  R.P = A[0]->ctx->nparts;
  for (int i = 0; i < n; ++i) {
    CHECK_ARG(A[i] && x[i] && b[i] && u[i] && r[i] && c[i] && idx[i], "null handle");
    const int64_t m = x[i]->n;
    for (const pa_vec* v : {(const pa_vec*)x[i], b[i], (const pa_vec*)u[i], (const pa_vec*)r[i], (const pa_vec*)c[i]}) {
      CHECK_ARG(v->dtype == dt, "cg!: element types differ");
      CHECK_ARG(v->n == m && v->ctx == A[i]->ctx, "cg!: x, b and the work vectors must share a.cols' partition");
    }
    CHECK_ARG(idx[i]->nlids == m && idx[i]->own_contig, "cg!: the device CG needs contiguous owned lids");
    CHECK_ARG(A[i]->ctx->nparts == R.P, "cg!: parts of different partitions");
    R.ctxs.push_back(A[i]->ctx);
  }
  R.remote = R.ctxs[0]->comm && !R.ctxs[0]->rank_of_part && n == 1;  // one part per process
  CHECK_ARG(R.remote || n == R.P, "cg!: pass every part held by this process, or use one part per process with RCCL");
  std::vector<int> part_pos(R.P + 1, -1);
  for (int i = 0; i < n; ++i) part_pos[R.ctxs[i]->part] = i;
  R.st.assign(n, nullptr);
  R.hist.assign(n, nullptr);
  R.ptrs.assign(n, nullptr);
  R.ev_red.assign(n, nullptr);
  R.ev_gat.assign(n, nullptr);
  for (int i = 0; i < n; ++i) {
    pa_ctx* cx = R.ctxs[i];
    HIPC(hipSetDevice(cx->device));
    HIPC(hipMalloc((void**)&R.st[i], sizeof(CGState)));
    if (history && maxiter > 0) HIPC(hipMalloc((void**)&R.hist[i], (size_t)maxiter * sizeof(double)));
    if (!R.remote) {
      std::vector<void*> tab(R.P, nullptr);
      for (int p = 1; p <= R.P; ++p) tab[p - 1] = R.ctxs[part_pos[p]]->d_result;
      if (dev_upload(&R.ptrs[i], tab)) return -1;
      HIPC(hipEventCreateWithFlags(&R.ev_red[i], hipEventDisableTiming));
      HIPC(hipEventCreateWithFlags(&R.ev_gat[i], hipEventDisableTiming));
      for (int j = 0; j < n; ++j) {  // the gather kernel reads the other devices' results
        const int dj = R.ctxs[j]->device;
        if (dj == cx->device) continue;
        int ok = 0;
        HIPC(hipDeviceCanAccessPeer(&ok, cx->device, dj));
        CHECK_ARG(ok, "cg!: the device CG over parts on several devices of one process needs peer access");
        hipError_t e = hipDeviceEnablePeerAccess(dj, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPC(e);
        (void)hipGetLastError();
      }
    }
  }
  if (!R.remote) {  // the destinations of the one-kernel all-gather (local parts in position order)
    std::vector<void*> d(n);
    for (int i = 0; i < n; ++i) d[i] = R.ctxs[i]->d_gather;
    HIPC(hipSetDevice(R.ctxs[0]->device));
    if (dev_upload(&R.dsts, d)) return -1;
  }
  // setup (cg_iterator!): u = 0; r = b; c = A*x; r .-= c; residual = norm(r);
  // tolerance = max(reltol*norm(b), abstol)
  unsigned char one[16], zero[16];
  scalar_one(dt, one, 1.0);
  scalar_one(dt, zero, 0.0);
  for (int i = 0; i < n; ++i) {
    HIPC(hipSetDevice(R.ctxs[i]->device));
    launch_fill(dt, u[i]->n, 0, nullptr, u[i]->d, zero, R.ctxs[i]->s_main);
    launch_copy(dt, r[i]->n, nullptr, r[i]->d, nullptr, b[i]->d, R.ctxs[i]->s_main);
  }
  HIPC(hipGetLastError());
  if (spmv_impl(n, A, c, idx, x, idx, xg, one, zero, false)) return -1;
  for (int i = 0; i < n; ++i) {
    HIPC(hipSetDevice(R.ctxs[i]->device));
    launch_axpby(dt, r[i]->n, nullptr, r[i]->d, c[i]->d, zero, 3, R.ctxs[i]->s_main);
  }
  double res0 = 0.0, nb = 0.0;
  if (pa_norm2_all(n, (const pa_vec* const*)r, idx, &res0)) return -1;
  if (pa_norm2_all(n, b, idx, &nb)) return -1;
  CGState h{};
  h.res = res0;
  h.prev = 1.0;
  h.tol = std::max(reltol * nb, abstol);
  h.it = 0;
  h.maxiter = maxiter;
  h.done = (0 >= maxiter || res0 <= h.tol) ? 1 : 0;
  for (int i = 0; i < n; ++i) {
    HIPC(hipSetDevice(R.ctxs[i]->device));
    HIPC(hipMemcpyAsync(R.st[i], &h, sizeof(CGState), hipMemcpyHostToDevice, R.ctxs[i]->s_main));
    HIPC(hipStreamSynchronize(R.ctxs[i]->s_main));
  }
  const size_t accsz = cplx ? 16 : 8;
  // one part in this process and no other process: the folds end in the
  // scalar updates themselves (no gather, no scalar kernels)
  const bool tail = !R.remote && R.P == 1;
  // The u update (pa_tune cg_fuse): 0 its own sweep, in place on u; 1 inside
  // the SpMV, u = r .+ β.*u_old evaluated per gathered element (the halo
  // carries r), u in two buffers (an iteration reads ucur, writes uoth, then
  // they swap), the deferred x .+= α.*u riding along; 2 auto: with all parts
  // in this process and at least three batches, the first batch runs the
  // sweep, the second the fused update, the rest the faster of the two (HIP
  // events on part 1's stream), remembered on the matrix.  The variants give
  // the same values bit for bit, so switching between batches changes no
  // result.  Fused: not for matrices with long rows (their kernel gathers x
  // directly).
  bool can_fuse = true;
  // (the fused u update is written by the main structure's waves: not for
  // rows that long-row kernels or the triple SELL compute)
  for (int i = 0; i < n; ++i) can_fuse = can_fuse && A[i]->n_long == 0 && A[i]->t_nrows == 0;
  if (R.remote && knobs().cg_fuse != 0) {  // every rank the same (cg_agree_fuse): RCCL max over the ranks
    pa_ctx* c0 = R.ctxs[0];
    const std::function<int(float*)> red = [&](float* v) -> int {
      HIPC(hipMemcpyAsync(c0->d_fold, v, 2 * sizeof(float), hipMemcpyHostToDevice, c0->s_main));
      NCCLC(ncclAllReduce(c0->d_fold, c0->d_fold, 2, ncclFloat32, ncclMax, (ncclComm_t)c0->comm, c0->s_main));
      HIPC(hipMemcpyAsync(v, c0->d_fold, 2 * sizeof(float), hipMemcpyDeviceToHost, c0->s_main));
      HIPC(hipStreamSynchronize(c0->s_main));
      return 0;
    };
    HIPC(hipSetDevice(c0->device));
    const int ok = cg_agree_fuse(can_fuse, red);
    if (ok < 0) return -1;
    can_fuse = ok == 1;
  }
  // (every rank of a one-part-per-process solve takes the same branches:
  // maxiter, batch, the done flag and the reduced batch times agree)
  int mode = can_fuse ? knobs().cg_fuse : 0;
  if (mode == 2 && maxiter < 3 * (int64_t)batch) mode = A[0]->cg_fuse_choice >= 0 ? A[0]->cg_fuse_choice : 0;
  if (mode == 2 && A[0]->cg_fuse_choice >= 0) mode = A[0]->cg_fuse_choice;
  std::vector<pa_vec*> u2(n, nullptr);
  struct U2Free {
    std::vector<pa_vec*>& v;
    ~U2Free() { for (pa_vec* p : v) if (p) pa_vec_destroy(p); }
  } u2_free{u2};
  if (mode != 0)
    for (int i = 0; i < n; ++i)
      if (pa_vec_create(R.ctxs[i], dt, u[i]->n, &u2[i])) return -1;
  std::vector<pa_vec*> ucur(u, u + n), uoth(u2);
  hipEvent_t tev[2] = {nullptr, nullptr};
  struct EvFree {
    hipEvent_t* e;
    ~EvFree() { for (int j = 0; j < 2; ++j) if (e[j]) (void)hipEventDestroy(e[j]); }
  } ev_free{tev};
  if (mode == 2) {
    HIPC(hipSetDevice(R.ctxs[0]->device));
    HIPC(hipEventCreate(&tev[0]));
    HIPC(hipEventCreate(&tev[1]));
  }
  float batch_ms[2] = {0.f, 0.f};
  int64_t enqueued = 0, nbatch = 0;
  bool done = h.done != 0;
  while (!done && enqueued < maxiter) {
    const int64_t k = std::min<int64_t>(batch, maxiter - enqueued);  // the same on every rank
    // (a batch that ended the solve before the choice was made runs the sweep)
    const int variant = mode == 2 ? (nbatch < 2 ? (int)nbatch : std::max(0, A[0]->cg_fuse_choice)) : mode;
    // the timed batches start their clock after their first iteration (which
    // builds the variant's launch tables) and need two iterations at least
    const bool timed = mode == 2 && nbatch < 2 && k >= 2;
    for (int64_t t = 0; t < k; ++t) {
      if (timed && t == 1) {
        HIPC(hipSetDevice(R.ctxs[0]->device));
        HIPC(hipEventRecord(tev[0], R.ctxs[0]->s_main));
      }
      if (variant == 1) {
        // mul!(c, A, u) with u = r .+ β.*u_old evaluated inside the SpMV (its
        // halo carries r), the owned u written, x .+= α.*u_old of the
        // previous iteration applied; dot(u, c) accumulated by the SpMV
        CGFuse fz;
        for (int i = 0; i < n; ++i) {
          fz.u_old.push_back(ucur[i]->d);
          fz.u_new.push_back(uoth[i]->d);
          fz.xacc.push_back(x[i]->d);
          fz.st.push_back(R.st[i]);
        }
        if (spmv_impl(n, A, c, idx, r, idx, xg, one, zero, true, tail ? R.st.data() : nullptr, &fz)) return -1;
        std::swap(ucur, uoth);
      } else {
        for (int i = 0; i < n; ++i) {  // (x .+= α.*u of the previous iteration); u .= r .+ β.*u
          HIPC(hipSetDevice(R.ctxs[i]->device));
          launch_cg_xu(dt, ucur[i]->n, x[i]->d, ucur[i]->d, r[i]->d, R.st[i], R.ctxs[i]->s_main);
        }
        // mul!(c, A, u) with dot(u, c) accumulated by the SpMV; α = residual² / dot(u, c)
        if (spmv_impl(n, A, c, idx, ucur.data(), idx, xg, one, zero, true, tail ? R.st.data() : nullptr)) return -1;
      }
      if (!tail) {
        if (cg_gather(R, accsz)) return -1;
        for (int i = 0; i < n; ++i) {
          HIPC(hipSetDevice(R.ctxs[i]->device));
          launch_cg_alpha(dt, R.P, R.ctxs[i]->d_gather, R.st[i], R.ctxs[i]->s_main);
        }
      }
      for (int i = 0; i < n; ++i) {  // r .-= α.*c; Σ|r|²
        pa_ctx* cx = R.ctxs[i];
        HIPC(hipSetDevice(cx->device));
        const int64_t m = x[i]->n;
        const int nbk = (int)std::min<int64_t>(8192, std::max<int64_t>(1, (m + 255) / 256));
        launch_cg_xr(dt, m, idx[i]->noids, nullptr, x[i]->d, r[i]->d, u[i]->d, c[i]->d, nullptr, R.st[i],
                     (double*)cx->d_partials, nbk, cx->s_main);
        if (tail)  // prev = residual; residual = norm(r); it += 1; done?
          launch_fold_cg_step(dt, nbk, cx->d_partials, cx->d_fold, cx->d_result, cx->d_ticket, R.st[i], R.hist[i],
                              cx->s_main);
        else
          launch_fold(0, nbk, cx->d_partials, cx->d_fold, cx->d_result, cx->d_ticket, cx->s_main);
      }
      if (!tail) {
        if (cg_gather(R, 8)) return -1;
        for (int i = 0; i < n; ++i) {  // prev = residual; residual = norm(r); it += 1; done?
          HIPC(hipSetDevice(R.ctxs[i]->device));
          launch_cg_step(dt, R.P, (const double*)R.ctxs[i]->d_gather, R.st[i], R.hist[i], R.ctxs[i]->s_main);
        }
      }
      HIPC(hipGetLastError());
    }
    enqueued += k;
    // every part holds the same state; read part 0's
    pa_ctx* c0 = R.ctxs[0];
    HIPC(hipSetDevice(c0->device));
    if (timed) HIPC(hipEventRecord(tev[1], c0->s_main));
    HIPC(hipMemcpyAsync(c0->h_pinned, R.st[0], sizeof(CGState), hipMemcpyDeviceToHost, c0->s_main));
    for (int i = 0; i < n; ++i) {
      HIPC(hipSetDevice(R.ctxs[i]->device));
      HIPC(hipStreamSynchronize(R.ctxs[i]->s_main));
    }
    std::memcpy(&h, c0->h_pinned, sizeof(CGState));
    done = h.done != 0;
    if (timed && !done) {  // a batch that converged part-way is no measurement
      float ms = 0.f;
      HIPC(hipEventElapsedTime(&ms, tev[0], tev[1]));
      batch_ms[nbatch] = ms / (float)(k - 1);
      if (nbatch == 1) {
        std::function<int(float*)> red;
        if (R.remote)  // the ranks' times, max over the ranks (RCCL, part 1's stream)
          red = [&](float* v) -> int {
            HIPC(hipMemcpyAsync(c0->d_fold, v, 2 * sizeof(float), hipMemcpyHostToDevice, c0->s_main));
            NCCLC(ncclAllReduce(c0->d_fold, c0->d_fold, 2, ncclFloat32, ncclMax, (ncclComm_t)c0->comm, c0->s_main));
            HIPC(hipMemcpyAsync(v, c0->d_fold, 2 * sizeof(float), hipMemcpyDeviceToHost, c0->s_main));
            HIPC(hipStreamSynchronize(c0->s_main));
            return 0;
          };
        const int ch = cg_agree_choice(batch_ms, red);
        if (ch == -2) return -1;
        if (ch >= 0) A[0]->cg_fuse_choice = ch;
      }
    } else if (mode == 2 && nbatch < 2) {
      mode = A[0]->cg_fuse_choice >= 0 ? A[0]->cg_fuse_choice : 0;  // no choice this solve: keep it unset
    }
    ++nbatch;
  }
  if (h.it > h.xit) {  // the last iteration's deferred x .+= α.*u (u untouched: done)
    for (int i = 0; i < n; ++i) {
      HIPC(hipSetDevice(R.ctxs[i]->device));
      launch_cg_xu(dt, ucur[i]->n, x[i]->d, ucur[i]->d, r[i]->d, R.st[i], R.ctxs[i]->s_main);
    }
    for (int i = 0; i < n; ++i) {
      HIPC(hipSetDevice(R.ctxs[i]->device));
      HIPC(hipStreamSynchronize(R.ctxs[i]->s_main));
    }
  }
  *iterations = h.it;
  *residual = h.res;
  if (history && h.it > 0) {
    HIPC(hipSetDevice(R.ctxs[0]->device));
    HIPC(hipMemcpy(history, R.hist[0], (size_t)h.it * sizeof(double), hipMemcpyDeviceToHost));
  }
  return 0;
}

int pa_cg_variant_agree(const float local_ms[2], pa_allreduce_max_fn fn, void* user, int* choice) {
  CHECK_ARG(local_ms && choice, "null argument");
  float ms[2] = {local_ms[0], local_ms[1]};
  std::function<int(float*)> red;
  if (fn) red = [&](float* v) -> int { return fn(v, 2, user) ? (pa::set_error("allreduce callback failed"), -1) : 0; };
  const int ch = cg_agree_choice(ms, red);
  if (ch == -2) return -1;
  *choice = ch;
  return 0;
}

int pa_cg_fuse_agree(int local_can_fuse, pa_allreduce_max_fn fn, void* user, int* agreed) {
  CHECK_ARG(agreed, "null argument");
  std::function<int(float*)> red;
  if (fn) red = [&](float* v) -> int { return fn(v, 2, user) ? (pa::set_error("allreduce callback failed"), -1) : 0; };
  const int ok = cg_agree_fuse(local_can_fuse != 0, red);
  if (ok < 0) return -1;
  *agreed = ok;
  return 0;
}

int pa_mat_cg_choice(const pa_mat* A, int* choice) {
  CHECK_ARG(A && choice, "null argument");
  *choice = A->cg_fuse_choice;
  return 0;
}

int pa_dot_all(int n, const pa_vec* const a[], const pa_index* const ia[], const pa_vec* const b[],
               const pa_index* const ib[], void* result) {
  CHECK_ARG(result, "null result");
  std::vector<c128> vals;
  if (reduce_all(n, a, ia, b, ib, 0, &vals)) return -1;
  store_scalar(a[0]->dtype, fold_parts(a[0]->dtype, vals, false), result);
  return 0;
}

int pa_norm2_all(int n, const pa_vec* const a[], const pa_index* const ia[], void* result) {
  CHECK_ARG(result, "null result");
  std::vector<c128> vals;
  if (reduce_all(n, a, ia, nullptr, nullptr, 1, &vals)) return -1;
  // (…)^(1/p) with p = 2 (Interfaces.jl:1771); Julia promotes to Float64.
  // x^0.5 correctly rounded is sqrt(x) (the device CG uses the same)
  *(double*)result = std::sqrt(fold_parts(a[0]->dtype, vals, true).re);
  return 0;
}

int pa_sum_all(int n, const pa_vec* const a[], const pa_index* const ia[], void* result) {
  CHECK_ARG(result, "null result");
  std::vector<c128> vals;
  if (reduce_all(n, a, ia, nullptr, nullptr, 2, &vals)) return -1;
  store_scalar(a[0]->dtype, fold_parts(a[0]->dtype, vals, false), result);
  return 0;
}

// ---------------------------------------------------------------------------
// Synthetic Cartesian stencil operator of one part box, built on the device
// (benchmark driver; equals pa_mat_from_csc of the CSC the oracle's drivers
// assemble, see tests/test_gpu_parity.py).
int pa_mat_stencil(pa_ctx* c, int dtype, int kind, const int64_t gdims[3], const int64_t box_lo[3],
                   const int64_t box_n[3], int64_t nlids_cols, const int32_t* shell_lid,
                   const double* coeffs, int ncoeffs, pa_mat** out) {
  CHECK_ARG(c && out && gdims && box_lo && box_n && coeffs, "null argument");
  TuneScope ts(c);
  CHECK_ARG(valid_dtype(dtype), "invalid dtype");
  CHECK_ARG(kind == 7 || kind == 27, "kind must be 7 or 27");
  CHECK_ARG((kind == 7 && ncoeffs == 2) || (kind == 27 && ncoeffs == 64), "coefficient count");
  for (int d = 0; d < 3; ++d) {
    CHECK_ARG(gdims[d] >= 2 && box_n[d] >= 1 && box_lo[d] >= 0 && box_lo[d] + box_n[d] <= gdims[d],
              "box outside the grid");
  }
  const int64_t nrows = box_n[0] * box_n[1] * box_n[2];
  CHECK_ARG(nrows < (int64_t)INT32_MAX && nlids_cols >= nrows && nlids_cols < (int64_t)INT32_MAX, "sizes");
  HIPC(hipSetDevice(c->device));
  pa_mat* A = new pa_mat();
  A->ctx = c;
  A->dtype = dtype;
  A->R = sell_rows_per_lane(dtype);
  A->H = 64 * A->R;
  A->nrows = nrows;
  A->ncols_lids = nlids_cols;
  StencilGeom g;
  for (int d = 0; d < 3; ++d) { g.N[d] = gdims[d]; g.lo[d] = box_lo[d]; g.n[d] = box_n[d]; }
  g.kind = kind;
  const int64_t ns = (nrows + A->H - 1) / A->H;
  const int64_t ext = (box_n[0] + 2) * (box_n[1] + 2) * (box_n[2] + 2);
  int32_t *d_shell = nullptr, *d_slen = nullptr, *d_sg = nullptr, *d_err = nullptr;
  double* d_coef = nullptr;
  auto cleanup = [&]() { dev_free(d_shell); dev_free(d_slen); dev_free(d_sg); dev_free(d_err); dev_free(d_coef); };
  if (shell_lid) {
    HIPC(hipMalloc((void**)&d_shell, ext * 4));
    HIPC(hipMemcpy(d_shell, shell_lid, ext * 4, hipMemcpyHostToDevice));
  }
  HIPC(hipMalloc((void**)&d_coef, ncoeffs * 8));
  HIPC(hipMemcpy(d_coef, coeffs, ncoeffs * 8, hipMemcpyHostToDevice));
  HIPC(hipMalloc((void**)&d_slen, std::max<int64_t>(ns, 1) * 4));
  HIPC(hipMalloc((void**)&d_sg, std::max<int64_t>(ns, 1) * 4));
  HIPC(hipMalloc((void**)&d_err, 4));
  // zeroed on the compute stream the kernels below run on (a hipMemset on
  // the null stream is not ordered before work on a non-blocking stream)
  HIPC(hipMemsetAsync(d_slen, 0, std::max<int64_t>(ns, 1) * 4, c->s_main));
  HIPC(hipMemsetAsync(d_sg, 0, std::max<int64_t>(ns, 1) * 4, c->s_main));
  HIPC(hipMemsetAsync(d_err, 0, 4, c->s_main));
  launch_stencil_count(g, d_shell, d_coef, nrows, (int)nrows, A->H, d_slen, d_sg, d_err, c->s_main);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->s_main));
  std::vector<int32_t> slen(ns), sg(ns);
  int32_t herr = 0;
  HIPC(hipMemcpy(slen.data(), d_slen, ns * 4, hipMemcpyDeviceToHost));
  HIPC(hipMemcpy(sg.data(), d_sg, ns * 4, hipMemcpyDeviceToHost));
  HIPC(hipMemcpy(&herr, d_err, 4, hipMemcpyDeviceToHost));
  if (herr) { cleanup(); delete A; PA_FAIL("stencil: a neighbour inside the domain has no lid (ghost shell table incomplete)"); }
  std::vector<char> sghost(ns);
  for (int64_t s = 0; s < ns; ++s) sghost[s] = sg[s] != 0;
  if (finish_sell_layout(A, slen, sghost, nullptr)) { cleanup(); pa_mat_destroy(A); return -1; }
  const size_t S = dtype_size(dtype);
  int64_t nnz_owned = 0;
  (void)nnz_owned;
  hipError_t e1 = hipMalloc((void**)&A->d_col, std::max<int64_t>(A->slots, 1) * 4);
  hipError_t e2 = hipErrorMemoryAllocation;
  // PA_DIAG_VAL_CONTIGUOUS (placement diagnostics only, tools/placement_pmc.py,
  // DESIGN.md §4.1): the values in physically contiguous memory when the
  // driver can provide it
  if (std::getenv("PA_DIAG_VAL_CONTIGUOUS")) {
    e2 = hipExtMallocWithFlags(&A->d_val, std::max<int64_t>(A->slots, 1) * S, hipDeviceMallocContiguous);
    if (e2 != hipSuccess)
      std::fprintf(stderr, "PA_DIAG_VAL_CONTIGUOUS: contiguous allocation of %lld B failed (%s): hipMalloc\n",
                   (long long)(std::max<int64_t>(A->slots, 1) * S), hipGetErrorString(e2));
  }
  if (e2 != hipSuccess) {
    (void)hipGetLastError();
    e2 = hipMalloc(&A->d_val, std::max<int64_t>(A->slots, 1) * S);
  }
  if (e1 != hipSuccess || e2 != hipSuccess) { cleanup(); pa_mat_destroy(A); PA_FAIL("hipMalloc(matrix) failed: out of device memory"); }
  launch_stencil_fill(g, d_shell, d_coef, nrows, (int)nrows, A, d_err, c->s_main);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->s_main));
  cleanup();
  // owned nnz: count from the structure (interior rows kind, boundary 1)
  int64_t nnz = 0;
  {
    // rows with Dirichlet status have 1 entry, others `kind`
    int64_t inner = 1;
    for (int d = 0; d < 3; ++d) {
      const int64_t lo = std::max<int64_t>(box_lo[d], 1), hi = std::min<int64_t>(box_lo[d] + box_n[d], gdims[d] - 1);
      inner *= std::max<int64_t>(0, hi - lo);
    }
    nnz = inner * kind + (nrows - inner);
  }
  A->nnz = nnz;
  {
    int kmax = 0;
    for (int32_t l : slen) kmax = std::max(kmax, l);
    if (finalize_pattern(A, kmax, nrows, false)) { pa_mat_destroy(A); return -1; }
  }
  *out = A;
  return 0;
}

}  // extern "C"
