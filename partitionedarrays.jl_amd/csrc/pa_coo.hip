// pa_coo.hip — `sparse(I, J, V, m, n, +)` and the owned-row SELL build on
// the device (the COO assembly path that feeds A10).
//
// Reference: PSparseMatrix(I,J,V,rows,cols;ids) (Interfaces.jl:2194-2244)
// → compresscoo / sparse (SparseUtils.jl:80-94): duplicates are combined with
// `+` in input order, rows ascend within each column.  Then the SELL layout
// of pa_mat_from_csc: each owned row's entries in the reference's summation
// order (owned columns by oid, then ghost columns by hid; SparseUtils.jl:
// 176-185 over the owned_owned and owned_ghost blocks), ghost rows' stored
// values kept after the SELL slots.
//
// Integer/byte work: two stable radix sorts (rocPRIM) over 64-bit keys, scans
// and scatters.  Duplicate sums run one thread per (i, j) in input order, so
// the result equals the host restatement bit for bit.
#include "pa_internal.h"

#include <cstring>
#include <rocprim/rocprim.hpp>

namespace pa {

// a blocking copy ordered after the work queued on stream st (a plain
// hipMemcpy goes to the null stream, which a non-blocking stream's kernels
// are not ordered against)
static inline hipError_t copy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t st) {
  hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  return e;
}


// key = (J-1)*m + (I-1) (column-major = CSC order), or (I-1)*ncols + (J-1)
// (row-major = CSR order, sparsecsr), payload = input position
template <typename IT>
__global__ void k_coo_keys(int64_t n, const IT* __restrict__ I, const IT* __restrict__ J, int64_t m,
                           int64_t ncols, int csr, uint64_t* __restrict__ key, int64_t* __restrict__ idx,
                           int* __restrict__ bad) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = (int64_t)I[k] - 1, j = (int64_t)J[k] - 1;
    if (i < 0 || i >= m || j < 0 || j >= ncols) {
      *bad = 1;
      key[k] = 0;
    } else {
      key[k] = csr ? (uint64_t)i * (uint64_t)ncols + (uint64_t)j : (uint64_t)j * (uint64_t)m + (uint64_t)i;
    }
    idx[k] = k;
  }
}

__global__ void k_heads(int64_t n, const uint64_t* __restrict__ key, int64_t* __restrict__ head) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    head[k] = (k == 0 || key[k] != key[k - 1]) ? 1 : 0;
}

// segid = inclusive scan of heads (1-based); start[segid-1] = k at each head
__global__ void k_seg_start(int64_t n, const int64_t* __restrict__ head, const int64_t* __restrict__ segid,
                            int64_t* __restrict__ start) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    if (head[k]) start[segid[k] - 1] = k;
}

// one thread per distinct (i, j): acc = V[first]; acc = acc + V[next] ... in
// input order (the sort is stable)
template <typename T>
__global__ void k_seg_sum(int64_t nu, int64_t n, const int64_t* __restrict__ start, const uint64_t* __restrict__ key,
                          const int64_t* __restrict__ idx, const T* __restrict__ V, int64_t m, int64_t ncols, int csr,
                          int32_t* __restrict__ crow, int32_t* __restrict__ ccol, T* __restrict__ cval) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < nu; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = start[s], b = (s + 1 < nu) ? start[s + 1] : n;
    T acc = V[idx[a]];
    for (int64_t k = a + 1; k < b; ++k) acc = acc + V[idx[k]];
    const uint64_t kk = key[a];
    crow[s] = (int32_t)(csr ? kk / (uint64_t)ncols : kk % (uint64_t)m);
    ccol[s] = (int32_t)(csr ? kk % (uint64_t)ncols : kk / (uint64_t)m);
    cval[s] = acc;
  }
}

// colptr[j] = first nz of column j (lower bound in the column-sorted list);
// for a CSR the same over the rows (ccol = the row of each nz)
__global__ void k_colptr(int64_t ncols, int64_t nu, const int32_t* __restrict__ ccol, int64_t* __restrict__ colptr) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j <= ncols; j += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nu;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ccol[mid] < j) lo = mid + 1; else hi = mid;
    }
    colptr[j] = lo;
  }
}

// owned-row order: key2 = oid*ncols + colpos (colpos = oid of an owned column,
// noids_c + hid of a ghost column); ghost rows sort last (key2 = max)
__global__ void k_own_keys(int64_t nu, const int32_t* __restrict__ crow, const int32_t* __restrict__ ccol,
                           const int32_t* __restrict__ rl2o, const int32_t* __restrict__ cl2o, int64_t noids_c,
                           int64_t ncols, uint64_t* __restrict__ key2, int64_t* __restrict__ idx2,
                           int64_t* __restrict__ gflag) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nu; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t o = rl2o[crow[p]];
    const int32_t oc = cl2o[ccol[p]];
    const int64_t colpos = oc > 0 ? (int64_t)oc - 1 : noids_c + (int64_t)(-oc) - 1;
    key2[p] = o > 0 ? (uint64_t)(o - 1) * (uint64_t)ncols + (uint64_t)colpos : ~0ull;
    idx2[p] = p;
    gflag[p] = o > 0 ? 0 : 1;
  }
}

// rowptr[r] = first owned entry of row r in key2 order
__global__ void k_rowptr(int64_t nrows, int64_t nnz, const uint64_t* __restrict__ key2, int64_t ncols,
                         int64_t* __restrict__ rowptr) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t target = (uint64_t)r * (uint64_t)ncols;
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (key2[mid] < target) lo = mid + 1; else hi = mid;
    }
    rowptr[r] = lo;
  }
}

// per slice: max row length, and whether any row reads a ghost column (its
// last entry, ghost columns sorting after owned ones)
__global__ void k_slice_len(int64_t ns, int64_t nrows, int H, const int64_t* __restrict__ rowptr,
                            const uint64_t* __restrict__ key2, int64_t ncols, int64_t noids_c,
                            const int32_t* __restrict__ lidx, int32_t* __restrict__ slen,
                            int32_t* __restrict__ sghost) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < ns; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r0 = s * H, r1 = (r0 + H < nrows) ? r0 + H : nrows;
    int32_t L = 0, g = 0;
    for (int64_t r = r0; r < r1; ++r) {
      if (lidx && lidx[r] >= 0) continue;  // long rows leave the SELL
      const int64_t a = rowptr[r], b = rowptr[r + 1];
      if (b - a > L) L = (int32_t)(b - a);
      if (b > a && (int64_t)(key2[b - 1] % (uint64_t)ncols) >= noids_c) g = 1;
    }
    slen[s] = L;
    sghost[s] = g;
  }
}

// lidx[r] >= 0: long row r, its entries go to the long CSR at lptr[lidx[r]]
// (values at val[long_off + ..], nz_slot = -(ngh + pos + 1))
template <typename T>
__global__ void k_fill_slots(int64_t nnz, const uint64_t* __restrict__ key2, const int64_t* __restrict__ idx2,
                             const int64_t* __restrict__ rowptr, const int64_t* __restrict__ soff, int H, int R,
                             int64_t ncols, const int32_t* __restrict__ ccol, const T* __restrict__ cval,
                             int32_t* __restrict__ col, T* __restrict__ val, int64_t* __restrict__ nz_slot,
                             const int32_t* __restrict__ lidx, const int64_t* __restrict__ lptr,
                             int32_t* __restrict__ lcol, int64_t long_off, int64_t ngh) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nnz; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = (int64_t)(key2[t] / (uint64_t)ncols);
    const int64_t k = t - rowptr[r];
    if (lidx && lidx[r] >= 0) {
      const int64_t pos = lptr[lidx[r]] + k;
      const int64_t p = idx2[t];
      lcol[pos] = ccol[p];
      val[long_off + pos] = cval[p];
      nz_slot[p] = -(ngh + pos + 1);
      continue;
    }
    const int64_t s = r / H, w = r - s * H;
    const int64_t slot = soff[s] + (k * 64 + w / R) * R + (w % R);
    const int64_t p = idx2[t];
    col[slot] = ccol[p];
    val[slot] = cval[p];
    nz_slot[p] = slot;
  }
}

// ghost-row nonzeros in CSC order after the slots: nz_slot = -(rank+1)
template <typename T>
__global__ void k_fill_ghost(int64_t nu, const int64_t* __restrict__ gflag, const int64_t* __restrict__ grank,
                             const T* __restrict__ cval, int64_t slots, T* __restrict__ val,
                             int64_t* __restrict__ nz_slot) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nu; p += (int64_t)gridDim.x * blockDim.x)
    if (gflag[p]) {
      const int64_t g = grank[p];
      nz_slot[p] = -(g + 1);
      val[slots + g] = cval[p];
    }
}

__global__ void k_fill_i32(int64_t n, int32_t* __restrict__ a, int32_t v) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    a[k] = v;
}

namespace {

inline dim3 grid1(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > 16384) g = 16384;
  return dim3((unsigned)g);
}

inline int bits_for(uint64_t maxkey) {
  int b = 1;
  while (b < 64 && (maxkey >> b)) ++b;
  return b;
}

// stable sort of (key, idx) pairs in place (double buffer + temp storage)
hipError_t sort_pairs(uint64_t*& key, int64_t*& idx, int64_t n, int end_bit, hipStream_t st) {
  if (n <= 1) return hipSuccess;
  uint64_t* k2 = nullptr;
  int64_t* i2 = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  hipError_t e = hipMalloc((void**)&k2, n * 8);
  if (e == hipSuccess) e = hipMalloc((void**)&i2, n * 8);
  rocprim::double_buffer<uint64_t> kb(key, k2);
  rocprim::double_buffer<int64_t> ib(idx, i2);
  if (e == hipSuccess) e = rocprim::radix_sort_pairs(nullptr, tb, kb, ib, (size_t)n, 0, (unsigned)end_bit, st);
  if (e == hipSuccess) e = hipMalloc(&tmp, tb ? tb : 1);
  if (e == hipSuccess) e = rocprim::radix_sort_pairs(tmp, tb, kb, ib, (size_t)n, 0, (unsigned)end_bit, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (tmp) (void)hipFree(tmp);
  // keep the buffers holding the result
  if (kb.current() != key) { (void)hipFree(key); key = kb.current(); } else (void)hipFree(k2);
  if (ib.current() != idx) { (void)hipFree(idx); idx = ib.current(); } else (void)hipFree(i2);
  return e;
}

hipError_t inclusive_sum(const int64_t* in, int64_t* out, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  size_t tb = 0;
  void* tmp = nullptr;
  hipError_t e = rocprim::inclusive_scan(nullptr, tb, in, out, (size_t)n, rocprim::plus<int64_t>(), st);
  if (e == hipSuccess) e = hipMalloc(&tmp, tb ? tb : 1);
  if (e == hipSuccess) e = rocprim::inclusive_scan(tmp, tb, in, out, (size_t)n, rocprim::plus<int64_t>(), st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (tmp) (void)hipFree(tmp);
  return e;
}

hipError_t exclusive_sum(const int64_t* in, int64_t* out, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  size_t tb = 0;
  void* tmp = nullptr;
  hipError_t e = rocprim::exclusive_scan(nullptr, tb, in, out, (int64_t)0, (size_t)n, rocprim::plus<int64_t>(), st);
  if (e == hipSuccess) e = hipMalloc(&tmp, tb ? tb : 1);
  if (e == hipSuccess) e = rocprim::exclusive_scan(tmp, tb, in, out, (int64_t)0, (size_t)n, rocprim::plus<int64_t>(), st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (tmp) (void)hipFree(tmp);
  return e;
}

template <typename T>
void seg_sum_t(int64_t nu, int64_t n, const int64_t* start, const uint64_t* key, const int64_t* idx,
               const void* V, int64_t m, int64_t ncols, int csr, int32_t* crow, int32_t* ccol, void* cval,
               hipStream_t st) {
  hipLaunchKernelGGL(k_seg_sum<T>, grid1(nu), dim3(256), 0, st, nu, n, start, key, idx, (const T*)V, m, ncols, csr,
                     crow, ccol, (T*)cval);
}

}  // namespace

#define PA_HIP_TRY(expr)                     \
  do {                                       \
    hipError_t e_ = (expr);                  \
    if (e_ != hipSuccess) {                  \
      err = e_;                              \
      goto done;                             \
    }                                        \
  } while (0)

// Phase A: sparse(I, J, V, m, n, +) → CSC on the device (0-based rows/cols,
// values combined).  I, J: 1-based device arrays (index_bytes 4 or 8).
// On success the caller owns *crow, *ccol, *cval (nu entries) and *colptr
// (ncols+1, 0-based offsets).  Returns 1 on an out-of-range index.
// csr: sparsecsr instead — the nonzeros in row-major (CSR) order and
// *colptr the row pointers (m+1).
int coo_compress(int dtype, int index_bytes, int64_t m, int64_t ncols, int64_t n, const void* dI, const void* dJ,
                 const void* dV, int csr, int64_t* nu_out, int32_t** crow, int32_t** ccol, void** cval,
                 int64_t** colptr, hipStream_t st, hipError_t* err_out) {
  hipError_t err = hipSuccess;
  const size_t S = dtype_size(dtype);
  uint64_t* key = nullptr;
  int64_t *idx = nullptr, *head = nullptr, *segid = nullptr, *start = nullptr;
  int* bad = nullptr;
  int hbad = 0;
  int64_t nu = 0;
  *crow = nullptr;
  *ccol = nullptr;
  *cval = nullptr;
  *colptr = nullptr;
  int rc = 0;
  const int64_t nptr = csr ? m : ncols;  // columns (CSC) or rows (CSR) of the compressed axis
  PA_HIP_TRY(hipMalloc((void**)colptr, (nptr + 1) * 8));
  if (n > 0) {
    PA_HIP_TRY(hipMalloc((void**)&key, n * 8));
    PA_HIP_TRY(hipMalloc((void**)&idx, n * 8));
    PA_HIP_TRY(hipMalloc((void**)&bad, sizeof(int)));
    PA_HIP_TRY(hipMemsetAsync(bad, 0, sizeof(int), st));
    if (index_bytes == 8)
      hipLaunchKernelGGL(k_coo_keys<int64_t>, grid1(n), dim3(256), 0, st, n, (const int64_t*)dI, (const int64_t*)dJ,
                         m, ncols, csr, key, idx, bad);
    else
      hipLaunchKernelGGL(k_coo_keys<int32_t>, grid1(n), dim3(256), 0, st, n, (const int32_t*)dI, (const int32_t*)dJ,
                         m, ncols, csr, key, idx, bad);
    PA_HIP_TRY(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, st));
    PA_HIP_TRY(hipStreamSynchronize(st));
    if (hbad) { rc = 1; goto done; }
    PA_HIP_TRY(sort_pairs(key, idx, n, bits_for((uint64_t)m * (uint64_t)ncols), st));
    PA_HIP_TRY(hipMalloc((void**)&head, n * 8));
    PA_HIP_TRY(hipMalloc((void**)&segid, n * 8));
    hipLaunchKernelGGL(k_heads, grid1(n), dim3(256), 0, st, n, key, head);
    PA_HIP_TRY(inclusive_sum(head, segid, n, st));
    PA_HIP_TRY(copy_sync(&nu, segid + n - 1, 8, hipMemcpyDeviceToHost, st));
    PA_HIP_TRY(hipMalloc((void**)&start, nu * 8));
    hipLaunchKernelGGL(k_seg_start, grid1(n), dim3(256), 0, st, n, head, segid, start);
    PA_HIP_TRY(hipMalloc((void**)crow, nu * 4));
    PA_HIP_TRY(hipMalloc((void**)ccol, nu * 4));
    PA_HIP_TRY(hipMalloc(cval, nu * S));
    switch (dtype) {
      case PA_F32: seg_sum_t<float>(nu, n, start, key, idx, dV, m, ncols, csr, *crow, *ccol, *cval, st); break;
      case PA_F64: seg_sum_t<double>(nu, n, start, key, idx, dV, m, ncols, csr, *crow, *ccol, *cval, st); break;
      case PA_C64: seg_sum_t<c64>(nu, n, start, key, idx, dV, m, ncols, csr, *crow, *ccol, *cval, st); break;
      case PA_C128: seg_sum_t<c128>(nu, n, start, key, idx, dV, m, ncols, csr, *crow, *ccol, *cval, st); break;
    }
  }
  hipLaunchKernelGGL(k_colptr, grid1(nptr + 1), dim3(256), 0, st, nptr, nu, csr ? *crow : *ccol, *colptr);
  PA_HIP_TRY(hipGetLastError());
  PA_HIP_TRY(hipStreamSynchronize(st));
done:
  for (void* p : {(void*)key, (void*)idx, (void*)head, (void*)segid, (void*)start, (void*)bad})
    if (p) (void)hipFree(p);
  *nu_out = nu;
  *err_out = err;
  if (err != hipSuccess || rc) {
    for (void** p : {(void**)crow, (void**)ccol, cval, (void**)colptr})
      if (*p) { (void)hipFree(*p); *p = nullptr; }
    return err != hipSuccess ? -1 : rc;
  }
  return 0;
}

// Phase B, first half: order the owned rows' entries (key2/idx2, nnz owned
// entries first), row pointers, per-slice lengths / ghost flags, ghost-row
// flags and ranks.  Device outputs are owned by the caller.
int coo_row_order(int64_t nu, const int32_t* crow, const int32_t* ccol, const int32_t* rl2o, const int32_t* cl2o,
                  int64_t nrows, int64_t noids_c, int64_t ncols, int H, uint64_t** key2, int64_t** idx2,
                  int64_t** rowptr, int64_t** gflag, int64_t** grank, int32_t** slen, int32_t** sghost,
                  int64_t* nnz_out, int64_t* ngh_out, hipStream_t st, hipError_t* err_out) {
  hipError_t err = hipSuccess;
  const int64_t ns = (nrows + H - 1) / H;
  int64_t nnz = 0, ngh = 0, last = 0, lastf = 0;
  *key2 = nullptr; *idx2 = nullptr; *rowptr = nullptr; *gflag = nullptr; *grank = nullptr;
  *slen = nullptr; *sghost = nullptr;
  const int64_t nb = nu > 0 ? nu : 1;
  PA_HIP_TRY(hipMalloc((void**)key2, nb * 8));
  PA_HIP_TRY(hipMalloc((void**)idx2, nb * 8));
  PA_HIP_TRY(hipMalloc((void**)gflag, nb * 8));
  PA_HIP_TRY(hipMalloc((void**)grank, nb * 8));
  PA_HIP_TRY(hipMalloc((void**)rowptr, (nrows + 1) * 8));
  PA_HIP_TRY(hipMalloc((void**)slen, (ns > 0 ? ns : 1) * 4));
  PA_HIP_TRY(hipMalloc((void**)sghost, (ns > 0 ? ns : 1) * 4));
  if (nu > 0) {
    hipLaunchKernelGGL(k_own_keys, grid1(nu), dim3(256), 0, st, nu, crow, ccol, rl2o, cl2o, noids_c, ncols, *key2,
                       *idx2, *gflag);
    PA_HIP_TRY(exclusive_sum(*gflag, *grank, nu, st));
    PA_HIP_TRY(copy_sync(&last, *grank + nu - 1, 8, hipMemcpyDeviceToHost, st));
    PA_HIP_TRY(copy_sync(&lastf, *gflag + nu - 1, 8, hipMemcpyDeviceToHost, st));
    ngh = last + lastf;
    nnz = nu - ngh;
    // ghost rows carry key2 = ~0: sort all bits of the owned range + 1
    const uint64_t maxk = (uint64_t)(nrows > 0 ? nrows : 1) * (uint64_t)ncols;
    PA_HIP_TRY(sort_pairs(*key2, *idx2, nu, ngh ? 64 : bits_for(maxk), st));
  }
  hipLaunchKernelGGL(k_rowptr, grid1(nrows + 1), dim3(256), 0, st, nrows, nnz, *key2, ncols, *rowptr);
  PA_HIP_TRY(hipGetLastError());
  PA_HIP_TRY(hipStreamSynchronize(st));
done:
  *nnz_out = nnz;
  *ngh_out = ngh;
  *err_out = err;
  if (err != hipSuccess) {
    for (void** p : {(void**)key2, (void**)idx2, (void**)rowptr, (void**)gflag, (void**)grank, (void**)slen,
                     (void**)sghost})
      if (*p) { (void)hipFree(*p); *p = nullptr; }
    return -1;
  }
  return 0;
}

// Phase B, second half: scatter into the SELL slots (col pre-filled with -1,
// val zeroed by the caller) and the ghost-row values after them.
// per-slice max row length and ghost flag of the SELL rows (long rows skipped)
void coo_slices(int64_t ns, int64_t nrows, int H, const int64_t* rowptr, const uint64_t* key2, int64_t ncols,
                int64_t noids_c, const int32_t* lidx, int32_t* slen, int32_t* sghost, hipStream_t st) {
  if (ns > 0)
    hipLaunchKernelGGL(k_slice_len, grid1(ns), dim3(256), 0, st, ns, nrows, H, rowptr, key2, ncols, noids_c, lidx,
                       slen, sghost);
}

void coo_fill(int dtype, int64_t nnz, int64_t nu, const uint64_t* key2, const int64_t* idx2, const int64_t* rowptr,
              const int64_t* soff, int H, int R, int64_t ncols, const int32_t* ccol, const void* cval,
              const int64_t* gflag, const int64_t* grank, int64_t slots, int32_t* col, void* val, int64_t* nz_slot,
              const int32_t* lidx, const int64_t* lptr, int32_t* lcol, int64_t long_off, hipStream_t st) {
  const int64_t ngh = long_off - slots;
#define PA_FILL(T)                                                                                             \
  if (nnz > 0)                                                                                                 \
    hipLaunchKernelGGL(k_fill_slots<T>, grid1(nnz), dim3(256), 0, st, nnz, key2, idx2, rowptr, soff, H, R,     \
                       ncols, ccol, (const T*)cval, col, (T*)val, nz_slot, lidx, lptr, lcol, long_off, ngh);   \
  if (nu > 0)                                                                                                  \
    hipLaunchKernelGGL(k_fill_ghost<T>, grid1(nu), dim3(256), 0, st, nu, gflag, grank, (const T*)cval, slots, \
                       (T*)val, nz_slot);
  switch (dtype) {
    case PA_F32: { PA_FILL(float) } break;
    case PA_F64: { PA_FILL(double) } break;
    case PA_C64: { PA_FILL(c64) } break;
    case PA_C128: { PA_FILL(c128) } break;
  }
#undef PA_FILL
}

void launch_fill_i32(int64_t n, int32_t* a, int32_t v, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_fill_i32, grid1(n), dim3(256), 0, st, n, a, v);
}

}  // namespace pa

// ---------------------------------------------------------------------------
// Global ids on the device: the gid → lid table of an
// index set (sorted gids + their lids), `to_lids!` (Interfaces.jl:1541-1543)
// and the first-touch ghost discovery of `add_gids!` (579-603, 1515-1533).

namespace pa {

__global__ void k_iota_i64(int64_t n, int64_t* __restrict__ a) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    a[k] = k;
}

// lid (0-based) of gid, or -1: binary search in the sorted gid table
__device__ inline int64_t gid_lookup(int64_t g, const uint64_t* __restrict__ sgid, const int64_t* __restrict__ slid,
                                     int64_t nl) {
  int64_t lo = 0, hi = nl;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)sgid[mid] < g) lo = mid + 1; else hi = mid;
  }
  return (lo < nl && (int64_t)sgid[lo] == g) ? slid[lo] : -1;
}

// ids (1-based gids) → 1-based lids in place; *bad = 1 if a gid is absent
__global__ void k_to_lids(int64_t n, int64_t* __restrict__ ids, const uint64_t* __restrict__ sgid,
                          const int64_t* __restrict__ slid, int64_t nl, int* __restrict__ bad) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = gid_lookup(ids[k], sgid, slid, nl);
    if (l < 0) *bad = 1;
    ids[k] = l + 1;
  }
}

// flag[k] = gid absent from the table
__global__ void k_absent(int64_t n, const int64_t* __restrict__ gids, const uint64_t* __restrict__ sgid,
                         const int64_t* __restrict__ slid, int64_t nl, int64_t* __restrict__ flag) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    flag[k] = gid_lookup(gids[k], sgid, slid, nl) < 0 ? 1 : 0;
}

__global__ void k_compact(int64_t n, const int64_t* __restrict__ gids, const int64_t* __restrict__ flag,
                          const int64_t* __restrict__ pos, uint64_t* __restrict__ key, int64_t* __restrict__ val) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    if (flag[k]) {
      key[pos[k]] = (uint64_t)gids[k];
      val[pos[k]] = k;
    }
}

// after sorting (gid, position) pairs: at each distinct gid, its first
// position becomes the key and the gid the payload
__global__ void k_first_touch(int64_t m, const uint64_t* __restrict__ key, const int64_t* __restrict__ val,
                              const int64_t* __restrict__ head, const int64_t* __restrict__ rank,
                              uint64_t* __restrict__ key2, int64_t* __restrict__ val2) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
    if (head[k]) {
      key2[rank[k] - 1] = (uint64_t)val[k];
      val2[rank[k] - 1] = (int64_t)key[k];
    }
}

// sorted (gid, lid) table of lid_to_gid (device input, n lids)
int gid_table(int64_t n, const int64_t* d_lid_to_gid, uint64_t** sgid, int64_t** slid, hipStream_t st) {
  *sgid = nullptr;
  *slid = nullptr;
  if (n <= 0) return 0;
  int64_t maxg = 0;
  if (hipMalloc((void**)sgid, n * 8) != hipSuccess || hipMalloc((void**)slid, n * 8) != hipSuccess) return -1;
  if (hipMemcpyAsync(*sgid, d_lid_to_gid, n * 8, hipMemcpyDeviceToDevice, st) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_iota_i64, grid1(n), dim3(256), 0, st, n, *slid);
  // the largest gid bounds the radix passes
  {
    size_t tb = 0;
    void* tmp = nullptr;
    int64_t* dmax = nullptr;
    if (hipMalloc((void**)&dmax, 8) != hipSuccess) return -1;
    hipError_t e = rocprim::reduce(nullptr, tb, d_lid_to_gid, dmax, (int64_t)0, (size_t)n, rocprim::maximum<int64_t>(), st);
    if (e == hipSuccess) e = hipMalloc(&tmp, tb ? tb : 1);
    if (e == hipSuccess) e = rocprim::reduce(tmp, tb, d_lid_to_gid, dmax, (int64_t)0, (size_t)n, rocprim::maximum<int64_t>(), st);
    if (e == hipSuccess) e = hipMemcpyAsync(&maxg, dmax, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (tmp) (void)hipFree(tmp);
    (void)hipFree(dmax);
    if (e != hipSuccess) return -1;
  }
  return sort_pairs(*sgid, *slid, n, bits_for((uint64_t)(maxg > 0 ? maxg : 1)), st) == hipSuccess ? 0 : -1;
}

// ids (n, device, 1-based gids) → 1-based lids; returns 1 if a gid is absent
int gids_to_lids(int64_t n, int64_t* ids, const uint64_t* sgid, const int64_t* slid, int64_t nl, hipStream_t st) {
  if (n <= 0) return 0;
  int* bad = nullptr;
  int hbad = 0;
  if (hipMalloc((void**)&bad, sizeof(int)) != hipSuccess) return -1;
  hipError_t e = hipMemsetAsync(bad, 0, sizeof(int), st);
  hipLaunchKernelGGL(k_to_lids, grid1(n), dim3(256), 0, st, n, ids, sgid, slid, nl, bad);
  if (e == hipSuccess) e = hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(bad);
  if (e != hipSuccess) return -1;
  return hbad ? 1 : 0;
}

// add_gids!: the gids (device, n) absent from the table, each once, in order
// of first occurrence.  *out (device, *m entries) is owned by the caller.
int gids_first_touch(int64_t n, const int64_t* gids, const uint64_t* sgid, const int64_t* slid, int64_t nl,
                     int64_t** out, int64_t* m_out, hipStream_t st) {
  *out = nullptr;
  *m_out = 0;
  if (n <= 0) return 0;
  int64_t *flag = nullptr, *pos = nullptr, *val = nullptr, *head = nullptr, *rank = nullptr, *val2 = nullptr;
  uint64_t *key = nullptr, *key2 = nullptr;
  int64_t m = 0, lastf = 0, u = 0, maxg = 0;
  hipError_t e = hipMalloc((void**)&flag, n * 8);
  if (e == hipSuccess) e = hipMalloc((void**)&pos, n * 8);
  if (e != hipSuccess) goto fail;
  hipLaunchKernelGGL(k_absent, grid1(n), dim3(256), 0, st, n, gids, sgid, slid, nl, flag);
  e = exclusive_sum(flag, pos, n, st);
  if (e == hipSuccess) e = copy_sync(&m, pos + n - 1, 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = copy_sync(&lastf, flag + n - 1, 8, hipMemcpyDeviceToHost, st);
  if (e != hipSuccess) goto fail;
  m += lastf;
  if (m > 0) {
    e = hipMalloc((void**)&key, m * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&val, m * 8);
    if (e != hipSuccess) goto fail;
    hipLaunchKernelGGL(k_compact, grid1(n), dim3(256), 0, st, n, gids, flag, pos, key, val);
    (void)hipFree(flag); flag = nullptr;
    (void)hipFree(pos); pos = nullptr;
    {
      size_t tb = 0;
      void* tmp = nullptr;
      int64_t* dmax = nullptr;
      e = hipMalloc((void**)&dmax, 8);
      if (e == hipSuccess) e = rocprim::reduce(nullptr, tb, (const int64_t*)key, dmax, (int64_t)0, (size_t)m, rocprim::maximum<int64_t>(), st);
      if (e == hipSuccess) e = hipMalloc(&tmp, tb ? tb : 1);
      if (e == hipSuccess) e = rocprim::reduce(tmp, tb, (const int64_t*)key, dmax, (int64_t)0, (size_t)m, rocprim::maximum<int64_t>(), st);
      if (e == hipSuccess) e = hipMemcpyAsync(&maxg, dmax, 8, hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      if (tmp) (void)hipFree(tmp);
      if (dmax) (void)hipFree(dmax);
      if (e != hipSuccess) goto fail;
    }
    e = sort_pairs(key, val, m, bits_for((uint64_t)(maxg > 0 ? maxg : 1)), st);
    if (e == hipSuccess) e = hipMalloc((void**)&head, m * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&rank, m * 8);
    if (e != hipSuccess) goto fail;
    hipLaunchKernelGGL(k_heads, grid1(m), dim3(256), 0, st, m, key, head);
    e = inclusive_sum(head, rank, m, st);
    if (e == hipSuccess) e = copy_sync(&u, rank + m - 1, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMalloc((void**)&key2, u * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&val2, u * 8);
    if (e != hipSuccess) goto fail;
    hipLaunchKernelGGL(k_first_touch, grid1(m), dim3(256), 0, st, m, key, val, head, rank, key2, val2);
    e = sort_pairs(key2, val2, u, bits_for((uint64_t)n), st);
    if (e != hipSuccess) goto fail;
    *out = val2;
    val2 = nullptr;
    *m_out = u;
  }
fail:
  for (void* p : {(void*)flag, (void*)pos, (void*)val, (void*)head, (void*)rank, (void*)val2, (void*)key, (void*)key2})
    if (p) (void)hipFree(p);
  return e == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------
// async_assemble!(I, J, V, rows) (Interfaces.jl:2406-2492) on the device: the
// triplets whose row is owned by another part are grouped by owner (segments
// in rows.exchanger.parts_rcv order, input order inside each), copied out
// and their local value set to zero; the host side (pa_api.cpp) moves the
// segments to the owners, which append them in parts_snd order.

// seg_of_lid[lids_rcv[t]] = the segment of slot t (every ghost lid is in
// exactly one receive segment: the one of its owner, Interfaces.jl:740-762)
__global__ void k_seg_of_lid(int64_t nslots, const int32_t* __restrict__ lids_rcv, const int64_t* __restrict__ ptrs,
                             int nseg, int32_t* __restrict__ seg_of_lid) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nslots; t += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = nseg;  // last segment whose start <= t
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (ptrs[mid] <= t) lo = mid; else hi = mid;
    }
    seg_of_lid[lids_rcv[t]] = lo;
  }
}

// key[k] = 0 for a row owned here, 1 + segment of the row's owner otherwise
// (rows' gid table: an absent gid is the KeyError of to_lids!; a ghost row
// that no receive segment lists is the KeyError of owner_to_i,
// Interfaces.jl:2428-2430: the exchanger does not match the rows)
__global__ void k_coo_seg(int64_t n, const int64_t* __restrict__ I, const uint64_t* __restrict__ sgid,
                          const int64_t* __restrict__ slid, int64_t nl, const int32_t* __restrict__ seg_of_lid,
                          uint64_t* __restrict__ key, int64_t* __restrict__ idx, int* __restrict__ bad) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = gid_lookup(I[k], sgid, slid, nl);
    const int32_t sg = l < 0 ? -1 : seg_of_lid[l];
    if (l < 0) *bad = 1;
    else if (sg == -2) *bad = 2;  // a ghost row whose owner is not in parts_rcv
    key[k] = sg < 0 ? 0 : (uint64_t)(sg + 1);
    idx[k] = k;
  }
}

// first[key] = the first position of each key of the sorted keys
__global__ void k_key_first(int64_t n, const uint64_t* __restrict__ key, int64_t* __restrict__ first) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    if (t == 0 || key[t] != key[t - 1]) first[key[t]] = t;
}

// the nr sent triplets in segment order: sI/sJ/sV[t] = I/J/V[idx[t]], and
// the local value becomes zero(v) (the entry stays in the local list)
template <typename T>
__global__ void k_coo_pack(int64_t nr, const int64_t* __restrict__ idx, const int64_t* __restrict__ I,
                           const int64_t* __restrict__ J, T* __restrict__ V, int64_t* __restrict__ sI,
                           int64_t* __restrict__ sJ, T* __restrict__ sV) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nr; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = idx[t];
    sI[t] = I[k];
    sJ[t] = J[k];
    sV[t] = V[k];
    V[k] = zero_of<T>();
  }
}

// One part's send side.  Outputs (device, owned by the caller): *sI, *sJ,
// *sV (the sent triplets, segment after segment) and cnt[0..nseg) on the
// host.  Returns 1 when a row gid is not a local id of rows (KeyError), 2
// when a ghost row's owner has no receive segment (KeyError).
int coo_assemble_pack(int dtype, int64_t n, const int64_t* I, const int64_t* J, void* V, const uint64_t* sgid,
                      const int64_t* slid, int64_t nl, const std::vector<int32_t>& lid_to_ohid, int nseg,
                      const int32_t* d_lids_rcv,
                      const std::vector<int64_t>& ptrs_rcv, int64_t** sI, int64_t** sJ, void** sV,
                      std::vector<int64_t>* cnt, hipStream_t st) {
  const size_t S = dtype_size(dtype);
  *sI = nullptr; *sJ = nullptr; *sV = nullptr;
  cnt->assign(nseg, 0);
  if (n <= 0) return 0;
  hipError_t e = hipSuccess;
  int32_t* sol = nullptr;
  int64_t *dptrs = nullptr, *idx = nullptr, *first = nullptr;
  uint64_t* key = nullptr;
  int* bad = nullptr;
  int hbad = 0, rc = 0;
  std::vector<int64_t> hfirst(nseg + 2, -1);
  const int64_t nslots = ptrs_rcv.empty() ? 0 : ptrs_rcv.back();
  int64_t nloc = n;
  {
    // -1: owned lid, -2: ghost lid (k_seg_of_lid then sets its segment)
    std::vector<int32_t> hs(nl > 0 ? nl : 1, -1);
    for (int64_t l = 0; l < nl; ++l) hs[l] = lid_to_ohid[l] > 0 ? -1 : -2;
    e = hipMalloc((void**)&sol, hs.size() * 4);
    if (e == hipSuccess) e = copy_sync(sol, hs.data(), hs.size() * 4, hipMemcpyHostToDevice, st);
  }
  if (e == hipSuccess && nslots > 0) e = hipMalloc((void**)&dptrs, ptrs_rcv.size() * 8);
  if (e == hipSuccess && nslots > 0)
    e = hipMemcpyAsync(dptrs, ptrs_rcv.data(), ptrs_rcv.size() * 8, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) goto done;
  if (nslots > 0) hipLaunchKernelGGL(k_seg_of_lid, grid1(nslots), dim3(256), 0, st, nslots, d_lids_rcv, dptrs, nseg, sol);
  e = hipMalloc((void**)&key, n * 8);
  if (e == hipSuccess) e = hipMalloc((void**)&idx, n * 8);
  if (e == hipSuccess) e = hipMalloc((void**)&bad, sizeof(int));
  if (e == hipSuccess) e = hipMemsetAsync(bad, 0, sizeof(int), st);
  if (e != hipSuccess) goto done;
  hipLaunchKernelGGL(k_coo_seg, grid1(n), dim3(256), 0, st, n, I, sgid, slid, nl, sol, key, idx, bad);
  e = hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) goto done;
  if (hbad) { rc = hbad; goto done; }  // 1: unknown gid, 2: ghost row without a segment
  e = sort_pairs(key, idx, n, bits_for((uint64_t)nseg + 1), st);  // stable: input order inside a segment
  if (e == hipSuccess) e = hipMalloc((void**)&first, (nseg + 2) * 8);
  if (e == hipSuccess) e = hipMemsetAsync(first, 0xff, (nseg + 2) * 8, st);
  if (e != hipSuccess) goto done;
  hipLaunchKernelGGL(k_key_first, grid1(n), dim3(256), 0, st, n, key, first);
  e = hipMemcpyAsync(hfirst.data(), first, (nseg + 1) * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) goto done;
  {
    // end of key q = start of the next present key, or n
    hfirst[nseg + 1] = n;
    std::vector<int64_t> start(nseg + 2, n);
    for (int q = nseg; q >= 0; --q) start[q] = hfirst[q] >= 0 ? hfirst[q] : start[q + 1];
    nloc = start[1];
    for (int q = 0; q < nseg; ++q) (*cnt)[q] = start[q + 2] - start[q + 1];
  }
  if (n - nloc > 0) {
    const int64_t nr = n - nloc;
    e = hipMalloc((void**)sI, nr * 8);
    if (e == hipSuccess) e = hipMalloc((void**)sJ, nr * 8);
    if (e == hipSuccess) e = hipMalloc(sV, nr * S);
    if (e != hipSuccess) goto done;
#define PA_PK(T) hipLaunchKernelGGL(k_coo_pack<T>, grid1(nr), dim3(256), 0, st, nr, idx + nloc, I, J, (T*)V, *sI, *sJ, (T*)*sV)
    switch (dtype) {
      case PA_F32: PA_PK(float); break;
      case PA_F64: PA_PK(double); break;
      case PA_C64: PA_PK(c64); break;
      case PA_C128: PA_PK(c128); break;
    }
#undef PA_PK
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
done:
  for (void* p : {(void*)sol, (void*)dptrs, (void*)idx, (void*)first, (void*)key, (void*)bad})
    if (p) (void)hipFree(p);
  if (e != hipSuccess || rc) {
    for (void** p : {(void**)sI, (void**)sJ, sV})
      if (*p) { (void)hipFree(*p); *p = nullptr; }
    return e != hipSuccess ? -1 : rc;
  }
  return 0;
}

}  // namespace pa
