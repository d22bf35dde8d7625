// pa_kernels.hip — gfx950 kernels of libpa_hip.so.
//
// Hot path: the owned-row SELL SpMV (k_spmv_sell), the halo pack/unpack
// kernels and the deterministic reductions.  Everything here is HBM-bound
// integer/byte + f32/f64 work: no MFMA (≈0.17 flop/byte).
//
// Numerics: compiled with -ffp-contract=off so that each row is accumulated
// exactly like the reference's CSC loop (SparseUtils.jl:176-185):
//   acc = β-init; for each stored entry of the row in (own oid, ghost hid)
//   order: acc = acc + v * (x*α)
// which makes the SpMV bit-identical to SequentialBackend/MPIBackend.
#include "pa_internal.h"

#include <hip/hip_ext.h>

namespace pa {

// One kernel launch whose completion is recorded in ev (null: none): the
// launch and the record as one runtime call (hipExtLaunchKernel binds ev to
// the kernel's dispatch), what the barrier issue of a stream-pair mul! pays
// per part for its pack and its pull (pa_api.cpp spmv_barrier_issue).
template <typename K, typename... Args>
static void launch_ev(K kernel, dim3 grid, hipStream_t st, hipEvent_t ev, Args... args) {
  if (ev) hipExtLaunchKernelGGL(kernel, grid, dim3(256), 0, st, nullptr, ev, 0, args...);
  else hipLaunchKernelGGL(kernel, grid, dim3(256), 0, st, args...);
}


// SELL SpMV kernels: pa_spmv.hip

// pa_tune("fault_inject"): a launch the runtime rejects before anything runs
// (more threads per block than the hardware allows): the error path of the
// threaded issue, tested without a faulting kernel
__global__ void k_never_runs() {}
void launch_invalid_config() { hipLaunchKernelGGL(k_never_runs, dim3(1), dim3(4096), 0, nullptr); }

// ---------------------------------------------------------------------------
// Halo pack / unpack (Interfaces.jl:858-866 and 878-886).

template <typename T>
__global__ void k_pack(int64_t n, const int32_t* __restrict__ lids, const T* __restrict__ v,
                       T* __restrict__ buf) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x)
    buf[p] = v[lids[p]];
}

// every target lid appears once: plain scatter (replace) or one combine (add)
template <typename T, int OP>
__global__ void k_unpack_unique(int64_t n, const int32_t* __restrict__ lids,
                                const T* __restrict__ buf, T* __restrict__ v) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = lids[p];
    v[l] = (OP == PA_ADD) ? v[l] + buf[p] : buf[p];
  }
}

// a lid may receive several contributions: fold them in buffer order
// (values_rcv[lid] = combine_op(values_rcv[lid], data_rcv.data[p]), p ascending)
template <typename T, int OP>
__global__ void k_unpack_ordered(int64_t ntargets, const int32_t* __restrict__ target,
                                 const int32_t* __restrict__ ptr, const int32_t* __restrict__ pos,
                                 const T* __restrict__ buf, T* __restrict__ v) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < ntargets;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = target[t];
    T acc = v[l];
    for (int32_t q = ptr[t]; q < ptr[t + 1]; ++q) {
      const T b = buf[pos[q]];
      acc = (OP == PA_ADD) ? acc + b : b;
    }
    v[l] = acc;
  }
}

static inline int grid_for(int64_t n, int block = 256, int64_t cap = 4096) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

template <typename T>
static void pack_t(int64_t n, const int32_t* lids, const void* v, void* buf, hipStream_t st, hipEvent_t ev) {
  if (n <= 0) {
    if (ev) (void)hipEventRecord(ev, st);
    return;
  }
  launch_ev(k_pack<T>, dim3(grid_for(n)), st, ev, n, lids, (const T*)v, (T*)buf);
}

template <typename T>
static void unpack_t(int64_t n, const int32_t* lids, const pa_combine_plan& plan, int op,
                     const void* buf, void* v, hipStream_t st) {
  if (n <= 0) return;
  if (plan.unique) {
    if (op == PA_ADD)
      hipLaunchKernelGGL((k_unpack_unique<T, PA_ADD>), dim3(grid_for(n)), dim3(256), 0, st, n, lids,
                         (const T*)buf, (T*)v);
    else
      hipLaunchKernelGGL((k_unpack_unique<T, PA_REPLACE>), dim3(grid_for(n)), dim3(256), 0, st, n,
                         lids, (const T*)buf, (T*)v);
  } else {
    const int64_t nt = plan.ntargets;
    if (op == PA_ADD)
      hipLaunchKernelGGL((k_unpack_ordered<T, PA_ADD>), dim3(grid_for(nt)), dim3(256), 0, st, nt,
                         plan.d_target, plan.d_ptr, plan.d_pos, (const T*)buf, (T*)v);
    else
      hipLaunchKernelGGL((k_unpack_ordered<T, PA_REPLACE>), dim3(grid_for(nt)), dim3(256), 0, st, nt,
                         plan.d_target, plan.d_ptr, plan.d_pos, (const T*)buf, (T*)v);
  }
}

// Pull-unpack (parts of one process): receive slot p reads its value straight
// from the sender's send buffer, bases[bid[p]][elem[p]] (peer memory over
// xGMI when the sender is on another device) — no staging copy.
template <typename T, int OP>
__global__ void k_pull_unique(int64_t n, const int32_t* __restrict__ lids, const int32_t* __restrict__ bid,
                              const int64_t* __restrict__ elem, const T* const* __restrict__ bases,
                              T* __restrict__ v) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = lids[p];
    const T b = bases[bid[p]][elem[p]];
    v[l] = (OP == PA_ADD) ? v[l] + b : b;
  }
}

template <typename T, int OP>
__global__ void k_pull_ordered(int64_t ntargets, const int32_t* __restrict__ target,
                               const int32_t* __restrict__ ptr, const int32_t* __restrict__ pos,
                               const int32_t* __restrict__ bid, const int64_t* __restrict__ elem,
                               const T* const* __restrict__ bases, T* __restrict__ v) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < ntargets;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = target[t];
    T acc = v[l];
    for (int32_t q = ptr[t]; q < ptr[t + 1]; ++q) {
      const int32_t s = pos[q];
      const T b = bases[bid[s]][elem[s]];
      acc = (OP == PA_ADD) ? acc + b : b;
    }
    v[l] = acc;
  }
}

template <typename T>
static void pull_t(int64_t n, const int32_t* lids, const pa_combine_plan& plan, int op, const int32_t* bid,
                   const int64_t* elem, const void* const* bases, void* v, hipStream_t st, hipEvent_t ev) {
  if (n <= 0) {
    if (ev) (void)hipEventRecord(ev, st);
    return;
  }
  const T* const* b = (const T* const*)bases;
  if (plan.unique) {
    if (op == PA_ADD)
      launch_ev(k_pull_unique<T, PA_ADD>, dim3(grid_for(n)), st, ev, n, lids, bid, elem, b, (T*)v);
    else
      launch_ev(k_pull_unique<T, PA_REPLACE>, dim3(grid_for(n)), st, ev, n, lids, bid, elem, b, (T*)v);
  } else {
    const int64_t nt = plan.ntargets;
    if (op == PA_ADD)
      launch_ev(k_pull_ordered<T, PA_ADD>, dim3(grid_for(nt)), st, ev, nt, (const int32_t*)plan.d_target,
                (const int32_t*)plan.d_ptr, (const int32_t*)plan.d_pos, bid, elem, b, (T*)v);
    else
      launch_ev(k_pull_ordered<T, PA_REPLACE>, dim3(grid_for(nt)), st, ev, nt, (const int32_t*)plan.d_target,
                (const int32_t*)plan.d_ptr, (const int32_t*)plan.d_pos, bid, elem, b, (T*)v);
  }
}

void launch_pull(int dtype, int64_t n, const int32_t* lids, const pa_combine_plan& plan, int op, const int32_t* bid,
                 const int64_t* elem, const void* const* bases, void* v, hipStream_t st, hipEvent_t ev) {
  switch (dtype) {
    case PA_F32: pull_t<float>(n, lids, plan, op, bid, elem, bases, v, st, ev); break;
    case PA_F64: pull_t<double>(n, lids, plan, op, bid, elem, bases, v, st, ev); break;
    case PA_C64: pull_t<c64>(n, lids, plan, op, bid, elem, bases, v, st, ev); break;
    case PA_C128: pull_t<c128>(n, lids, plan, op, bid, elem, bases, v, st, ev); break;
  }
}

void launch_pack(int dtype, int64_t n, const int32_t* lids, const void* v, void* buf,
                 hipStream_t st, hipEvent_t ev) {
  switch (dtype) {
    case PA_F32: pack_t<float>(n, lids, v, buf, st, ev); break;
    case PA_F64: pack_t<double>(n, lids, v, buf, st, ev); break;
    case PA_C64: pack_t<c64>(n, lids, v, buf, st, ev); break;
    case PA_C128: pack_t<c128>(n, lids, v, buf, st, ev); break;
  }
}

void launch_unpack(int dtype, int64_t n, const int32_t* lids, const pa_combine_plan& plan, int op,
                   const void* buf, void* v, hipStream_t st) {
  switch (dtype) {
    case PA_F32: unpack_t<float>(n, lids, plan, op, buf, v, st); break;
    case PA_F64: unpack_t<double>(n, lids, plan, op, buf, v, st); break;
    case PA_C64: unpack_t<c64>(n, lids, plan, op, buf, v, st); break;
    case PA_C128: unpack_t<c128>(n, lids, plan, op, buf, v, st); break;
  }
}

// ---------------------------------------------------------------------------
// Grouped pack / pull for the parts of one process that share a stream pair
// (pa_spmv_all's grouped path): one launch for all parts, blockIdx.y = part,
// so the per-part pointers are wave-uniform kernel arguments.

template <typename T>
__global__ void k_pack_group(const PackGroup g) {
  const int p = blockIdx.y;
  const int64_t n = g.n[p];
  const int32_t* __restrict__ lids = g.lids[p];
  const T* __restrict__ v = (const T*)g.v[p];
  T* __restrict__ buf = (T*)g.buf[p];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    buf[i] = v[lids[i]];
}

// forward halo (every ghost lid received once): v[lids[i]] = bases[bid[i]][elem[i]]
// (staging the base pointers in LDS, two dependent global loads per ghost
// instead of three, changed nothing: C5 F32 0.0766 -> 0.0773 ms, F64 0.1029
// -> 0.1038, alternating library A/B, profiles/r05/o/)
template <typename T>
__global__ void k_pull_group(const PullGroup g) {
  const int p = blockIdx.y;
  const int64_t n = g.n[p];
  const int32_t* __restrict__ lids = g.lids[p];
  const int32_t* __restrict__ bid = g.bid[p];
  const int64_t* __restrict__ elem = g.elem[p];
  const T* const* __restrict__ bases = (const T* const*)g.bases[p];
  T* __restrict__ v = (T*)g.v[p];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[lids[i]] = bases[bid[i]][elem[i]];
}

static inline dim3 group_grid(const int64_t* n, int np) {
  int64_t m = 1;
  for (int i = 0; i < np; ++i) m = n[i] > m ? n[i] : m;
  return dim3((unsigned)grid_for(m, 256, 1024), (unsigned)np);
}

void launch_pack_group(int dtype, const PackGroup& g, hipStream_t st) {
  if (g.np <= 0) return;
  const dim3 grid = group_grid(g.n, g.np);
  switch (dtype) {
    case PA_F32: hipLaunchKernelGGL(k_pack_group<float>, grid, dim3(256), 0, st, g); break;
    case PA_F64: hipLaunchKernelGGL(k_pack_group<double>, grid, dim3(256), 0, st, g); break;
    case PA_C64: hipLaunchKernelGGL(k_pack_group<c64>, grid, dim3(256), 0, st, g); break;
    case PA_C128: hipLaunchKernelGGL(k_pack_group<c128>, grid, dim3(256), 0, st, g); break;
  }
}

void launch_pull_group(int dtype, const PullGroup& g, hipStream_t st) {
  if (g.np <= 0) return;
  const dim3 grid = group_grid(g.n, g.np);
  switch (dtype) {
    case PA_F32: hipLaunchKernelGGL(k_pull_group<float>, grid, dim3(256), 0, st, g); break;
    case PA_F64: hipLaunchKernelGGL(k_pull_group<double>, grid, dim3(256), 0, st, g); break;
    case PA_C64: hipLaunchKernelGGL(k_pull_group<c64>, grid, dim3(256), 0, st, g); break;
    case PA_C128: hipLaunchKernelGGL(k_pull_group<c128>, grid, dim3(256), 0, st, g); break;
  }
}

// ---------------------------------------------------------------------------
// Elementwise vector kernels.  Index maps: null → identity over [0,n) (plus
// base offset), else lid = map[i].

template <typename T>
__global__ void k_fill_range(int64_t n, int64_t base, const int32_t* __restrict__ map, T* v, T s) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    v[map ? (int64_t)map[i] : base + i] = s;
}

template <typename T>
__global__ void k_copy_map(int64_t n, const int32_t* __restrict__ dmap, T* __restrict__ d,
                           const int32_t* __restrict__ smap, const T* __restrict__ s) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    d[dmap ? (int64_t)dmap[i] : i] = s[smap ? (int64_t)smap[i] : i];
}

// The scalar of a broadcast and the type its elements are evaluated in:
// SK 0 a scalar of the element type T (arithmetic in T); SK 1 a Float64
// (Real * element componentwise, arithmetic in Float64 / ComplexF64, one
// rounding to T on the store); SK 2 a ComplexF64 (complex T only).  Julia's
// promotion rules for `y .= x .+ a.*y` with those scalars.
template <typename T, int SK> struct BcastScalar { using A = T; using W = T; };
template <typename T> struct BcastScalar<T, 1> { using A = double; using W = typename wide_of<T>::type; };
template <typename T> struct BcastScalar<T, 2> { using A = c128; using W = c128; };

template <typename W, typename T> __device__ inline W to_w(T v) {
  if constexpr (std::is_same<W, T>::value) return v; else return widen(v);
}
template <typename T, typename W> __device__ inline T from_w(W v) {
  if constexpr (std::is_same<W, T>::value) return v; else return narrow<T>(v);
}
template <typename A, typename W> __device__ inline W scale(A a, W v) {
  if constexpr (std::is_same<A, double>::value) return rscale(a, v); else return a * v;
}

template <typename T, int MODE, int SK>
__global__ void k_axpby(int64_t n, const int32_t* __restrict__ map, T* __restrict__ y,
                        const T* __restrict__ x, typename BcastScalar<T, SK>::A a) {
  using W = typename BcastScalar<T, SK>::W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = map ? (int64_t)map[i] : i;
    const W yi = to_w<W>(y[l]);
    W r;
    if (MODE == 0) r = to_w<W>(x[l]) + scale(a, yi);        // u .= r .+ β.*u
    else if (MODE == 1) r = yi + scale(a, to_w<W>(x[l]));   // x .+= α.*u
    else if (MODE == 2) r = yi - scale(a, to_w<W>(x[l]));   // r .-= α.*c
    else if (MODE == 3) r = yi - to_w<W>(x[l]);             // r .-= c
    else r = scale(a, yi);                                  // rmul!(y, a): a * y[i]
    y[l] = from_w<T>(r);
  }
}

template <typename T>
static void fill_t(int64_t n, int64_t base, const int32_t* map, void* v, const void* s,
                   hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_fill_range<T>, dim3(grid_for(n)), dim3(256), 0, st, n, base, map, (T*)v,
                     *(const T*)s);
}
void launch_fill(int dtype, int64_t n, int64_t base, const int32_t* map, void* v, const void* s,
                 hipStream_t st) {
  switch (dtype) {
    case PA_F32: fill_t<float>(n, base, map, v, s, st); break;
    case PA_F64: fill_t<double>(n, base, map, v, s, st); break;
    case PA_C64: fill_t<c64>(n, base, map, v, s, st); break;
    case PA_C128: fill_t<c128>(n, base, map, v, s, st); break;
  }
}

template <typename T>
static void copy_t(int64_t n, const int32_t* dmap, void* d, const int32_t* smap, const void* s,
                   hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_copy_map<T>, dim3(grid_for(n)), dim3(256), 0, st, n, dmap, (T*)d, smap,
                     (const T*)s);
}
void launch_copy(int dtype, int64_t n, const int32_t* dmap, void* d, const int32_t* smap,
                 const void* s, hipStream_t st) {
  switch (dtype) {
    case PA_F32: copy_t<float>(n, dmap, d, smap, s, st); break;
    case PA_F64: copy_t<double>(n, dmap, d, smap, s, st); break;
    case PA_C64: copy_t<c64>(n, dmap, d, smap, s, st); break;
    case PA_C128: copy_t<c128>(n, dmap, d, smap, s, st); break;
  }
}

template <typename T, int SK>
static void axpby_t(int64_t n, const int32_t* map, void* y, const void* x, const void* a, int mode,
                    hipStream_t st) {
  if (n <= 0) return;
  using A = typename BcastScalar<T, SK>::A;
  const A av = *(const A*)a;
  const dim3 g(grid_for(n, 256, 8192)), b(256);
  switch (mode) {
    case 0: hipLaunchKernelGGL((k_axpby<T, 0, SK>), g, b, 0, st, n, map, (T*)y, (const T*)x, av); break;
    case 1: hipLaunchKernelGGL((k_axpby<T, 1, SK>), g, b, 0, st, n, map, (T*)y, (const T*)x, av); break;
    case 2: hipLaunchKernelGGL((k_axpby<T, 2, SK>), g, b, 0, st, n, map, (T*)y, (const T*)x, av); break;
    case 3: hipLaunchKernelGGL((k_axpby<T, 3, SK>), g, b, 0, st, n, map, (T*)y, (const T*)x, av); break;
    default: hipLaunchKernelGGL((k_axpby<T, 4, SK>), g, b, 0, st, n, map, (T*)y, (const T*)x, av); break;
  }
}
template <typename T>
static void axpby_sk(int64_t n, const int32_t* map, void* y, const void* x, const void* a, int mode, int sk,
                     hipStream_t st) {
  constexpr bool cplx = std::is_same<T, c64>::value || std::is_same<T, c128>::value;
  if (sk == 1) {
    axpby_t<T, 1>(n, map, y, x, a, mode, st);
  } else if (sk == 2) {
    if constexpr (cplx) axpby_t<T, 2>(n, map, y, x, a, mode, st);
  } else {
    axpby_t<T, 0>(n, map, y, x, a, mode, st);
  }
}
// mode 0..4 (pa_vec_axpby); scalar kind sk (BcastScalar): 0 element type,
// 1 Float64, 2 ComplexF64 (complex vectors only)
void launch_axpby(int dtype, int64_t n, const int32_t* map, void* y, const void* x, const void* a,
                  int mode, hipStream_t st, int sk) {
  switch (dtype) {
    case PA_F32: axpby_sk<float>(n, map, y, x, a, mode, sk == 2 ? 0 : sk, st); break;
    case PA_F64: axpby_sk<double>(n, map, y, x, a, mode, sk == 2 ? 0 : sk, st); break;
    case PA_C64: axpby_sk<c64>(n, map, y, x, a, mode, sk, st); break;
    case PA_C128: axpby_sk<c128>(n, map, y, x, a, mode, sk, st); break;
  }
}

// ---------------------------------------------------------------------------
// Deterministic reductions: fixed grid, per-block tree in a fixed order,
// then the last block to finish folds the block partials in order (one
// launch; block_reduce / publish_arrive / k_fold in pa_internal.h).
// Accumulator type: double (F32, F64) / c128 (C64, C128).

template <typename T> struct acc_of { using type = double; };
template <> struct acc_of<c64> { using type = c128; };
template <> struct acc_of<c128> { using type = c128; };

__device__ inline double to_acc(float a) { return (double)a; }
__device__ inline double to_acc(double a) { return a; }
__device__ inline c128 to_acc(c64 a) { return c128{(double)a.re, (double)a.im}; }
__device__ inline c128 to_acc(c128 a) { return a; }
template <typename A> __device__ inline A acc_real(double v);
template <> __device__ inline double acc_real<double>(double v) { return v; }
template <> __device__ inline c128 acc_real<c128>(double v) { return c128{v, 0.0}; }

// KIND 0: dot(a,b) (conj(a)·b); 1: Σ|a|²; 2: Σ a.  Block partials go to
// out[blockIdx]; the last block folds them (block order) into result[0].
template <typename T, int KIND>
__global__ __launch_bounds__(256) void k_reduce_partial(int64_t n, const int32_t* __restrict__ ma,
                                                        const T* __restrict__ a,
                                                        const int32_t* __restrict__ mb,
                                                        const T* __restrict__ b,
                                                        typename acc_of<T>::type* out,
                                                        typename acc_of<T>::type* __restrict__ result,
                                                        unsigned* ticket) {
  using A = typename acc_of<T>::type;
  A s = zero_of<A>();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const T ai = a[ma ? (int64_t)ma[i] : i];
    if (KIND == 0) {
      const T bi = b[mb ? (int64_t)mb[i] : i];
      s = s + to_acc(cdot(ai, bi));
    } else if (KIND == 1) {
      s = s + acc_real<A>((double)abs2(ai));
    } else {
      s = s + to_acc(ai);
    }
  }
  A r = block_reduce(s);
  if (!publish_arrive(out, r, ticket)) return;
  A f = zero_of<A>();
  for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) f = f + ld_wt(&out[i]);
  f = block_reduce(f);
  if (threadIdx.x == 0) result[0] = f;
}

constexpr int kReduceBlocks = 1024;

template <typename T, int KIND>
static void reduce_t(int64_t n, const int32_t* ma, const void* a, const int32_t* mb,
                     const void* b, void* partials, void* result, unsigned* ticket, hipStream_t st) {
  using A = typename acc_of<T>::type;
  int nb = grid_for(n, 256, kReduceBlocks);
  hipLaunchKernelGGL((k_reduce_partial<T, KIND>), dim3(nb), dim3(256), 0, st, n, ma, (const T*)a,
                     mb, (const T*)b, (A*)partials, (A*)result, ticket);
}

// fold nb partials (double, or c128 when cplx) in a fixed order into out[0];
// scratch holds kFoldBlocks accumulators
void launch_fold(int cplx, int nb, const void* in, void* scratch, void* out, unsigned* ticket, hipStream_t st) {
  if (cplx) fold_launch<c128>(nb, (const c128*)in, (c128*)scratch, (c128*)out, ticket, NoTail{}, st);
  else fold_launch<double>(nb, (const double*)in, (double*)scratch, (double*)out, ticket, NoTail{}, st);
}

// result: device accumulator (double or c128) of the part's local value
void launch_reduce(int dtype, int kind, int64_t n, const int32_t* ma, const void* a,
                   const int32_t* mb, const void* b, void* partials, void* result,
                   unsigned* ticket, hipStream_t st) {
#define PA_RED(T)                                                                           \
  if (kind == 0) reduce_t<T, 0>(n, ma, a, mb, b, partials, result, ticket, st);             \
  else if (kind == 1) reduce_t<T, 1>(n, ma, a, mb, b, partials, result, ticket, st);        \
  else reduce_t<T, 2>(n, ma, a, mb, b, partials, result, ticket, st);
  switch (dtype) {
    case PA_F32: { PA_RED(float) } break;
    case PA_F64: { PA_RED(double) } break;
    case PA_C64: { PA_RED(c64) } break;
    case PA_C128: { PA_RED(c128) } break;
  }
#undef PA_RED
}

// ---------------------------------------------------------------------------
// Synthetic Cartesian stencil operators built on the device (driver side of
// the benchmark, see pa_api.cpp: pa_mat_stencil).  kind 7: test_fdm.jl's FD
// operator; kind 27: Q1-hex FE operator of test_fem_sa.jl's pattern.

__device__ inline bool is_dirichlet(const StencilGeom& g, int64_t gx, int64_t gy, int64_t gz) {
  return gx == 0 || gy == 0 || gz == 0 || gx == g.N[0] - 1 || gy == g.N[1] - 1 || gz == g.N[2] - 1;
}

// Column lid of neighbour (lx+dx,...) (local coords may be -1 or n): own lid
// inside the box, else the ghost-shell table.  -2: outside the domain.
__device__ inline int32_t nb_lid(const StencilGeom& g, const int32_t* __restrict__ shell,
                                 int64_t lx, int64_t ly, int64_t lz) {
  const int64_t gx = g.lo[0] + lx, gy = g.lo[1] + ly, gz = g.lo[2] + lz;
  if (gx < 0 || gy < 0 || gz < 0 || gx >= g.N[0] || gy >= g.N[1] || gz >= g.N[2]) return -2;
  if (lx >= 0 && ly >= 0 && lz >= 0 && lx < g.n[0] && ly < g.n[1] && lz < g.n[2])
    return (int32_t)(lx + g.n[0] * (ly + g.n[1] * lz));
  if (!shell) return -3;
  const int64_t ex = lx + 1, ey = ly + 1, ez = lz + 1;
  return shell[ex + (g.n[0] + 2) * (ey + (g.n[1] + 2) * ez)];
}

// FE27 value of entry (node, node+d): Σ over the cells holding both nodes,
// ascending cell gid (sparse() combines duplicates in COO order, and the
// cell loop of test_fem_sa.jl visits cells in ascending gid), of Ke[a][b].
__device__ inline double fe27_value(const StencilGeom& g, const double* __restrict__ Ke,
                                    int64_t gx, int64_t gy, int64_t gz, int dx, int dy, int dz) {
  double acc = 0.0;
  bool first = true;
  // candidate cell origins per dim, ascending
  for (int cz = -1; cz <= 0; ++cz) {
    const int64_t czg = gz + cz;
    if (czg < 0 || czg > g.N[2] - 2) continue;
    const int az = (int)(gz - czg), bz = (int)(gz + dz - czg);
    if (bz < 0 || bz > 1) continue;
    for (int cy = -1; cy <= 0; ++cy) {
      const int64_t cyg = gy + cy;
      if (cyg < 0 || cyg > g.N[1] - 2) continue;
      const int ay = (int)(gy - cyg), by = (int)(gy + dy - cyg);
      if (by < 0 || by > 1) continue;
      for (int cx = -1; cx <= 0; ++cx) {
        const int64_t cxg = gx + cx;
        if (cxg < 0 || cxg > g.N[0] - 2) continue;
        const int ax = (int)(gx - cxg), bx = (int)(gx + dx - cxg);
        if (bx < 0 || bx > 1) continue;
        const double v = Ke[(ax + 2 * ay + 4 * az) * 8 + (bx + 2 * by + 4 * bz)];
        acc = first ? v : acc + v;
        first = false;
      }
    }
  }
  return acc;
}

// number of cells touching a node (Dirichlet diagonal of the FE operator)
__device__ inline double fe27_ncells(const StencilGeom& g, int64_t gx, int64_t gy, int64_t gz) {
  double acc = 0.0;
  bool first = true;
  for (int cz = -1; cz <= 0; ++cz) {
    const int64_t c2 = gz + cz;
    if (c2 < 0 || c2 > g.N[2] - 2) continue;
    for (int cy = -1; cy <= 0; ++cy) {
      const int64_t c1 = gy + cy;
      if (c1 < 0 || c1 > g.N[1] - 2) continue;
      for (int cx = -1; cx <= 0; ++cx) {
        const int64_t c0 = gx + cx;
        if (c0 < 0 || c0 > g.N[0] - 2) continue;
        acc = first ? 1.0 : acc + 1.0;
        first = false;
      }
    }
  }
  return acc;
}

template <typename T> __device__ inline T from_real(double v);
template <> __device__ inline float from_real<float>(double v) { return (float)v; }
template <> __device__ inline double from_real<double>(double v) { return v; }
template <> __device__ inline c64 from_real<c64>(double v) {
  // Float32 operator times (1+0.5im), entrywise (BASELINE config 5)
  const float f = (float)v;
  return c64{f * 1.0f, f * 0.5f};
}
template <> __device__ inline c128 from_real<c128>(double v) { return c128{v * 1.0, v * 0.5}; }

// Row entries of the stencil in the reference's per-row summation order:
// own columns ascending oid, then ghost columns ascending hid.  Returns the
// count; cols/vals must hold 27.
__device__ inline int stencil_row(const StencilGeom& g, const int32_t* __restrict__ shell,
                                  const double* __restrict__ coef, int64_t r, int32_t* cols,
                                  double* vals, int* nghost, int noids, int* err) {
  const int64_t lx = r % g.n[0];
  const int64_t ly = (r / g.n[0]) % g.n[1];
  const int64_t lz = r / (g.n[0] * g.n[1]);
  const int64_t gx = g.lo[0] + lx, gy = g.lo[1] + ly, gz = g.lo[2] + lz;
  *nghost = 0;
  if (is_dirichlet(g, gx, gy, gz)) {
    cols[0] = (int32_t)r;
    vals[0] = (g.kind == 7) ? 1.0 : fe27_ncells(g, gx, gy, gz);
    return 1;
  }
  int nown = 0;
  int32_t gc[27];
  double gv[27];
  int ng = 0;
  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int nz = (dx != 0) + (dy != 0) + (dz != 0);
        if (g.kind == 7 && nz > 1) continue;
        const int32_t c = nb_lid(g, shell, lx + dx, ly + dy, lz + dz);
        if (c < 0) { *err = 1; continue; }
        double v;
        if (g.kind == 7) v = (nz == 0) ? coef[0] : coef[1];
        else v = fe27_value(g, coef, gx, gy, gz, dx, dy, dz);
        if (c < noids) { cols[nown] = c; vals[nown] = v; ++nown; }
        else { gc[ng] = c; gv[ng] = v; ++ng; }
      }
  // ghosts by ascending hid (= ascending lid, ghosts are appended)
  for (int i = 1; i < ng; ++i) {
    const int32_t c = gc[i];
    const double v = gv[i];
    int j = i - 1;
    while (j >= 0 && gc[j] > c) { gc[j + 1] = gc[j]; gv[j + 1] = gv[j]; --j; }
    gc[j + 1] = c; gv[j + 1] = v;
  }
  for (int i = 0; i < ng; ++i) { cols[nown + i] = gc[i]; vals[nown + i] = gv[i]; }
  *nghost = ng;
  return nown + ng;
}

// pass 1: per-slice max row length and ghost flag
__global__ __launch_bounds__(256) void k_stencil_count(StencilGeom g, const int32_t* __restrict__ shell,
                                                       const double* __restrict__ coef, int64_t nrows,
                                                       int noids, int H, int32_t* __restrict__ slen,
                                                       int32_t* __restrict__ sghost,
                                                       int32_t* __restrict__ err) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int len = 0, ng = 0, e = 0;
  if (r < nrows) {
    int32_t c[27];
    double v[27];
    len = stencil_row(g, shell, coef, r, c, v, &ng, noids, &e);
  }
  if (e) atomicOr(err, 1);
  if (r < nrows) {
    atomicMax(&slen[r / H], len);
    if (ng) atomicOr(&sghost[r / H], 1);
  }
}

template <typename T, int R>
__global__ __launch_bounds__(256) void k_stencil_fill(StencilGeom g, const int32_t* __restrict__ shell,
                                                      const double* __restrict__ coef, int64_t nrows,
                                                      int noids, const int64_t* __restrict__ soff,
                                                      const int32_t* __restrict__ slen,
                                                      int32_t* __restrict__ col, T* __restrict__ val,
                                                      int32_t* __restrict__ err) {
  constexpr int H = 64 * R;
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  const int64_t s = r / H;
  const int within = (int)(r - s * H);
  const int lane = within / R, rr = within % R;
  int32_t c[27];
  double v[27];
  int ng = 0, e = 0;
  const int len = stencil_row(g, shell, coef, r, c, v, &ng, noids, &e);
  if (e) atomicOr(err, 1);
  const int L = slen[s];
  const int64_t base = soff[s];
  for (int k = 0; k < L; ++k) {
    const int64_t slot = base + ((int64_t)k * 64 + lane) * R + rr;
    if (k < len) { col[slot] = c[k]; val[slot] = from_real<T>(v[k]); }
    else { col[slot] = -1; val[slot] = zero_of<T>(); }
  }
}

// padding rows of the last slice (rows >= nrows): mark their slots empty
template <typename T, int R>
__global__ void k_sell_pad_tail(int64_t nrows, int64_t nslices, const int64_t* __restrict__ soff,
                                const int32_t* __restrict__ slen, int32_t* __restrict__ col,
                                T* __restrict__ val) {
  constexpr int H = 64 * R;
  const int64_t s = nslices - 1;
  const int64_t first_pad = nrows - s * H;  // rows within slice >= this are padding
  const int L = slen[s];
  for (int t = threadIdx.x; t < H * L; t += blockDim.x) {
    const int k = t / H, within = t % H;
    if (within < first_pad) continue;
    const int lane = within / R, rr = within % R;
    const int64_t slot = soff[s] + ((int64_t)k * 64 + lane) * R + rr;
    col[slot] = -1;
    val[slot] = zero_of<T>();
  }
}

void launch_stencil_count(const StencilGeom& g, const int32_t* shell, const double* coef,
                          int64_t nrows, int noids, int H, int32_t* slen, int32_t* sghost,
                          int32_t* err, hipStream_t st) {
  const int64_t blocks = (nrows + 255) / 256;
  if (blocks == 0) return;
  hipLaunchKernelGGL(k_stencil_count, dim3(blocks), dim3(256), 0, st, g, shell, coef, nrows, noids,
                     H, slen, sghost, err);
}

template <typename T, int R>
static void stencil_fill_t(const StencilGeom& g, const int32_t* shell, const double* coef,
                           int64_t nrows, int noids, pa_mat* A, int32_t* err, hipStream_t st) {
  const int64_t blocks = (nrows + 255) / 256;
  if (blocks == 0) return;
  hipLaunchKernelGGL((k_stencil_fill<T, R>), dim3(blocks), dim3(256), 0, st, g, shell, coef, nrows,
                     noids, A->d_slice_off, A->d_slice_len, A->d_col, (T*)A->d_val, err);
  if (A->nslices > 0 && nrows % (64 * R) != 0)
    hipLaunchKernelGGL((k_sell_pad_tail<T, R>), dim3(1), dim3(256), 0, st, nrows, A->nslices,
                       A->d_slice_off, A->d_slice_len, A->d_col, (T*)A->d_val);
}

void launch_stencil_fill(const StencilGeom& g, const int32_t* shell, const double* coef,
                         int64_t nrows, int noids, pa_mat* A, int32_t* err, hipStream_t st) {
  switch (A->dtype) {
    case PA_F32:
      if (A->R == 2) stencil_fill_t<float, 2>(g, shell, coef, nrows, noids, A, err, st);
      else stencil_fill_t<float, 4>(g, shell, coef, nrows, noids, A, err, st);
      break;
    case PA_F64: stencil_fill_t<double, 2>(g, shell, coef, nrows, noids, A, err, st); break;
    case PA_C64: stencil_fill_t<c64, 2>(g, shell, coef, nrows, noids, A, err, st); break;
    case PA_C128: stencil_fill_t<c128, 1>(g, shell, coef, nrows, noids, A, err, st); break;
  }
}

// ---------------------------------------------------------------------------
// HBM calibration (pa_hbm_probe): the attainable read and copy rates of the
// box, measured with the SpMV's own load idiom (16 B non-temporal vector
// loads, 4 or 8 in flight per lane, grid-stride).  Not on the hot path.

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void k_probe_read(int64_t n16, const u32x4* __restrict__ a,
                                                    u32x4* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) {
    const u32x4 v = __builtin_nontemporal_load(a + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[threadIdx.x] = u32x4{acc, 0u, 0u, 0u};  // keeps the loads live
}

template <int U>
__global__ __launch_bounds__(256) void k_probe_copy(int64_t n16, const u32x4* __restrict__ a,
                                                    u32x4* __restrict__ b) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], b + i + u * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}

void launch_probe(int copy, int unroll, int64_t n16, const void* a, void* b, int blocks, hipStream_t st) {
  const u32x4* ia = (const u32x4*)a;
  u32x4* ob = (u32x4*)b;
  if (copy && unroll == 8) hipLaunchKernelGGL(k_probe_copy<8>, dim3(blocks), dim3(256), 0, st, n16, ia, ob);
  else if (copy) hipLaunchKernelGGL(k_probe_copy<4>, dim3(blocks), dim3(256), 0, st, n16, ia, ob);
  else if (unroll == 8) hipLaunchKernelGGL(k_probe_read<8>, dim3(blocks), dim3(256), 0, st, n16, ia, ob);
  else hipLaunchKernelGGL(k_probe_read<4>, dim3(blocks), dim3(256), 0, st, n16, ia, ob);
}

}  // namespace pa
