// pa_spmv.hip — the hot kernel: owned-row SELL SpMV for gfx950, and the
// one-time conversion of its int32-column layout to pattern slices.
//
// Layout: a slice is H = 64*R consecutive owned rows; lane l
// owns rows l*R .. l*R+R-1; entry k of those rows sits at slot
// off[s] + (k*64 + l)*R + r.  A wave-instruction streams 64*R consecutive
// values (16 B per lane).
//
// Two column encodings share the value slots:
//  * int32 slices: column id (x lid) per slot, -1 = padding;
//  * pattern slices: the rows whose columns are `row + pat[k]`, k < plen
//    (mask bit set) carry no column ids at all; the slice's other rows are
//    computed from a small side SELL (int32 columns + row map).
// Either way each row is accumulated sequentially in the reference's order
// (SparseUtils.jl:176-185: owned columns by oid, then ghost columns by hid):
//   acc = β-init; acc = acc + v_k * (x_{c_k} * α)   (-ffp-contract=off)
#include "pa_internal.h"

#include <cstddef>

#include <algorithm>
#include <cstring>
#include <type_traits>

// Build split: the file is compiled once per element type with
// -DPA_SPMV_DT=0..3 (F32, F64, C64, C128: that type's SpMV kernels and
// launchers, the bulk of the code) and once without (the dtype dispatchers,
// the CG, pattern and layout kernels, the knobs), so that the hipcc runs go
// in parallel (__graft_entry__.build).
#if defined(PA_SPMV_DT)
#define PA_DT_DEFINE 0
#else
#define PA_DT_DEFINE 1
#endif
#define PA_CAT2(a, b) a##b
#define PA_CAT(a, b) PA_CAT2(a, b)

namespace pa {

template <typename T, int R>
struct alignas(sizeof(T) * R) Pack {
  T v[R];
};
template <int R>
struct alignas(4 * R) IPack {
  int32_t c[R];
};
template <int R>
struct alignas(2 * R) S16Pack {
  uint16_t c[R];
};

// Bits 9 (lane-shared x runs), the old bit 1 (XCD remap) and the old bit 7
// (x runs in int32 slices) were negative A/Bs of rounds 1-3
// and are gone; bits 7 (SPMV_SHORT7) and 1 (SPMV_DESC) are r06's.
enum { SPMV_NT = 1, SPMV_DESC = 2 /* pattern / triple-SELL slices: one descriptor load (make_args) */, SPMV_XPAIR = 4, SPMV_TAILB = 8, SPMV_IDLIST = 16, SPMV_YNT = 32, SPMV_SHORT = 64,
       SPMV_SHORT7 = 128 /* Float64 rows <= 7 entries: k_spmv_group_short7 */,
       SPMV_PRODA = 256 /* per matrix: CSR parent, α scales the product */,
       SPMV_TPACK = 512 /* per matrix: Float32 pair slices with per-triple value packs (pa_mat::t_pack bit 0) */ };

typedef unsigned int spmv_u32x4 __attribute__((ext_vector_type(4)));
// Process-wide knobs (pa_tune).  Defaults from the A/Bs in
// profiles/r01_ab_spmv.txt and profiles/r01/ab_xpair.txt: non-temporal
// streams on, U = 8, 16 B x runs on (FE27 256³: F64 −9 %,
// F32 −33 %, C64 −5 % kernel time), predicated tail batch on
// (profiles/r01/ab_tail.txt: FD7 256³ F64 −31 %, F32 −42 %; FE27 −1…−3 %),
// identity slice lists dropped (profiles/r01/ab_idlist.txt: FD7 −0.9 %, FE27 ±0),
// the Float64 7-entry short-row tail launch (C2 0.0281 -> 0.0278 ms, both
// orders of 7 interleaved rounds, profiles/r06/j/), the pattern slices'
// one-load descriptor (C2 -4.6 %, profiles/r06/o/).
// (the knob defaults: pa_api.cpp kDefaults; spmv_flags 223 = NT | DESC |
// XPAIR | TAILB | IDLIST | SHORT | SHORT7)
static_assert((SPMV_NT | SPMV_DESC | SPMV_XPAIR | SPMV_TAILB | SPMV_IDLIST | SPMV_SHORT | SPMV_SHORT7) == 223,
              "kDefaults.spmv_flags");
template <int R>
constexpr int kDescWords = desc_words(R);

// SpmvArgs' pointers are global memory.  The merged launch reads them from a
// device-resident table, where the compiler cannot see their address space:
// typed global in device code, its loads are global_load (scalar s_load for
// the wave-uniform ones: patterns, slice offsets) instead of flat_load.
#if defined(__HIP_DEVICE_COMPILE__)
#define PA_GLB __attribute__((address_space(1)))
#else
#define PA_GLB
#endif

template <int BYTES> struct RawOf;
template <> struct RawOf<2> { typedef unsigned short type; };
template <> struct RawOf<4> { typedef unsigned int type; };
template <> struct RawOf<8> { typedef unsigned int type __attribute__((ext_vector_type(2))); };
template <> struct RawOf<16> { typedef unsigned int type __attribute__((ext_vector_type(4))); };

template <bool NT, typename V>
__device__ __forceinline__ V ld(const V* p) {
  typedef typename RawOf<sizeof(V)>::type Raw;
  Raw r;
  if (NT) r = __builtin_nontemporal_load(reinterpret_cast<const Raw*>(p));
  else r = *reinterpret_cast<const Raw*>(p);
  V v;
  __builtin_memcpy(&v, &r, sizeof(V));
  return v;
}

template <typename T>
struct SpmvArgs {
  int64_t nwork;            // slices of this launch
  const PA_GLB int32_t* list;      // slice ids (null: 0..nwork-1)
  const PA_GLB int64_t* soff;
  const PA_GLB int32_t* slen;      // entries per row of the slice
  const PA_GLB int32_t* col;
  const PA_GLB T* val;
  const PA_GLB int32_t* pat;       // kmax offsets per slice
  const PA_GLB uint64_t* mask;     // H/64 words per slice
  int kmax;
  const PA_GLB int32_t* rowmap;    // structure row → oid (side SELL), null: identity
  int64_t nrows;            // rows of this structure
  const PA_GLB T* x;
  int64_t nx;               // x length (lids)
  PA_GLB T* y;
  const PA_GLB int32_t* ymap;      // oid → y lid, null: identity
  T alpha, beta;
  int flags;
  // fused dot(u, c) (CG): u = x indexed by oid (contiguous own layout);
  // one partial per slice at dotp[dot_base + s] (deterministic fold later)
  const PA_GLB T* dotu;
  void* dotp;
  int64_t dot_base;
  // long rows (k_spmv_long) inside int32-column slices: slices with
  // sflags[s] != 0 skip the rows whose lmask bit is set (null: none)
  const PA_GLB int32_t* sflags;
  const PA_GLB uint64_t* lmask;
  int maxlen;               // longest row (entries) of the launch's slices: <= U selects the SH kernels
  // delta16 slices: 16-bit column codes and the per-slice ghost base
  const PA_GLB uint16_t* col16;
  const PA_GLB int32_t* gbase;
  // int32-column launches over delta16 slices (spmv_format 0): the slices'
  // kinds; kind 3 = interleaved rows (null: every slice blocked)
  const PA_GLB int32_t* ilv;
  // the device CG's fused u update (XV kernels, pa_cg_solve_all): x is r,
  // the gathered values are u_new = r .+ β.*u_old (β = res²/prev² of cg);
  // waves of the main structure write u_new of their rows to un and apply
  // the deferred x .+= α.*u_old to xacc (while cg->it > cg->xit)
  const PA_GLB T* xu;
  PA_GLB T* un;
  PA_GLB T* xacc;
  const PA_GLB CGState* cg;
  int xcd_chunk;            // xcd_block (the k_spmv_sell / _group launches; merged: a kernel argument)
  // pattern slices (SPMV_DESC): per slice one descriptor of kDescWords
  // int32 {offset / H, length word, 0, 0, the slice's H/64 mask words} read
  // with one scalar load (dedup_patterns); null: soff, slen and mask
  // triple-SELL slices (SPMV_DESC): 4 int32 {offset / H, length word,
  // ghost base, 0} per slice, one scalar load (build_triple_sell)
  const PA_GLB int32_t* desc;
  // the uniform layout of short pattern rows (build_uniform; pattern
  // launches of Float64 matrices with it): values at slice * H * uK in the
  // order of the offsets upat[0 .. uK-1]
  const PA_GLB T* uval;
  int uK;
  int32_t upat[8];
};

template <typename T> struct DAcc { using type = double; };
template <> struct DAcc<c64> { using type = c128; };
template <> struct DAcc<c128> { using type = c128; };
__device__ inline double dacc(float a) { return (double)a; }
__device__ inline double dacc(double a) { return a; }
__device__ inline c128 dacc(c64 a) { return c128{(double)a.re, (double)a.im}; }
__device__ inline c128 dacc(c128 a) { return a; }
__device__ inline double shfl_down_acc(double v, int d) { return __shfl_down(v, d, 64); }
__device__ inline c128 shfl_down_acc(c128 v, int d) {
  return c128{__shfl_down(v.re, d, 64), __shfl_down(v.im, d, 64)};
}

// Branch-free select.  Complex values are selected per component: a select
// of the whole struct made clang route c128 through scratch (a stack slot
// indexed by the condition) on every entry.
__device__ __forceinline__ float pick(bool c, float a, float b) { return c ? a : b; }
__device__ __forceinline__ double pick(bool c, double a, double b) { return c ? a : b; }
__device__ __forceinline__ c64 pick(bool c, c64 a, c64 b) { return c64{c ? a.re : b.re, c ? a.im : b.im}; }
__device__ __forceinline__ c128 pick(bool c, c128 a, c128 b) { return c128{c ? a.re : b.re, c ? a.im : b.im}; }

// the R consecutive x values x[i .. i+R-1] as one 16 B load (i only
// dword-aligned: global loads need 4 B alignment); pa_vec pads 64 B on both
// sides, so i in [-(R-1), n-1] stays inside the allocation
typedef unsigned int u4a __attribute__((ext_vector_type(4))) __attribute__((aligned(4)));
typedef unsigned int u2r __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));
template <typename T, int R>
__device__ __forceinline__ Pack<T, R> ld_xrun(const T* p) {
  Pack<T, R> v;
  if constexpr (sizeof(Pack<T, R>) == 8) {  // Float32 with 2 rows per lane (pa_tune "f32_rows")
    const u2r r = *reinterpret_cast<const u2r*>(p);
    __builtin_memcpy(&v, &r, 8);
  } else {
    static_assert(sizeof(Pack<T, R>) == 16, "16 B runs");
    const u4a r = *reinterpret_cast<const u4a*>(p);
    __builtin_memcpy(&v, &r, 16);
  }
  return v;
}

// What an SpMV gathers as x.  XV false: a vector.  XV true (the device
// CG's fused u update, pa_cg_solve_all): u_new = r .+ β.*u_old evaluated per
// gathered element, in the wide type and rounded to T once (k_cg_xu's
// arithmetic, IterativeSolvers' `u .= r .+ β.*u`), so iteration k's SpMV
// reads r and u_{k-1} instead of a materialised u_k: the same values bit for
// bit, one vector sweep less per iteration.
// x[j], x[j+1], x[j+2] with the fewest loads (4 B aligned: global loads of
// several dwords need only dword alignment): one 12 B load for 4 B
// elements, a 16 B and an 8 B load for 8 B elements, three 16 B loads for
// 16 B elements.  j + 2 stays inside the vector's 64 B back padding.
typedef unsigned int u3a __attribute__((ext_vector_type(3))) __attribute__((aligned(4)));
typedef unsigned int u2a __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));
template <typename T>
__device__ __forceinline__ void ld_xtrip(const T* p, T (&o)[3]) {
  if constexpr (sizeof(T) == 4) {
    const u3a r = *reinterpret_cast<const u3a*>(p);
    __builtin_memcpy(&o[0], &r, 12);
  } else if constexpr (sizeof(T) == 8) {
    const u4a r = *reinterpret_cast<const u4a*>(p);
    const u2a q = *reinterpret_cast<const u2a*>(p + 2);
    __builtin_memcpy(&o[0], &r, 16);
    __builtin_memcpy(&o[2], &q, 8);
  } else {
#pragma unroll
    for (int j = 0; j < 3; ++j) o[j] = p[j];
  }
}

// x[j .. j+3] (a pair slice's triple: row a reads j..j+2, row a+1 j+1..j+3)
// as one 16 B load for 4 B elements, two for 8 B elements
template <typename T>
__device__ __forceinline__ void ld_xquad(const T* p, T (&o)[4]) {
  if constexpr (sizeof(T) == 4) {
    const u4a r = *reinterpret_cast<const u4a*>(p);
    __builtin_memcpy(&o[0], &r, 16);
  } else if constexpr (sizeof(T) == 8) {
    const u4a r0 = *reinterpret_cast<const u4a*>(p);
    const u4a r1 = *reinterpret_cast<const u4a*>(p + 2);
    __builtin_memcpy(&o[0], &r0, 16);
    __builtin_memcpy(&o[2], &r1, 16);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = p[j];
  }
}

template <typename T, bool XV>
struct XSrc {
  const T* __restrict__ x;
  __device__ __forceinline__ T get(int64_t j) const { return x[j]; }
  __device__ __forceinline__ void quad(int64_t j, T (&o)[4]) const { ld_xquad<T>(x + j, o); }
  template <int R>
  __device__ __forceinline__ Pack<T, R> run(int64_t j) const { return ld_xrun<T, R>(x + j); }
  __device__ __forceinline__ void trip(int64_t j, T (&o)[3]) const { ld_xtrip<T>(x + j, o); }
};
template <typename T>
struct XSrc<T, true> {
  const T* __restrict__ r;
  const T* __restrict__ u;
  double b;
  __device__ __forceinline__ T f(T rv, T uv) const { return narrow<T>(widen(rv) + rscale(b, widen(uv))); }
  __device__ __forceinline__ T get(int64_t j) const { return f(r[j], u[j]); }
  __device__ __forceinline__ void trip(int64_t j, T (&o)[3]) const {
#pragma unroll
    for (int k = 0; k < 3; ++k) o[k] = get(j + k);
  }
  __device__ __forceinline__ void quad(int64_t j, T (&o)[4]) const {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = get(j + k);
  }
  template <int R>
  __device__ __forceinline__ Pack<T, R> run(int64_t j) const {
    const Pack<T, R> a = ld_xrun<T, R>(r + j), c = ld_xrun<T, R>(u + j);
    Pack<T, R> o;
#pragma unroll
    for (int k = 0; k < R; ++k) o.v[k] = f(a.v[k], c.v[k]);
    return o;
  }
};

// the x values of a lane's R rows at one entry: R gathers (c < 0: padding,
// read x[0], never used)
template <typename T, int R, typename XS>
__device__ __forceinline__ void gather_x(T (&xv)[R], const int32_t (&c)[R], const XS& x) {
#pragma unroll
  for (int r = 0; r < R; ++r) xv[r] = x.get(c[r] >= 0 ? c[r] : 0);
}

// One term of a row's sum.  A CSC parent scales x first, v*(x*α)
// (SparseUtils.jl:177, 182); a CSR parent scales the product, (v*x)*α
// (SparseUtils.jl:247: nzv[p]*B[j]*α).  ALPHA false (α == 1): v*x either way.
template <bool ALPHA, typename T>
__device__ __forceinline__ T term(T v, T x, T alpha, bool pf) {
  if (!ALPHA) return v * x;
  if (pf) return (v * x) * alpha;
  return v * (x * alpha);
}

// Column ids one batch ahead (IPF in rows_int32 / rows_d16) for Float64:
// same-copy A/B (profiles/r04/i/): C5 F64 0.1240 -> 0.1217 ms (-1.9 %), FE27
// 256^3 F64 +-0; Float32 (R = 4, 134 -> 155 VGPRs) C5 0.0832 -> 0.0852 ms
// (+2.4 %): off.
// Float32 with 2 rows per lane (f32_rows): C5 F32 median 0.0663 -> 0.0656 ms,
// within the noise (profiles/r05/af/ab_f32_ids_ahead_c5.log); 4 rows per lane
// keep them off (the register cost above)
template <typename T, int R>
constexpr bool kIdsAhead = std::is_same<T, double>::value || (std::is_same<T, float>::value && R == 2);

// int32-column rows: c < 0 is padding (skipped: never multiplied)
// TB: the entries past the last full U batch run as one masked batch
// (entries >= len re-read entry len-1 and are never accumulated)
template <typename T, int R, bool ALPHA, bool NT, int U, bool SH = false, bool IPF = false, typename XS>
__device__ __forceinline__ void rows_int32(T (&acc)[R], const IPack<R>* __restrict__ cp,
                                           const Pack<T, R>* __restrict__ vp, int len,
                                           const XS& x, T alpha, bool pf, bool TB) {
  int k = 0;
  if (SH) TB = true;  // short rows (len <= U): the one masked batch is the whole row
  if constexpr (IPF && !SH) {
    // column ids one batch ahead: batch k+1's ids load while batch k's
    // gathers are in flight, so a batch waits for one load latency (the
    // gather), not two (ids, then gather)
    if (U <= len) {
      IPack<R> cn[U];
#pragma unroll
      for (int u = 0; u < U; ++u) cn[u] = ld<NT>(&cp[u * 64]);
      for (; k + U <= len; k += U) {
        IPack<R> c[U];
        Pack<T, R> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = cn[u];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(&vp[(k + u) * 64]);
        T xv[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u) gather_x<T, R>(xv[u], c[u].c, x);
        const int kn = k + U;
        if (kn + U <= len) {
#pragma unroll
          for (int u = 0; u < U; ++u) cn[u] = ld<NT>(&cp[(kn + u) * 64]);
        } else if (TB && kn < len) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (kn + u < len) cn[u] = ld<NT>(&cp[(kn + u) * 64]);
            else for (int r = 0; r < R; ++r) cn[u].c[r] = -1;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const T t = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
            acc[r] = pick(c[u].c[r] >= 0, t, acc[r]);
          }
      }
      if (TB && k < len) {  // the masked tail batch, its ids already loaded
        Pack<T, R> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (k + u < len) v[u] = ld<NT>(&vp[(k + u) * 64]);
        T xv[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (k + u < len) gather_x<T, R>(xv[u], cn[u].c, x);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const T t = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
            acc[r] = pick(k + u < len && cn[u].c[r] >= 0, t, acc[r]);
          }
        k = len;
      }
    }
  }
  for (; !SH && k + U <= len; k += U) {
    IPack<R> c[U];
    Pack<T, R> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = ld<NT>(&cp[(k + u) * 64]);
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(&vp[(k + u) * 64]);
    T xv[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u) gather_x<T, R>(xv[u], c[u].c, x);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const T t = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
        acc[r] = pick(c[u].c[r] >= 0, t, acc[r]);
      }
  }
  if (TB && k < len) {  // the last len % U entries as one masked batch (loads issued together)
    IPack<R> c[U];
    Pack<T, R> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (k + u < len) c[u] = ld<NT>(&cp[(k + u) * 64]);
      else for (int r = 0; r < R; ++r) c[u].c[r] = -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k + u < len) v[u] = ld<NT>(&vp[(k + u) * 64]);
    T xv[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k + u < len) gather_x<T, R>(xv[u], c[u].c, x);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const T t = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
        acc[r] = pick(k + u < len && c[u].c[r] >= 0, t, acc[r]);
      }
    k = len;
  }
  for (; !SH && k < len; ++k) {
    const IPack<R> c = ld<NT>(&cp[k * 64]);
    const Pack<T, R> v = ld<NT>(&vp[k * 64]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int32_t cc = c.c[r];
      const T t = acc[r] + term<ALPHA>(v.v[r], x.get(cc >= 0 ? cc : 0), alpha, pf);
      acc[r] = pick(cc >= 0, t, acc[r]);
    }
  }
}

// delta16 code → x lid (-1: padding): bit 15 clear = owned column, row +
// the signed 15-bit delta; set = ghost column, the slice's ghost base + the
// 15-bit offset; 0xFFFF = padding
__device__ __forceinline__ int32_t d16_col(uint32_t q, int32_t row, int32_t gb) {
  if (q == 0xFFFFu) return -1;
  return (q & 0x8000u) ? gb + (int32_t)(q & 0x7FFFu) : row + (((int32_t)(q << 17)) >> 17);
}

// delta16 rows: rows_int32 with the column ids decoded from 2 B codes.
// Float32 (R = 4) delta16 slices have interleaved rows (k_delta16): row0 =
// the slice's first row + lane, the lane's rows row0 + r*64.  Same-box A/B
// (profiles/r04/l/): C5 F32 0.0855 -> 0.0757 ms (-11.5 %), F64 (R = 2)
// 0.1191 -> 0.1232 (+3.4 %), so the other types keep blocked rows.
template <int R> constexpr bool kInterleaveD16 = R == 4;
template <int R> constexpr int kD16RowStride = kInterleaveD16<R> ? 64 : 1;
template <typename T, int R, bool ALPHA, bool NT, int U, bool SH = false, bool IPF = false, typename XS>
__device__ __forceinline__ void rows_d16(T (&acc)[R], const S16Pack<R>* __restrict__ cp,
                                         const Pack<T, R>* __restrict__ vp, int len,
                                         const XS& x, T alpha, bool pf, bool TB, const int32_t (&rw)[R], int32_t gb) {
  int k = 0;
  if (SH) TB = true;
  if constexpr (IPF && !SH) {  // codes one batch ahead, as in rows_int32
    if (U <= len) {
      S16Pack<R> qn[U];
#pragma unroll
      for (int u = 0; u < U; ++u) qn[u] = ld<NT>(&cp[u * 64]);
      for (; k + U <= len; k += U) {
        int32_t c[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < R; ++r) c[u][r] = d16_col(qn[u].c[r], rw[r], gb);
        Pack<T, R> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(&vp[(k + u) * 64]);
        T xv[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u) gather_x<T, R>(xv[u], c[u], x);
        const int kn = k + U;
        if (kn + U <= len) {
#pragma unroll
          for (int u = 0; u < U; ++u) qn[u] = ld<NT>(&cp[(kn + u) * 64]);
        } else if (TB && kn < len) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (kn + u < len) qn[u] = ld<NT>(&cp[(kn + u) * 64]);
            else for (int r = 0; r < R; ++r) qn[u].c[r] = 0xFFFFu;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const T t = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
            acc[r] = pick(c[u][r] >= 0, t, acc[r]);
          }
      }
      if (TB && k < len) {  // the masked tail batch, its codes already loaded
        int32_t c[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < R; ++r) c[u][r] = d16_col(qn[u].c[r], rw[r], gb);
        Pack<T, R> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (k + u < len) v[u] = ld<NT>(&vp[(k + u) * 64]);
        T xv[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (k + u < len) gather_x<T, R>(xv[u], c[u], x);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const T t = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
            acc[r] = pick(k + u < len && c[u][r] >= 0, t, acc[r]);
          }
        k = len;
      }
    }
  }
  for (; !SH && k + U <= len; k += U) {
    S16Pack<R> q[U];
    Pack<T, R> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) q[u] = ld<NT>(&cp[(k + u) * 64]);
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(&vp[(k + u) * 64]);
    int32_t c[U][R];
    T xv[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < R; ++r) c[u][r] = d16_col(q[u].c[r], rw[r], gb);
      gather_x<T, R>(xv[u], c[u], x);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const T t = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
        acc[r] = pick(c[u][r] >= 0, t, acc[r]);
      }
  }
  if (TB && k < len) {  // the last len % U entries as one masked batch
    S16Pack<R> q[U];
    Pack<T, R> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (k + u < len) q[u] = ld<NT>(&cp[(k + u) * 64]);
      else for (int r = 0; r < R; ++r) q[u].c[r] = 0xFFFFu;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k + u < len) v[u] = ld<NT>(&vp[(k + u) * 64]);
    int32_t c[U][R];
    T xv[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < R; ++r) c[u][r] = d16_col(q[u].c[r], rw[r], gb);
      if (k + u < len) gather_x<T, R>(xv[u], c[u], x);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const T t = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
        acc[r] = pick(k + u < len && c[u][r] >= 0, t, acc[r]);
      }
    k = len;
  }
  for (; !SH && k < len; ++k) {
    const S16Pack<R> q = ld<NT>(&cp[k * 64]);
    const Pack<T, R> v = ld<NT>(&vp[k * 64]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int32_t cc = d16_col(q.c[r], rw[r], gb);
      const T t = acc[r] + term<ALPHA>(v.v[r], x.get(cc >= 0 ? cc : 0), alpha, pf);
      acc[r] = pick(cc >= 0, t, acc[r]);
    }
  }
}

// triples per batch: 12 entries in flight per lane (library A/B, profiles/r04/ag/: FE27
// 256^3 2 triples 0.6590 ms, 3 0.6549-0.6554, 4 0.6500 at the same VGPR count;
// 6: 0.6627, the merged kernel 122 -> 132 VGPRs, halo leg +12 %, r04/ai/)
constexpr int kTriBatch = 4;

// Triple-SELL tri slices: every row's columns are consecutive triples (c,
// c+1, c+2), entry 3t..3t+2; the code of triple t (relative to the row, as
// in rows_d16) sits in code group t, and the lane reads the triple's x with
// ld_xtrip.  Padding triples (code 0xFFFF) are never accumulated.  Four
// triples (12 values) in flight per lane, as in rows_pattern_tri.  The
// terms and their order are those of rows_d16.
template <typename T, int R, bool ALPHA, bool NT, typename XS>
__device__ __forceinline__ void rows_t16_tri(T (&acc)[R], const S16Pack<R>* __restrict__ cp,
                                             const Pack<T, R>* __restrict__ vp, int len, const XS& x, T alpha,
                                             bool pf, const int32_t (&rw)[R], int32_t gb) {
  const int ntri = len / 3;
  // Batches of 4 triples for every element type.  Float32 (2 rows per lane)
  // ran batches of 9 (r05-r06: 8, then 9 triples, per-triple value packs and
  // batch code packs, profiles/r05/af/, r06/n/, r06/s/), which held the
  // merged Float32 kernel at 158 VGPRs (3 waves per SIMD); since the pair
  // slices (rows_t16_pair) took most triple rows, the batches of 4 (118
  // VGPRs, 4 waves per SIMD) run C5 F32 0.0640 -> 0.0631 ms (four
  // alternating library rounds, profiles/r06/aa/).  8 B elements: 6 triples
  // cost C5 F64 0.1056 -> 0.1094 ms, ComplexF32 0.1083 -> 0.1149
  // (r05/af/ab_f64_c64_tri_batch6_c5.log)
  constexpr int TB = kTriBatch;
  auto step = [&](const S16Pack<R>* q, const Pack<T, R>* v, auto nb) {
    constexpr int B = decltype(nb)::value;
    T xv[B][3][R];
    bool ok[B][R];
#pragma unroll
    for (int u = 0; u < B; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int32_t c = d16_col(q[u].c[r], rw[r], gb);
        ok[u][r] = c >= 0;
        T t3[3];
        x.trip(c >= 0 ? c : 0, t3);
#pragma unroll
        for (int j = 0; j < 3; ++j) xv[u][j][r] = t3[j];
      }
#pragma unroll
    for (int u = 0; u < B; ++u)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const T t = acc[r] + term<ALPHA>(v[3 * u + j].v[r], xv[u][j][r], alpha, pf);
          acc[r] = pick(ok[u][r], t, acc[r]);
        }
  };
  int t = 0;
  for (; t + TB <= ntri; t += TB) {
    S16Pack<R> q[TB];
    Pack<T, R> v[3 * TB];
#pragma unroll
    for (int u = 0; u < TB; ++u) q[u] = ld<NT>(&cp[(t + u) * 64]);
#pragma unroll
    for (int u = 0; u < 3 * TB; ++u) v[u] = ld<NT>(&vp[(3 * t + u) * 64]);
    step(q, v, std::integral_constant<int, TB>{});
  }
  for (; t < ntri; ++t) {
    S16Pack<R> q[1];
    Pack<T, R> v[3];
    q[0] = ld<NT>(&cp[t * 64]);
#pragma unroll
    for (int u = 0; u < 3; ++u) v[u] = ld<NT>(&vp[(3 * t + u) * 64]);
    step(q, v, std::integral_constant<int, 1>{});
  }
}

// Pair slices of the triple SELL (spmv_tri_pack bit 2, build_triple_sell):
// lane l holds the rows a and a + 1 of one pair, whose columns are those of
// row a plus one, entry for entry (the x-neighbours of an FE27 part: pattern
// rows without a pattern).  One code per triple and lane (row a's, Rc = 1,
// t_code_slot) and one x run x[c .. c+3] serve both rows: row a reads
// x[c .. c+2], row a+1 x[c+1 .. c+3].  Values as in tri slices (Float32
// with TP: per-triple packs).  Batches of 9 triples (4 B elements) or 4 (8 B
// elements); full batches read their codes as 8 B packs of 4.  The terms and
// their order per row are those of rows_t16_tri.
// pair_batch: NB triples of a pair slice from triple t (FULL: all exist, the codes of
// a batch of B = NB in their packs; otherwise clamped to the last triple and
// never accumulated past it)
template <typename T, bool ALPHA, typename XS, bool TP, int NB, bool FULL>
__device__ __forceinline__ void pair_batch(T (&acc)[2], const uint16_t* __restrict__ cs,
                                           const Pack<T, 2>* __restrict__ vp, int t, int ntri, const XS& x, T alpha,
                                           bool pf, int32_t rowa, int32_t gb, bool packs) {
  constexpr int R = 2, NQ = NB / 4;
  const int lane = threadIdx.x % 64;
  uint16_t q[NB];
  if (FULL && packs) {
    const uint16_t* __restrict__ cb = cs + (int64_t)t * 64;
#pragma unroll
    for (int h = 0; h < NQ; ++h) {
      const S16Pack<4> q4 = ld<true>(reinterpret_cast<const S16Pack<4>*>(cb + h * 4 * 64) + lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) q[4 * h + i] = q4.c[i];
    }
#pragma unroll
    for (int u = 4 * NQ; u < NB; ++u) q[u] = ld<true>(reinterpret_cast<const S16Pack<1>*>(cb + u * 64) + lane).c[0];
  } else {
#pragma unroll
    for (int u = 0; u < NB; ++u)
      q[u] = ld<true>(reinterpret_cast<const S16Pack<1>*>(cs + (int64_t)(FULL ? t + u : min(t + u, ntri - 1)) * 64) +
                      lane).c[0];
  }
  Pack<T, R> v[3 * NB];
  const Pack<T, R>* __restrict__ vb = vp - lane;  // the slice's values
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int tu = FULL ? t + u : min(t + u, ntri - 1);
    if constexpr (TP) {
      const Pack<T, R>* tb = vb + (int64_t)tu * 3 * 64;
      const Pack<T, 2 * R> p01 = ld<true>(reinterpret_cast<const Pack<T, 2 * R>*>(tb) + lane);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        v[3 * u].v[r] = p01.v[r];
        v[3 * u + 1].v[r] = p01.v[R + r];
      }
      v[3 * u + 2] = ld<true>(tb + 2 * 64 + lane);
    } else {
#pragma unroll
      for (int j = 0; j < 3; ++j) v[3 * u + j] = ld<true>(&vp[(3 * tu + j) * 64]);
    }
  }
  T xq[NB][4];
  bool ok[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int32_t c = d16_col(q[u], rowa, gb);
    ok[u] = c >= 0 && (FULL || t + u < ntri);
    x.quad(c >= 0 ? c : 0, xq[u]);
  }
#pragma unroll
  for (int u = 0; u < NB; ++u)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const T t0 = acc[0] + term<ALPHA>(v[3 * u + j].v[0], xq[u][j], alpha, pf);
      const T t1 = acc[1] + term<ALPHA>(v[3 * u + j].v[1], xq[u][j + 1], alpha, pf);
      acc[0] = pick(ok[u], t0, acc[0]);
      acc[1] = pick(ok[u], t1, acc[1]);
    }
}

template <typename T, bool ALPHA, typename XS, bool TP>
__device__ __forceinline__ void rows_t16_pair(T (&acc)[2], const uint16_t* __restrict__ cs,
                                              const Pack<T, 2>* __restrict__ vp, int len, const XS& x, T alpha,
                                              bool pf, int32_t rowa, int32_t gb) {
  constexpr int B = sizeof(T) == 4 ? 9 : kTriBatch;
  const int ntri = len / 3;
  int t = 0;
  for (; t + B <= ntri; t += B) pair_batch<T, ALPHA, XS, TP, B, true>(acc, cs, vp, t, ntri, x, alpha, pf, rowa, gb, true);
  if constexpr (sizeof(T) == 4) {  // the rest as one clamped batch (Float32's 9-triple batches, rows_t16_tri)
    if (t < ntri) pair_batch<T, ALPHA, XS, TP, B, false>(acc, cs, vp, t, ntri, x, alpha, pf, rowa, gb, false);
  } else {  // then single triples (8 B elements, as rows_t16_tri)
    for (; t < ntri; ++t) pair_batch<T, ALPHA, XS, TP, 1, true>(acc, cs, vp, t, ntri, x, alpha, pf, rowa, gb, false);
  }
}

// pattern rows: column of row `rbase + r` at entry k is rbase + r + pat[k].
// XP: the lane's R rows read R consecutive x values per entry, fetched as
// one 16 B run (rows that are not regular get values they never use).
template <typename T, int R, bool ALPHA, bool NT, int U, bool XP, bool SH = false, typename XS>
__device__ __forceinline__ void rows_pattern(T (&acc)[R], const int32_t* __restrict__ pat,
                                             const Pack<T, R>* __restrict__ vp, int len,
                                             const XS& x, int64_t rbase,
                                             const bool (&ok)[R], T alpha, bool pf, bool TB) {
  if (SH) TB = true;  // short rows (len <= U): the one masked batch is the whole row
  int64_t xb[R];
  bool any = false;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    xb[r] = ok[r] ? rbase + r : -1;
    any = any || ok[r];
  }
  int k = 0;
  for (; !SH && k + U <= len; k += U) {
    int32_t o[U];
    Pack<T, R> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) o[u] = pat[k + u];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(&vp[(k + u) * 64]);
    T xv[U][R];
    if constexpr (XP && R > 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const Pack<T, R> xr = x.template run<R>(any ? rbase + o[u] : 0);
#pragma unroll
        for (int r = 0; r < R; ++r) xv[u][r] = xr.v[r];
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r) xv[u][r] = x.get(xb[r] >= 0 ? xb[r] + o[u] : 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        acc[r] = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
      }
  }
  if (TB && k < len) {  // masked tail batch, as in rows_int32
    int32_t o[U];
    Pack<T, R> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) o[u] = pat[min(k + u, len - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k + u < len) v[u] = ld<NT>(&vp[(k + u) * 64]);
    T xv[U][R];
    if constexpr (XP && R > 1) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k + u < len) {
          const Pack<T, R> xr = x.template run<R>(any ? rbase + o[u] : 0);
#pragma unroll
          for (int r = 0; r < R; ++r) xv[u][r] = xr.v[r];
        }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k + u < len)
#pragma unroll
          for (int r = 0; r < R; ++r) xv[u][r] = x.get(xb[r] >= 0 ? xb[r] + o[u] : 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k + u < len) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          acc[r] = acc[r] + term<ALPHA>(v[u].v[r], xv[u][r], alpha, pf);
        }
      }
    k = len;
  }
  for (; !SH && k < len; ++k) {
    const int32_t o = pat[k];
    const Pack<T, R> v = ld<NT>(&vp[k * 64]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      acc[r] = acc[r] + term<ALPHA>(v.v[r], x.get(xb[r] >= 0 ? xb[r] + o : 0), alpha, pf);
    }
  }
}

// Pattern rows whose pattern is consecutive column triples (o, o+1, o+2),
// tri bit of the slice's length word: the lane's R rows read the three x
// runs x[rbase+o .. +R-1], x[rbase+o+1 .. +R], x[rbase+o+2 .. +R+1] as two
// 16 B loads, A = x[rbase+o ..] and B = x[rbase+o+2 ..]: run 0 = A, run 2 =
// B, run 1 = A[1..R-1] followed by B[R-2].  Three triples (9 entries) per
// batch, then single triples; the terms and their order are those of
// rows_pattern.  Library A/B on one box (profiles/r04/p/): FE27 256^3 one
// part 0.6744 -> 0.6523 ms, the (2,2,2) halo leg 0.714 -> 0.688 ms, C5 F64
// -1.0 %: one x load in three fewer relieves the per-CU memory pipeline.
template <typename T, int R, bool ALPHA, bool NT, typename XS>
__device__ __forceinline__ void rows_pattern_tri(T (&acc)[R], const int32_t* __restrict__ pat,
                                                 const Pack<T, R>* __restrict__ vp, int len, const XS& x,
                                                 int64_t rbase, const bool (&ok)[R], T alpha, bool pf) {
  static_assert(R > 1, "runs of R > 1 values");
  bool any = false;
#pragma unroll
  for (int r = 0; r < R; ++r) any = any || ok[r];
  auto triple = [&](int32_t o, T (&xv)[3][R]) {
    Pack<T, R> A, B;
    if constexpr (R == 2 && sizeof(T) == 4) {  // Float32, 2 rows per lane: x[o .. o+3] as one 16 B load
      T q[4];
      x.quad(any ? rbase + o : 0, q);
      A.v[0] = q[0];
      A.v[1] = q[1];
      B.v[0] = q[2];
      B.v[1] = q[3];
    } else {
      A = x.template run<R>(any ? rbase + o : 0);
      B = x.template run<R>(any ? rbase + o + 2 : 0);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      xv[0][r] = A.v[r];
      xv[1][r] = r + 1 < R ? A.v[r + 1] : B.v[R - 2];
      xv[2][r] = B.v[r];
    }
  };
  int k = 0;
  constexpr int TB = kTriBatch;  // triples per batch
  for (; k + 3 * TB <= len; k += 3 * TB) {
    int32_t o[TB];
#pragma unroll
    for (int t = 0; t < TB; ++t) o[t] = pat[k + 3 * t];
    Pack<T, R> v[3 * TB];
#pragma unroll
    for (int u = 0; u < 3 * TB; ++u) v[u] = ld<NT>(&vp[(k + u) * 64]);
    T xv[TB][3][R];
#pragma unroll
    for (int t = 0; t < TB; ++t) triple(o[t], xv[t]);
#pragma unroll
    for (int t = 0; t < TB; ++t)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = acc[r] + term<ALPHA>(v[3 * t + j].v[r], xv[t][j][r], alpha, pf);
  }
  for (; k < len; k += 3) {
    const int32_t o = pat[k];
    Pack<T, R> v[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] = ld<NT>(&vp[(k + j) * 64]);
    T xv[3][R];
    triple(o, xv);
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = acc[r] + term<ALPHA>(v[j].v[r], xv[j][r], alpha, pf);
  }
}

// α of the device CG state in the wide type W (Float64 / ComplexF64)
template <typename W> __device__ inline W cg_alpha_of(const CGState* st);
template <> __device__ inline double cg_alpha_of<double>(const CGState* st) { return st->alpha.re; }
template <> __device__ inline c128 cg_alpha_of<c128>(const CGState* st) { return st->alpha; }

// The fused CG update of one lane's R rows i0 + k*rs (< nrows; owned lids
// = oids, contiguous; rs = 1 blocked rows, 64 interleaved): x[i] .+= α.*u_old[i] when an x update is pending
// (xpend), and with U: u_new[i] = r[i] .+ β.*u_old[i] stored to un and
// returned in unv.  16 B accesses when all R rows exist.  The arithmetic of
// k_cg_xu, element for element.
template <typename T, int R, bool UPD, typename XS, typename W>
__device__ __forceinline__ void cg_rows_update(const SpmvArgs<T>& a, const XS& xs, int64_t i0, int rs, W alpha,
                                               bool xpend = true, T* unv = nullptr) {
  T* xacc = (T*)a.xacc;
  T* un = (T*)a.un;
  if (rs == 1 && i0 + R <= a.nrows) {
    const Pack<T, R> uo = *reinterpret_cast<const Pack<T, R>*>(xs.u + i0);
    if (UPD) {
      const Pack<T, R> rv = *reinterpret_cast<const Pack<T, R>*>(xs.r + i0);
      Pack<T, R> o;
#pragma unroll
      for (int k = 0; k < R; ++k) o.v[k] = xs.f(rv.v[k], uo.v[k]);
      *reinterpret_cast<Pack<T, R>*>(un + i0) = o;
#pragma unroll
      for (int k = 0; k < R; ++k) unv[k] = o.v[k];
    }
    if (xpend) {  // x is next read one iteration later: non-temporal, as in k_cg_xu
      Pack<T, R> xv = ld<true>(reinterpret_cast<const Pack<T, R>*>(xacc + i0));
#pragma unroll
      for (int k = 0; k < R; ++k) xv.v[k] = narrow<T>(widen(xv.v[k]) + alpha * widen(uo.v[k]));
      if constexpr (sizeof(Pack<T, R>) == 16) {
        spmv_u32x4 w;
        __builtin_memcpy(&w, &xv, 16);
        __builtin_nontemporal_store(w, reinterpret_cast<spmv_u32x4*>(xacc + i0));
      } else {
        *reinterpret_cast<Pack<T, R>*>(xacc + i0) = xv;
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int64_t i = i0 + (int64_t)k * rs;
    if (i >= a.nrows) {
      if (UPD) unv[k] = zero_of<T>();
      continue;
    }
    const T uo = xs.u[i];
    if (UPD) {
      unv[k] = xs.f(xs.r[i], uo);
      un[i] = unv[k];
    }
    if (xpend) xacc[i] = narrow<T>(widen(xacc[i]) + alpha * widen(uo));
  }
}

// BMODE: 0 → acc = 0 (β == 0: fill!(co,0)), 1 → acc = y (β == 1),
//        2 → acc = y*β (rmul!(co,β)).  Interfaces.jl:2262-2263.
// PK: the launch's slices are int32-column slices (0), pattern slices (1:
// implied columns for the rows of their mask), delta16 slices (3: 2 B
// column codes decoded against the row) or the triple SELL (4: rows through
// a row map, one code per triple in its tri slices); one kernel per kind
// keeps the hot loop free of the others' code and registers.
// One wave computes work item w (slice a.list[w], or w) of the structure a.
// SH: every row of the launch has at most U entries (FD7: 7) — the masked
// batch alone, no loop code (fewer registers, more waves per SIMD).
// XV: the device CG's fused u update (SpmvArgs::xu/un/xacc/cg; BMODE 0,
// ALPHA false): x.get(j) = r[j] + β*u_old[j] on the fly, and the waves of the
// main structure (no rowmap) write u_new and the deferred x update of all
// their rows (whoever computes the row's product); once the solve is done a
// wave only applies a pending x update.
template <typename T, int R, bool ALPHA, int BMODE, int U, int PK, bool SH = false, bool XV = false>
__device__ __forceinline__ void spmv_wave(const SpmvArgs<T>& a, const int64_t w) {
  constexpr bool PAT = PK == 1;  // implied columns (mask of regular rows)
  constexpr int H = 64 * R;
  const int lane = threadIdx.x & 63;
  const int64_t s = a.list ? (int64_t)a.list[w] : w;
  // the slice's row layout: blocked (the lane's rows lane*R + r) or, for
  // delta16 slices, interleaved (rows r*64 + lane; k_delta16)
  bool il = false;
  if constexpr (PK == 3) il = kInterleaveD16<R>;
  if constexpr (PK == 4) il = true;
  if constexpr (PK == 0 && kInterleaveD16<R>) il = a.ilv && a.ilv[s] == 3;
  const int rs = il ? 64 : 1;
  const int64_t row0 = s * H + (il ? (int64_t)lane : (int64_t)lane * R);  // the lane's first row
  XSrc<T, XV> xs;
  bool xpend = false, main_rows = false;
  typename wide_of<T>::type xalpha{};
  if constexpr (XV) {
    const CGState* cg = (const CGState*)a.cg;
    xpend = cg->it > cg->xit;
    xalpha = cg_alpha_of<typename wide_of<T>::type>(cg);
    xs.r = (const T*)a.x;
    xs.u = (const T*)a.xu;
    xs.b = (cg->res * cg->res) / (cg->prev * cg->prev);
    main_rows = a.rowmap == nullptr;
    if (cg->done) {  // nothing left but a pending x .+= α.*u_old
      if (xpend && main_rows) cg_rows_update<T, R, false>(a, xs, row0, rs, xalpha);
      return;
    }
  } else {
    xs.x = (const T*)a.x;
  }
  // the slice's metadata: offset, length word (and, pattern slices, the
  // lane's mask word; triple-SELL slices, the ghost base).  With SPMV_DESC
  // pattern and triple-SELL slices read all of it as one descriptor (32 B,
  // 64 B for 4 rows per lane; 16 B) with one scalar load instead of three
  // loads on two paths.  Same-copy A/Bs (profiles/r06/o/, p/, q/): FD7 128^3
  // 0.0287 -> 0.0277 ms, C5 F32 0.0658 -> 0.0649, C5 F64 -0.3 %, FE27 256^3
  // and the (2,2,2) halo leg -0.1 %
  int64_t off;
  int32_t lraw;
  uint64_t dmask = 0;
  int32_t tgb = 0;
  if (PAT && a.desc) {
    constexpr int W = H / 64, DW = kDescWords<R>;
    typedef int iv __attribute__((ext_vector_type(DW)));
    const iv d = *reinterpret_cast<const iv*>(a.desc + DW * s);
    off = (int64_t)d[0] * H;
    lraw = d[1];
    const int wi = (lane * R) / 64;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      const uint64_t mw = (uint64_t)(uint32_t)d[4 + 2 * i] | ((uint64_t)(uint32_t)d[5 + 2 * i] << 32);
      if (i == 0 || wi == i) dmask = mw;
    }
  } else if (PK == 4 && a.desc) {
    typedef int i4v __attribute__((ext_vector_type(4)));
    const i4v d = *reinterpret_cast<const i4v*>(a.desc + 4 * s);
    off = (int64_t)d[0] * H;
    lraw = d[1];
    tgb = d[2];
  } else {
    off = a.soff[s];
    lraw = a.slen[s];
  }
  // pattern slices: len | tri << 8 | pattern id << 9 (dedup_patterns); triple SELL: len | kTriSlice
  const int len = PAT ? (lraw & 0xff) : (PK == 4 ? (lraw & kTriLen) : lraw);
  bool ok[R];
  if (PAT) {
    const uint64_t m = a.desc ? dmask : a.mask[s * (H / 64) + (lane * R) / 64];
#pragma unroll
    for (int r = 0; r < R; ++r) ok[r] = ((m >> ((lane * R + r) & 63)) & 1ull) && (row0 + r < a.nrows);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) ok[r] = row0 + (int64_t)r * rs < a.nrows;
    if (a.sflags && a.sflags[s]) {  // rows handed to the long-row kernel (blocked slices only)
      const uint64_t m = a.lmask[s * (H / 64) + (lane * R) / 64];
#pragma unroll
      for (int r = 0; r < R; ++r) ok[r] = ok[r] && !((m >> ((lane * R + r) & 63)) & 1ull);
    }
  }
  int64_t orow[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = row0 + (int64_t)r * rs;
    orow[r] = ok[r] ? (a.rowmap ? (int64_t)a.rowmap[i] : i) : 0;
    if constexpr (PK == 4) {  // padding positions of the triple SELL (row map -1: before a pair group)
      if (orow[r] < 0) {
        ok[r] = false;
        orow[r] = 0;
      }
    }
  }

  T acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (BMODE == 0) {
      acc[r] = zero_of<T>();
    } else {
      T yo = zero_of<T>();
      if (ok[r]) yo = a.y[a.ymap ? (int64_t)a.ymap[orow[r]] : orow[r]];
      acc[r] = (BMODE == 2) ? yo * a.beta : yo;
    }
  }

  const Pack<T, R>* __restrict__ vp = reinterpret_cast<const Pack<T, R>*>(a.val + off) + lane;
  const bool tb = (a.flags & SPMV_TAILB) != 0;
  const bool pf = (a.flags & SPMV_PRODA) != 0;
  if constexpr (PK == 1) {
    const int32_t* pat = a.pat + (int64_t)(lraw >> 9) * a.kmax;
    bool tri_done = false;
    if constexpr (R > 1 && !SH) {
      if ((lraw & 0x100) && (a.flags & SPMV_XPAIR)) {  // triples of consecutive columns
        if (a.flags & SPMV_NT) rows_pattern_tri<T, R, ALPHA, true>(acc, pat, vp, len, xs, row0, ok, a.alpha, pf);
        else rows_pattern_tri<T, R, ALPHA, false>(acc, pat, vp, len, xs, row0, ok, a.alpha, pf);
        tri_done = true;
      }
    }
    if (tri_done) {
    } else if (a.flags & SPMV_XPAIR) {
      if (a.flags & SPMV_NT) rows_pattern<T, R, ALPHA, true, U, true, SH>(acc, pat, vp, len, xs, row0, ok, a.alpha, pf, tb);
      else rows_pattern<T, R, ALPHA, false, U, true, SH>(acc, pat, vp, len, xs, row0, ok, a.alpha, pf, tb);
    } else {
      if (a.flags & SPMV_NT) rows_pattern<T, R, ALPHA, true, U, false, SH>(acc, pat, vp, len, xs, row0, ok, a.alpha, pf, tb);
      else rows_pattern<T, R, ALPHA, false, U, false, SH>(acc, pat, vp, len, xs, row0, ok, a.alpha, pf, tb);
    }
  } else if constexpr (PK == 3) {
    const S16Pack<R>* __restrict__ cp = reinterpret_cast<const S16Pack<R>*>(a.col16 + off) + lane;
    const int32_t gb = a.gbase[s];
    int32_t rw[R];  // the rows the codes are relative to
#pragma unroll
    for (int r = 0; r < R; ++r) rw[r] = (int32_t)row0 + r * kD16RowStride<R>;
    if (a.flags & SPMV_NT) rows_d16<T, R, ALPHA, true, U, SH, kIdsAhead<T, R>>(acc, cp, vp, len, xs, a.alpha, pf, tb, rw, gb);
    else rows_d16<T, R, ALPHA, false, U, SH, kIdsAhead<T, R>>(acc, cp, vp, len, xs, a.alpha, pf, tb, rw, gb);
  } else if constexpr (PK == 4) {
    // triple SELL (rows through the row map, interleaved): tri slices carry
    // one code per triple, the others one per entry (rows_d16)
    const S16Pack<R>* __restrict__ cp = reinterpret_cast<const S16Pack<R>*>(a.col16 + off) + lane;
    const int32_t gb = a.desc ? tgb : a.gbase[s];
    int32_t rw[R];
#pragma unroll
    for (int r = 0; r < R; ++r) rw[r] = (int32_t)orow[r];
    if (lraw & kTriSlice) {
      bool packed = false;
      if constexpr (R == 2) {
        // pair slices, per-triple value packs (Float32) and/or batch code
        // packs (k_t_fill, pa_mat::t_pack), non-temporal
        using XS = XSrc<T, XV>;
        const bool tp = sizeof(T) == 4 && (a.flags & SPMV_TPACK);
        packed = true;
        if (lraw & kTriPair) {
          const uint16_t* cs = (const uint16_t*)a.col16 + off;
          if constexpr (sizeof(T) == 4) {
            if (tp) rows_t16_pair<T, ALPHA, XS, true>(acc, cs, vp, len, xs, a.alpha, pf, rw[0], gb);
            else rows_t16_pair<T, ALPHA, XS, false>(acc, cs, vp, len, xs, a.alpha, pf, rw[0], gb);
          } else {
            rows_t16_pair<T, ALPHA, XS, false>(acc, cs, vp, len, xs, a.alpha, pf, rw[0], gb);
          }
        } else {
          packed = false;
        }
      }
      if (packed) {
      } else if (a.flags & SPMV_NT) rows_t16_tri<T, R, ALPHA, true>(acc, cp, vp, len, xs, a.alpha, pf, rw, gb);
      else rows_t16_tri<T, R, ALPHA, false>(acc, cp, vp, len, xs, a.alpha, pf, rw, gb);
    } else {
      if (a.flags & SPMV_NT) rows_d16<T, R, ALPHA, true, U, SH, kIdsAhead<T, R>>(acc, cp, vp, len, xs, a.alpha, pf, tb, rw, gb);
      else rows_d16<T, R, ALPHA, false, U, SH, kIdsAhead<T, R>>(acc, cp, vp, len, xs, a.alpha, pf, tb, rw, gb);
    }
  } else {
    const IPack<R>* __restrict__ cp = reinterpret_cast<const IPack<R>*>(a.col + off) + lane;
    if (a.flags & SPMV_NT) rows_int32<T, R, ALPHA, true, U, SH, kIdsAhead<T, R>>(acc, cp, vp, len, xs, a.alpha, pf, tb);
    else rows_int32<T, R, ALPHA, false, U, SH, kIdsAhead<T, R>>(acc, cp, vp, len, xs, a.alpha, pf, tb);
  }

  // XV: u_new (and the deferred x update) of the main structure's rows
  T un[R];
  if constexpr (XV) {
    if (main_rows) cg_rows_update<T, R, true>(a, xs, row0, rs, xalpha, xpend, un);
  }
  if (a.dotp) {  // fused dot(u, c): Σ conj(u_i)·c_i over this slice's rows
    using DA = typename DAcc<T>::type;
    DA part = zero_of<DA>();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      T uv;
      if constexpr (XV) uv = main_rows ? un[r] : xs.get(orow[r]);
      else uv = a.dotu[orow[r]];
      if (ok[r]) part = part + dacc(cdot(uv, acc[r]));
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) part = part + shfl_down_acc(part, d);
    if (lane == 0) reinterpret_cast<DA*>(a.dotp)[a.dot_base + s] = part;
  }

  bool all = true;
#pragma unroll
  for (int r = 0; r < R; ++r) all = all && ok[r];
  if (all && !a.ymap && !a.rowmap && !il) {
    Pack<T, R> o;
#pragma unroll
    for (int r = 0; r < R; ++r) o.v[r] = acc[r];
    if constexpr (sizeof(Pack<T, R>) == 16) {
      if (a.flags & SPMV_YNT) {  // y as a non-temporal 16 B store per lane
        spmv_u32x4 w;
        __builtin_memcpy(&w, &o, 16);
        __builtin_nontemporal_store(w, reinterpret_cast<spmv_u32x4*>(a.y + row0));
      } else {
        *reinterpret_cast<Pack<T, R>*>(a.y + row0) = o;
      }
    } else {
      *reinterpret_cast<Pack<T, R>*>(a.y + row0) = o;
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (ok[r]) a.y[a.ymap ? (int64_t)a.ymap[orow[r]] : orow[r]] = acc[r];
  }
}

// XCD-chunked block order (pa_tune "spmv_xcd_chunk" C > 0): the hardware
// deals workgroups to the 8 XCDs round robin (block b on XCD b % 8), so
// consecutive slices land on different XCDs and each XCD's L2 fetches the x
// lines of its neighbours' slices too (C2: x fetched 1.59 times,
// profiles/r05/a/c2_pmc_per_kind.json).  With C, XCD k works on runs of C
// consecutive logical blocks: logical = (b / 8C)·8C + (b % 8)·C + (b / 8) % C
// (blocks past the last full group of 8C keep their order).  C = 4 keeps a
// block and the one 32 blocks away (128 slices: FD7 128³'s z neighbour; a
// divisor of FE27 256³'s) on the same XCD, as the round robin does.
__device__ __forceinline__ int64_t xcd_block(int chunk) {
  const int64_t b = blockIdx.x;
  if (chunk <= 0) return b;
  const int64_t G = 8 * (int64_t)chunk, full = ((int64_t)gridDim.x / G) * G;
  if (b >= full) return b;
  return (b / G) * G + (b % 8) * chunk + (b / 8) % chunk;
}

template <typename T, int R, bool ALPHA, int BMODE, int U, int PK, bool SH = false, bool XV = false>
__global__ __launch_bounds__(256) void k_spmv_sell(SpmvArgs<T> a) {
  const int64_t w = xcd_block(a.xcd_chunk) * 4 + (threadIdx.x >> 6);
  if (w >= a.nwork) return;
  spmv_wave<T, R, ALPHA, BMODE, U, PK, SH, XV>(a, w);
}

// One wave of the short-row tail launch over the uniform layout
// (build_uniform): the slice's values at s * H * K and its x runs at
// rbase + upat[e] (clamped into x: entries and rows the slice does not hold
// read some x and are never accumulated) are issued from the slice index
// and the kernel arguments alone; the descriptor (scalar load) supplies
// only the row mask and emask, which select the terms.  A lane's R rows are
// blocked, as in rows_pattern with 16 B x runs; the terms of a row and
// their order are rows_pattern's (U's order restricted to the slice's
// pattern = the pattern's own order).
template <typename T, int R, bool ALPHA, int BMODE, int U>
__device__ __forceinline__ void spmv_wave_u(const SpmvArgs<T>& a, const int64_t w) {
  constexpr int H = 64 * R, DW = kDescWords<R>;
  const int lane = threadIdx.x & 63;
  const int64_t s = a.list ? (int64_t)a.list[w] : w;
  const int64_t row0 = s * H + (int64_t)lane * R;
  const int K = a.uK;
  typedef int iv __attribute__((ext_vector_type(DW)));
  const iv d = *reinterpret_cast<const iv*>(a.desc + DW * s);
  const Pack<T, R>* __restrict__ vp = reinterpret_cast<const Pack<T, R>*>(a.uval + s * H * K) + lane;
  Pack<T, R> v[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (u < K) v[u] = ld<true>(&vp[u * 64]);
  Pack<T, R> xr[U];
  const int64_t xmax = a.nx - R;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (u < K) {
      const int64_t j = row0 + a.upat[u];
      xr[u] = ld_xrun<T, R>((const T*)a.x + (j < 0 ? 0 : j > xmax ? xmax : j));
    }
  const int emask = d[2];
  uint64_t m = 0;
#pragma unroll
  for (int i = 0; i < H / 64; ++i) {
    const uint64_t mw = (uint64_t)(uint32_t)d[4 + 2 * i] | ((uint64_t)(uint32_t)d[5 + 2 * i] << 32);
    if (i == 0 || (lane * R) / 64 == i) m = mw;
  }
  bool ok[R];
#pragma unroll
  for (int r = 0; r < R; ++r) ok[r] = ((m >> ((lane * R + r) & 63)) & 1ull) && (row0 + r < a.nrows);
  T acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (BMODE == 0) {
      acc[r] = zero_of<T>();
    } else {
      T yo = zero_of<T>();
      if (ok[r]) yo = a.y[a.ymap ? (int64_t)a.ymap[row0 + r] : row0 + r];
      acc[r] = (BMODE == 2) ? yo * a.beta : yo;
    }
  }
  const bool pf = (a.flags & SPMV_PRODA) != 0;
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const T t = acc[r] + term<ALPHA>(v[u].v[r], xr[u].v[r], a.alpha, pf);
      acc[r] = pick(u < K && ((emask >> u) & 1), t, acc[r]);
    }
  if (a.dotp) {  // fused dot(u, c), as in spmv_wave
    using DA = typename DAcc<T>::type;
    DA part = zero_of<DA>();
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (ok[r]) part = part + dacc(cdot(a.dotu[row0 + r], acc[r]));
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) part = part + shfl_down_acc(part, dd);
    if (lane == 0) reinterpret_cast<DA*>(a.dotp)[a.dot_base + s] = part;
  }
  bool all = true;
#pragma unroll
  for (int r = 0; r < R; ++r) all = all && ok[r];
  if (all && !a.ymap) {
    Pack<T, R> o;
#pragma unroll
    for (int r = 0; r < R; ++r) o.v[r] = acc[r];
    if constexpr (sizeof(Pack<T, R>) == 16) {
      if (a.flags & SPMV_YNT) {  // as spmv_wave: y as a non-temporal 16 B store per lane
        spmv_u32x4 yw;
        __builtin_memcpy(&yw, &o, 16);
        __builtin_nontemporal_store(yw, reinterpret_cast<spmv_u32x4*>(a.y + row0));
      } else {
        *reinterpret_cast<Pack<T, R>*>(a.y + row0) = o;
      }
    } else {
      *reinterpret_cast<Pack<T, R>*>(a.y + row0) = o;
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (ok[r]) a.y[a.ymap ? (int64_t)a.ymap[row0 + r] : row0 + r] = acc[r];
  }
}

// Several parts of one device in ONE launch (parts sharing a stream pair):
// the work items of part p are [start[p], start[p+1]) of the grid's waves,
// so a mul! over P small parts fills the GPU once instead of P times and
// costs one launch per phase instead of P.  Each wave computes exactly what
// the per-part launch computes (same slice, same order).
template <typename T>
struct SpmvGroup {
  int np;
  int tail0;  // entries [tail0, np) are side rows (int32 columns, <= 8 entries), TAIL kernels only
  int64_t start[PA_GROUP_MAX + 1];
  SpmvArgs<T> a[PA_GROUP_MAX];
};

// TAIL: the group's last entries are the parts' side rows (spmv_grouped's
// side tail, pa_tune "spmv_side_tail"): their few short waves run as the
// launch's trailing waves with the short-row int32 code (one masked batch:
// few registers, so the kernel keeps the pattern code's), instead of a
// launch of their own after the pattern slices (FE27 256³: 1,008 waves of
// one entry each, 6.8 µs as a separate launch, profiles/r04/am/)
template <typename T, int R, bool ALPHA, int BMODE, int U, int PK, bool SH = false, bool XV = false,
          bool TAIL = false>
__device__ __forceinline__ void group_wave(const SpmvGroup<T>& g) {
  // wave-uniform: the part's arguments are read with scalar loads
  const int64_t w = xcd_block(g.a[0].xcd_chunk) * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (w >= g.start[g.np]) return;
  int p = 0;
  while (p + 1 < g.np && w >= g.start[p + 1]) ++p;
  p = __builtin_amdgcn_readfirstlane(p);
  if constexpr (TAIL) {
    if (p >= g.tail0) {
      // the side rows in batches of 4 (one masked batch for the 1-entry
      // Dirichlet rows): the short-row launch then holds the pattern code's
      // registers (C2: 98 -> 84 VGPRs, 6 waves per SIMD instead of 5)
      spmv_wave<T, R, ALPHA, BMODE, 4, 0, false, false>(g.a[p], w - g.start[p]);
      return;
    }
  }
  if constexpr (PK == 1 && SH && !XV && U == 7) {
    if (g.a[p].uval) {  // the short-row tail launch over the uniform layout
      spmv_wave_u<T, R, ALPHA, BMODE, U>(g.a[p], w - g.start[p]);
      return;
    }
  }
  spmv_wave<T, R, ALPHA, BMODE, U, PK, SH, XV>(g.a[p], w - g.start[p]);
}

template <typename T, int R, bool ALPHA, int BMODE, int U, int PK, bool SH = false, bool XV = false,
          bool TAIL = false>
__global__ __launch_bounds__(256) void k_spmv_sell_group(const SpmvGroup<T> g) {
  group_wave<T, R, ALPHA, BMODE, U, PK, SH, XV, TAIL>(g);
}

// Float64 pattern slices whose rows have at most 7 entries (FD7: C2) with
// their side rows: the short-row batch of 7 (not 8) and 7 waves per SIMD
// (72 VGPRs instead of 84; the rare side rows' loop spills a few)
template <typename T, int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void k_spmv_group_short7(
    const SpmvGroup<T> g) {
  group_wave<T, R, false, 0, 7, 1, true, false, true>(g);
}

template <typename T, int R, bool ALPHA, int BMODE, int PAT>
static void launch_group_t(const SpmvGroup<T>& g, hipStream_t st) {
  const int64_t blocks = (g.start[g.np] + 3) / 4;
  if (blocks == 0) return;
  bool sh = (knobs().spmv_flags & SPMV_SHORT) != 0;
  for (int i = 0; i < g.np && i < g.tail0; ++i) sh = sh && g.a[i].maxlen <= 8;
  if constexpr (!ALPHA && BMODE == 0 && PAT != 4) {
    if (g.a[0].cg) {  // the device CG's fused u update
      if (sh)
        hipLaunchKernelGGL((k_spmv_sell_group<T, R, false, 0, 8, PAT, true, true>), dim3(blocks), dim3(256), 0, st, g);
      else
        hipLaunchKernelGGL((k_spmv_sell_group<T, R, false, 0, 8, PAT, false, true>), dim3(blocks), dim3(256), 0, st, g);
      return;
    }
  }
  if constexpr (PAT == 1) {
    if (g.tail0 < g.np) {  // pattern entries, then side rows (group_which, which 6)
      if constexpr (std::is_same<T, double>::value && !ALPHA && BMODE == 0) {
        bool sh7 = sh && (knobs().spmv_flags & SPMV_SHORT7) != 0 && knobs().spmv_xcd_chunk < 0;
        for (int i = 0; i < g.np && i < g.tail0; ++i) sh7 = sh7 && g.a[i].maxlen <= 7;
        if (sh7) {
          SpmvGroup<T> g2 = g;
          for (int i = 0; i < g2.np; ++i) g2.a[i].xcd_chunk = 0;
          hipLaunchKernelGGL((k_spmv_group_short7<T, R>), dim3(blocks), dim3(256), 0, st, g2);
          return;
        }
      }
      if (sh && knobs().spmv_xcd_chunk < 0) {
        // short rows (one batch per wave, latency-bound): the auto XCD runs
        // cost more than their x locality gives (C2: 0.0282 with the round
        // robin vs 0.0283-0.0284 with runs of 4, profiles/r05/y/)
        SpmvGroup<T> g2 = g;
        for (int i = 0; i < g2.np; ++i) g2.a[i].xcd_chunk = 0;
        hipLaunchKernelGGL((k_spmv_sell_group<T, R, ALPHA, BMODE, 8, PAT, true, false, true>), dim3(blocks),
                           dim3(256), 0, st, g2);
      } else if (sh)
        hipLaunchKernelGGL((k_spmv_sell_group<T, R, ALPHA, BMODE, 8, PAT, true, false, true>), dim3(blocks),
                           dim3(256), 0, st, g);
      else
        hipLaunchKernelGGL((k_spmv_sell_group<T, R, ALPHA, BMODE, 8, PAT, false, false, true>), dim3(blocks),
                           dim3(256), 0, st, g);
      return;
    }
  }
  if (sh)
    hipLaunchKernelGGL((k_spmv_sell_group<T, R, ALPHA, BMODE, 8, PAT, true>), dim3(blocks), dim3(256), 0, st, g);
  else
    hipLaunchKernelGGL((k_spmv_sell_group<T, R, ALPHA, BMODE, 8, PAT>), dim3(blocks), dim3(256), 0, st, g);
}

template <typename T, int R, int PAT>
static void launch_group_ab(const SpmvGroup<T>& g, bool has_alpha, int bmode, hipStream_t st) {
  if (!has_alpha) {
    if (bmode == 0) launch_group_t<T, R, false, 0, PAT>(g, st);
    else if (bmode == 1) launch_group_t<T, R, false, 1, PAT>(g, st);
    else launch_group_t<T, R, false, 2, PAT>(g, st);
  } else {
    if (bmode == 0) launch_group_t<T, R, true, 0, PAT>(g, st);
    else if (bmode == 1) launch_group_t<T, R, true, 1, PAT>(g, st);
    else launch_group_t<T, R, true, 2, PAT>(g, st);
  }
}

template <typename T, int R, bool ALPHA, int BMODE, int PAT>
static void launch_t(const SpmvArgs<T>& a, hipStream_t st) {
  const int64_t blocks = (a.nwork + 3) / 4;
  if (blocks == 0) return;
  if constexpr (!ALPHA && BMODE == 0 && PAT != 4) {
    if (a.cg) {  // the device CG's fused u update
      if ((knobs().spmv_flags & SPMV_SHORT) && a.maxlen <= 8)
        hipLaunchKernelGGL((k_spmv_sell<T, R, false, 0, 8, PAT, true, true>), dim3(blocks), dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL((k_spmv_sell<T, R, false, 0, 8, PAT, false, true>), dim3(blocks), dim3(256), 0, st, a);
      return;
    }
  }
  if ((knobs().spmv_flags & SPMV_SHORT) && a.maxlen <= 8)
    hipLaunchKernelGGL((k_spmv_sell<T, R, ALPHA, BMODE, 8, PAT, true>), dim3(blocks), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((k_spmv_sell<T, R, ALPHA, BMODE, 8, PAT>), dim3(blocks), dim3(256), 0, st, a);
}

template <typename T, int R, int PAT>
static void launch_ab(const SpmvArgs<T>& a, bool has_alpha, int bmode, hipStream_t st) {
  if (!has_alpha) {
    if (bmode == 0) launch_t<T, R, false, 0, PAT>(a, st);
    else if (bmode == 1) launch_t<T, R, false, 1, PAT>(a, st);
    else launch_t<T, R, false, 2, PAT>(a, st);
  } else {
    if (bmode == 0) launch_t<T, R, true, 0, PAT>(a, st);
    else if (bmode == 1) launch_t<T, R, true, 1, PAT>(a, st);
    else launch_t<T, R, true, 2, PAT>(a, st);
  }
}

// which = 0: pattern slices of the main structure; 1: int32-column slices
// of the main structure; 2: side SELL; 4: delta16 slices of the main
// structure; 5: triple SELL.  list/nwork select the slices.
template <typename T>
static SpmvArgs<T> make_args(int which, int64_t nwork, const int32_t* list, const pa_mat* A, const void* x,
                             void* y, const int32_t* ymap, const void* alpha, const void* beta, void* dotp,
                             const SpmvPart* cgp = nullptr) {
  SpmvArgs<T> a{};
  if (cgp && cgp->cg) {
    a.xu = (decltype(a.xu))((const T*)cgp->xu);
    a.un = (decltype(a.un))((T*)cgp->un);
    a.xacc = (decltype(a.xacc))((T*)cgp->xacc);
    a.cg = (decltype(a.cg))(cgp->cg);
  }
  a.dotu = (decltype(a.dotu))((const T*)x);
  a.dotp = dotp;
  a.dot_base = which == 2 ? A->nslices : which == 5 ? A->nslices + A->s_nslices : 0;
  a.nwork = nwork;
  a.list = (decltype(a.list))(list);
  a.x = (decltype(a.x))((const T*)x);
  a.nx = A->ncols_lids;
  a.y = (decltype(a.y))((T*)y);
  a.ymap = (decltype(a.ymap))(ymap);
  a.alpha = *(const T*)alpha;
  a.beta = *(const T*)beta;
  a.flags = knobs().spmv_flags | (A->csr ? SPMV_PRODA : 0) | (which == 5 && (A->t_pack & 1) ? SPMV_TPACK : 0);
  a.xcd_chunk = knobs().spmv_xcd_chunk >= 0 ? knobs().spmv_xcd_chunk : A->xcd_auto;
  a.maxlen = which == 0   ? A->maxlen_pat
             : which == 2 ? A->maxlen_side
             : which == 1 ? ((knobs().spmv_format == 1 && A->has_pat) ? A->maxlen_pm_int : A->maxlen_all)
             : which == 4 ? A->maxlen_d16
             : which == 5 ? std::max(A->maxlen_t, 9)  // never the short-row kernels (merged_wave)
                          : INT32_MAX;
  if (which == 5) {  // triple SELL
    a.soff = (decltype(a.soff))(A->d_t_off);
    a.slen = (decltype(a.slen))(A->d_t_len);
    a.col16 = (decltype(a.col16))(A->d_t_col16);
    a.gbase = (decltype(a.gbase))(A->d_t_gbase);
    a.val = (decltype(a.val))((const T*)A->d_t_val);
    a.rowmap = (decltype(a.rowmap))(A->d_t_rowmap);
    a.nrows = A->t_nrows;
    if (knobs().spmv_flags & SPMV_DESC) a.desc = (decltype(a.desc))(A->d_t_desc);
  } else if (which == 2) {
    a.soff = (decltype(a.soff))(A->d_s_off);
    a.slen = (decltype(a.slen))(A->d_s_len);
    a.col = (decltype(a.col))(A->d_s_col);
    a.val = (decltype(a.val))((const T*)A->d_s_val);
    a.rowmap = (decltype(a.rowmap))(A->d_s_rowmap);
    a.nrows = A->s_nrows;
  } else {
    a.soff = (decltype(a.soff))(A->d_slice_off);
    a.col = (decltype(a.col))(A->d_col);
    a.val = (decltype(a.val))((const T*)A->d_val);
    a.nrows = A->nrows;
    if (which == 0) {
      a.slen = (decltype(a.slen))(A->d_plen);
      a.pat = (decltype(a.pat))(A->d_pat);
      a.mask = (decltype(a.mask))(A->d_mask);
      a.kmax = A->kmax;
      if (knobs().spmv_flags & SPMV_DESC) a.desc = (decltype(a.desc))(A->d_pdesc);
      if (A->d_uval && a.desc) {
        a.uval = (decltype(a.uval))((const T*)A->d_uval);
        a.uK = A->uK;
        for (int e = 0; e < 8; ++e) a.upat[e] = A->upat[e];
      }
    } else {
      a.slen = (decltype(a.slen))(A->d_slice_len);
      if (which == 4) {
        a.col16 = (decltype(a.col16))(A->d_col16);
        a.gbase = (decltype(a.gbase))(A->d_gbase);
      }
    }
  }
  if (which == 1) {
    a.sflags = (decltype(a.sflags))(A->d_sflags);
    a.lmask = (decltype(a.lmask))(A->d_lmask);
    // spmv_format 0 runs the delta16 slices (Float32: interleaved rows) as int32
    if (A->d_col16 && A->R == 4 && !(knobs().spmv_format == 1 && A->has_pat)) a.ilv = (decltype(a.ilv))(A->d_kind);
  }
  return a;
}

template <typename T, int R>
static void launch_which(int which, int64_t nwork, const int32_t* list, const pa_mat* A, const void* x,
                         void* y, const int32_t* ymap, bool has_alpha, int bmode, const void* alpha,
                         const void* beta, void* dotp, hipStream_t st, const SpmvPart* cgp) {
  const SpmvArgs<T> a = make_args<T>(which, nwork, list, A, x, y, ymap, alpha, beta, dotp, cgp);
  if (which == 0) launch_ab<T, R, 1>(a, has_alpha, bmode, st);
  else if (which == 4) launch_ab<T, R, 3>(a, has_alpha, bmode, st);
  else if (which == 5) {
    if constexpr (R <= 2) launch_ab<T, R, 4>(a, has_alpha, bmode, st);  // (build_triple_sell: R <= 2 only)
  } else launch_ab<T, R, 0>(a, has_alpha, bmode, st);
}

// the same slices of np parts as one launch per PA_GROUP_MAX parts
template <typename T, int R>
static void group_which(int which, int np, const SpmvPart* parts, bool has_alpha, int bmode, const void* alpha,
                        const void* beta, hipStream_t st) {
  // which 6: pattern entries followed by side-row entries (SpmvPart::side;
  // the caller passes at most PA_GROUP_MAX entries, pattern ones first): one
  // TAIL launch
  SpmvGroup<T> g{};
  g.tail0 = PA_GROUP_MAX + 1;
  auto flush = [&]() {
    if (g.np == 0) return;
    if (which == 0 || which == 6) launch_group_ab<T, R, 1>(g, has_alpha, bmode, st);
    else if (which == 4) launch_group_ab<T, R, 3>(g, has_alpha, bmode, st);
    else if (which == 5) {
      if constexpr (R <= 2) launch_group_ab<T, R, 4>(g, has_alpha, bmode, st);  // (R <= 2 only)
    }
    else launch_group_ab<T, R, 0>(g, has_alpha, bmode, st);
    g = SpmvGroup<T>{};
    g.tail0 = PA_GROUP_MAX + 1;
  };
  for (int i = 0; i < np; ++i) {
    const SpmvPart& q = parts[i];
    if (q.nwork <= 0) continue;
    const int kind = which == 6 ? (q.side ? 2 : 0) : which;
    if (which == 6 && q.side && g.tail0 > g.np) g.tail0 = g.np;
    const int32_t* list = q.list;
    if ((knobs().spmv_flags & SPMV_IDLIST) && list && kind != 2 && kind != 5 && q.nwork == q.A->nslices) list = nullptr;
    g.a[g.np] = make_args<T>(kind, q.nwork, list, q.A, q.x, q.y, q.ymap, alpha, beta, q.dotp, &q);
    g.start[g.np + 1] = g.start[g.np] + q.nwork;
    if (++g.np == PA_GROUP_MAX) flush();
  }
  flush();
}

// the per-element-type entry points (one translation unit each, PA_SPMV_DT)
#define PA_DT_DECL(k)                                                                                          \
  void spmv_group_##k(int which, int np, const SpmvPart* parts, bool has_alpha, int bmode, const void* alpha,  \
                      const void* beta, hipStream_t st);                                                        \
  int spmv_merged_##k(int n, const int* which, const SpmvPart* parts, bool has_alpha, int bmode,              \
                      const void* alpha, const void* beta, pa_ctx* owner, hipStream_t st);                     \
  void spmv_long_##k(const pa_mat* A, const void* x, void* y, const int32_t* ymap, bool has_alpha, int bmode,  \
                     const void* alpha, const void* beta, void* dotp, int64_t dot_base, hipStream_t st);       \
  void spmv_part_##k(int which, int64_t nwork, const int32_t* list, const pa_mat* A, const void* x, void* y,  \
                     const int32_t* ymap, bool has_alpha, int bmode, const void* alpha, const void* beta,     \
                     void* dotp, hipStream_t st, const SpmvPart* cgp);
PA_DT_DECL(0)
PA_DT_DECL(1)
PA_DT_DECL(2)
PA_DT_DECL(3)
#undef PA_DT_DECL
#if defined(PA_SPMV_DT)
#if PA_SPMV_DT == 0
using DtT = float;
constexpr int kDtR = 4;
#elif PA_SPMV_DT == 1
using DtT = double;
constexpr int kDtR = 2;
#elif PA_SPMV_DT == 2
using DtT = c64;
constexpr int kDtR = 2;
#else
using DtT = c128;
constexpr int kDtR = 1;
#endif
// Float32 matrices hold 4 or 2 rows per lane (pa_tune "f32_rows", fixed when
// a matrix is built): a call's parts run as runs of equal R
constexpr bool kDtR2 = PA_SPMV_DT == 0;
void PA_CAT(spmv_group_, PA_SPMV_DT)(int which, int np, const SpmvPart* parts, bool has_alpha, int bmode,
                                     const void* alpha, const void* beta, hipStream_t st) {
  if constexpr (kDtR2) {
    for (int i = 0; i < np;) {
      int j = i + 1;
      while (j < np && parts[j].A->R == parts[i].A->R) ++j;
      if (parts[i].A->R == 2) group_which<DtT, 2>(which, j - i, parts + i, has_alpha, bmode, alpha, beta, st);
      else group_which<DtT, kDtR>(which, j - i, parts + i, has_alpha, bmode, alpha, beta, st);
      i = j;
    }
  } else {
    group_which<DtT, kDtR>(which, np, parts, has_alpha, bmode, alpha, beta, st);
  }
}
#else
void launch_spmv_group(int which, int np, const SpmvPart* parts, bool has_alpha, int bmode, const void* alpha,
                       const void* beta, hipStream_t st) {
  if (np <= 0) return;
#define spmv_group_(k) spmv_group_##k(which, np, parts, has_alpha, bmode, alpha, beta, st)
  switch (parts[0].A->dtype) {
    case PA_F32: spmv_group_(0); break;
    case PA_F64: spmv_group_(1); break;
    case PA_C64: spmv_group_(2); break;
    case PA_C128: spmv_group_(3); break;
  }
#undef spmv_group_
}
#endif

// ---------------------------------------------------------------------------
// Merged launch: every slice kind of every part of the call in ONE launch
// (when no halo is in flight: the ghosts are already in x), instead of one
// launch per kind and phase.  Each entry of the table is (kind, the
// arguments of one part's launch of that kind); waves pick their entry with
// a wave-uniform search and run exactly the per-kind wave code, so results
// equal the separate launches bit for bit.  The small latency-bound launches
// (side rows, the few int32 slices) then overlap the big ones instead of
// each adding its own tail.  The table lives in device memory (too large for
// kernel arguments), one cached copy per distinct call.
constexpr int kMergeMax = 48;

template <typename T>
struct SpmvTable {
  int n;
  int pk[kMergeMax];
  int64_t start[kMergeMax + 1];
  SpmvArgs<T> a[kMergeMax];
};

// The wave -> entry map that follows a merged table in device memory (one
// byte per wave, at the 16 B boundary after the table's n used entries):
// a wave finds its entry with one load instead of a binary search over the
// table's start offsets (log2(n) dependent loads ahead of every wave's
// stream; C5's tables hold 20-40 entries)
template <typename T>
__host__ __device__ constexpr size_t merged_map_offset(int n) {
  return (offsetof(SpmvTable<T>, a) + (size_t)n * sizeof(SpmvArgs<T>) + 15) & ~(size_t)15;
}

template <typename T, int R, bool ALPHA, int BMODE, int U, bool SH, bool XV = false>
__device__ __forceinline__ void merged_wave(const SpmvTable<T>* __restrict__ tab, int n, int64_t waves, int xc) {
  // n and the wave count come as kernel arguments (with the kernarg load, not
  // two dependent table loads ahead of the search)
  const int64_t w = xcd_block(xc) * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (w >= waves) return;
  const uint8_t* __restrict__ map = reinterpret_cast<const uint8_t*>(tab) + merged_map_offset<T>(n);
  const int p = __builtin_amdgcn_readfirstlane((int)map[w]);
  const int pk = __builtin_amdgcn_readfirstlane(tab->pk[p]);
  const int64_t lw = w - tab->start[p];
  const SpmvArgs<T>& a = tab->a[p];
  if (pk == 1) spmv_wave<T, R, ALPHA, BMODE, U, 1, SH, XV>(a, lw);
  else if (pk == 3) spmv_wave<T, R, ALPHA, BMODE, U, 3, SH, XV>(a, lw);
  else if (pk == 4) {
    // the triple SELL never runs in the short-row (make_args: maxlen >= 9)
    // or fused-u kernels (pa_cg_solve_all: no fused update with it): their
    // registers stay those of the other kinds
    // (and slices of R <= 2 rows per lane only: build_triple_sell)
    if constexpr (!SH && !XV && R <= 2) spmv_wave<T, R, ALPHA, BMODE, U, 4, SH, XV>(a, lw);
  }
  else spmv_wave<T, R, ALPHA, BMODE, U, 0, SH, XV>(a, lw);
}

// No occupancy cap: amdgpu_waves_per_eu(4) (F32 134 -> 128 VGPRs, a small
// spill) lost in a same-box A/B: C5 F32 +4.5 %, FE27 F64 +0.4 %, F32 +0.6 %
// (profiles/r02/stream/ab_waves4.txt).
template <typename T, int R, bool ALPHA, int BMODE, int U, bool SH, bool XV = false>
__global__ __launch_bounds__(256) void k_spmv_merged(const SpmvTable<T>* __restrict__ tab, int n,
                                                         int64_t waves, int xc) {
  merged_wave<T, R, ALPHA, BMODE, U, SH, XV>(tab, n, waves, xc);
}

// F64 short rows (FD7): 5 waves per SIMD instead of 4 (96 VGPRs instead of
// 102; the pattern path keeps its registers, a few int32-path values spill).
// C2 FD7 128^3: 0.0312-0.0317 -> 0.0303 ms (profiles/r02/waves/).  Not for
// F32/C64 (R = 4 / complex: ~200 spills) nor for longer rows (FE27: -10 %).
template <typename T, int R, bool ALPHA, int BMODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_spmv_merged_short(
    const SpmvTable<T>* __restrict__ tab, int n, int64_t waves, int xc) {
  merged_wave<T, R, ALPHA, BMODE, 8, true>(tab, n, waves, xc);
}

template <typename T, int R, bool ALPHA, int BMODE>
static void launch_merged_t(const SpmvTable<T>* d, int n, int64_t waves, bool sh, hipStream_t st) {
  const int xc = std::max(knobs().spmv_xcd_chunk, 0);  // (auto: merged launches keep the round robin)
  const int64_t blocks = (waves + 3) / 4;
  if (blocks == 0) return;
  if constexpr (std::is_same<T, double>::value) {
    if (sh) {
      hipLaunchKernelGGL((k_spmv_merged_short<T, R, ALPHA, BMODE>), dim3(blocks), dim3(256), 0, st, d, n, waves, xc);
      return;
    }
  }
  if (sh)
    hipLaunchKernelGGL((k_spmv_merged<T, R, ALPHA, BMODE, 8, true>), dim3(blocks), dim3(256), 0, st, d, n, waves, xc);
  else
    hipLaunchKernelGGL((k_spmv_merged<T, R, ALPHA, BMODE, 8, false>), dim3(blocks), dim3(256), 0, st, d, n, waves, xc);
}

static int pk_of(int which) { return which == 0 ? 1 : which == 4 ? 3 : which == 5 ? 4 : 0; }

// One merged launch, prepared: its device table (cached) and launch shape
template <typename T>
struct MergedLaunch {
  const SpmvTable<T>* dt = nullptr;
  int n = 0;
  int64_t waves = 0;
  bool sh = false, cg = false;
};

template <typename T, int R>
static int merged_prepare(int n, const int* which, const SpmvPart* parts, bool has_alpha, int bmode,
                          const void* alpha, const void* beta, pa_ctx* owner, hipStream_t st, MergedLaunch<T>* out) {
  // the table's used bytes (header + n entries) are its cache key: only
  // those are zeroed, compared and uploaded (a 48-entry table is ≈15 KB, a
  // call's tables hold 1-4 entries: per-call host work of the stream-pair
  // path)
  SpmvTable<T> h;
  constexpr size_t kHdr = offsetof(SpmvTable<T>, a);
  std::memset(&h, 0, kHdr);
  bool sh = (knobs().spmv_flags & SPMV_SHORT) != 0;
  for (int i = 0; i < n; ++i) {
    const SpmvPart& q = parts[i];
    if (q.nwork <= 0) continue;
    if (h.n == kMergeMax) return 1;
    const int32_t* list = q.list;
    if ((knobs().spmv_flags & SPMV_IDLIST) && list && which[i] != 2 && which[i] != 5 && q.nwork == q.A->nslices) list = nullptr;
    h.a[h.n] = make_args<T>(which[i], q.nwork, list, q.A, q.x, q.y, q.ymap, alpha, beta, q.dotp, &q);
    h.pk[h.n] = pk_of(which[i]);
    sh = sh && h.a[h.n].maxlen <= 8;
    h.start[h.n + 1] = h.start[h.n] + q.nwork;
    ++h.n;
  }
  *out = MergedLaunch<T>{};
  if (h.n == 0) return 0;
  static_assert(kMergeMax <= 255, "the wave map holds entry indices in bytes");
  const size_t used = kHdr + (size_t)h.n * sizeof(SpmvArgs<T>);  // the device reads entries < n only
  const int64_t nwaves = h.start[h.n];
  const size_t moff = merged_map_offset<T>(h.n), total = moff + (size_t)nwaves;
  // cached device copy of this exact table (most recent first)
  auto& C = owner->merged_cache;
  const char* hb = reinterpret_cast<const char*>(&h);
  void* d = nullptr;
  for (size_t k = 0; k < C.size(); ++k)
    if (C[k].first.size() == used && std::memcmp(C[k].first.data(), hb, used) == 0) {
      if (k) std::swap(C[k], C[0]);
      d = C[0].second;
      break;
    }
  if (!d) {
    if (hipMalloc(&d, total) != hipSuccess) return -1;
    std::vector<char> m((size_t)nwaves);  // entry of every wave (merged_wave)
    for (int e = 0; e < h.n; ++e) std::memset(m.data() + h.start[e], e, (size_t)(h.start[e + 1] - h.start[e]));
    if (hipMemcpy(d, &h, used, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy((char*)d + moff, m.data(), m.size(), hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(d);
      return -1;
    }
    if (C.size() >= 16) {
      (void)hipStreamSynchronize(st);  // the evicted table may still be read
      (void)hipFree(C.back().second);
      C.pop_back();
    }
    C.insert(C.begin(), {std::vector<char>(hb, hb + used), d});
  }
  out->dt = (const SpmvTable<T>*)d;
  out->n = h.n;
  out->waves = nwaves;
  out->sh = sh;
  out->cg = h.a[0].cg != nullptr;
  return 0;
}

template <typename T, int R>
static void merged_launch(const MergedLaunch<T>& m, bool has_alpha, int bmode, hipStream_t st) {
  if (m.n == 0) return;
  if (m.cg) {  // the device CG's fused u update (α = 1, β = 0)
    const int64_t blocks = (m.waves + 3) / 4;
    if (blocks == 0) return;
    const int xc = std::max(knobs().spmv_xcd_chunk, 0);  // (auto: merged launches keep the round robin)
    if (m.sh) hipLaunchKernelGGL((k_spmv_merged<T, R, false, 0, 8, true, true>), dim3(blocks), dim3(256), 0, st, m.dt, m.n, m.waves, xc);
    else hipLaunchKernelGGL((k_spmv_merged<T, R, false, 0, 8, false, true>), dim3(blocks), dim3(256), 0, st, m.dt, m.n, m.waves, xc);
    return;
  }
  if (!has_alpha) {
    if (bmode == 0) launch_merged_t<T, R, false, 0>(m.dt, m.n, m.waves, m.sh, st);
    else if (bmode == 1) launch_merged_t<T, R, false, 1>(m.dt, m.n, m.waves, m.sh, st);
    else launch_merged_t<T, R, false, 2>(m.dt, m.n, m.waves, m.sh, st);
  } else {
    if (bmode == 0) launch_merged_t<T, R, true, 0>(m.dt, m.n, m.waves, m.sh, st);
    else if (bmode == 1) launch_merged_t<T, R, true, 1>(m.dt, m.n, m.waves, m.sh, st);
    else launch_merged_t<T, R, true, 2>(m.dt, m.n, m.waves, m.sh, st);
  }
}

template <typename T, int R>
static int merged_t(int n, const int* which, const SpmvPart* parts, bool has_alpha, int bmode, const void* alpha,
                    const void* beta, pa_ctx* owner, hipStream_t st) {
  MergedLaunch<T> m;
  const int rc = merged_prepare<T, R>(n, which, parts, has_alpha, bmode, alpha, beta, owner, st, &m);
  if (rc) return rc;
  merged_launch<T, R>(m, has_alpha, bmode, st);
  return 0;
}

// n (which, part) entries as one launch; returns 1 when they do not fit one
// table (the caller launches per kind), -1 on an allocation/copy error
#if defined(PA_SPMV_DT)
int PA_CAT(spmv_merged_, PA_SPMV_DT)(int n, const int* which, const SpmvPart* parts, bool has_alpha, int bmode,
                                     const void* alpha, const void* beta, pa_ctx* owner, hipStream_t st) {
  if constexpr (kDtR2) {
    bool mixed = false;
    for (int i = 1; i < n; ++i) mixed = mixed || parts[i].A->R != parts[0].A->R;
    if (mixed) {  // parts of both layouts: one merged launch per layout
      if (n > kMergeMax) return 1;  // (nothing launched: the caller runs per kind)
      std::vector<int> w[2];
      std::vector<SpmvPart> q[2];
      for (int i = 0; i < n; ++i) {
        const int k = parts[i].A->R == 2 ? 0 : 1;
        w[k].push_back(which[i]);
        q[k].push_back(parts[i]);
      }
      // both tables before either launch: a table that does not fit or
      // fails leaves nothing launched for the caller's per-kind fallback to
      // repeat (with β ≠ 0, y would accumulate twice)
      MergedLaunch<DtT> m2, m4;
      int rc = merged_prepare<DtT, 2>((int)w[0].size(), w[0].data(), q[0].data(), has_alpha, bmode, alpha, beta,
                                      owner, st, &m2);
      if (rc == 0)
        rc = merged_prepare<DtT, kDtR>((int)w[1].size(), w[1].data(), q[1].data(), has_alpha, bmode, alpha, beta,
                                       owner, st, &m4);
      if (rc) return rc;
      merged_launch<DtT, 2>(m2, has_alpha, bmode, st);
      merged_launch<DtT, kDtR>(m4, has_alpha, bmode, st);
      return 0;
    }
    if (n > 0 && parts[0].A->R == 2) return merged_t<DtT, 2>(n, which, parts, has_alpha, bmode, alpha, beta, owner, st);
  }
  return merged_t<DtT, kDtR>(n, which, parts, has_alpha, bmode, alpha, beta, owner, st);
}
#else
int launch_spmv_merged(int n, const int* which, const SpmvPart* parts, bool has_alpha, int bmode,
                       const void* alpha, const void* beta, pa_ctx* owner, hipStream_t st) {
  if (n <= 0) return 0;
#define spmv_merged_(k) spmv_merged_##k(n, which, parts, has_alpha, bmode, alpha, beta, owner, st)
  switch (parts[0].A->dtype) {
    case PA_F32: return spmv_merged_(0);
    case PA_F64: return spmv_merged_(1);
    case PA_C64: return spmv_merged_(2);
    case PA_C128: return spmv_merged_(3);
  }
#undef spmv_merged_
  return 0;
}
#endif

// ---------------------------------------------------------------------------
// Long rows (row-length histogram): rows far longer than the
// rest leave the SELL (whose slices would pad every row to their length)
// and run one wave per row over their own CSR, entries in the reference's
// order.  EXACT: the wave adds the 64 products of each chunk one after the
// other (readlane), so the row is summed exactly as SparseUtils.jl:176-185
// sums it; otherwise each lane keeps a strided partial sum and the wave
// folds them in a fixed tree (deterministic, within 1e-12 of the reference).

template <typename T> struct LaneOf;
template <> struct LaneOf<float> { static __device__ float get(float v, int j) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j)); } };
template <> struct LaneOf<double> {
  static __device__ double get(double v, int j) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), j);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
  }
};
template <> struct LaneOf<c64> { static __device__ c64 get(c64 v, int j) { return c64{LaneOf<float>::get(v.re, j), LaneOf<float>::get(v.im, j)}; } };
template <> struct LaneOf<c128> { static __device__ c128 get(c128 v, int j) { return c128{LaneOf<double>::get(v.re, j), LaneOf<double>::get(v.im, j)}; } };

__device__ inline float shfl_xor_t(float v, int m) { return __shfl_xor(v, m, 64); }
__device__ inline double shfl_xor_t(double v, int m) { return __shfl_xor(v, m, 64); }
__device__ inline c64 shfl_xor_t(c64 v, int m) { return c64{__shfl_xor(v.re, m, 64), __shfl_xor(v.im, m, 64)}; }
__device__ inline c128 shfl_xor_t(c128 v, int m) { return c128{__shfl_xor(v.re, m, 64), __shfl_xor(v.im, m, 64)}; }

// EXACT: one wave (one 64-thread block) per long row.  The wave computes
// the products of 512 entries at a time (8 per lane, the next 512 loading
// while the current ones are summed), stages them in LDS and every lane adds
// them one after the other: the reference's summation chain.
template <typename T, bool ALPHA, int BMODE>
__global__ __launch_bounds__(64) void k_spmv_long_exact(int64_t nlong, const int32_t* __restrict__ lrow,
                                                        const int64_t* __restrict__ lptr,
                                                        const int32_t* __restrict__ lcol, const T* __restrict__ lval,
                                                        const T* __restrict__ x, T* __restrict__ y,
                                                        const int32_t* __restrict__ ymap, T alpha, bool pf, T beta,
                                                        const T* __restrict__ dotu, void* dotp, int64_t dot_base) {
  constexpr int U = 8, B = U * 64;
  __shared__ T buf[B];
  const int lane = threadIdx.x;
  const int64_t w = blockIdx.x;
  if (w >= nlong) return;
  const int64_t r = lrow[w];
  const int64_t yl = ymap ? (int64_t)ymap[r] : r;
  T acc;
  if (BMODE == 0) acc = zero_of<T>();
  else acc = (BMODE == 2) ? y[yl] * beta : y[yl];
  const int64_t b0 = lptr[w], b1 = lptr[w + 1];
  T p[U];
  auto load = [&](int64_t b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = b + u * 64 + lane;
      T q = zero_of<T>();
      if (k < b1) {
        q = term<ALPHA>(lval[k], x[lcol[k]], alpha, pf);
      }
      p[u] = q;
    }
  };
  if (b0 < b1) load(b0);
  for (int64_t b = b0; b < b1; b += B) {
#pragma unroll
    for (int u = 0; u < U; ++u) buf[u * 64 + lane] = p[u];
    __syncthreads();
    if (b + B < b1) load(b + B);  // in flight while the chain below runs
    const int cnt = (int)((b1 - b) < B ? (b1 - b) : B);
    int t = 0;
    for (; t + 16 <= cnt; t += 16) {  // reads ahead of the dependent adds
      T v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = buf[t + i];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc = acc + v[i];
    }
    for (; t < cnt; ++t) acc = acc + buf[t];
    __syncthreads();
  }
  if (lane == 0) {
    y[yl] = acc;
    if (dotp) {
      using DA = typename DAcc<T>::type;
      reinterpret_cast<DA*>(dotp)[dot_base + w] = dacc(cdot(dotu[r], acc));
    }
  }
}

// Fast (long_rows_exact = 0): the long rows are cut into chunks of
// kLongChunk entries, one wave per chunk (lane-strided partial sums, then a
// fixed xor tree); k_spmv_long_fold adds each row's chunk partials in chunk
// order after the β-init.  Deterministic, within 1e-12 of the reference.
template <typename T, bool ALPHA>
__global__ __launch_bounds__(256) void k_spmv_long_chunks(int64_t nchunks, const int64_t* __restrict__ cstart,
                                                          const int64_t* __restrict__ cend,
                                                          const int32_t* __restrict__ lcol,
                                                          const T* __restrict__ lval, const T* __restrict__ x,
                                                          T alpha, bool pf, T* __restrict__ part) {
  constexpr int U = 8;
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  const int64_t b1 = cend[c];
  T s = zero_of<T>();
  for (int64_t b = cstart[c]; b < b1; b += U * 64) {
    T q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = b + u * 64 + lane;
      q[u] = zero_of<T>();
      if (k < b1) {
        q[u] = term<ALPHA>(lval[k], x[lcol[k]], alpha, pf);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s = s + q[u];
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) s = s + shfl_xor_t(s, m);
  if (lane == 0) part[c] = s;
}

template <typename T, int BMODE>
__global__ void k_spmv_long_fold(int64_t nlong, const int32_t* __restrict__ lrow, const int64_t* __restrict__ cptr,
                                 const T* __restrict__ part, T* __restrict__ y, const int32_t* __restrict__ ymap,
                                 T beta, const T* __restrict__ dotu, void* dotp, int64_t dot_base) {
  const int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (w >= nlong) return;
  const int64_t r = lrow[w];
  const int64_t yl = ymap ? (int64_t)ymap[r] : r;
  T acc;
  if (BMODE == 0) acc = zero_of<T>();
  else acc = (BMODE == 2) ? y[yl] * beta : y[yl];
  for (int64_t c = cptr[w]; c < cptr[w + 1]; ++c) acc = acc + part[c];
  y[yl] = acc;
  if (dotp) {
    using DA = typename DAcc<T>::type;
    reinterpret_cast<DA*>(dotp)[dot_base + w] = dacc(cdot(dotu[r], acc));
  }
}

template <typename T, bool ALPHA, int BMODE>
static void long_t(const pa_mat* A, const void* x, void* y, const int32_t* ymap, const void* alpha, const void* beta,
                   void* dotp, int64_t dot_base, hipStream_t st) {
  const T* val = (const T*)A->d_val + A->long_off;
  const T al = *(const T*)alpha, be = *(const T*)beta;
  if (knobs().long_exact) {
    hipLaunchKernelGGL((k_spmv_long_exact<T, ALPHA, BMODE>), dim3((unsigned)A->n_long), dim3(64), 0, st, A->n_long,
                       A->d_long_row, A->d_long_ptr, A->d_long_col, val, (const T*)x, (T*)y, ymap, al, A->csr, be,
                       (const T*)x, dotp, dot_base);
  } else {
    hipLaunchKernelGGL((k_spmv_long_chunks<T, ALPHA>), dim3((unsigned)((A->n_lchunks + 3) / 4)), dim3(256), 0, st,
                       A->n_lchunks, A->d_lchunk_start, A->d_lchunk_start + 1, A->d_long_col, val, (const T*)x, al,
                       A->csr, (T*)A->d_lpart);
    hipLaunchKernelGGL((k_spmv_long_fold<T, BMODE>), dim3((unsigned)((A->n_long + 63) / 64)), dim3(64), 0, st,
                       A->n_long, A->d_long_row, A->d_lrow_chunk, (const T*)A->d_lpart, (T*)y, ymap, be,
                       (const T*)x, dotp, dot_base);
  }
}

template <typename T>
static void long_ab(const pa_mat* A, const void* x, void* y, const int32_t* ymap, bool has_alpha, int bmode,
                    const void* alpha, const void* beta, void* dotp, int64_t dot_base, hipStream_t st) {
#define PA_L(AL, BM) long_t<T, AL, BM>(A, x, y, ymap, alpha, beta, dotp, dot_base, st)
  if (!has_alpha) {
    if (bmode == 0) PA_L(false, 0); else if (bmode == 1) PA_L(false, 1); else PA_L(false, 2);
  } else {
    if (bmode == 0) PA_L(true, 0); else if (bmode == 1) PA_L(true, 1); else PA_L(true, 2);
  }
#undef PA_L
}

// dotp: partial of long row w at dotp[dot_base + w] (the fused CG dot)
#if defined(PA_SPMV_DT)
void PA_CAT(spmv_long_, PA_SPMV_DT)(const pa_mat* A, const void* x, void* y, const int32_t* ymap, bool has_alpha,
                                    int bmode, const void* alpha, const void* beta, void* dotp, int64_t dot_base,
                                    hipStream_t st) {
  long_ab<DtT>(A, x, y, ymap, has_alpha, bmode, alpha, beta, dotp, dot_base, st);
}
void PA_CAT(spmv_part_, PA_SPMV_DT)(int which, int64_t nwork, const int32_t* list, const pa_mat* A, const void* x,
                                    void* y, const int32_t* ymap, bool has_alpha, int bmode, const void* alpha,
                                    const void* beta, void* dotp, hipStream_t st, const SpmvPart* cgp) {
  if constexpr (kDtR2) {
    if (A->R == 2) {
      launch_which<DtT, 2>(which, nwork, list, A, x, y, ymap, has_alpha, bmode, alpha, beta, dotp, st, cgp);
      return;
    }
  }
  launch_which<DtT, kDtR>(which, nwork, list, A, x, y, ymap, has_alpha, bmode, alpha, beta, dotp, st, cgp);
}
#else
// dotp: partial of long row w at dotp[dot_base + w] (the fused CG dot)
void launch_spmv_long(const pa_mat* A, const void* x, void* y, const int32_t* ymap, bool has_alpha, int bmode,
                      const void* alpha, const void* beta, void* dotp, int64_t dot_base, hipStream_t st) {
  if (A->n_long <= 0) return;
#define spmv_long_(k) spmv_long_##k(A, x, y, ymap, has_alpha, bmode, alpha, beta, dotp, dot_base, st)
  switch (A->dtype) {
    case PA_F32: spmv_long_(0); break;
    case PA_F64: spmv_long_(1); break;
    case PA_C64: spmv_long_(2); break;
    case PA_C128: spmv_long_(3); break;
  }
#undef spmv_long_
}

void launch_spmv_part(int which, int64_t nwork, const int32_t* list, const pa_mat* A, const void* x,
                      void* y, const int32_t* ymap, bool has_alpha, int bmode, const void* alpha,
                      const void* beta, void* dotp, hipStream_t st, const SpmvPart* cgp) {
  // a slice list as long as the structure is 0..nslices-1 (lists are
  // ascending subsets): launch without it, one dependent load less per wave
  if ((knobs().spmv_flags & SPMV_IDLIST) && list && which != 2 && which != 5 && nwork == A->nslices) list = nullptr;
#define spmv_part_(k) spmv_part_##k(which, nwork, list, A, x, y, ymap, has_alpha, bmode, alpha, beta, dotp, st, cgp)
  switch (A->dtype) {
    case PA_F32: spmv_part_(0); break;
    case PA_F64: spmv_part_(1); break;
    case PA_C64: spmv_part_(2); break;
    case PA_C128: spmv_part_(3); break;
  }
#undef spmv_part_
}
#endif

#if PA_DT_DEFINE  // ---- everything below: the dispatcher translation unit only

// x .+= α.*u; r .-= α.*c (all lids, Interfaces.jl:1710-1737) and the owned
// Σ|r|² of norm(r) (1767-1772) in one pass (contiguous owned lids
// 0..noids-1); per-block partials, folded in block order afterwards.  α is
// Float64 (ComplexF64 for complex T) as in IterativeSolvers: each element
// is evaluated in that wide type and rounded to T once.  V elements per
// 16 B access (V = 1: unaligned fallback).  DEV: α comes from the device CG
// state (pa_cg_solve_all), x is left alone (its update is deferred into the
// next k_cg_xu, which reads u anyway) and a finished solve is a no-op.
template <typename T, int V, bool DEV>
__global__ __launch_bounds__(256) void k_cg_xr(int64_t n, int64_t noids, T* __restrict__ x, T* __restrict__ r,
                                               const T* __restrict__ u, const T* __restrict__ c,
                                               typename wide_of<T>::type alpha, const CGState* __restrict__ st,
                                               double* __restrict__ part) {
  using W = typename wide_of<T>::type;
  if (DEV) {
    if (st->done) return;
    alpha = cg_alpha_of<W>(st);
  }
  using P = Pack<T, V>;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nv = n / V;
  double s = 0.0;
  for (int64_t j = t; j < nv; j += stride) {
    if (!DEV) {
      P xv = reinterpret_cast<const P*>(x)[j];
      const P uv = reinterpret_cast<const P*>(u)[j];
#pragma unroll
      for (int e = 0; e < V; ++e) xv.v[e] = narrow<T>(widen(xv.v[e]) + alpha * widen(uv.v[e]));
      reinterpret_cast<P*>(x)[j] = xv;
    }
    P rv = reinterpret_cast<const P*>(r)[j];
    // c's last read in the iteration: non-temporal (with r's in k_cg_xu, CG
    // 0.8952 -> 0.8558 ms, profiles/r04/ad/)
    const P cv = ld<true>(&reinterpret_cast<const P*>(c)[j]);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      rv.v[e] = narrow<T>(widen(rv.v[e]) - alpha * widen(cv.v[e]));
      if (j * V + e < noids) s = s + (double)abs2(rv.v[e]);
    }
    reinterpret_cast<P*>(r)[j] = rv;
  }
  for (int64_t i = nv * V + t; i < n; i += stride) {
    if (!DEV) x[i] = narrow<T>(widen(x[i]) + alpha * widen(u[i]));
    const T ri = narrow<T>(widen(r[i]) - alpha * widen(c[i]));
    r[i] = ri;
    if (i < noids) s = s + (double)abs2(ri);
  }
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_down(s, d, 64);
  __shared__ double sm[4];
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((sm[0] + sm[1]) + sm[2]) + sm[3];
}

template <typename T>
static void cg_xr_t(int64_t n, int64_t noids, void* x, void* r, const void* u, const void* c,
                    const void* alpha, const CGState* st, double* part, int nb, hipStream_t st_) {
  using W = typename wide_of<T>::type;
  constexpr int V = 16 / sizeof(T);
  const bool aligned = ((uintptr_t)x | (uintptr_t)r | (uintptr_t)u | (uintptr_t)c) % 16 == 0;
  const W a = alpha ? *(const W*)alpha : zero_of<W>();
#define PA_XR(VV, DD)                                                                                  \
  hipLaunchKernelGGL((k_cg_xr<T, VV, DD>), dim3(nb), dim3(256), 0, st_, n, noids, (T*)x, (T*)r,      \
                     (const T*)u, (const T*)c, a, st, part)
  if (st) {
    if (aligned) PA_XR(V, true); else PA_XR(1, true);
  } else {
    if (aligned) PA_XR(V, false); else PA_XR(1, false);
  }
#undef PA_XR
}

// alpha: host scalar in the wide type (st == nullptr) or read from the device CG state
void launch_cg_xr(int dtype, int64_t n, int64_t noids, const int32_t* own, void* x, void* r, const void* u,
                  const void* c, const void* alpha, const CGState* st, double* part, int nb, hipStream_t s) {
  (void)own;  // owned lids are 0..noids-1 (checked by the caller)
  switch (dtype) {
    case PA_F32: cg_xr_t<float>(n, noids, x, r, u, c, alpha, st, part, nb, s); break;
    case PA_F64: cg_xr_t<double>(n, noids, x, r, u, c, alpha, st, part, nb, s); break;
    case PA_C64: cg_xr_t<c64>(n, noids, x, r, u, c, alpha, st, part, nb, s); break;
    case PA_C128: cg_xr_t<c128>(n, noids, x, r, u, c, alpha, st, part, nb, s); break;
  }
}

// ---------------------------------------------------------------------------
// Device-driven CG scalars (pa_cg_solve_all).  The same arithmetic as the
// host-driven loop (pvector.cg_ over pa_spmv_dot_all / pa_cg_update_all),
// on one thread, so the device recurrence equals it bit for bit.

// u .= r .+ β.*u over all lids, β = residual²/prev_residual² (Float64,
// IterativeSolvers 0.9 cg iterate; Real * Complex componentwise), preceded
// per element by the previous iteration's deferred x .+= α.*u (while it >
// xit: α is still that iteration's, u not yet overwritten).  Each element in
// the wide type, rounded to T once.  V elements per 16 B access (V = 1:
// unaligned fallback).
template <typename T, int V>
__global__ __launch_bounds__(256) void k_cg_xu(int64_t n, T* __restrict__ x, T* __restrict__ u,
                                               const T* __restrict__ r, const CGState* __restrict__ st) {
  using W = typename wide_of<T>::type;
  const bool xpend = st->it > st->xit;
  const bool upd = !st->done;
  if (!xpend && !upd) return;
  const W a = cg_alpha_of<W>(st);
  const double b = (st->res * st->res) / (st->prev * st->prev);
  using P = Pack<T, V>;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nv = n / V;
  for (int64_t j = t; j < nv; j += stride) {
    P uv = reinterpret_cast<const P*>(u)[j];
    if (xpend) {  // x is next read one iteration later: non-temporal (CG 0.9234 -> 0.895 ms, profiles/r04/ab/)
      P xv = ld<true>(&reinterpret_cast<const P*>(x)[j]);
#pragma unroll
      for (int e = 0; e < V; ++e) xv.v[e] = narrow<T>(widen(xv.v[e]) + a * widen(uv.v[e]));
      if constexpr (sizeof(P) == 16) {
        spmv_u32x4 w;
        __builtin_memcpy(&w, &xv, 16);
        __builtin_nontemporal_store(w, reinterpret_cast<spmv_u32x4*>(x) + j);
      } else {
        reinterpret_cast<P*>(x)[j] = xv;
      }
    }
    if (upd) {
      const P rv = ld<true>(&reinterpret_cast<const P*>(r)[j]);  // r is next read after the SpMV's stream
#pragma unroll
      for (int e = 0; e < V; ++e) uv.v[e] = narrow<T>(widen(rv.v[e]) + rscale(b, widen(uv.v[e])));
      reinterpret_cast<P*>(u)[j] = uv;
    }
  }
  for (int64_t i = nv * V + t; i < n; i += stride) {
    const T ui = u[i];
    if (xpend) x[i] = narrow<T>(widen(x[i]) + a * widen(ui));
    if (upd) u[i] = narrow<T>(widen(r[i]) + rscale(b, widen(ui)));
  }
}

// Julia's inv(::ComplexF64) (base/complex.jl, the scaled Smith algorithm):
// Float64 / ComplexF64 is a * inv(z), componentwise.
__host__ __device__ inline c128 julia_inv(c128 w) {
  double c = w.re, d = w.im;
  if (isinf(c) || isinf(d)) return c128{copysign(0.0, c), signbit(d) ? 0.0 : -0.0};  // flipsign(-0.0, d)
  const double half = 0.5, two = 2.0;
  const double cd = fmax(fabs(c), fabs(d));
  const double ov = 1.7976931348623157e308, un = 2.2250738585072014e-308, eps = 2.220446049250313e-16;
  const double bs = two / (eps * eps);
  double s = 1.0;
  if (cd >= half * ov) { c = half * c; d = half * d; s = s * half; }
  if (cd <= un * two / eps) { c = c * bs; d = d * bs; s = s * bs; }
  double p, q;
  if (fabs(d) <= fabs(c)) {
    const double r = d / c;
    const double t = 1.0 / (c + d * r);
    p = t;
    q = -r * t;
  } else {
    const double c2 = d, d2 = c;
    const double r = d2 / c2;
    const double t = 1.0 / (c2 + d2 * r);
    p = r * t;
    q = -t;
  }
  return c128{p * s, q * s};
}

// the dot partials of the P parts (accumulators, part order) → dot =
// reduce(+; init=0) over the part values in T (each part's value rounded to
// T: Julia's local dot returns T) → α = residual² / dot in Float64 /
// ComplexF64.  It also records that the previous iteration's x update has
// been applied (k_cg_xu ran before this iteration's SpMV).
template <typename T>
__device__ inline void cg_alpha(int P, const void* __restrict__ gathered, CGState* __restrict__ st) {
  st->xit = st->it;
  if (st->done) return;
  const double res2 = st->res * st->res;
  if constexpr (std::is_same<T, float>::value || std::is_same<T, double>::value) {
    const double* g = (const double*)gathered;
    T s = (T)0;
    for (int p = 0; p < P; ++p) s = s + (T)g[p];
    st->alpha = c128{res2 / (double)s, 0.0};
  } else {
    const c128* g = (const c128*)gathered;
    T s = zero_of<T>();
    for (int p = 0; p < P; ++p) s = s + narrow<T>(g[p]);
    st->alpha = rscale(res2, julia_inv(widen(s)));
  }
}

template <typename T>
__global__ void k_cg_alpha(int P, const void* __restrict__ gathered, CGState* __restrict__ st) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  cg_alpha<T>(P, gathered, st);
}

// Σ|r|² partials of the P parts → prev = residual; residual = sqrt(Σ);
// it += 1; history[it] = residual; done = it >= maxiter || residual <= tol.
// F32 (Float32 / ComplexF32 vectors): each part's norm(r)^2 is a Float32 and
// their reduce(+) runs in Float32 before the Float64 ^(1/2) (Interfaces.jl:
// 1767-1772).
template <bool F32>
__device__ inline void cg_step(int P, const double* __restrict__ gathered, CGState* __restrict__ st,
                               double* __restrict__ history) {
  if (st->done) return;
  double s;
  if (F32) {
    float f = 0.f;
    for (int p = 0; p < P; ++p) f = f + (float)gathered[p];
    s = (double)f;
  } else {
    s = 0.0;
    for (int p = 0; p < P; ++p) s = s + gathered[p];
  }
  const double res = sqrt(s);
  st->prev = st->res;
  st->res = res;
  const int64_t it = st->it + 1;
  st->it = it;
  if (history) history[it - 1] = res;
  st->done = (it >= st->maxiter || res <= st->tol) ? 1 : 0;
}

template <bool F32>
__global__ void k_cg_step(int P, const double* __restrict__ gathered, CGState* __restrict__ st,
                          double* __restrict__ history) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  cg_step<F32>(P, gathered, st, history);
}

// One part in one process: the fold of the part's partials ends in the
// scalar update itself (no gather, no extra launch).
template <typename T>
struct AlphaTail {
  CGState* st;
  __device__ void operator()(const void* out) const { cg_alpha<T>(1, out, st); }
};
template <bool F32>
struct StepTail {
  CGState* st;
  double* hist;
  __device__ void operator()(const void* out) const { cg_step<F32>(1, (const double*)out, st, hist); }
};

// gathered[p] = *srcs[p] (accsz bytes each): the part values of the parts
// held by this process, read straight from their devices
__global__ void k_gather_ptrs(int P, const void* const* __restrict__ srcs, int accsz, char* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const double* s = (const double*)srcs[p];
  double* d = (double*)(out + (int64_t)p * accsz);
  d[0] = s[0];
  if (accsz == 16) d[1] = s[1];
}

// dsts[d][p] = *srcs[p] for every destination d (accsz bytes each): the
// part values gathered once and written to every local part's d_gather (peer
// stores across the devices of one process), the device CG's one-kernel
// all-gather (pa_api.cpp cg_gather)
__global__ void k_gather_scatter(int P, const void* const* __restrict__ srcs, int accsz, int nd,
                                 void* const* __restrict__ dsts) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)P * nd) return;
  const int p = (int)(t % P), d = (int)(t / P);
  const double* s = (const double*)srcs[p];
  double* o = (double*)((char*)dsts[d] + (int64_t)p * accsz);
  o[0] = s[0];
  if (accsz == 16) o[1] = s[1];
}

template <typename T>
static void cg_xu_t(int64_t n, void* x, void* u, const void* r, const CGState* st, hipStream_t s) {
  constexpr int V = 16 / sizeof(T);
  const bool aligned = ((uintptr_t)x | (uintptr_t)u | (uintptr_t)r) % 16 == 0;
  const int64_t nw = aligned ? (n + V - 1) / V : n;
  const int nb = (int)std::min<int64_t>(8192, std::max<int64_t>(1, (nw + 255) / 256));
  if (aligned) hipLaunchKernelGGL((k_cg_xu<T, V>), dim3(nb), dim3(256), 0, s, n, (T*)x, (T*)u, (const T*)r, st);
  else hipLaunchKernelGGL((k_cg_xu<T, 1>), dim3(nb), dim3(256), 0, s, n, (T*)x, (T*)u, (const T*)r, st);
}

// The fused CG's ghost lids [lo, hi) (after the halo of r): u_new = r .+
// β.*u_old (while the solve runs) and the deferred x .+= α.*u_old (while
// it > xit) — k_cg_xu's arithmetic on the lids the SpMV waves do not own.
template <typename T>
__global__ __launch_bounds__(256) void k_cg_ghost(int64_t lo, int64_t hi, const T* __restrict__ r,
                                                  const T* __restrict__ uo, T* __restrict__ un, T* __restrict__ x,
                                                  const CGState* __restrict__ st) {
  using W = typename wide_of<T>::type;
  const bool xpend = st->it > st->xit;
  const bool upd = !st->done;
  if (!xpend && !upd) return;
  const W a = cg_alpha_of<W>(st);
  const double b = (st->res * st->res) / (st->prev * st->prev);
  for (int64_t i = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < hi; i += (int64_t)gridDim.x * blockDim.x) {
    const T ui = uo[i];
    if (upd) un[i] = narrow<T>(widen(r[i]) + rscale(b, widen(ui)));
    if (xpend) x[i] = narrow<T>(widen(x[i]) + a * widen(ui));
  }
}

void launch_cg_ghost(int dtype, int64_t lo, int64_t hi, const void* r, const void* uo, void* un, void* x,
                     const CGState* st, hipStream_t s) {
  if (hi <= lo) return;
  const int nb = (int)std::min<int64_t>(1024, (hi - lo + 255) / 256);
#define PA_CGG(T) hipLaunchKernelGGL(k_cg_ghost<T>, dim3(nb), dim3(256), 0, s, lo, hi, (const T*)r, (const T*)uo, \
                                     (T*)un, (T*)x, st)
  switch (dtype) {
    case PA_F32: PA_CGG(float); break;
    case PA_F64: PA_CGG(double); break;
    case PA_C64: PA_CGG(c64); break;
    case PA_C128: PA_CGG(c128); break;
  }
#undef PA_CGG
}

void launch_cg_xu(int dtype, int64_t n, void* x, void* u, const void* r, const CGState* st, hipStream_t s) {
  switch (dtype) {
    case PA_F32: cg_xu_t<float>(n, x, u, r, st, s); break;
    case PA_F64: cg_xu_t<double>(n, x, u, r, st, s); break;
    case PA_C64: cg_xu_t<c64>(n, x, u, r, st, s); break;
    case PA_C128: cg_xu_t<c128>(n, x, u, r, st, s); break;
  }
}

void launch_cg_alpha(int dtype, int P, const void* gathered, CGState* st, hipStream_t s) {
  switch (dtype) {
    case PA_F32: hipLaunchKernelGGL(k_cg_alpha<float>, dim3(1), dim3(64), 0, s, P, gathered, st); break;
    case PA_F64: hipLaunchKernelGGL(k_cg_alpha<double>, dim3(1), dim3(64), 0, s, P, gathered, st); break;
    case PA_C64: hipLaunchKernelGGL(k_cg_alpha<c64>, dim3(1), dim3(64), 0, s, P, gathered, st); break;
    case PA_C128: hipLaunchKernelGGL(k_cg_alpha<c128>, dim3(1), dim3(64), 0, s, P, gathered, st); break;
  }
}

void launch_cg_step(int dtype, int P, const double* gathered, CGState* st, double* history, hipStream_t s) {
  if (dtype == PA_F32 || dtype == PA_C64)
    hipLaunchKernelGGL(k_cg_step<true>, dim3(1), dim3(64), 0, s, P, gathered, st, history);
  else
    hipLaunchKernelGGL(k_cg_step<false>, dim3(1), dim3(64), 0, s, P, gathered, st, history);
}

// fold the SpMV's dot partials into out, then α (one part per process)
void launch_fold_cg_alpha(int dtype, int nb, const void* in, void* scratch, void* out, unsigned* ticket,
                          CGState* st, hipStream_t s) {
  switch (dtype) {
    case PA_F32:
      fold_launch<double>(nb, (const double*)in, (double*)scratch, (double*)out, ticket, AlphaTail<float>{st}, s);
      break;
    case PA_F64:
      fold_launch<double>(nb, (const double*)in, (double*)scratch, (double*)out, ticket, AlphaTail<double>{st}, s);
      break;
    case PA_C64:
      fold_launch<c128>(nb, (const c128*)in, (c128*)scratch, (c128*)out, ticket, AlphaTail<c64>{st}, s);
      break;
    case PA_C128:
      fold_launch<c128>(nb, (const c128*)in, (c128*)scratch, (c128*)out, ticket, AlphaTail<c128>{st}, s);
      break;
  }
}

// fold the Σ|r|² partials into out, then the residual step
void launch_fold_cg_step(int dtype, int nb, const void* in, void* scratch, void* out, unsigned* ticket,
                         CGState* st, double* history, hipStream_t s) {
  if (dtype == PA_F32 || dtype == PA_C64)
    fold_launch<double>(nb, (const double*)in, (double*)scratch, (double*)out, ticket, StepTail<true>{st, history}, s);
  else
    fold_launch<double>(nb, (const double*)in, (double*)scratch, (double*)out, ticket, StepTail<false>{st, history}, s);
}

void launch_gather_ptrs(int P, const void* const* srcs, int accsz, void* out, hipStream_t s) {
  hipLaunchKernelGGL(k_gather_ptrs, dim3((P + 63) / 64), dim3(64), 0, s, P, srcs, accsz, (char*)out);
}

void launch_gather_scatter(int P, const void* const* srcs, int accsz, int nd, void* const* dsts, hipStream_t s) {
  const int64_t n = (int64_t)P * nd;
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_scatter, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, srcs, accsz, nd, dsts);
}

// ---------------------------------------------------------------------------
// Pattern detection (one wave per slice).  Candidate 0: the middle valid row
// of the slice (or the row at 1/4 or 3/4 when more rows follow that one); its
// offsets pat[k] = col_k - row.  A row is regular for a
// candidate when its column sequence is exactly row + pat[k] (same length).
// The slice becomes a pattern slice when at least pattern_min_regular % of its rows are regular
// (the others go to the side SELL).

template <int R>
__global__ __launch_bounds__(256) void k_pattern_detect(int64_t nrows, int64_t nslices, int min_pct,
                                                        const int64_t* __restrict__ soff,
                                                        const int32_t* __restrict__ slen,
                                                        const int32_t* __restrict__ col, int64_t noids, int kmax,
                                                        int32_t* __restrict__ kind,
                                                        int32_t* __restrict__ plen,
                                                        int32_t* __restrict__ pat,
                                                        uint64_t* __restrict__ mask,
                                                        int32_t* __restrict__ pghost,
                                                        int32_t* __restrict__ nirreg) {
  constexpr int H = 64 * R;
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nslices) return;
  auto oid = [&](int ln, int r) -> int64_t { return s * H + (int64_t)ln * R + r; };
  const int64_t off = soff[s];
  const int L = slen[s];
  const int64_t rem = nrows - s * H;
  const int nvalid = (int)(rem < H ? rem : H);
  // candidate row length (entries before its first padding slot)
  auto cand_len = [&](int clane, int cr) {
    int l = 0;
    for (int k = 0; k < L; ++k) {
      if (col[off + ((int64_t)k * 64 + clane) * R + cr] < 0) break;
      ++l;
    }
    return l;
  };
  int mlane = (nvalid / 2) / R, mr = (nvalid / 2) % R;
  int Lp = cand_len(mlane, mr);
  // row lengths (entries before the first padding slot) and ghost columns
  int rlen[R];
  bool ghost_any = false;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = lane * R + r;
    const bool valid = i < nvalid;
    int l = 0;
    bool pad = false;
    for (int k = 0; k < L; ++k) {
      const int32_t c = col[off + ((int64_t)k * 64 + lane) * R + r];
      if (c < 0) pad = true;
      else if (pad) l = -(1 << 30);  // a column after padding: never regular
      else ++l;
      if (valid && c >= noids) ghost_any = true;
    }
    rlen[r] = valid ? l : -1;
  }
  // rows of this lane regular for candidate (clane, cr): bit r; g = reads a ghost
  auto follow = [&](int clane, int cr, bool& g) -> unsigned {
    const int64_t crow = oid(clane, cr);
    unsigned bits = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t row = oid(lane, r);
      bool reg = Lp > 0 && rlen[r] == Lp;
      bool gr = false;
      for (int k = 0; k < Lp; ++k) {
        const int32_t cm = col[off + ((int64_t)k * 64 + clane) * R + cr];
        const int32_t c = col[off + ((int64_t)k * 64 + lane) * R + r];
        const int64_t e = row + (int64_t)(cm - crow);
        if ((int64_t)c != e) reg = false;
        if (e >= noids) gr = true;
      }
      if (reg) {
        bits |= 1u << r;
        g = g || gr;
      }
    }
    return bits;
  };
  auto wave_count = [&](unsigned bits) {
    int t = __popc(bits);
    for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d, 64);
    return t;
  };
  bool g1 = false;
  unsigned bits1 = follow(mlane, mr, g1);
  int tot1 = wave_count(bits1);
  // the middle row may be an exception (a slice of several grid lines: the
  // first row of the second line); the rows at 1/4 and 3/4 are candidates too,
  // the one most rows follow wins (ties keep the earlier)
  if (tot1 < nvalid && nvalid >= 4) {
    for (int q = 1; q <= 3; q += 2) {
      const int m = q * nvalid / 4;
      const int cl = m / R, cr = m % R;
      const int keepL = Lp;
      Lp = cand_len(cl, cr);
      bool g = false;
      const unsigned b = follow(cl, cr, g);
      const int t = wave_count(b);
      if (t > tot1) {
        mlane = cl; mr = cr; bits1 = b; tot1 = t; g1 = g;
      } else {
        Lp = keepL;
      }
    }
  }
  // a pattern slice when at least min_pct % of its rows follow the pattern
  // (pa_tune pattern_min_regular, default 70 / 50 for Float32; the others go to the side
  // SELL) and its rows have at most 255 entries (the length has 8 bits)
  const bool best = Lp > 0 && Lp <= 255 && 100 * tot1 >= min_pct * nvalid;
  const bool gr = __any(g1);
  const bool ga = __any(ghost_any);
  if (lane == 0) {
    kind[s] = best ? 1 : 0;
    plen[s] = best ? Lp : L;
    pghost[s] = best ? (gr ? 1 : 0) : (ga ? 1 : 0);
    nirreg[s] = best ? nvalid - tot1 : 0;
  }
  if (best && bits1) {
    const int i0 = lane * R;
    atomicOr((unsigned long long*)&mask[s * (H / 64) + i0 / 64], (unsigned long long)bits1 << (i0 & 63));
  }
  if (best) {
    const int64_t crow = oid(mlane, mr);
    for (int k = lane; k < Lp; k += 64) pat[s * kmax + k] = col[off + ((int64_t)k * 64 + mlane) * R + mr] - (int32_t)crow;
  }
}

// delta16 eligibility and codes, one wave per slice: an int32-column slice
// (kind 0, no long rows) becomes delta16 when every owned column is within
// ±16383 of its row and every ghost column within 32766 of the slice's
// smallest ghost column.  Float32 slices' rows are then re-laid out
// interleaved (row w of the slice at lane w % 64, position w / 64, instead
// of lane w / R, position w % R), values and int32 ids moved in place,
// block k by block k; the codes go to col16 in the (new) slots: a gather
// instruction then reads x for 64 consecutive rows (a coalesced span)
// instead of 64 rows R apart.
template <int R>
__global__ __launch_bounds__(256) void k_delta16(int64_t nslices, const int64_t* __restrict__ soff,
                                                 const int32_t* __restrict__ slen, int32_t* __restrict__ col,
                                                 const int32_t* __restrict__ kind, const int32_t* __restrict__ sflags,
                                                 int64_t noids, uint16_t* __restrict__ col16,
                                                 int32_t* __restrict__ gbase, int32_t* __restrict__ ok,
                                                 unsigned char* __restrict__ val) {
  typedef typename RawOf<16 / R>::type E;  // one value (R values = 16 B per lane)
  constexpr int H = 64 * R;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nslices) return;
  const int lane = threadIdx.x & 63;
  if (kind[s] != 0 || (sflags && sflags[s])) {
    if (lane == 0) { ok[s] = 0; gbase[s] = 0; }
    return;
  }
  const int64_t off = soff[s];
  const int len = slen[s];
  const int64_t row0 = s * H + (int64_t)lane * R;
  int32_t gmin = INT32_MAX;
  for (int k = 0; k < len; ++k)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int32_t c = col[off + ((int64_t)k * 64 + lane) * R + r];
      if (c >= noids) gmin = min(gmin, c);
    }
  for (int d = 32; d >= 1; d >>= 1) gmin = min(gmin, __shfl_xor(gmin, d, 64));
  bool fit = true;
  for (int k = 0; k < len; ++k)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int32_t c = col[off + ((int64_t)k * 64 + lane) * R + r];
      if (c < 0) continue;
      if (c < noids) {
        const int64_t dlt = (int64_t)c - (row0 + r);
        fit = fit && dlt >= -16384 && dlt <= 16383;
      } else {
        fit = fit && (int64_t)c - gmin <= 32766;
      }
    }
  const bool all = __all(fit);
  if (lane == 0) { ok[s] = all ? 1 : 0; gbase[s] = gmin == INT32_MAX ? 0 : gmin; }
  if (!all) return;
  for (int k = 0; k < len; ++k) {
    // block k (64*R slots) in registers first: every lane's loads of the
    // block are issued before any lane stores into it
    int32_t c[R];
    E v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t slot = off + ((int64_t)k * 64 + lane) * R + r;
      c[r] = col[slot];
      v[r] = reinterpret_cast<const E*>(val)[slot];
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int w = lane * R + r;  // the row within the slice
      const int64_t slot = kInterleaveD16<R> ? off + ((int64_t)k * 64 + (w & 63)) * R + (w >> 6)
                                             : off + ((int64_t)k * 64 + lane) * R + r;
      uint16_t q;
      if (c[r] < 0) q = 0xFFFFu;
      else if (c[r] < noids) q = (uint16_t)((uint32_t)(c[r] - (int32_t)(row0 + r)) & 0x7FFFu);
      else q = (uint16_t)(0x8000u | (uint32_t)(c[r] - gmin));
      col16[slot] = q;
      if (kInterleaveD16<R>) {
        col[slot] = c[r];
        reinterpret_cast<E*>(val)[slot] = v[r];
      }
    }
  }
}

void launch_delta16(pa_mat* A, int64_t noids, const int32_t* kind, int32_t* ok, hipStream_t st) {
  const int64_t blocks = (A->nslices + 3) / 4;
  if (blocks == 0) return;
#define PA_D16(RR)                                                                                          \
  hipLaunchKernelGGL(k_delta16<RR>, dim3(blocks), dim3(256), 0, st, A->nslices, A->d_slice_off,              \
                     A->d_slice_len, A->d_col, kind, A->d_sflags, noids, A->d_col16, A->d_gbase, ok,  \
                     (unsigned char*)A->d_val)
  switch (A->R) {
    case 1: PA_D16(1); break;
    case 2: PA_D16(2); break;
    case 4: PA_D16(4); break;
  }
#undef PA_D16
}

void launch_pattern_detect(pa_mat* A, int64_t noids, int min_pct, int32_t* kind, int32_t* plen, int32_t* pat,
                           uint64_t* mask, int32_t* pghost, int32_t* nirreg, hipStream_t st) {
  const int64_t blocks = (A->nslices + 3) / 4;
  if (blocks == 0) return;
#define PA_DET(RR)                                                                                      \
  hipLaunchKernelGGL(k_pattern_detect<RR>, dim3(blocks), dim3(256), 0, st, A->nrows, A->nslices, min_pct, \
                     A->d_slice_off, A->d_slice_len, A->d_col, noids, A->kmax, kind, plen, pat, mask,  \
                     pghost, nirreg)
  switch (A->R) {
    case 1: PA_DET(1); break;
    case 2: PA_DET(2); break;
    case 4: PA_DET(4); break;
  }
#undef PA_DET
}

// Side SELL: the irregular rows (oids, ascending), copied from the int32 layout.
template <int R>
__global__ void k_side_len(int64_t n, const int32_t* __restrict__ rows, const int64_t* __restrict__ soff,
                           const int32_t* __restrict__ slen, const int32_t* __restrict__ col,
                           int32_t* __restrict__ len, int64_t noids, int32_t* __restrict__ sghost, int sH) {
  constexpr int H = 64 * R;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t row = rows[i];
  const int64_t s = row / H;
  const int w = (int)(row - s * H);
  const int lane = w / R, r = w % R;
  int l = 0;
  bool g = false;
  for (int k = 0; k < slen[s]; ++k) {
    const int32_t c = col[soff[s] + ((int64_t)k * 64 + lane) * R + r];
    if (c < 0) break;
    if (c >= noids) g = true;
    ++l;
  }
  len[i] = l;
  if (g) atomicOr(&sghost[i / sH], 1);
}

template <typename T, int R>
__global__ void k_side_fill(int64_t n, const int32_t* __restrict__ rows, const int64_t* __restrict__ soff,
                            const int32_t* __restrict__ col, const T* __restrict__ val,
                            const int64_t* __restrict__ s_off, const int32_t* __restrict__ s_len,
                            const int32_t* __restrict__ len, int32_t* __restrict__ s_col,
                            T* __restrict__ s_val, int64_t s_nslices) {
  constexpr int H = 64 * R;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= s_nslices * H) return;
  const int64_t ss = i / H;
  const int wi = (int)(i - ss * H);
  const int sl = wi / R, sr = wi % R;
  int l = 0;
  int64_t base = 0;
  int lane = 0, r = 0;
  if (i < n) {
    const int64_t row = rows[i];
    const int64_t s = row / H;
    const int w = (int)(row - s * H);
    lane = w / R;
    r = w % R;
    l = len[i];
    base = soff[s];
  }
  for (int k = 0; k < s_len[ss]; ++k) {
    const int64_t dst = s_off[ss] + ((int64_t)k * 64 + sl) * R + sr;
    if (k < l) {
      const int64_t src = base + ((int64_t)k * 64 + lane) * R + r;
      s_col[dst] = col[src];
      s_val[dst] = val[src];
    } else {
      s_col[dst] = -1;
      s_val[dst] = zero_of<T>();
    }
  }
}

void launch_side_len(pa_mat* A, int64_t n, const int32_t* rows, int32_t* len, int64_t noids,
                     int32_t* sghost, hipStream_t st) {
  if (n == 0) return;
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  switch (A->R) {
    case 1: hipLaunchKernelGGL(k_side_len<1>, g, b, 0, st, n, rows, A->d_slice_off, A->d_slice_len, A->d_col, len, noids, sghost, A->H); break;
    case 2: hipLaunchKernelGGL(k_side_len<2>, g, b, 0, st, n, rows, A->d_slice_off, A->d_slice_len, A->d_col, len, noids, sghost, A->H); break;
    case 4: hipLaunchKernelGGL(k_side_len<4>, g, b, 0, st, n, rows, A->d_slice_off, A->d_slice_len, A->d_col, len, noids, sghost, A->H); break;
  }
}

template <typename T, int R>
static void side_fill_t(pa_mat* A, const int32_t* rows, const int32_t* len, hipStream_t st) {
  const int64_t tot = A->s_nslices * 64 * R;
  if (tot == 0) return;
  hipLaunchKernelGGL((k_side_fill<T, R>), dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st,
                     A->s_nrows, rows, A->d_slice_off, A->d_col, (const T*)A->d_val, A->d_s_off,
                     A->d_s_len, len, A->d_s_col, (T*)A->d_s_val, A->s_nslices);
}

void launch_side_fill(pa_mat* A, const int32_t* rows, const int32_t* len, hipStream_t st) {
  switch (A->dtype) {
    case PA_F32:
      if (A->R == 2) side_fill_t<float, 2>(A, rows, len, st);
      else side_fill_t<float, 4>(A, rows, len, st);
      break;
    case PA_F64: side_fill_t<double, 2>(A, rows, len, st); break;
    case PA_C64: side_fill_t<c64, 2>(A, rows, len, st); break;
    case PA_C128: side_fill_t<c128, 1>(A, rows, len, st); break;
  }
}

// ---------------------------------------------------------------------------
// Triple SELL build (pa_api.cpp build_triple_sell).  Main-layout slot of
// entry k of row w of slice s (after k_delta16): Float32 delta16 slices are
// interleaved (lane w % 64, position w / 64), the others blocked (lane
// w / R, position w % R).
template <int R>
__device__ __forceinline__ int64_t main_slot0(int64_t soff, int w) {
  return kInterleaveD16<R> ? soff + (int64_t)(w & 63) * R + (w >> 6) : soff + (int64_t)(w / R) * R + (w % R);
}

// per candidate row (oids of the delta16 slices): entries, consecutive
// triples (len % 3 == 0 and c[3t+1] = c[3t]+1, c[3t+2] = c[3t]+2), ghost
// reads; info = len | regular << 28 | ghost << 29 | bad << 30 (a column
// after padding: the layout is not one the triple SELL can take)
template <int R>
__global__ void k_t_rowinfo(int64_t n, const int32_t* __restrict__ rows, int H, const int64_t* __restrict__ soff,
                            const int32_t* __restrict__ slen, const int32_t* __restrict__ col, int64_t noids,
                            int32_t* __restrict__ info) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t row = rows[i], s = row / H;
  const int64_t b = main_slot0<R>(soff[s], (int)(row - s * H));
  const int L = slen[s];
  int len = 0;
  bool reg = true, ghost = false, pad = false, bad = false;
  int32_t prev = 0;
  for (int k = 0; k < L; ++k) {
    const int32_t c = col[b + (int64_t)k * 64 * R];
    if (c < 0) { pad = true; continue; }
    if (pad) bad = true;
    if (len % 3 != 0 && c != prev + 1) reg = false;
    ghost = ghost || c >= noids;
    prev = c;
    ++len;
  }
  reg = reg && len > 0 && len % 3 == 0;
  info[i] = len | (reg ? 1 << 28 : 0) | (ghost ? 1 << 29 : 0) | (bad ? 1 << 30 : 0);
}

// per candidate row i (oids of the delta16 slices, ascending): 1 when the
// next candidate is row + 1 and its columns are row i's plus one, entry for
// entry (a pair of the triple SELL's pair slices), else 0
template <int R>
__global__ void k_t_pairinfo(int64_t n, const int32_t* __restrict__ rows, int H, const int64_t* __restrict__ soff,
                             const int32_t* __restrict__ slen, const int32_t* __restrict__ col,
                             int32_t* __restrict__ pairable) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t ok = 0;
  if (i + 1 < n && rows[i + 1] == rows[i] + 1) {
    const int64_t ra = rows[i], rb = ra + 1, sa = ra / H, sb = rb / H;
    const int64_t ba = main_slot0<R>(soff[sa], (int)(ra - sa * H)), bb = main_slot0<R>(soff[sb], (int)(rb - sb * H));
    const int La = slen[sa], Lb = slen[sb];
    ok = 1;
    for (int k = 0; k < max(La, Lb); ++k) {
      const int32_t ca = k < La ? col[ba + (int64_t)k * 64 * R] : -1;
      const int32_t cb = k < Lb ? col[bb + (int64_t)k * 64 * R] : -1;
      if (ca < 0 && cb < 0) break;
      if (ca < 0 || cb != ca + 1) {
        ok = 0;
        break;
      }
    }
  }
  pairable[i] = ok;
}

// the uniform layout's values (build_uniform): one thread per (slice, entry
// < 8, lane) of the pattern slices; entry k of the slice's pattern goes to
// U's position emap[pattern id][k]
template <typename E, int R>
__global__ void k_u_fill(int64_t ns, int H, int K, const int32_t* __restrict__ kind, const int64_t* __restrict__ soff,
                         const int32_t* __restrict__ plen, const int32_t* __restrict__ emap,
                         const E* __restrict__ val, E* __restrict__ uval) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= ns * 8 * 64) return;
  const int64_t s = i / (8 * 64);
  const int k = (int)((i / 64) % 8), l = (int)(i % 64);
  if (kind[s] != 1) return;
  const int32_t lraw = plen[s];
  if (k >= (lraw & 0xff)) return;
  const int e = emap[(lraw >> 9) * 8 + k];
#pragma unroll
  for (int r = 0; r < R; ++r)
    uval[s * H * K + ((int64_t)e * 64 + l) * R + r] = val[soff[s] + ((int64_t)k * 64 + l) * R + r];
}

void launch_u_fill(const pa_mat* A, hipStream_t st) {
  const int64_t n = A->nslices * 8 * 64;
  if (n == 0 || !A->d_uval) return;
  hipLaunchKernelGGL((k_u_fill<double, 2>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A->nslices, A->H,
                     A->uK, A->d_kind, A->d_slice_off, A->d_plen, A->d_uemap, (const double*)A->d_val,
                     (double*)A->d_uval);
}

void launch_t_pairinfo(const pa_mat* A, int64_t n, const int32_t* rows, int32_t* pairable, hipStream_t st) {
  if (n == 0) return;
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
#define PA_TPI(RR) hipLaunchKernelGGL(k_t_pairinfo<RR>, g, b, 0, st, n, rows, A->H, A->d_slice_off, A->d_slice_len, \
                                      A->d_col, pairable)
  switch (A->R) {
    case 1: PA_TPI(1); break;
    case 2: PA_TPI(2); break;
    case 4: PA_TPI(4); break;
  }
#undef PA_TPI
}

// one wave per triple-SELL slice: the smallest ghost column of its rows
// (the ghost codes' base) and whether every ghost code fits 15 bits
template <int R>
__global__ __launch_bounds__(256) void k_t_gbase(int64_t ns, int64_t nrows, int H, const int32_t* __restrict__ rowlen,
                                                 const int64_t* __restrict__ src, const int32_t* __restrict__ col,
                                                 int64_t noids, int32_t* __restrict__ gbase, int32_t* __restrict__ ok) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= ns) return;
  const int lane = threadIdx.x & 63;
  int32_t gmin = INT32_MAX, gmax = -1;
  for (int w = lane; w < H; w += 64) {
    const int64_t i = s * H + w;
    if (i >= nrows) break;
    for (int k = 0; k < rowlen[i]; ++k) {
      const int32_t c = col[src[i] + (int64_t)k * 64 * R];
      if (c >= noids) { gmin = min(gmin, c); gmax = max(gmax, c); }
    }
  }
  for (int d = 32; d >= 1; d >>= 1) {
    gmin = min(gmin, __shfl_xor(gmin, d, 64));
    gmax = max(gmax, __shfl_xor(gmax, d, 64));
  }
  if (lane == 0) {
    gbase[s] = gmin == INT32_MAX ? 0 : gmin;
    ok[s] = gmin == INT32_MAX || (int64_t)gmax - gmin <= 32766;
  }
}

// Slot of code group g (triple g of a tri slice, entry g otherwise) of lane
// `lane`, row r, in a triple-SELL slice at code offset d, R codes per lane
// and triple.  Packed (pair slices, R = 1, rows_t16_pair): each full batch
// of B triples (9 for 4 B elements, 4 for 8 B) holds packs of 4 triples per
// lane, then single triples; a last batch of fewer triples keeps one code
// per triple, as unpacked slices do.
__device__ __forceinline__ int64_t t_code_slot(int64_t d, int g, int ntri, int lane, int r, int R, bool packed,
                                               int B) {
  const int b = g / B, i = g % B, nq = 4 * (B / 4);
  if (!packed || B * (b + 1) > ntri) return d + ((int64_t)g * 64 + lane) * R + r;
  const int64_t bb = d + (int64_t)b * B * 64 * R;
  return i < nq ? bb + (int64_t)(i / 4) * 4 * 64 * R + (int64_t)lane * 4 * R + (i % 4) * R + r
                : bb + (int64_t)i * 64 * R + (int64_t)lane * R + r;
}

// one thread per triple-SELL row: its values (and, with codes, its 16-bit
// codes relative to its oid: tri slices one per triple in code group t,
// the others one per entry) from the main layout; padding: value 0, code
// 0xFFFF.  values only (codes false): the refresh after new values.
template <typename E, int R>
__global__ void k_t_fill(int64_t nrows, int H, const int32_t* __restrict__ rowmap, const int32_t* __restrict__ rowlen,
                         const int64_t* __restrict__ src, const int64_t* __restrict__ toff,
                         const int32_t* __restrict__ tlen, const int32_t* __restrict__ gbase,
                         const int32_t* __restrict__ col, const E* __restrict__ val, int64_t noids, bool codes,
                         int pack, uint16_t* __restrict__ col16, E* __restrict__ tval) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= nrows) return;
  const int64_t ts = i / H;
  const int w = (int)(i - ts * H), lane = w & 63, r = w >> 6;
  if (rowmap[i] < 0) return;  // a padding position (memset: values 0, codes 0xFFFF)
  const int32_t lraw = tlen[ts];
  const int L = lraw & kTriLen;
  const bool tri = (lraw & kTriSlice) != 0, pair = (lraw & kTriPair) != 0;
  constexpr int B = sizeof(E) == 4 ? 9 : 4;  // rows_t16_tri's batches
  const int n = rowlen[i];
  const int64_t b = src[i], d = toff[ts];
  const int32_t oid = rowmap[i], gb = gbase[ts];
  for (int k = 0; k < L; ++k) {
    const int64_t sk = b + (int64_t)k * 64 * R;
    E v;
    __builtin_memset(&v, 0, sizeof(E));
    if (k < n) v = val[sk];
    if ((pack & 1) && pair && sizeof(E) == 4) {  // triple t: entries 3t, 3t+1 as one 2R-value pack per lane, entry 3t+2 as an R pack
      const int64_t tb = d + (int64_t)(k / 3) * 3 * 64 * R;
      const int j = k % 3;
      tval[j < 2 ? tb + (int64_t)lane * 2 * R + j * R + r : tb + 2 * 64 * R + (int64_t)lane * R + r] = v;
    } else {
      tval[d + ((int64_t)k * 64 + lane) * R + r] = v;
    }
    if (!codes || (tri && k % 3 != 0) || (pair && r != 0)) continue;  // pair slices: row a's codes
    uint16_t q = 0xFFFFu;
    if (k < n) {
      const int32_t c = col[sk];
      q = c < noids ? (uint16_t)((uint32_t)(c - oid) & 0x7FFFu) : (uint16_t)(0x8000u | (uint32_t)(c - gb));
    }
    const int g = tri ? k / 3 : k;
    col16[pair ? t_code_slot(d, g, L / 3, lane, 0, 1, true, B)
               : t_code_slot(d, g, L / 3, lane, r, R, false, B)] = q;
  }
}

// build check, one thread per row position of every slice (past the last
// row too): every code the SpMV will decode gives a column in [-1, ncols)
// (a tri slice's run c, c+1, c+2 inside x); *bad counts the others
__global__ void k_t_check(int64_t npos, int64_t nrows, int H, int R, const int32_t* __restrict__ rowmap,
                          const int64_t* __restrict__ toff, const int32_t* __restrict__ tlen,
                          const int32_t* __restrict__ gbase, const uint16_t* __restrict__ col16, int64_t ncols,
                          int pack, int B, unsigned* bad) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= npos) return;
  const int64_t ts = i / H;
  const int w = (int)(i - ts * H), lane = w & 63, r = w >> 6;
  const int32_t lraw = tlen[ts];
  const bool tri = (lraw & kTriSlice) != 0, pair = (lraw & kTriPair) != 0;
  const int L = lraw & kTriLen, G = tri ? L / 3 : L;
  const int32_t row = i < nrows ? rowmap[i] : 0;
  if (pair && r != 0) return;  // pair slices: row a's codes serve both rows
  unsigned nb = 0;
  for (int g = 0; g < G; ++g) {
    const int64_t at = pair ? t_code_slot(toff[ts], g, L / 3, lane, 0, 1, true, B)
                            : t_code_slot(toff[ts], g, L / 3, lane, r, R, false, B);
    const int32_t c = d16_col(col16[at], row, gbase[ts]);
    if (c < -1 || (c >= 0 && c + (pair ? 3 : tri ? 2 : 0) >= ncols)) ++nb;
  }
  if (nb) atomicAdd(bad, nb);
}

void launch_t_check(const pa_mat* A, unsigned* bad, hipStream_t st) {
  const int64_t npos = A->t_nslices * A->H;
  if (npos == 0) return;
  hipLaunchKernelGGL(k_t_check, dim3((unsigned)((npos + 255) / 256)), dim3(256), 0, st, npos, A->t_nrows, A->H, A->R,
                     A->d_t_rowmap, A->d_t_off, A->d_t_len, A->d_t_gbase, A->d_t_col16, A->ncols_lids, A->t_pack,
                     dtype_size(A->dtype) == 4 ? 9 : 4, bad);
}

void launch_t_rowinfo(const pa_mat* A, int64_t n, const int32_t* rows, int64_t noids, int32_t* info, hipStream_t st) {
  if (n == 0) return;
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
#define PA_TRI(RR) hipLaunchKernelGGL(k_t_rowinfo<RR>, g, b, 0, st, n, rows, A->H, A->d_slice_off, A->d_slice_len, \
                                      A->d_col, noids, info)
  switch (A->R) {
    case 1: PA_TRI(1); break;
    case 2: PA_TRI(2); break;
    case 4: PA_TRI(4); break;
  }
#undef PA_TRI
}

void launch_t_gbase(const pa_mat* A, int64_t noids, int32_t* ok, hipStream_t st) {
  const int64_t blocks = (A->t_nslices + 3) / 4;
  if (blocks == 0) return;
#define PA_TGB(RR) hipLaunchKernelGGL(k_t_gbase<RR>, dim3((unsigned)blocks), dim3(256), 0, st, A->t_nslices, \
                                      A->t_nrows, A->H, A->d_t_rowlen, A->d_t_src, A->d_col, noids, A->d_t_gbase, ok)
  switch (A->R) {
    case 1: PA_TGB(1); break;
    case 2: PA_TGB(2); break;
    case 4: PA_TGB(4); break;
  }
#undef PA_TGB
}

// codes false: values only (pa_mat_set_values, fillstored, exchange!(A))
void launch_t_fill(const pa_mat* A, int64_t noids, bool codes, hipStream_t st) {
  if (A->t_nrows == 0) return;
  const dim3 g((unsigned)((A->t_nrows + 255) / 256)), b(256);
#define PA_TF(E, RR)                                                                                           \
  hipLaunchKernelGGL((k_t_fill<E, RR>), g, b, 0, st, A->t_nrows, A->H, A->d_t_rowmap, A->d_t_rowlen, A->d_t_src, \
                     A->d_t_off, A->d_t_len, A->d_t_gbase, A->d_col, (const E*)A->d_val, noids, codes,          \
                     A->t_pack, A->d_t_col16, (E*)A->d_t_val)
  switch (A->dtype) {
    case PA_F32:
      if (A->R == 2) PA_TF(float, 2);
      else PA_TF(float, 4);
      break;
    case PA_F64: PA_TF(double, 2); break;
    case PA_C64: PA_TF(c64, 2); break;
    case PA_C128: PA_TF(c128, 1); break;
  }
#undef PA_TF
}

#endif  // PA_DT_DEFINE

}  // namespace pa
