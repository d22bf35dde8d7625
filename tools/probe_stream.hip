// Stream probe (standalone, not part of the library): where does the headline
// SpMV's value stream lose rate against a plain read sweep on the same box?
// Same 3.57 GB of values (131,072 FE27 slices × 27 entries × 1 KB), variants:
//   lin_ro     grid-stride read sweep, no writes (pa_hbm_probe's idiom)
//   lin_w      the same + 1 KB of y per slice written after the sweep
//   slice_ro   wave w streams its own contiguous 27 KB slice, no y write
//   slice_w    the same + its 1 KB of y (the SELL kernel's traffic shape)
//   slice_wnt  the same with a non-temporal y store
//   slice_b64  slice_w launched as one wave per workgroup
//   slice_2    slice_w with two slices per wave (grid halved)
//   (with a 3rd argument) write-only sweeps of y / of 3.57 GB, memset, and
//   slice_w with y folded into a 1 / 16 / 64 MB ring
//   (3rd argument "x") slice_w plus the FE27 pattern kernel's x reads (16 B
//   runs at row + 27 stencil offsets of a 256³ x), or the same folded into
//   a 1 MB window (L2 hits), or with each dx triple's x shared between
//   neighbouring lanes (one 16 B run per lane per triple; __shfl or DPP)
//   (3rd argument "c") slice_w behind a list → offset load chain, with 1,
//   2, 4 or 8 slices per wave, the next slice's metadata prefetched or not
//   (3rd argument "e") persistent blocks staging y in LDS per epoch of C
//   slices and writing it in one burst, with or without a grid barrier
// hipcc --offload-arch=gfx950 -O3 tools/probe_stream.hip -o probe_stream
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));     \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

constexpr int L = 27;  // entries per slice (FE27)
constexpr int U = 8;   // loads in flight per lane
constexpr unsigned MAGIC = 0x9e3779b9u;

__device__ __forceinline__ u32x4 ldnt(const u32x4* p) { return __builtin_nontemporal_load(p); }

template <int UU = U>
__device__ __forceinline__ u32x4 stream_slice(const u32x4* __restrict__ v, int64_t s, int lane) {
  const int64_t base = s * L * 64;
  u32x4 acc = {0, 0, 0, 0};
  int k = 0;
  for (; k + UU <= L; k += UU) {
    u32x4 t[UU];
#pragma unroll
    for (int u = 0; u < UU; ++u) t[u] = ldnt(v + base + (k + u) * 64 + lane);
#pragma unroll
    for (int u = 0; u < UU; ++u) acc ^= t[u];
  }
  for (; k < L; ++k) acc ^= ldnt(v + base + k * 64 + lane);
  return acc;
}

// WMODE 0: no write (kept live by a never-true test), 1: plain store, 2: non-temporal store
template <int WMODE, int WPB, int SPW, int UU = U>
__global__ __launch_bounds__(64 * WPB) void k_slice(const u32x4* __restrict__ v, u32x4* __restrict__ y,
                                                   int64_t nslices) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
#pragma unroll
  for (int j = 0; j < SPW; ++j) {
    const int64_t s = w * SPW + j;
    if (s >= nslices) return;
    const u32x4 acc = stream_slice<UU>(v, s, lane);
    if (WMODE == 0) {
      if (acc.x == MAGIC) y[s * 64 + lane] = acc;
    } else if (WMODE == 1) {
      y[s * 64 + lane] = acc;
    } else {
      __builtin_nontemporal_store(acc, y + s * 64 + lane);
    }
  }
}

// slice_w + the x reads of the FE27 pattern kernel: entry k of lane l's two
// rows (r0 = slice*128 + 2l) reads x[r0 + off[k]] as one 16 B run, off = the
// 27 offsets {dz*N² + dy*N + dx}, N = 256 (x: N³ doubles).  XWIN: x indices
// folded into a 1 MB window (always L2 hits) instead of the real 134 MB x.
__constant__ int c_off[L];
template <bool XWIN>
__global__ __launch_bounds__(256) void k_slice_x(const u32x4* __restrict__ v, const double* __restrict__ x,
                                                 u32x4* __restrict__ y, int64_t nslices, int64_t nx) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nslices) return;
  const int64_t base = s * L * 64;
  const int64_t r0 = s * 128 + 2 * lane;
  u32x4 acc = {0, 0, 0, 0};
  double xa = 0.0;
  int k = 0;
  for (; k + U <= L; k += U) {
    u32x4 t[U];
    double2 xr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = ldnt(v + base + (k + u) * 64 + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t i = r0 + c_off[k + u];
      i = i < 0 ? 0 : (i >= nx - 1 ? nx - 2 : i);
      if (XWIN) i &= (1 << 17) - 2;
      xr[u] = *reinterpret_cast<const double2*>(x + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc ^= t[u];
      xa = xa + xr[u].x * xr[u].y;
    }
  }
  for (; k < L; ++k) {
    acc ^= ldnt(v + base + k * 64 + lane);
    int64_t i = r0 + c_off[k];
    i = i < 0 ? 0 : (i >= nx - 1 ? nx - 2 : i);
    if (XWIN) i &= (1 << 17) - 2;
    xa = xa + x[i];
  }
  acc.x ^= (unsigned)(xa != 0.5);
  y[s * 64 + lane] = acc;
}

// slice_wx with the x of each (dx = -1, 0, +1) triple shared between
// neighbouring lanes: one 16 B run per lane at dx = 0, the dx = ±1 runs
// assembled from the neighbours' values (DPP wave shift, or __shfl when
// DPP is 0), lanes 0 and 63 fetch the one value past the slice's edge
template <int DPP>
__device__ __forceinline__ double shift_from_lower(double v) {  // lane l gets lane l-1's v
  if (DPP) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x138, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
  }
  return __shfl_up(v, 1, 64);
}
template <int DPP>
__device__ __forceinline__ double shift_from_upper(double v) {  // lane l gets lane l+1's v
  if (DPP) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x130, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
  }
  return __shfl_down(v, 1, 64);
}
template <int DPP, bool ROLL = false>
__global__ __launch_bounds__(256) void k_slice_x3(const u32x4* __restrict__ v, const double* __restrict__ x,
                                                  u32x4* __restrict__ y, int64_t nslices, int64_t nx) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nslices) return;
  const int64_t base = s * L * 64;
  const int64_t r0 = s * 128 + 2 * lane;
  u32x4 acc = {0, 0, 0, 0};
  double xa = 0.0;
  // 27 entries = 9 triples; 3 triples (9 entries) per batch
#pragma unroll(ROLL ? 1 : 3)
  for (int g = 0; g < 9; g += 3) {
    u32x4 t[9];
#pragma unroll
    for (int u = 0; u < 9; ++u) t[u] = ldnt(v + base + (3 * g + u) * 64 + lane);
    double2 c[3];
    double e[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      int64_t i = r0 + c_off[3 * (g + q) + 1];
      i = i < 2 ? 2 : (i >= nx - 3 ? nx - 4 : i);
      c[q] = *reinterpret_cast<const double2*>(x + i);
      e[q] = 0.0;
      if (lane == 0 || lane == 63) e[q] = x[lane == 0 ? i - 1 : i + 2];
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      double lo = shift_from_lower<DPP>(c[q].y);
      double hi = shift_from_upper<DPP>(c[q].x);
      if (lane == 0) lo = e[q];
      if (lane == 63) hi = e[q];
      acc ^= t[3 * q] ^ t[3 * q + 1] ^ t[3 * q + 2];
      xa = xa + lo * c[q].x + c[q].x * c[q].y + c[q].y * hi;
    }
  }
  acc.x ^= (unsigned)(xa != 0.5);
  y[s * 64 + lane] = acc;
}

// slice_w behind the SpMV's metadata chain: the slice's offset comes from
// soff[list[w]] (two dependent loads) before its first value load; CHAIN 2:
// each wave streams SPW slices and loads the next slice's metadata while
// the current one streams (software-pipelined across slices)
template <int SPW, bool PREF>
__global__ __launch_bounds__(256) void k_slice_chain(const u32x4* __restrict__ v, u32x4* __restrict__ y,
                                                     const int32_t* __restrict__ list, const int64_t* __restrict__ soff,
                                                     int64_t nslices) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t w0 = w * SPW;
  if (w0 >= nslices) return;
  int64_t s = list[w0];
  int64_t off = soff[s];
  for (int j = 0; j < SPW; ++j) {
    int64_t s_next = 0, off_next = 0;
    const bool more = j + 1 < SPW && w0 + j + 1 < nslices;
    if (PREF && more) {
      s_next = list[w0 + j + 1];
      off_next = soff[s_next];
    }
    u32x4 acc = {0, 0, 0, 0};
    int k = 0;
    for (; k + U <= L; k += U) {
      u32x4 t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) t[u] = ldnt(v + off + (k + u) * 64 + lane);
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= t[u];
    }
    for (; k < L; ++k) acc ^= ldnt(v + off + k * 64 + lane);
    y[s * 64 + lane] = acc;
    if (!more) break;
    if (PREF) {
      s = s_next;
      off = off_next;
    } else {
      s = list[w0 + j + 1];
      off = soff[s];
    }
  }
}

// write-only sweep of n16 16 B values (NT: non-temporal stores)
template <bool NT>
__global__ __launch_bounds__(256) void k_wonly(u32x4* __restrict__ y, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const u32x4 v = {1u, 2u, 3u, (unsigned)threadIdx.x};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
    if (NT) __builtin_nontemporal_store(v, y + i);
    else y[i] = v;
  }
}

// slice_w with the y store folded into a small ring (RING 16 B slots): same
// store instructions, but the bytes stay in L2
template <int RINGLOG>
__global__ __launch_bounds__(256) void k_slice_ring(const u32x4* __restrict__ v, u32x4* __restrict__ y,
                                                    int64_t nslices) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nslices) return;
  const u32x4 acc = stream_slice(v, s, lane);
  y[(s * 64 + lane) & ((1ll << RINGLOG) - 1)] = acc;
}

// Persistent blocks of 16 waves (one per CU): epoch e of block b streams the
// C consecutive slices [(e*nb + b)*C, +C), stages their y (1 KB each) in LDS
// and writes the C KB at once after the block's waves finish the epoch.
// SYNC: all blocks meet at a grid barrier before the write burst, so the
// whole GPU reads, then writes (the barrier gives up after 2^18 polls:
// never a hang, only a wrong time).
__device__ unsigned g_bar[2];
template <int C, bool SYNC>
__global__ __launch_bounds__(1024) void k_slice_epoch(const u32x4* __restrict__ v, u32x4* __restrict__ y,
                                                      int64_t nslices) {
  __shared__ u32x4 sy[C * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nb = gridDim.x;
  const int64_t nep = (nslices + nb * C - 1) / (nb * C);
  for (int64_t e = 0; e < nep; ++e) {
    const int64_t s0 = (e * nb + blockIdx.x) * C;
    for (int j = wv; j < C; j += 16)
      if (s0 + j < nslices) sy[j * 64 + lane] = stream_slice(v, s0 + j, lane);
    __syncthreads();
    if (SYNC) {
      if (threadIdx.x == 0) {
        __threadfence();
        const unsigned target = (unsigned)((e + 1) * nb);
        atomicAdd(&g_bar[0], 1u);
        for (int it = 0; it < (1 << 18); ++it)
          if (__hip_atomic_load(&g_bar[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      }
      __syncthreads();
    }
    for (int i = threadIdx.x; i < C * 64; i += 1024)
      if (s0 + i / 64 < nslices) y[s0 * 64 + i] = sy[i];
    __syncthreads();
  }
}

__global__ void k_bar_reset() { g_bar[0] = 0; g_bar[1] = 0; }

template <int WRITE>
__global__ __launch_bounds__(256) void k_linear(const u32x4* __restrict__ v, u32x4* __restrict__ y,
                                                int64_t n16, int64_t nslices) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  u32x4 acc = {0, 0, 0, 0};
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = ldnt(v + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= t[u];
  }
  for (; i < n16; i += stride) acc ^= ldnt(v + i);
  if (WRITE) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < nslices * 64; j += stride) y[j] = acc;
  } else if (acc.x == MAGIC) {
    y[threadIdx.x] = acc;
  }
}

int main(int argc, char** argv) {
  const int64_t nslices = argc > 1 ? std::atoll(argv[1]) : 131072;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
  const int64_t n16 = nslices * L * 64;
  const size_t vbytes = (size_t)n16 * 16, ybytes = (size_t)nslices * 1024;
  u32x4 *v, *y;
  CK(hipMalloc(&v, vbytes));
  CK(hipMalloc(&y, ybytes));
  CK(hipMemset(v, 0x5a, vbytes));
  CK(hipMemset(y, 0, ybytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, bool writes, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double bytes = (double)vbytes + (writes ? (double)ybytes : 0.0);
    std::printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f, \"gbs_median\": %.1f}\n", name,
                ms[ms.size() / 2], ms[0], bytes / (ms[ms.size() / 2] * 1e-3) / 1e9);
    std::fflush(stdout);
  };
  if (argc > 3 && argv[3][0] == 'c') {  // metadata-chain variants
    std::vector<int32_t> hl(nslices);
    std::vector<int64_t> ho(nslices);
    for (int64_t i = 0; i < nslices; ++i) { hl[i] = (int32_t)i; ho[i] = i * L * 64; }
    int32_t* dl;
    int64_t* dof;
    CK(hipMalloc(&dl, nslices * 4));
    CK(hipMalloc(&dof, nslices * 8));
    CK(hipMemcpy(dl, hl.data(), nslices * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dof, ho.data(), nslices * 8, hipMemcpyHostToDevice));
    const int64_t b4 = (nslices + 3) / 4;
    for (int round = 0; round < 2; ++round) {
      run("slice_w", true, [&] { hipLaunchKernelGGL((k_slice<1, 4, 1>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
      run("chain1", true, [&] { hipLaunchKernelGGL((k_slice_chain<1, false>), dim3(b4), dim3(256), 0, 0, v, y, dl, dof, nslices); });
      run("chain2", true, [&] { hipLaunchKernelGGL((k_slice_chain<2, false>), dim3((nslices + 7) / 8), dim3(256), 0, 0, v, y, dl, dof, nslices); });
      run("chain2_pref", true, [&] { hipLaunchKernelGGL((k_slice_chain<2, true>), dim3((nslices + 7) / 8), dim3(256), 0, 0, v, y, dl, dof, nslices); });
      run("chain4_pref", true, [&] { hipLaunchKernelGGL((k_slice_chain<4, true>), dim3((nslices + 15) / 16), dim3(256), 0, 0, v, y, dl, dof, nslices); });
      run("chain8_pref", true, [&] { hipLaunchKernelGGL((k_slice_chain<8, true>), dim3((nslices + 31) / 32), dim3(256), 0, 0, v, y, dl, dof, nslices); });
    }
    CK(hipFree(dl));
    CK(hipFree(dof));
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'x') {  // x-read variants
    const int64_t N = 256, nx = N * N * N;
    double* x;
    CK(hipMalloc(&x, (size_t)nx * 8));
    CK(hipMemset(x, 0, (size_t)nx * 8));
    int off[L], t = 0;
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) off[t++] = (int)(dz * N * N + dy * N + dx);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_off), off, sizeof off));
    const int64_t b4 = (nslices + 3) / 4;
    for (int round = 0; round < 2; ++round) {
      run("slice_w", true, [&] { hipLaunchKernelGGL((k_slice<1, 4, 1>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
      run("slice_wx", true, [&] { hipLaunchKernelGGL(k_slice_x<false>, dim3(b4), dim3(256), 0, 0, v, x, y, nslices, nx); });
      run("slice_wx_l2", true, [&] { hipLaunchKernelGGL(k_slice_x<true>, dim3(b4), dim3(256), 0, 0, v, x, y, nslices, nx); });
      run("slice_wx3_shfl", true, [&] { hipLaunchKernelGGL(k_slice_x3<0>, dim3(b4), dim3(256), 0, 0, v, x, y, nslices, nx); });
      run("slice_wx3_dpp", true, [&] { hipLaunchKernelGGL(k_slice_x3<1>, dim3(b4), dim3(256), 0, 0, v, x, y, nslices, nx); });
      run("slice_wx3_dpp_rolled", true, [&] { hipLaunchKernelGGL((k_slice_x3<1, true>), dim3(b4), dim3(256), 0, 0, v, x, y, nslices, nx); });
      run("slice_w_u9", true, [&] { hipLaunchKernelGGL((k_slice<1, 4, 1, 9>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
      run("slice_w_u27", true, [&] { hipLaunchKernelGGL((k_slice<1, 4, 1, 27>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
    }
    CK(hipFree(x));
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'e') {  // epoch-staged y variants
    int ncu = 256;
    {
      hipDeviceProp_t pr;
      CK(hipGetDeviceProperties(&pr, 0));
      ncu = pr.multiProcessorCount;
    }
    const int64_t b4 = (nslices + 3) / 4;
    for (int round = 0; round < 2; ++round) {
      run("slice_ro", false, [&] { hipLaunchKernelGGL((k_slice<0, 4, 1>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
      run("slice_w", true, [&] { hipLaunchKernelGGL((k_slice<1, 4, 1>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
      run("epoch128_nosync", true, [&] { hipLaunchKernelGGL((k_slice_epoch<128, false>), dim3(ncu), dim3(1024), 0, 0, v, y, nslices); });
      run("epoch32_nosync", true, [&] { hipLaunchKernelGGL((k_slice_epoch<32, false>), dim3(ncu), dim3(1024), 0, 0, v, y, nslices); });
      run("epoch128_sync", true, [&] {
        hipLaunchKernelGGL(k_bar_reset, dim3(1), dim3(1), 0, 0);
        void* args[] = {(void*)&v, (void*)&y, (void*)&nslices};
        CK(hipLaunchCooperativeKernel((const void*)k_slice_epoch<128, true>, dim3(ncu), dim3(1024), args, 0, 0));
      });
    }
    return 0;
  }
  if (argc > 3) {  // write-side variants only
    const int64_t yn16 = (int64_t)ybytes / 16;
    u32x4* big;
    CK(hipMalloc(&big, vbytes));
    for (int round = 0; round < 2; ++round) {
      for (int blocks : {4096, 16384}) {
        char nm[48];
        std::snprintf(nm, sizeof nm, "wonly_y_%d", blocks);
        run(nm, false, [&] { hipLaunchKernelGGL(k_wonly<false>, dim3(blocks), dim3(256), 0, 0, y, yn16); });
        std::snprintf(nm, sizeof nm, "wonly_y_nt_%d", blocks);
        run(nm, false, [&] { hipLaunchKernelGGL(k_wonly<true>, dim3(blocks), dim3(256), 0, 0, y, yn16); });
        std::snprintf(nm, sizeof nm, "wonly_big_%d", blocks);
        run(nm, false, [&] { hipLaunchKernelGGL(k_wonly<false>, dim3(blocks), dim3(256), 0, 0, big, n16); });
        std::snprintf(nm, sizeof nm, "wonly_big_nt_%d", blocks);
        run(nm, false, [&] { hipLaunchKernelGGL(k_wonly<true>, dim3(blocks), dim3(256), 0, 0, big, n16); });
      }
      run("memset_y", false, [&] { CK(hipMemsetAsync(y, round, ybytes, 0)); });
      const int64_t b4 = (nslices + 3) / 4;
      run("slice_ro", false, [&] { hipLaunchKernelGGL((k_slice<0, 4, 1>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
      run("slice_w", true, [&] { hipLaunchKernelGGL((k_slice<1, 4, 1>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
      run("slice_ring1MB", true, [&] { hipLaunchKernelGGL((k_slice_ring<16>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
      run("slice_ring16MB", true, [&] { hipLaunchKernelGGL((k_slice_ring<20>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
      run("slice_ring64MB", true, [&] { hipLaunchKernelGGL((k_slice_ring<22>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
    }
    CK(hipFree(big));
    return 0;
  }
  for (int round = 0; round < 2; ++round) {
    for (int blocks : {4096, 16384}) {
      char nm[32];
      std::snprintf(nm, sizeof nm, "lin_ro_%d", blocks);
      run(nm, false, [&] { hipLaunchKernelGGL(k_linear<0>, dim3(blocks), dim3(256), 0, 0, v, y, n16, nslices); });
      std::snprintf(nm, sizeof nm, "lin_w_%d", blocks);
      run(nm, true, [&] { hipLaunchKernelGGL(k_linear<1>, dim3(blocks), dim3(256), 0, 0, v, y, n16, nslices); });
    }
    const int64_t b4 = (nslices + 3) / 4;
    run("slice_ro", false, [&] { hipLaunchKernelGGL((k_slice<0, 4, 1>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
    run("slice_w", true, [&] { hipLaunchKernelGGL((k_slice<1, 4, 1>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
    run("slice_wnt", true, [&] { hipLaunchKernelGGL((k_slice<2, 4, 1>), dim3(b4), dim3(256), 0, 0, v, y, nslices); });
    run("slice_b64", true, [&] { hipLaunchKernelGGL((k_slice<1, 1, 1>), dim3(nslices), dim3(64), 0, 0, v, y, nslices); });
    run("slice_2", true, [&] { hipLaunchKernelGGL((k_slice<1, 4, 2>), dim3((nslices + 7) / 8), dim3(256), 0, 0, v, y, nslices); });
  }
  CK(hipFree(v));
  CK(hipFree(y));
  return 0;
}
