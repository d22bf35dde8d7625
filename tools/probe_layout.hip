// Layout probe (standalone, not part of the library): does the order in
// which concurrently running waves touch HBM change the read rate of the
// SpMV's value stream?  Same bytes, four access orders:
//   linear   — grid-stride sweep, 1 KB per wave per step (the pa_hbm_probe order)
//   slice    — wave w streams its own contiguous L KB region (the SELL layout:
//              one slice = L entries × 64 lanes × 16 B)
//   group G  — G consecutive slices interleaved entry-major: entry k of the
//              G slices of a group sits in G adjacent 1 KB chunks
// Every variant also writes 1 KB per slice (y).  Non-temporal 16 B loads as in
// k_spmv_sell.  hipcc --offload-arch=gfx950 -O3 tools/probe_layout.hip -o probe_layout
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

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

__device__ __forceinline__ u32x4 ldnt(const u32x4* p) { return __builtin_nontemporal_load(p); }

// MODE 0: slice-contiguous; MODE 1: group-interleaved (G slices)
template <int MODE>
__global__ __launch_bounds__(256) void k_slices(const u32x4* __restrict__ v, u32x4* __restrict__ y,
                                                int64_t nslices, int G) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= nslices) return;
  int64_t base, stride;
  if (MODE == 0) {
    base = w * L * 64;
    stride = 64;
  } else {
    const int64_t g = w / G, j = w % G;
    base = g * (int64_t)L * G * 64 + j * 64;
    stride = (int64_t)G * 64;
  }
  u32x4 acc = {0, 0, 0, 0};
  int k = 0;
  for (; k + U <= L; k += U) {
    u32x4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = ldnt(v + base + (k + u) * stride + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= t[u];
  }
  for (; k < L; ++k) acc ^= ldnt(v + base + k * stride + lane);
  y[w * 64 + lane] = acc;
}

__global__ __launch_bounds__(256) void k_linear(const u32x4* __restrict__ v, u32x4* __restrict__ y,
                                                int64_t nchunks, int64_t nslices) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  u32x4 acc = {0, 0, 0, 0};
  int64_t c = w0;
  for (; c + (U - 1) * nw < nchunks; c += U * nw) {
    u32x4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = ldnt(v + (c + u * nw) * 64 + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= t[u];
  }
  for (; c < nchunks; c += nw) acc ^= ldnt(v + c * 64 + lane);
  for (int64_t s = w0; s < nslices; s += nw) y[s * 64 + lane] = acc;
}

int main(int argc, char** argv) {
  const int64_t nslices = argc > 1 ? std::atoll(argv[1]) : 131072;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
  const int64_t nchunks = nslices * L;  // 1 KB each
  const size_t vbytes = (size_t)nchunks * 1024, ybytes = (size_t)nslices * 1024;
  u32x4 *v, *y;
  CK(hipMalloc(&v, vbytes));
  CK(hipMalloc(&y, ybytes));
  CK(hipMemset(v, 1, vbytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)vbytes + (double)ybytes;
  auto run = [&](const char* name, auto launch) {
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
    std::printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f, \"gbs_median\": %.1f}\n", name,
                ms[ms.size() / 2], ms[0], bytes / (ms[ms.size() / 2] * 1e-3) / 1e9);
    std::fflush(stdout);
  };
  const int64_t blocks = (nslices + 3) / 4;
  int ncu = 256;
  {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    ncu = p.multiProcessorCount;
  }
  for (int round = 0; round < 2; ++round) {
    run("linear", [&] { hipLaunchKernelGGL(k_linear, dim3(ncu * 16), dim3(256), 0, 0, v, y, nchunks, nslices); });
    run("slice", [&] { hipLaunchKernelGGL(k_slices<0>, dim3(blocks), dim3(256), 0, 0, v, y, nslices, 1); });
    for (int G : {2, 4, 16, 64, 256}) {
      char nm[32];
      std::snprintf(nm, sizeof nm, "group%d", G);
      run(nm, [&] { hipLaunchKernelGGL(k_slices<1>, dim3(blocks), dim3(256), 0, 0, v, y, nslices, G); });
    }
  }
  CK(hipFree(v));
  CK(hipFree(y));
  return 0;
}
