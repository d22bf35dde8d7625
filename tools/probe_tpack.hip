// Standalone check of the Float32 triple SELL's packed code layout
// (pa_spmv.hip t_code_slot / rows_t16_tri): a writer kernel stores each
// (triple, lane, row) code at t_code_slot, a reader wave loads them the way
// the SpMV does; prints the mismatches.  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int R> struct alignas(2 * R) S16Pack { uint16_t c[R]; };
template <int BYTES> struct RawOf;
template <> struct RawOf<4> { typedef unsigned int type; };
template <> struct RawOf<16> { typedef unsigned int type __attribute__((ext_vector_type(4))); };
template <bool NT, typename V> __device__ __forceinline__ V ld(const V* p) {
  typedef typename RawOf<sizeof(V)>::type Raw;
  Raw r;
  if (NT) r = __builtin_nontemporal_load(reinterpret_cast<const Raw*>(p));
  else r = *reinterpret_cast<const Raw*>(p);
  V v;
  __builtin_memcpy(&v, &r, sizeof(V));
  return v;
}
__device__ __forceinline__ int64_t t_code_slot(int64_t d, int g, int ntri, int lane, int r, int R, bool packed) {
  const int b = g / 9, i = g % 9;
  if (!packed || 9 * (b + 1) > ntri) return d + ((int64_t)g * 64 + lane) * R + r;
  const int64_t bb = d + (int64_t)b * 9 * 64 * R;
  return i < 8 ? bb + (int64_t)(i / 4) * 4 * 64 * R + (int64_t)lane * 4 * R + (i % 4) * R + r
               : bb + 8 * 64 * R + (int64_t)lane * R + r;
}
__global__ void wr(uint16_t* col16, int64_t d, int ntri) {
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;
  for (int g = 0; g < ntri; ++g) col16[t_code_slot(d, g, ntri, lane, r, 2, true)] = (uint16_t)(g << 8 | lane << 1 | r);
}
__global__ void rd(const uint16_t* col16, int64_t off, int ntri, int* bad) {
  constexpr int R = 2, MB = 9;
  const int lane = threadIdx.x & 63;
  const S16Pack<R>* __restrict__ cp = reinterpret_cast<const S16Pack<R>*>(col16 + off) + lane;
  for (int t = 0; t < ntri; t += MB) {
    S16Pack<R> q[MB];
    if (t + MB <= ntri) {
      const S16Pack<R>* __restrict__ cb = cp - threadIdx.x % 64 + (int64_t)t * 64;
      for (int h = 0; h < 2; ++h) {
        const S16Pack<4 * R> q4 = ld<true>(reinterpret_cast<const S16Pack<4 * R>*>(cb + h * 4 * 64) + threadIdx.x % 64);
        for (int i = 0; i < 4; ++i)
          for (int r = 0; r < R; ++r) q[4 * h + i].c[r] = q4.c[i * R + r];
      }
      q[8] = ld<true>(cb + 8 * 64 + threadIdx.x % 64);
    } else {
      for (int u = 0; u < MB; ++u) q[u] = ld<true>(&cp[min(t + u, ntri - 1) * 64]);
    }
    for (int u = 0; u < MB && t + u < ntri; ++u)
      for (int r = 0; r < R; ++r) {
        const int want = (t + u) << 8 | lane << 1 | r;
        if (q[u].c[r] != want) {
          atomicAdd(bad, 1);
          if (lane < 2) printf("t %d u %d lane %d r %d got %x want %x\n", t, u, lane, r, q[u].c[r], want);
        }
      }
  }
}
int main() {
  uint16_t* c;
  int* bad;
  const int64_t d = 128 * 27 * 3;
  hipMalloc(&c, 1 << 20);
  hipMalloc(&bad, 4);
  int fails = 0;
  for (int ntri : {9, 6, 18, 3}) {
    hipMemset(bad, 0, 4);
    hipMemset(c, 0xff, 1 << 20);
    wr<<<1, 128>>>(c, d, ntri);
    rd<<<1, 64>>>(c, d, ntri, bad);
    int b = 0;
    hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost);
    printf("ntri %d: %d mismatches\n", ntri, b);
    fails += b;
  }
  return fails ? 1 : 0;
}
