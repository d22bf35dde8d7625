// capture_probe.cpp — which multi-stream capture structures hipStreamEndCapture
// accepts on this ROCm runtime (the r01 capture of the eager
// fork/join mul! crashed inside hipStreamEndCapture; the library captures a
// single in-order chain instead).  One variant per process (a crash ends only
// that process); prints one JSON line per variant with the error codes.
//
//   hipcc --offload-arch=gfx950 -O2 -o build/capture_probe tools/capture_probe.cpp
//   build/capture_probe <variant>      variant 0..5 (see below)
//
//  0  fork/join: origin records e0; side waits e0, runs a kernel, records e1;
//     origin waits e1 before EndCapture                        (valid CUDA rule)
//  1  fork without join: the side stream's last work is not waited on by the
//     origin before EndCapture                                  (unjoined fork)
//  2  the side stream waits an event recorded OUTSIDE the capture (before
//     BeginCapture) and then joins                              (external event)
//  3  the origin waits an event recorded outside the capture   (external event)
//  4  fork/join where the side stream is recorded into with the join event
//     but the origin's capture ends before the side's last kernel is joined
//     (record e1 on side AFTER origin's wait)                   (late record)
//  5  like 0 but with 16 side streams, as the eager multi-part mul! had
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_touch(int* p, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += v;
}

#define CK(x) (int)(x)

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 0;
  int* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 2;
  (void)hipMemset(d, 0, 64);
  const int nside = variant == 5 ? 16 : 1;
  hipStream_t s0;
  std::vector<hipStream_t> side(nside);
  (void)hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
  for (auto& s : side) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t e0, ext;
  std::vector<hipEvent_t> e1(nside);
  (void)hipEventCreateWithFlags(&e0, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&ext, hipEventDisableTiming);
  for (auto& e : e1) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  (void)hipEventRecord(ext, side[0]);  // recorded before the capture
  (void)hipStreamSynchronize(side[0]);

  int rb = CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
  hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s0, d, 1);
  int rr = CK(hipEventRecord(e0, s0));
  int rw = 0, rj = 0;
  for (int i = 0; i < nside; ++i) {
    if (variant == 2) rw |= CK(hipStreamWaitEvent(side[i], ext, 0));
    rw |= CK(hipStreamWaitEvent(side[i], e0, 0));
    hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, side[i], d, 2);
    if (variant != 4) rj |= CK(hipEventRecord(e1[i], side[i]));
  }
  if (variant == 3) rw |= CK(hipStreamWaitEvent(s0, ext, 0));
  if (variant != 1)
    for (int i = 0; i < nside; ++i) rj |= CK(hipStreamWaitEvent(s0, e1[i], 0));
  if (variant == 4)
    for (int i = 0; i < nside; ++i) {
      hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, side[i], d, 4);
      rj |= CK(hipEventRecord(e1[i], side[i]));
    }
  hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s0, d, 8);
  hipGraph_t g = nullptr;
  fprintf(stderr, "variant %d: before EndCapture\n", variant);
  int re = CK(hipStreamEndCapture(s0, &g));
  int ri = -1, rl = -1, rs = -1;
  int val = -1;
  if (re == 0 && g) {
    hipGraphExec_t ge = nullptr;
    ri = CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    if (ri == 0) {
      rl = CK(hipGraphLaunch(ge, s0));
      rs = CK(hipStreamSynchronize(s0));
      (void)hipMemcpy(&val, d, 4, hipMemcpyDeviceToHost);
    }
  }
  const int last = CK(hipGetLastError());
  printf("{\"variant\": %d, \"begin\": %d, \"record\": %d, \"waits\": %d, \"join\": %d, \"end_capture\": %d, "
         "\"end_capture_str\": \"%s\", \"instantiate\": %d, \"launch\": %d, \"sync\": %d, \"value\": %d, \"last\": %d}\n",
         variant, rb, rr, rw, rj, re, hipGetErrorString((hipError_t)re), ri, rl, rs, val, last);
  return 0;
}
