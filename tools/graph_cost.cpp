// graph_cost.cpp — host cost of hipGraphLaunch on this ROCm runtime by graph
// shape (the one-process-drives-several-GPUs design of DESIGN.md §6: per-part
// graphs with external event nodes vs eager launches).  Prints one JSON line
// per shape: host µs per launch (the enqueue alone, measured over back-to-back
// launches with the device kept busy) and device µs per replay.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/graph_cost.bin tools/graph_cost.cpp
//   tools/graph_cost.bin                      the shapes of profiles/r05/g/
//   tools/graph_cost.bin K W R [--trace]      one shape (K kernels, W external
//                                             waits, R external records); --trace
//                                             prints a line after every HIP call
//                                             of the capture
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <vector>

__global__ void k_small(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.0f;
}

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));       \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

static bool g_trace = false;
#define STEP(x)                                        \
  do {                                                 \
    CK(x);                                             \
    if (g_trace) std::printf("ok %s\n", #x);           \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// kernels: kernel nodes in a chain; waits: external event-wait nodes before
// them (events recorded on other streams before each launch); records:
// external event-record nodes after them
static int shape(int kernels, int waits, int records, int reps) {
  std::printf("# shape %d %d %d\n", kernels, waits, records);
  const int n = 1 << 16;
  float* d = nullptr;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemset(d, 0, n * sizeof(float)));
  hipStream_t s, o;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&o, hipStreamNonBlocking));
  std::vector<hipEvent_t> ew(waits), er(records);
  for (auto& e : ew) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : er) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : ew) STEP(hipEventRecord(e, o));
  STEP(hipStreamSynchronize(o));
  hipGraph_t g;
  STEP(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  for (auto& e : ew) STEP(hipStreamWaitEvent(s, e, hipEventWaitExternal));
  for (int k = 0; k < kernels; ++k) {
    hipLaunchKernelGGL(k_small, dim3(n / 256), dim3(256), 0, s, d, n);
    STEP(hipGetLastError());
  }
  for (auto& e : er) STEP(hipEventRecordWithFlags(e, s, hipEventRecordExternal));
  STEP(hipStreamEndCapture(s, &g));
  if (g_trace) {
    size_t nn = 0;
    STEP(hipGraphGetNodes(g, nullptr, &nn));
    std::printf("graph nodes %zu\n", nn);
  }
  hipGraphExec_t x;
  STEP(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  for (int r = 0; r < 5; ++r) STEP(hipGraphLaunch(x, s));
  STEP(hipStreamSynchronize(s));
  // host: enqueue reps launches back to back (events re-recorded on the
  // other stream before each, as the callers of the real graphs would)
  double t0 = now_us();
  for (int r = 0; r < reps; ++r) {
    for (auto& e : ew) CK(hipEventRecord(e, o));
    CK(hipGraphLaunch(x, s));
  }
  const double host = (now_us() - t0) / reps;
  CK(hipStreamSynchronize(s));
  const double dev_total = (now_us() - t0) / reps;
  // the same work eager: waits + kernels + records
  t0 = now_us();
  for (int r = 0; r < reps; ++r) {
    for (auto& e : ew) CK(hipEventRecord(e, o));
    for (auto& e : ew) CK(hipStreamWaitEvent(s, e, 0));
    for (int k = 0; k < kernels; ++k) hipLaunchKernelGGL(k_small, dim3(n / 256), dim3(256), 0, s, d, n);
    for (auto& e : er) CK(hipEventRecord(e, s));
  }
  const double eager = (now_us() - t0) / reps;
  CK(hipStreamSynchronize(s));
  std::printf("{\"kernels\": %d, \"waits\": %d, \"records\": %d, \"graph_launch_host_us\": %.2f, "
              "\"graph_wall_us_per_replay\": %.2f, \"eager_host_us\": %.2f, \"other_stream_records_per_launch\": %d}\n",
              kernels, waits, records, host, dev_total, eager, waits);
  CK(hipGraphExecDestroy(x));
  CK(hipGraphDestroy(g));
  for (auto& e : ew) CK(hipEventDestroy(e));
  for (auto& e : er) CK(hipEventDestroy(e));
  CK(hipStreamDestroy(s));
  CK(hipStreamDestroy(o));
  CK(hipFree(d));
  return 0;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  if (argc >= 4) {
    g_trace = argc >= 5;
    return shape(std::atoi(argv[1]), std::atoi(argv[2]), std::atoi(argv[3]), 200);
  }
  // more than one external event-wait node per capture ({2, 7, 1}) crashed
  // the HIP runtime of the box inside the capture (segfault, profiles/r05/g/)
  const int shapes[][3] = {{1, 0, 0}, {2, 0, 0}, {4, 0, 0}, {8, 0, 0}, {16, 0, 0}, {32, 0, 0}, {2, 1, 1}};
  for (auto& sh : shapes)
    if (shape(sh[0], sh[1], sh[2], 200)) return 1;
  return 0;
}
