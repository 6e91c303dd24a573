// Does a HIP graph captured with hipEventRecord around its kernels time them?
// Captures [event 0, n x spin kernel, event 1] from a stream, replays it, and
// compares hipEventElapsedTime(event 0, event 1) of the replay with the same
// sequence recorded outside a graph. Build: hipcc --offload-arch=gfx950 -O2
// graph_event.hip -o graph_event
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void spin(long long cycles, int* out) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += 1;
}

int main() {
  const int n = 20;
  const long long cycles = 20000;  // ~10 us at 2 GHz
  int* d = nullptr;
  CK(hipMalloc(&d, 4));
  CK(hipMemset(d, 0, 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1, f0, f1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&f0));
  CK(hipEventCreate(&f1));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < n; ++i) spin<<<1, 64, 0, s>>>(cycles, d);
  CK(hipEventRecord(e1, s));
  CK(hipStreamEndCapture(s, &g));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  std::printf("graph nodes after capture: %zu\n", nn);
  if (std::getenv("EXPLICIT")) {  // event record nodes added by hand: e0 before the roots, e1 after the leaves
    size_t nr = 0, nl = 0;
    CK(hipGraphGetRootNodes(g, nullptr, &nr));
    hipGraphNode_t roots[64], leaves[64];
    CK(hipGraphGetRootNodes(g, roots, &nr));
    hipGraphNode_t all[256];
    size_t na = 256;
    CK(hipGraphGetNodes(g, all, &na));
    for (size_t i = 0; i < na; ++i) {
      size_t nd = 0;
      CK(hipGraphNodeGetDependentNodes(all[i], nullptr, &nd));
      if (nd == 0) leaves[nl++] = all[i];
    }
    hipGraphNode_t r0, r1;
    CK(hipGraphAddEventRecordNode(&r0, g, nullptr, 0, e0));
    for (size_t i = 0; i < nr; ++i) CK(hipGraphAddDependencies(g, &r0, &roots[i], 1));
    CK(hipGraphAddEventRecordNode(&r1, g, leaves, nl, e1));
    CK(hipGraphGetNodes(g, nullptr, &nn));
    std::printf("graph nodes with explicit records: %zu (roots %zu, leaves %zu)\n", nn, nr, nl);
  }
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    const auto t1 = std::chrono::steady_clock::now();
    float ms = -1.f;
    const hipError_t er = hipEventElapsedTime(&ms, e0, e1);
    // the same sequence outside a graph
    CK(hipEventRecord(f0, s));
    for (int i = 0; i < n; ++i) spin<<<1, 64, 0, s>>>(cycles, d);
    CK(hipEventRecord(f1, s));
    CK(hipStreamSynchronize(s));
    float ms2 = -1.f;
    CK(hipEventElapsedTime(&ms2, f0, f1));
    std::printf("rep %d: graph window %s %.3f us (wall %.1f us), stream window %.3f us\n", rep,
                er == hipSuccess ? "ok" : hipGetErrorString(er), ms * 1e3,
                std::chrono::duration<double, std::micro>(t1 - t0).count(), ms2 * 1e3);
  }
  int h = 0;
  CK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
  std::printf("kernel runs: %d (expect %d)\n", h, 10 * n);
  return 0;
}
