// Probe: multi-stream fork/join hipGraph capture on this ROCm runtime.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(float* p, int i) { if (threadIdx.x == 0) p[i] += 1.0f; }
#define CK(x) do { hipError_t rr_ = (x); if (rr_ != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(rr_)); return 1; } } while (0)
int run(int variant) {
  hipStream_t s[4];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t ev[16];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  float* p; CK(hipMalloc(&p, 64 * 4)); CK(hipMemset(p, 0, 256));
  int ne = 0;
  auto dep = [&](hipStream_t a, hipStream_t b) { (void)hipEventRecord(ev[ne], a); (void)hipStreamWaitEvent(b, ev[ne], 0); ++ne; };
  CK(hipStreamBeginCapture(s[0], variant == 3 ? hipStreamCaptureModeGlobal : hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s[0], p, 0);
  dep(s[0], s[1]);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s[1], p, 1);
  if (variant >= 1) {
    dep(s[0], s[2]);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s[2], p, 2);
    dep(s[1], s[3]);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s[3], p, 3);
    dep(s[3], s[1]);
    dep(s[2], s[1]);
  }
  if (variant == 2) { dep(s[1], s[0]); dep(s[2], s[0]); dep(s[3], s[0]); }
  else dep(s[1], s[0]);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s[0], p, 4);
  hipGraph_t g;
  printf("variant %d: end capture...\n", variant); fflush(stdout);
  CK(hipStreamEndCapture(s[0], &g));
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, s[0]));
  CK(hipStreamSynchronize(s[0]));
  float h[5]; CK(hipMemcpy(h, p, 20, hipMemcpyDeviceToHost));
  printf("variant %d ok: %g %g %g %g %g\n", variant, h[0], h[1], h[2], h[3], h[4]); fflush(stdout);
  return 0;
}
// variant 4: two single-stream captured child graphs joined by explicit dependencies
int run_child() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* p; CK(hipMalloc(&p, 256)); CK(hipMemset(p, 0, 256));
  hipGraph_t top; CK(hipGraphCreate(&top, 0));
  hipGraphNode_t nodes[3];
  for (int i = 0; i < 3; ++i) {
    hipGraph_t g;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s, p, i);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s, p, i);
    CK(hipStreamEndCapture(s, &g));
    const hipGraphNode_t* deps = (i == 2) ? nodes : nullptr;
    CK(hipGraphAddChildGraphNode(&nodes[i], top, deps, (i == 2) ? 2 : 0, g));
  }
  hipGraphExec_t x; CK(hipGraphInstantiate(&x, top, nullptr, nullptr, 0));
  for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(x, s));
  CK(hipStreamSynchronize(s));
  float h[3]; CK(hipMemcpy(h, p, 12, hipMemcpyDeviceToHost));
  printf("variant 4 ok: %g %g %g\n", h[0], h[1], h[2]); fflush(stdout);
  return 0;
}
int main(int argc, char** argv) { int v = atoi(argv[1]); return v == 4 ? run_child() : run(v); }
