// Per-kernel cost inside a replayed HIP graph: K back-to-back launches of a kernel that does almost
// nothing, for several grid sizes and written footprints.  Separates the fixed cost of a kernel
// boundary (dispatch + end-of-kernel cache maintenance across the XCDs) from the work of the small
// C2 kernels.   hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o tools/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_touch(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.0f;
}

int main() {
  const int K = 100;
  float* buf;
  const size_t maxn = 64u << 20;
  CK(hipMalloc(&buf, maxn * sizeof(float)));
  CK(hipMemset(buf, 0, maxn * sizeof(float)));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int sizes[] = {64, 256 * 64, 1356 * 256, 1 << 20, 1 << 22};
  for (int n : sizes) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, st, buf, n);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int R = 20;
    CK(hipEventRecord(a, st));
    for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"elements\": %d, \"blocks\": %d, \"bytes_rw\": %zu, \"us_per_kernel\": %.3f}\n", n, (n + 255) / 256,
           (size_t)n * 8, 1000.0 * ms / (R * K));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  // the same kernels launched directly on the stream (no graph)
  {
    const int n = 256 * 64;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, st, buf, n);
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int k = 0; k < 10 * K; ++k) hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, st, buf, n);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"stream_launch\": true, \"elements\": %d, \"us_per_kernel\": %.3f}\n", n, 1000.0 * ms / (10 * K));
  }
  CK(hipFree(buf));
  return 0;
}
