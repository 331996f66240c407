// Inter-kernel gap probe: K back-to-back launches of a fixed-work kernel on one stream,
// plain launches vs one hipGraph of the same K launches.  Prints per-launch time of each
// and the implied gap.  hipcc --offload-arch=gfx950 -O3 tools/gap_probe.cpp -o /tmp/gap_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ __launch_bounds__(256) void work(float* out, int iters, int write_floats) {
  float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) a = __builtin_fmaf(a, 0.999f, b);
  // write a slab so the L2 holds dirty lines at kernel end
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (size_t i = t; i < (size_t)write_floats; i += (size_t)gridDim.x * 256) out[i] = a + i;
}

int main(int argc, char** argv) {
  const int K = 50;
  const int blocks = argc > 1 ? atoi(argv[1]) : 2048;
  const int iters = argc > 2 ? atoi(argv[2]) : 20000;
  const int wf = argc > 3 ? atoi(argv[3]) : (64 << 20);
  float* out;
  CK(hipMalloc(&out, (size_t)wf * 4 + 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;
  // single launch duration
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, st, out, iters, wf);
  CK(hipEventRecord(e0, st));
  hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, st, out, iters, wf);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  const float one = ms;
  CK(hipEventRecord(e0, st));
  for (int k = 0; k < K; ++k) hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, st, out, iters, wf);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  const float plain = ms / K;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < K; ++k) hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, st, out, iters, wf);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  const float graph = ms / K;
  printf("blocks %d iters %d write %d MB: single %.1f us, plain %.1f us/launch, graph %.1f us/launch\n", blocks, iters,
         wf / (1 << 18), one * 1e3f, plain * 1e3f, graph * 1e3f);
  return 0;
}
