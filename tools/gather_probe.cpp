// Diagnostic harness (NOT part of the product): the dconv8 gather (dconv8_gather_kernel) at
// the config-2 shape on a synthetic projection array (64 images x 3 planes x 4 phases x 8 x 8
// tiles x 25 taps x 64 px fp32 = 315 MB), beside a plain streaming read of the same bytes:
//   gather      the kernel on clean data (repeated launches)
//   gather+dirty the kernel right after a kernel that rewrote the whole projection array (as
//               dconv7 does in the decoder)
//   stream      float4 reads of the 315 MB (sum per thread, one store per block)
// Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I neural_network_image_compression_amd/csrc tools/gather_probe.cpp -o /tmp/gather_probe && /tmp/gather_probe
#include "../neural_network_image_compression_amd/csrc/nic_kernels.hip"

#include <cstdio>
#include <vector>

using namespace nic;

#define CK(x)                                                \
  do {                                                       \
    hipError_t e = (x);                                      \
    if (e != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                               \
    }                                                        \
  } while (0)

__global__ void stream_read(const f32x4* __restrict__ p, size_t n4, float* out) {
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const f32x4 v = p[i];
    s += v[0] + v[1] + v[2] + v[3];
  }
  if (s == 12345.f) out[blockIdx.x] = s;  // keeps the loads
}

// rewrite the array with 16-B buffer stores of cache policy AUX (gfx950 CPol bits: 1 = sc0,
// 2 = nt, 16 = sc1); chunked so every offset fits the 32-bit buffer range
template <int AUX>
__global__ void dirty(f32x4* __restrict__ p, size_t n4, float v) {
  const size_t chunk = (size_t)1 << 26;  // f32x4 per resource (1 GiB)
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const size_t c = i / chunk;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p + c * chunk), (short)0, 0x40000000, kBufWord3);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, (f32x4){v, v, v, v}), rs, (unsigned)((i - c * chunk) * 16), 0, AUX);
  }
}

int main() {
  const int N = 64, H = 128, W = 128;  // dconv8 input (= dconv7 output) grid
  float lut[256], k9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, off[3] = {0, .5f, .5f};
  for (int i = 0; i < 256; ++i) lut[i] = i / 255.f;
  CK(upload_constants(lut, k9, k9, off));
  const int ty7 = 8, tx7 = 8;  // dconv7's 8x8 tile grid over its 64x64 input
  const size_t nf = (size_t)3 * N * 4 * ty7 * tx7 * 25 * 64;
  float *proj, *bias, *sink;
  uint8_t* out;
  CK(hipMalloc(&proj, nf * 4));
  CK(hipMalloc(&out, (size_t)N * 4 * H * W * 3));
  CK(hipMalloc(&bias, 64));
  CK(hipMemset(bias, 0, 64));
  CK(hipMalloc(&sink, 1 << 20));
  hipLaunchKernelGGL(dirty<0>, dim3(4096), dim3(256), 0, 0, (f32x4*)proj, nf / 4, 0.01f);
  Dconv8Args a{};
  a.out_u8 = out;
  a.bias = bias;
  a.nimg = N;
  a.H = H;
  a.W = W;
  a.proj = proj;
  a.tiles_y7 = ty7;
  a.tiles_x7 = tx7;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double gb = (nf * 4.0 + (double)N * 4 * H * W * 3) / 1e9;  // GB moved by the gather
  auto timeit = [&](const char* name, auto&& pre, auto&& body, double bytes) {
    float best = 1e9, sum = 0;
    const int reps = 20;
    for (int it = 0; it < 10; ++it) {
      pre();
      body();
    }
    for (int it = 0; it < reps; ++it) {
      pre();
      CK(hipEventRecord(e0, 0));
      body();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    printf("%-16s avg %.4f ms  best %.4f ms  %.2f TB/s (avg)\n", name, sum / reps, best, bytes / (sum / reps));  // GB per ms = TB/s
  };
  auto none = [] {};
  auto gather = [&] { CK(launch_dconv8_gather(a, 0)); };
  auto stream = [&] { hipLaunchKernelGGL(stream_read, dim3(4096), dim3(256), 0, 0, (const f32x4*)proj, nf / 4, sink); };
  timeit("gather", none, gather, gb);
  timeit("stream", none, stream, nf * 4.0 / 1e9);
  auto policy = [&](const char* nm, auto kern) {
    auto mk = [&] { hipLaunchKernelGGL(kern, dim3(4096), dim3(256), 0, 0, (f32x4*)proj, nf / 4, 0.01f); };
    char b[64];
    snprintf(b, sizeof b, "write %s", nm);
    timeit(b, none, mk, nf * 4.0 / 1e9);  // the write itself
    snprintf(b, sizeof b, "  gather after");
    timeit(b, mk, gather, gb);
    snprintf(b, sizeof b, "  stream after");
    timeit(b, mk, stream, nf * 4.0 / 1e9);
  };
  policy("plain", dirty<0>);
  policy("sc0", dirty<1>);
  policy("nt", dirty<2>);
  policy("sc1", dirty<16>);
  policy("sc0sc1", dirty<17>);
  policy("sc1nt", dirty<18>);
  policy("all", dirty<19>);
  return 0;
}
