// Diagnostic harness (NOT part of the product): could the dconv8 gather run beside dconv7 instead
// of after it?  dconv7 (conv_ws_kernel<..., PROJ>, launch_dconv7_proj_x3) and the gather
// (launch_dconv8_gather) at the config-2 shapes on synthetic data, timed as
//   seq      dconv7 then the gather on one stream (the decoder's order today)
//   overlap  dconv7 on stream A and the gather on stream B, both released by one event
//            (the gather reads a second projection array: timing only, not a data flow)
//   d7 / g   each alone
// Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I neural_network_image_compression_amd/csrc tools/overlap_probe.cpp -o /tmp/op && /tmp/op
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

template <class T>
static T* dev_random(size_t n, float lo, float hi) {
  std::vector<_Float16> h(n * sizeof(T) / 2);
  for (auto& v : h) v = (_Float16)(lo + (hi - lo) * (rand() / (float)RAND_MAX));
  T* d;
  CK(hipMalloc(&d, n * sizeof(T)));
  CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main() {
  const int N = 64, P = 3 * N, H = 64, W = 64;
  float lut[256], k9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, off[3] = {0, .5f, .5f};
  for (int i = 0; i < 256; ++i) lut[i] = i / 255.f;
  CK(upload_constants(lut, k9, k9, off));
  const size_t in_n = (size_t)P * H * W * 64 * 2;
  uint16_t* in = dev_random<uint16_t>(in_n, -1.f, 1.f);
  uint16_t* wx = dev_random<uint16_t>((size_t)2 * 25 * 64 * 64 * 2, -0.05f, 0.05f);
  uint16_t* pw = dev_random<uint16_t>((size_t)2 * 2 * 2 * 2 * 64 * 8, -0.05f, 0.05f);
  float* bias;
  CK(hipMalloc(&bias, 2 * 64 * 4));
  CK(hipMemset(bias, 0, 2 * 64 * 4));
  char* zero16;
  CK(hipMalloc(&zero16, 256));
  CK(hipMemset(zero16, 0, 256));
  const int ty = (H + 7) / 8, tx = (W + 7) / 8;
  const size_t nproj = (size_t)P * 4 * ty * tx * 25 * 64;
  float *proj_a, *proj_b;
  CK(hipMalloc(&proj_a, nproj * 4));
  CK(hipMalloc(&proj_b, nproj * 4));
  CK(hipMemset(proj_b, 0, nproj * 4));
  uint8_t* rgb;
  CK(hipMalloc(&rgb, (size_t)N * 4 * H * W * 3 * 4));

  ConvArgs a{};
  a.in_s = in;
  a.zero16 = zero16;
  a.wx = wx;
  a.wscale[0] = a.wscale[1] = 1.f;
  a.bias = bias;
  a.P = P;
  a.nimg = N;
  a.H = H;
  a.W = W;
  a.pad_y = a.pad_x = 1;
  a.OH = 2 * H;
  a.OW = 2 * W;
  a.proj = proj_a;
  a.proj_w = pw;
  a.proj_scale[0] = a.proj_scale[1] = 1.f;

  Dconv8Args g{};
  g.out_u8 = rgb;
  g.bias = bias;
  g.nimg = N;
  g.H = 2 * H;
  g.W = 2 * W;
  g.tiles_y7 = ty;
  g.tiles_x7 = tx;

  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t e0, e1, ea, eb;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));

  auto d7 = [&](hipStream_t s) { CK(launch_dconv7_proj_x3(a, s)); };
  auto gat = [&](hipStream_t s, float* proj) {
    g.proj = proj;
    CK(launch_dconv8_gather(g, s));
  };
  auto timeit = [&](const char* name, auto&& body) {
    const int reps = 30;
    for (int it = 0; it < 20; ++it) body();
    CK(hipDeviceSynchronize());
    float sum = 0, best = 1e9;
    for (int it = 0; it < reps; ++it) {
      CK(hipEventRecord(e0, sa));
      body();
      CK(hipEventRecord(e1, sa));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      sum += ms;
      best = ms < best ? ms : best;
    }
    printf("%-10s avg %.4f ms  best %.4f ms\n", name, sum / reps, best);
  };
  for (int round = 0; round < 2; ++round) {
    timeit("d7", [&] { d7(sa); });
    timeit("g", [&] { gat(sa, proj_a); });
    timeit("seq", [&] {
      d7(sa);
      gat(sa, proj_a);
    });
    timeit("overlap", [&] {  // both after the previous pair; sa waits for sb before the end event
      CK(hipEventRecord(ea, sa));
      CK(hipStreamWaitEvent(sb, ea, 0));
      d7(sa);
      gat(sb, proj_b);
      CK(hipEventRecord(eb, sb));
      CK(hipStreamWaitEvent(sa, eb, 0));
    });
  }
  return 0;
}
