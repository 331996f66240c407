// Diagnostic harness (NOT part of the product): conv8 (conv_ws2_kernel<64,32,4,4,U8 latent>)
// built with NIC_STAMPS at the config-2 shape (64 x 3 planes of 64 x 64 x 64 -> 32 x 32 x 32);
// per wave (ts = tap quarter), cycle sums per tile of: the top barrier (DMA wait + barrier) and
// the rest (epilogue (ts 0), next halo's DMA issue, MFMA stream, partial stores).  Random
// split data and weights (constant patterns draw less MFMA power).  Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNIC_STAMPS \
//     -I neural_network_image_compression_amd/csrc tools/c8_stamps.cpp -o /tmp/c8 && /tmp/c8
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

int main() {
  const int N = 64, H = 64, W = 64, OH = 32, OW = 32, P = 3 * N;
  auto rnd16 = [](size_t n, float s) {
    std::vector<_Float16> h(n);
    for (auto& v : h) v = (_Float16)(((rand() % 2000) / 1000.f - 1.f) * s);
    return h;
  };
  uint16_t *in, *wx;
  uint8_t* lat;
  float* bias;
  char* zero16;
  CK(hipMalloc(&in, (size_t)P * H * W * 64 * 4));
  auto hin = rnd16((size_t)P * H * W * 64 * 2, 0.5f);
  CK(hipMemcpy(in, hin.data(), hin.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&wx, (size_t)2 * 25 * 64 * 32 * 4));
  auto hw = rnd16((size_t)2 * 25 * 64 * 32 * 2, getenv("C8_ZERO") ? 0.f : 0.05f);  // C8_ZERO: all-zero weights
  CK(hipMemcpy(wx, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&lat, (size_t)N * OH * OW * 96));
  CK(hipMalloc(&bias, 2 * 32 * 4));
  CK(hipMemset(bias, 0, 2 * 32 * 4));
  CK(hipMalloc(&zero16, 256));
  CK(hipMemset(zero16, 0, 256));
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
  a.OH = OH;
  a.OW = OW;
  a.pad_y = a.pad_x = 1;
  a.out_u8 = lat;
  const int maxb = 1024;
  unsigned long long* st;
  CK(hipMalloc(&st, (size_t)maxb * 64 * 8));
  CK(hipMemset(st, 0, (size_t)maxb * 64 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 30; ++it) CK(launch_layer_x3(L_CONV8, a, 0));
  const int iters = 20;
  CK(hipEventRecord(e0, 0));
  for (int it = 0; it < iters; ++it) CK(launch_layer_x3(L_CONV8, a, 0));
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  std::vector<unsigned long long> hs((size_t)maxb * 64);
  CK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
  printf("conv8 %.4f ms (%.0f TFLOP/s)\n", ms, 20.133 / ms);
  const char* nm[7] = {"top-bar", "epilogue", "dma-issue", "stream", "partials", "drain", "tail"};
  for (int w = 0; w < 8; ++w) {
    double sum[7] = {}, nt = 0;
    for (int b = 0; b < 256; ++b) {
      const unsigned long long* o = &hs[((size_t)b * 8 + w) * 8];
      if (o[7] == 0) continue;
      for (int q = 0; q < 7; ++q) sum[q] += o[q];
      nt += o[7];
    }
    printf("  wave %d (cg %d, ts %d) per tile:", w, w % 2, w / 2);
    for (int q = 0; q < 7; ++q) printf(" %s %5.0f", nm[q], sum[q] / nt);
    printf("  (%.1f tiles/block)\n", nt / 256);
  }
  return 0;
}
