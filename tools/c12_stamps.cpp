// Diagnostic harness (NOT part of the product): the pipelined conv1+conv2 kernel built with
// NIC_STAMPS at the config-2 shape; per wave, cycle sums (s_memtime) per tile in: top
// barrier, epilogue (ts 0) / colour patch (ts 1), B1 barrier, conv1, RGB prefetch issue,
// conv2 stream + partials.  Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNIC_STAMPS \
//     -I neural_network_image_compression_amd/csrc tools/c12_stamps.cpp -o /tmp/c12 && /tmp/c12
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
  const int N = 64, H0 = 256, W0 = 256, H1 = 128, W1 = 128, OH = 64, OW = 64, P = 3 * N;
  float lut[256], k9[9] = {0.299f, 0.587f, 0.114f, -0.16874f, -0.33126f, 0.5f, 0.5f, -0.41869f, -0.08131f},
                  off[3] = {0, .5f, .5f};
  for (int i = 0; i < 256; ++i) lut[i] = i / 255.f;
  CK(upload_constants(lut, k9, k9, off));
  uint8_t* rgb;
  uint16_t *out, *wx, *wx1;
  float *bias, *bias1;
  char* zero16;
  CK(hipMalloc(&rgb, (size_t)N * H0 * W0 * 3));
  std::vector<uint8_t> hr((size_t)N * H0 * W0 * 3);
  for (auto& v : hr) v = rand() & 255;
  CK(hipMemcpy(rgb, hr.data(), hr.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)P * OH * OW * 64 * 4));
  // random f16 weights in [-0.05, 0.05] (constant patterns draw less MFMA power: the clock,
  // and so the cycle split, would not be the real kernel's)
  // C12_ZERO=1: all-zero weights (the schedule's clock, not the power budget's)
  const bool zero = getenv("C12_ZERO") && getenv("C12_ZERO")[0] == '1';
  auto rnd16 = [zero](size_t n) {
    std::vector<_Float16> h(n);
    for (auto& v : h) v = zero ? (_Float16)0.f : (_Float16)((rand() % 2000) / 20000.f - 0.05f);
    return h;
  };
  CK(hipMalloc(&wx, (size_t)2 * 25 * 32 * 64 * 4));
  auto hw = rnd16((size_t)2 * 25 * 32 * 64 * 2);
  CK(hipMemcpy(wx, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&wx1, 2 * 2 * 2 * 64 * 16));
  auto hw1 = rnd16(2 * 2 * 2 * 64 * 8);
  CK(hipMemcpy(wx1, hw1.data(), hw1.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&bias, 2 * 64 * 4));
  CK(hipMemset(bias, 0, 2 * 64 * 4));
  CK(hipMalloc(&bias1, 2 * 32 * 4));
  CK(hipMemset(bias1, 0, 2 * 32 * 4));
  CK(hipMalloc(&zero16, 256));
  CK(hipMemset(zero16, 0, 256));
  ConvArgs a{};
  a.out_s = out;
  a.zero16 = zero16;
  a.wx = wx;
  a.wscale[0] = a.wscale[1] = 1.f;
  a.bias = bias;
  a.P = P;
  a.nimg = N;
  a.H = H1;
  a.W = W1;
  a.OH = OH;
  a.OW = OW;
  a.pad_y = a.pad_x = 1;
  a.rgb = rgb;
  a.wx1 = wx1;
  a.wscale1[0] = a.wscale1[1] = 1.f;
  a.bias1 = bias1;
  a.H0 = H0;
  a.W0 = W0;
  a.p1y = a.p1x = 1;
  int oy, ox, hp, wp;  // padded split colour planes of the fused conv1
  c12_plane_geom(OH, OW, a.pad_y, a.pad_x, a.p1y, a.p1x, &oy, &ox, &hp, &wp);
  CK(hipMalloc(&a.cplane, (size_t)2 * P * hp * wp * 2));
  const int maxb = 1024;
  unsigned long long* st;
  CK(hipMalloc(&st, (size_t)maxb * 64 * 8));
  CK(hipMemset(st, 0, (size_t)maxb * 64 * 8));
#ifdef NIC_STAMPS
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
#endif
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 30; ++it) CK(launch_conv12_x3(a, 0));
  const int iters = 20;
  CK(hipEventRecord(e0, 0));
  for (int it = 0; it < iters; ++it) CK(launch_conv12_x3(a, 0));
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  std::vector<unsigned long long> hs((size_t)maxb * 64);
  CK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
#if NIC_C12R  // c12r_wave: wave 0 = R2 (stream), wave 4 = R1 (vector work)
  const char* nm[7] = {"top-bar", "acc+dma+epi", "flag+acc-st", "conv1", "dma-wait", "stream", "other"};
#else
  const char* nm[7] = {"top-bar", "epi|patch", "flag-wait", "(part+)conv1", "rgb-issue", "stream", "other"};
#endif
  printf("conv12 %.4f ms (%.0f TFLOP/s)\n", ms, 85.564 / ms);
#ifdef NIC_STAMPS
  for (int w = 0; w < 8; w += 4) {
    double s[7] = {}, nt = 0;
    for (int b = 0; b < 256; ++b) {  // one block per CU; the clock words follow block 255's stamps
      if (hs[((size_t)b * 8 + w) * 8 + 7] == 0) continue;
      for (int q = 0; q < 7; ++q) s[q] += hs[((size_t)b * 8 + w) * 8 + q];
      nt += hs[((size_t)b * 8 + w) * 8 + 7];
    }
    printf("  wave %d (ts %d) per tile:", w, w / 4);
    for (int q = 0; q < 7; ++q) printf("  %s %5.0f", nm[q], s[q] / nt);
    printf("\n");
  }
  double cyc = 0, rt = 0;
  for (int b = 0; b < 256; ++b) {
    cyc += hs[256 * 64 + 2 * b];
    rt += hs[256 * 64 + 2 * b + 1];
  }
  if (rt > 0) printf("  clock %.2f GHz\n", 0.1 * cyc / rt);
#endif
  return 0;
}
