// Diagnostic harness (NOT part of the product): the fused k3 residual pair
// (conv_k3pair_kernel) built with NIC_STAMPS at the config-2 shape (192 planes of 64 x 64 x 64
// split), synthetic data.  Wave 0 (conv_a) and wave 4 (conv_b) of every block sum their cycles
// (s_memtime) in: the step barrier (vmcnt drain + s_barrier), the MFMA stream, the epilogue
// and the next input row's DMA issue; s_memrealtime (100 MHz) gives the shader clock.
// Usage: k3p_stamps [zero]   ("zero": all-zero weights, the power probe's clock)
// Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNIC_STAMPS \
//     -I neural_network_image_compression_amd/csrc tools/k3p_stamps.cpp -o /tmp/k3p_stamps && /tmp/k3p_stamps
#include "../neural_network_image_compression_amd/csrc/nic_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
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

int main(int argc, char** argv) {
  const bool zero = argc > 1 && !strcmp(argv[1], "zero");
  const int N = 64, P = 3 * N, H = 64, W = 64;
  float lut[256], k9[9] = {0}, off[3] = {0, .5f, .5f};
  for (int i = 0; i < 256; ++i) lut[i] = i / 255.f;
  CK(upload_constants(lut, k9, k9, off));
  const size_t n = (size_t)P * H * W * 64;
  uint16_t *in, *out, *wx, *wx2;
  float* bias;
  CK(hipMalloc(&in, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&bias, 2 * 64 * 4));
  CK(hipMemset(bias, 0, 2 * 64 * 4));
  const size_t wn = (size_t)2 * 9 * 64 * 64 * 2;
  CK(hipMalloc(&wx, wn * 2));
  CK(hipMalloc(&wx2, wn * 2));
  std::vector<uint16_t> h(n * 2);
  for (auto& v : h) {
    _Float16 f = (_Float16)((rand() % 2000) / 1000.f - 1.f);
    std::memcpy(&v, &f, 2);
  }
  CK(hipMemcpy(in, h.data(), n * 4, hipMemcpyHostToDevice));
  std::vector<uint16_t> hw(wn);
  for (auto& v : hw) {
    _Float16 f = (_Float16)(zero ? 0.f : (rand() % 2000) / 20000.f - 0.05f);
    std::memcpy(&v, &f, 2);
  }
  CK(hipMemcpy(wx, hw.data(), wn * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(wx2, hw.data(), wn * 2, hipMemcpyHostToDevice));
  ConvArgs a{};
  a.in_s = in;
  a.out_s = out;
  a.res_s = in;
  a.wx = wx;
  a.wx2 = wx2;
  a.wscale[0] = a.wscale[1] = a.wscale2[0] = a.wscale2[1] = 1.f;
  a.bias = bias;
  a.bias2 = bias;
  a.P = P;
  a.nimg = N;
  a.H = a.OH = H;
  a.W = a.OW = W;
  a.pad_y = a.pad_x = 1;
  const int maxb = 1024;
  unsigned long long* st;
  CK(hipMalloc(&st, maxb * 16 * 8));
  CK(hipMemset(st, 0, maxb * 16 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 30; ++it) CK(launch_k3pair_x3(a, 0));
  CK(hipEventRecord(e0, 0));
  const int reps = 10;
  for (int it = 0; it < reps; ++it) CK(launch_k3pair_x3(a, 0));
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> hs(maxb * 16);
  CK(hipMemcpy(hs.data(), st, maxb * 16 * 8, hipMemcpyDeviceToHost));
  printf("k3pair%s: %.4f ms per launch\n", zero ? " (zero weights)" : "", ms / reps);
  for (int role = 0; role < 2; ++role) {
    double s[7] = {};
    int nb = 0;
    for (int b = 0; b < maxb; ++b) {
      const unsigned long long* o = &hs[b * 16 + role * 8];
      if (!o[7]) continue;
      ++nb;
      for (int k = 0; k < 7; ++k) s[k] += o[k];
    }
    if (!nb) continue;
    const double steps = s[4];
    // one row step: MT = 4 tiles x 9 taps x 2 k32-steps x 3 MFMAs of 16 cycles, two waves per SIMD
    printf("  %s: %d blocks, steps/block %.1f, clock %.2f GHz, life %.0f cyc; per step: wait %.0f  mfma %.0f  "
           "epi %.0f  dma-issue %.0f  (MFMA floor per SIMD step: 2 x 216 x 16 = 6912)\n",
           role ? "conv_b" : "conv_a", nb, steps / nb, 0.1 * s[5] / s[6], s[5] / nb, s[0] / steps, s[1] / steps,
           s[2] / steps, s[3] / steps);
  }
  return 0;
}
