// Diagnostic harness (NOT part of the product): dconv8_strip_kernel built with NIC_STAMPS at
// the config-2 shape; per MFMA wave, cycle sums (s_memtime) in: the row barrier, the DMA
// issue, the MFMA segment, the vmcnt wait for row y+2.  Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNIC_STAMPS \
//     -I neural_network_image_compression_amd/csrc tools/d8_stamps.cpp -o /tmp/d8_stamps && /tmp/d8_stamps
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
  const int N = 64, H = 128, W = 128;
  float lut[256], k9[9] = {0}, off[3] = {0, .5f, .5f};
  for (int i = 0; i < 256; ++i) lut[i] = i / 255.f;
  CK(upload_constants(lut, k9, k9, off));
  uint16_t *in, *wx;
  uint8_t* out;
  float* bias;
  char* zero16;
  CK(hipMalloc(&in, (size_t)3 * N * H * W * 256));
  CK(hipMemset(in, 0x11, (size_t)3 * N * H * W * 256));
  CK(hipMalloc(&out, (size_t)N * 4 * H * W * 3));
  CK(hipMalloc(&wx, 2 * 9 * 2 * 2 * 64 * 16));
  CK(hipMemset(wx, 0x22, 2 * 9 * 2 * 2 * 64 * 16));
  CK(hipMalloc(&bias, 64));
  CK(hipMemset(bias, 0, 64));
  CK(hipMalloc(&zero16, 256));
  CK(hipMemset(zero16, 0, 256));
  Dconv8Args a{};
  a.in_s = in;
  a.zero16 = zero16;
  a.out_u8 = out;
  a.wx = wx;
  a.wscale[0] = a.wscale[1] = 1.f;
  a.bias = bias;
  a.nimg = N;
  a.H = H;
  a.W = W;
  const int maxb = 8192;
  unsigned long long* st;
  CK(hipMalloc(&st, (size_t)maxb * 16 * 8));
  CK(hipMemset(st, 0, (size_t)maxb * 16 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 20; ++it) CK(launch_dconv8_x3(a, 0));
  CK(hipEventRecord(e0, 0));
  CK(launch_dconv8_x3(a, 0));
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> hs((size_t)maxb * 16);
  CK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
  double s[3][4] = {};
  int nb = 0;
  for (int b = 0; b < maxb; ++b) {
    if (hs[(size_t)b * 16 + 2] == 0) continue;
    ++nb;
    for (int w = 0; w < 3; ++w)
      for (int k = 0; k < 4; ++k) s[w][k] += hs[((size_t)b * 4 + w) * 4 + k];
  }
  printf("dconv8 strip %.4f ms, %d blocks, %d rows each\n", ms, nb, H);
  for (int w = 0; w < 3; ++w)
    printf("  wave %d per row: barrier %6.0f  issue %6.0f  mfma+ex %6.0f  vmcnt-wait %6.0f\n", w, s[w][0] / nb / H,
           s[w][1] / nb / H, s[w][2] / nb / H, s[w][3] / nb / H);
  return 0;
}
