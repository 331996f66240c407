// Diagnostic harness (NOT part of the product): the weight-stationary conv kernels built
// with NIC_STAMPS, run at the config-2 shapes on synthetic data.  Wave 0 of every block
// sums its cycles (s_memtime) in: waiting at the tile barrier (vmcnt drain + s_barrier),
// the epilogue, the next halo's DMA issue (+ residual loads), and the MFMA stream; s_memrealtime (100 MHz) gives the
// shader clock.  Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNIC_STAMPS \
//     -I neural_network_image_compression_amd/csrc tools/ws_stamps.cpp -o /tmp/ws_stamps && /tmp/ws_stamps
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

struct Case {
  const char* name;
  LayerId id;
  int H, W, OH, OW, taps;
  bool resid;
};

int main() {
  const int N = 64, P = 3 * N;
  const Case cases[] = {
      {"k3", L_CONV3, 64, 64, 64, 64, 9, false},
      {"k3_resid", L_CONV4, 64, 64, 64, 64, 9, true},
      {"dconv7", L_DCONV7, 64, 64, 128, 128, 25, false},
  };
  float lut[256], k9[9] = {0}, off[3] = {0, .5f, .5f};
  for (int i = 0; i < 256; ++i) lut[i] = i / 255.f;
  CK(upload_constants(lut, k9, k9, off));
  for (const Case& c : cases) {
    const size_t in_n = (size_t)P * c.H * c.W * 64, out_n = (size_t)P * c.OH * c.OW * 64;
    uint16_t *in, *out, *res, *wx;
    float* bias;
    char* zero16;
    CK(hipMalloc(&in, in_n * 4));
    CK(hipMalloc(&out, out_n * 4));
    CK(hipMalloc(&res, out_n * 4));
    CK(hipMalloc(&bias, 2 * 64 * 4));
    CK(hipMalloc(&zero16, 256));
    CK(hipMemset(zero16, 0, 256));
    CK(hipMemset(bias, 0, 2 * 64 * 4));
    const size_t wn = (size_t)2 * c.taps * 64 * 64 * 2;
    CK(hipMalloc(&wx, wn * 2));
    std::vector<uint16_t> h(in_n * 2);
    for (auto& v : h) {
      _Float16 f = (_Float16)((rand() % 2000) / 1000.f - 1.f);
      std::memcpy(&v, &f, 2);
    }
    CK(hipMemcpy(in, h.data(), in_n * 4, hipMemcpyHostToDevice));
    std::vector<uint16_t> hw(wn);
    for (auto& v : hw) {
      _Float16 f = (_Float16)((rand() % 2000) / 20000.f - 0.05f);
      std::memcpy(&v, &f, 2);
    }
    CK(hipMemcpy(wx, hw.data(), wn * 2, hipMemcpyHostToDevice));
    ConvArgs a{};
    a.in_s = in;
    a.out_s = out;
    a.res_s = res;
    a.zero16 = zero16;
    a.wx = wx;
    a.wscale[0] = a.wscale[1] = 1.f;
    a.bias = bias;
    a.P = P;
    a.nimg = N;
    a.H = c.H;
    a.W = c.W;
    a.OH = c.OH;
    a.OW = c.OW;
    a.pad_y = a.pad_x = 1;
    const int maxb = 4096;
    unsigned long long* st;
    CK(hipMalloc(&st, maxb * 8 * 8));
    CK(hipMemset(st, 0, maxb * 8 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int it = 0; it < 20; ++it) CK(launch_layer_x3(c.id, a, 0));
    CK(hipEventRecord(e0, 0));
    CK(launch_layer_x3(c.id, a, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> hs(maxb * 8);
    CK(hipMemcpy(hs.data(), st, maxb * 64, hipMemcpyDeviceToHost));
    // per tap-set group: sums
    double w[26] = {}, ep[26] = {}, mf[26] = {}, nt[26] = {}, life[26] = {}, rt[26] = {}, nb[26] = {};
    int nblk = 0;
    for (int b = 0; b < maxb; ++b) {
      if (hs[b * 8 + 5] == 0) continue;
      ++nblk;
      const int k = (int)hs[b * 8 + 6];
      w[k] += hs[b * 8 + 0];
      ep[k] += hs[b * 8 + 1];
      mf[k] += hs[b * 8 + 2];
      nt[k] += hs[b * 8 + 3];
      life[k] += hs[b * 8 + 4];
      rt[k] += hs[b * 8 + 5];
      nb[k] += 1;
    }
    printf("%-9s %.4f ms, %d blocks\n", c.name, ms, nblk);
    for (int k = 0; k < 26; ++k) {
      if (nb[k] == 0) continue;
      const double per = nt[k];
      printf("  taps %2d: %4.0f blocks, tiles/block %5.1f, clock %.2f GHz, life %8.0f cyc; per tile: wait %5.0f  "
             "epi+issue %5.0f  mfma %5.0f (ideal %5.0f = 2 waves x %d MFMA x 16)\n",
             k, nb[k], per / nb[k], 0.1 * life[k] / rt[k],
             life[k] / nb[k], w[k] / per, ep[k] / per, mf[k] / per, 2.0 * k * 2 * 4 * 3 * 16, k * 2 * 4 * 3);
    }
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(res));
    CK(hipFree(wx));
    CK(hipFree(bias));
    CK(hipFree(zero16));
    CK(hipFree(st));
  }
  return 0;
}
