// Diagnostic harness (NOT part of the product): compiles the codec kernels with
// NIC_STAMPS and NIC_WS=0 (the one-tile-per-block kernels), runs one split-f16 conv layer on synthetic data at the config-2 shape and
// reports the average per-block cycles in halo staging / MFMA main loop / epilogue, and
// the implied concurrency.  Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNIC_STAMPS \
//     -I neural_network_image_compression_amd/csrc tools/stamps.cpp -o /tmp/stamps && /tmp/stamps
#include "../neural_network_image_compression_amd/csrc/nic_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace nic;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

struct Case {
  const char* name;
  LayerId id;
  int cin, cout, H, W, OH, OW, taps, th, tw;
  bool tr, u8in, u8out, resid;
};

int main() {
  const int N = 64, P = 3 * N;
  std::vector<Case> cases = {
      {"conv2", L_CONV2, 32, 64, 128, 128, 64, 64, 25, 8, 8, false, false, false, false},
      {"conv3", L_CONV3, 64, 64, 64, 64, 64, 64, 9, 8, 16, false, false, false, false},
      {"conv4", L_CONV4, 64, 64, 64, 64, 64, 64, 9, 8, 16, false, false, false, true},
      {"conv8", L_CONV8, 64, 32, 64, 64, 32, 32, 25, 4, 8, false, false, true, false},
      {"dconv1", L_DCONV1, 32, 64, 32, 32, 64, 64, 25, 8, 8, true, true, false, false},
      {"dconv7", L_DCONV7, 64, 64, 64, 64, 128, 128, 25, 8, 16, true, false, false, false},
  };
  float lut[256], k9[9] = {0}, off[3] = {0, .5f, .5f};
  for (int i = 0; i < 256; ++i) lut[i] = i / 255.f;
  CK(upload_constants(lut, k9, k9, off));
  int clk_khz = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  for (const Case& c : cases) {
    const size_t in_n = (size_t)P * c.H * c.W * c.cin, out_n = (size_t)P * c.OH * c.OW * c.cout;
    float *in, *out, *res, *bias;
    uint8_t *in8, *out8;
    uint16_t* wx;
    CK(hipMalloc(&in, in_n * 4));
    CK(hipMalloc(&out, out_n * 4));
    CK(hipMalloc(&res, out_n * 4));
    CK(hipMalloc(&bias, 2 * c.cout * 4));
    CK(hipMalloc(&in8, (size_t)N * c.H * c.W * 96));
    CK(hipMalloc(&out8, (size_t)N * c.OH * c.OW * 96));
    const size_t wn = (size_t)2 * c.taps * c.cin * c.cout * 2;
    CK(hipMalloc(&wx, wn * 2));
    std::vector<float> h(in_n);
    for (auto& v : h) v = (rand() % 2000) / 1000.f - 1.f;
    CK(hipMemcpy(in, h.data(), in_n * 4, hipMemcpyHostToDevice));
    std::vector<uint16_t> hw(wn);
    for (auto& v : hw) {
      _Float16 f = (_Float16)((rand() % 2000) / 20000.f - 0.05f);
      std::memcpy(&v, &f, 2);
    }
    CK(hipMemcpy(wx, hw.data(), wn * 2, hipMemcpyHostToDevice));
    CK(hipMemset(bias, 0, 2 * c.cout * 4));
    CK(hipMemset(in8, 7, (size_t)N * c.H * c.W * 96));
    char* zero16;
    CK(hipMalloc(&zero16, 256));
    CK(hipMemset(zero16, 0, 256));
    ConvArgs a{};
    a.in = in;
    a.in_s = (const uint16_t*)in;
    a.zero16 = zero16;
    a.in_u8 = in8;
    a.out = out;
    a.out_s = (uint16_t*)out;
    a.res = c.resid ? res : nullptr;
    a.res_s = (const uint16_t*)res;
    a.out_u8 = out8;
    a.wx = wx;
    a.wscale[0] = a.wscale[1] = 1.f;
    a.bias = bias;
    a.P = P;
    a.nimg = N;
    a.H = c.H;
    a.W = c.W;
    a.OH = c.OH;
    a.OW = c.OW;
    a.pad_y = a.pad_x = c.taps == 9 ? 1 : 1;
    const int gy = c.tr ? c.H : c.OH, gx = c.tr ? c.W : c.OW;
    const size_t blocks = (size_t)((gy + c.th - 1) / c.th) * ((gx + c.tw - 1) / c.tw) * P;
    unsigned long long* st;
    CK(hipMalloc(&st, blocks * 4 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int it = 0; it < 3; ++it) CK(launch_layer_x3(c.id, a, 0));
    CK(hipEventRecord(e0, 0));
    CK(launch_layer_x3(c.id, a, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> hs(blocks * 4);
    CK(hipMemcpy(hs.data(), st, blocks * 32, hipMemcpyDeviceToHost));

    double s01 = 0, s12 = 0, s23 = 0;
    unsigned long long t_min = ~0ull, t_max = 0;
    for (size_t b = 0; b < blocks; ++b) {
      s01 += hs[b * 4 + 1] - hs[b * 4 + 0];
      s12 += hs[b * 4 + 2] - hs[b * 4 + 1];
      s23 += hs[b * 4 + 3] - hs[b * 4 + 2];
      t_min = std::min(t_min, hs[b * 4]);
      t_max = std::max(t_max, hs[b * 4 + 3]);
    }
    const double span = (double)(t_max - t_min), life = (s01 + s12 + s23) / blocks;
    printf("%-7s blocks %6zu  %.3f ms  cycles/block: staging %7.0f  mfma %7.0f  epilogue %6.0f  "
           "(%.0f%% / %.0f%% / %.0f%%)  concurrent blocks/CU %.2f\n",
           c.name, blocks, ms, s01 / blocks, s12 / blocks, s23 / blocks, 100 * s01 / blocks / life,
           100 * s12 / blocks / life, 100 * s23 / blocks / life, life * blocks / span / 256.0);
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(res));
    CK(hipFree(bias));
    CK(hipFree(in8));
    CK(hipFree(out8));
    CK(hipFree(wx));
    CK(hipFree(st));
    CK(hipFree(zero16));
  }
  return 0;
}
