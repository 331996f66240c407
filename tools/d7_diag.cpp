// Diagnostic harness (NOT part of the product): dconv7 with dconv8's projection fused
// (conv_ws_kernel<64,64,8,8,false,true,true>) and conv3 at the config-2 shapes on synthetic
// data, timed with hipEvents after 30 warm-up launches.  Built in variants with the
// NIC_DIAG_* switches of nic_kernels.hip (each removes one part of the work and gives wrong
// results) to bound what each part costs; with -DNIC_STAMPS it prints the per-tile cycle split.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off [-DNIC_DIAG_ONETILE ...] \
//     tools/d7_diag.cpp -o ab/d7_base
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

template <class T>
static T* dev_random(size_t n, float lo, float hi) {
  std::vector<_Float16> h(n * sizeof(T) / 2);
  for (auto& v : h) v = (_Float16)(lo + (hi - lo) * (rand() / (float)RAND_MAX));
  T* d;
  CK(hipMalloc(&d, n * sizeof(T)));
  CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int N = 64, P = 3 * N, H = 64, W = 64;
  const int iters = argc > 1 ? atoi(argv[1]) : 50;
  float lut[256], k9[9] = {0}, off[3] = {0, .5f, .5f};
  for (int i = 0; i < 256; ++i) lut[i] = i / 255.f;
  CK(upload_constants(lut, k9, k9, off));
  const size_t in_n = (size_t)P * H * W * 64 * 2;  // halves
  uint16_t* in = dev_random<uint16_t>(in_n, -1.f, 1.f);
  uint16_t* wx = dev_random<uint16_t>((size_t)2 * 25 * 64 * 64 * 2, -0.05f, 0.05f);
  uint16_t* pw = dev_random<uint16_t>((size_t)2 * 2 * 2 * 2 * 64 * 8, -0.05f, 0.05f);
  float* bias;
  CK(hipMalloc(&bias, 2 * 64 * 4));
  CK(hipMemset(bias, 0, 2 * 64 * 4));
  char* zero16;
  CK(hipMalloc(&zero16, 256));
  CK(hipMemset(zero16, 0, 256));
  // zero operands (the MFMAs' data-dependent power is minimal): 'z' all, 'w' weights, 'a' activations
  const char zm = argc > 2 ? argv[2][0] : 'r';
  if (zm == 'z' || zm == 'a') CK(hipMemset(in, 0, in_n * 2));
  if (zm == 'z' || zm == 'w') {
    CK(hipMemset(wx, 0, (size_t)2 * 25 * 64 * 64 * 2 * 2));
    CK(hipMemset(pw, 0, (size_t)2 * 2 * 2 * 2 * 64 * 8 * 2));
  }
  const int ty = (H + 7) / 8, tx = (W + 7) / 8;
  float* proj;
  CK(hipMalloc(&proj, (size_t)P * 4 * ty * tx * 25 * 64 * 4));
  uint16_t* out;  // conv3 output
  CK(hipMalloc(&out, in_n * 2));
  const int maxb = 4096;
  unsigned long long* st;
  CK(hipMalloc(&st, maxb * 8 * 8));
  CK(hipMemset(st, 0, maxb * 8 * 8));
#ifdef NIC_STAMPS
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
#endif
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int layer = 0; layer < 3; ++layer) {
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
    double gflop;
    if (layer == 0) {
      a.OH = 2 * H;
      a.OW = 2 * W;
      a.proj = proj;
      a.proj_w = pw;
      a.proj_scale[0] = a.proj_scale[1] = 1.f;
      gflop = 171.1276;
    } else {
      a.OH = H;
      a.OW = W;
      a.out_s = out;
      a.res_s = in;  // conv4: residual of the same shape
      gflop = 57.982;
    }
    auto go = [&] {
      return layer == 0 ? launch_dconv7_proj_x3(a, 0) : launch_layer_x3(layer == 1 ? L_CONV3 : L_CONV4, a, 0);
    };
    for (int it = 0; it < 30; ++it) CK(go());
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < iters; ++it) CK(go());
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("%-7s %.4f ms  %.1f TFLOP/s  frac %.3f\n", layer == 0 ? "dconv7" : layer == 1 ? "conv3" : "conv4", ms,
           gflop / ms, gflop / ms / 833.3);
#ifdef NIC_STAMPS
    std::vector<unsigned long long> hs(maxb * 8);
    CK(hipMemcpy(hs.data(), st, maxb * 64, hipMemcpyDeviceToHost));
    double w[26] = {}, ep[26] = {}, mf[26] = {}, nt[26] = {}, life[26] = {}, rt[26] = {}, nb[26] = {};
    for (int b = 0; b < maxb; ++b) {
      if (hs[b * 8 + 5] == 0) continue;
      const int k = (int)hs[b * 8 + 6];
      w[k] += hs[b * 8 + 0];
      ep[k] += hs[b * 8 + 1];
      mf[k] += hs[b * 8 + 2];
      nt[k] += hs[b * 8 + 3];
      life[k] += hs[b * 8 + 4];
      rt[k] += hs[b * 8 + 5];
      nb[k] += 1;
    }
    for (int k = 0; k < 26; ++k) {
      if (nb[k] == 0) continue;
      const double per = nt[k];
      printf("  taps %2d: %4.0f blocks, tiles/block %5.1f, clock %.2f GHz, life %8.0f cyc; per tile: wait %5.0f  "
             "epi+issue %5.0f  mfma %5.0f (one wave alone: %d MFMA x 16 = %d)\n",
             k, nb[k], per / nb[k], 0.1 * life[k] / rt[k], life[k] / nb[k], w[k] / per, ep[k] / per, mf[k] / per,
             k * 2 * 4 * 3, k * 2 * 4 * 3 * 16);
    }
    CK(hipMemset(st, 0, maxb * 8 * 8));
#endif
  }
  return 0;
}
