// Diagnostic (NOT part of the product): the v_fma_mix split (csrc/nic_kernels.hip split4,
// NIC_MIX_SPLIT) against the plain C++ split over 16M fp32 values; exit 0 iff bit-identical.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/mixcheck.hip -o /tmp/mixcheck
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split_ref(const f32x4& v, f16x4& hi, f16x4& lo) {
  for (int r = 0; r < 4; ++r) { _Float16 h = (_Float16)v[r]; hi[r] = h; lo[r] = (_Float16)(v[r] - (float)h); }
}
__device__ __forceinline__ void split_mix(const f32x4& v, f16x4& hi, f16x4& lo) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  u32x2 H, L;
  for (int k = 0; k < 2; ++k) {
    unsigned h, l = 0;
    asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h) : "v"(v[2 * k]), "v"(v[2 * k + 1]));
    asm volatile("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "+v"(l) : "v"(h), "v"(v[2 * k]));
    asm volatile("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(h), "v"(v[2 * k + 1]));
    H[k] = h; L[k] = l;
  }
  hi = __builtin_bit_cast(f16x4, H); lo = __builtin_bit_cast(f16x4, L);
}
__global__ void k(const float* in, uint64_t* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * i + 3 >= n) return;
  f32x4 v = {in[4*i], in[4*i+1], in[4*i+2], in[4*i+3]};
  f16x4 h1, l1, h2, l2;
  split_ref(v, h1, l1); split_mix(v, h2, l2);
  uint64_t a, b, c, d; memcpy(&a, &h1, 8); memcpy(&b, &l1, 8); memcpy(&c, &h2, 8); memcpy(&d, &l2, 8);
  out[i] = (a ^ c) | (b ^ d);
}
int main() {
  const int n = 1 << 24;
  std::vector<float> h(n);
  uint32_t s = 12345;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    uint32_t bits = s;
    int mode = i % 4;
    if (mode == 0) { float f = (float)((int)(s >> 8) - (1 << 23)) / (1 << 20); h[i] = f; }
    else if (mode == 1) { bits = (bits & 0x807fffffu) | ((100u + (bits >> 23) % 60u) << 23); memcpy(&h[i], &bits, 4); }  // exps around f16 range
    else if (mode == 2) { bits = (bits & 0x807fffffu) | ((90u + (bits >> 23) % 50u) << 23); memcpy(&h[i], &bits, 4); }   // small: f16 subnormal region
    else { memcpy(&h[i], &bits, 4); if (!(h[i] == h[i]) || fabsf(h[i]) > 60000.f) h[i] = 1.5f; }
  }
  float* d; uint64_t* o; hipMalloc(&d, n * 4); hipMalloc(&o, n / 4 * 8);
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  k<<<n / 4 / 256, 256>>>(d, o, n);
  std::vector<uint64_t> r(n / 4); hipMemcpy(r.data(), o, n / 4 * 8, hipMemcpyDeviceToHost);
  long bad = 0; for (auto x : r) bad += x != 0;
  printf("split_mix vs split_ref: %ld of %d quads differ\n", bad, n / 4);
  return bad != 0;
}
