// HIP kernels for the learned-image-codec hot path on gfx950 (MI355X / CDNA4).
//
// Reference path (AlexFuster/Neural_network_image_compression, tf2_0/src):
//   Encoder.__call__ (encoder.py:38-47): u8 RGB -> /255 -> YCbCr (utils.py:64-77)
//     -> BaseEncoder (encoder.py:19-32) per plane -> clip -> round(x*255) -> u8 latent (N,h,w,96)
//   Decoder.__call__ (decoder.py:39-48): u8 latent -> /255 -> split -> BaseDecoder
//     (decoder.py:19-32) per plane -> inverse YCbCr (utils.py:70-72) -> clip -> round -> u8 RGB
//
// Activations live in HBM as fp32 NHWC "plane batches": P = 3N planes ordered
// [Y_0..Y_{N-1}, Cb_0..Cb_{N-1}, Cr_0..Cr_{N-1}] (the concat order of training.py:81-85 /
// tf1_13/src/training.py:62).  Plane p uses model (p >= N) -- Y weights for p < N, the
// shared CbCr weights otherwise (utils.py:19-24).  One launch covers all 3N planes.
//
// Convolutions with Cin >= 32 are implicit GEMMs on the exact-fp32 MFMA
// v_mfma_f32_32x32x2_f32 (M = output pixels, N = Cout, K = taps x Cin): the input halo of a
// block's output tile is staged once in LDS and re-read by every tap; weights are
// pre-permuted on the host into MFMA fragment order and read from L2 as 16-B loads.
// Conv2DTranspose (stride 2) is run as its 4-phase sub-pixel decomposition (taps 2x2, 2x3,
// 3x2, 3x3) so no zero is ever multiplied.  Cin = 1 (conv1) and Cout = 1 (dconv8) layers
// fuse the colour transforms and use MFMA over taps / VALU dot products respectively.
//
// Numerics: this file is compiled with -ffp-contract=off so every elementwise op rounds
// like TF's one-op-at-a-time eager execution; products inside convolutions are exact-fp32
// FMA chains (MFMA or explicit fmaf).  Quantisers use rintf (round half to even, = np.round).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <utility>

#include "nic_kernels.h"


namespace nic {

static int device_cus();  // CUs of the current device (cached)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// Compile-time loop: f(std::integral_constant<int, I>{}) for I = 0 .. N-1 (register arrays
// indexed by I stay registers however large the body; #pragma unroll may give up).
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}


typedef float f32x16 __attribute__((ext_vector_type(16)));

__constant__ float c_u8_to_unit[256];  // fp32(i) / 255, correctly rounded (host-computed)
__constant__ float c_ycbcr[9];         // fp32(ycbcr_kernel), utils.py:7
__constant__ float c_ycbcr_inv[9];     // fp32(inv(ycbcr_kernel)), utils.py:8
__constant__ float c_ycbcr_off[3];     // fp32(ycbcr_off), utils.py:9

// Diagnostic build only (tools/stamps.cpp defines NIC_STAMPS): per-block s_memtime stamps
// at phase boundaries of the split-f16 conv kernel.  The shipped library never records.
#ifdef NIC_STAMPS
__device__ unsigned long long* g_stamps;
#define NIC_STAMP(k)                                                                         \
  do {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    if (threadIdx.x == 0)                                                                    \
      g_stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + (k)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                       \
  } while (0)
// persistent kernels: per-block cycle sums (tools/ws_stamps.cpp, tools/d8_stamps.cpp)
#define NIC_PNOW(v)                    \
  do {                                 \
    __builtin_amdgcn_sched_barrier(0); \
    v = __builtin_amdgcn_s_memtime();  \
    __builtin_amdgcn_sched_barrier(0); \
  } while (0)
#else
#define NIC_STAMP(k) \
  do {               \
  } while (0)
#endif

// b / 255 for a byte b, correctly rounded like the host table c_u8_to_unit (NumPy's
// x.astype(f32) / 255), in registers: r = b * fl(1/255), then one FMA correction step.  Exact
// for every b in 0..255 (checked against exact rationals: tests/test_oracle.py).
__device__ __forceinline__ float u8_unit(unsigned b) {
  const float f = (float)b, c = 0.0039215688593685627f;  // fl(1/255)
  const float r = __fmul_rn(f, c);
  return __builtin_fmaf(__builtin_fmaf(-r, 255.0f, f), c, r);
}

__device__ __forceinline__ float leaky02(float z) {
  // tf.nn.leaky_relu(z, alpha=0.2) = max(alpha*z, z)
  return fmaxf(__fmul_rn(z, 0.2f), z);
}
// conv sum * 2^-k (exact: k undoes the power-of-two weight pre-scale of the split-f16
// paths) + bias, rounded once -- bit-identical to TF's rounded BiasAdd of the fp32 sum
__device__ __forceinline__ float scale_bias(float acc, float scale_pow2, float b) {
  return __builtin_fmaf(acc, scale_pow2, b);
}
__device__ __forceinline__ float clip01(float v) {
  // tf.clip_by_value(v, 0, 1) = max(min(v, 1), 0)
  return fmaxf(fminf(v, 1.0f), 0.0f);
}
__device__ __forceinline__ uint8_t quant255(float v) {
  // np.round(v * 255).astype(np.uint8) for v in [0, 1]: fp32 multiply, round half to even
  return (uint8_t)(int)rintf(__fmul_rn(v, 255.0f));
}
// f16 range guard (RangeGuard, nic_kernels.h).  Every split-f16 producer keeps a running
// max of |v| over the values it splits (one v_max_f32 per value) and reports once per lane
// at the end: a value at or beyond the f16 limit would split into +-inf.  NaN needs an inf
// first (finite operands; products bounded by the weight pre-scale), so the max catches it.
__device__ __forceinline__ void range_track(float& m, const f32x4& v) {
  // two v_max3_f32 with |.| source modifiers (fmaxf's NaN canonicalisation would add a
  // v_max per value); NaN sources are not needed here (see above)
  asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(m) : "v"(m), "v"(v[0]), "v"(v[1]));
  asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(m) : "v"(m), "v"(v[2]), "v"(v[3]));
}
__device__ __forceinline__ void range_report(const RangeGuard& rg, float m) {
  if (!(m < kF16Limit) && rg.flag) atomicExch(rg.flag, rg.epoch);  // vector atomic, rare
}
// exact-fp32 re-run of a pass: the kernel does nothing unless the f16x3 pass it backs up
// (same epoch) tripped the guard
__device__ __forceinline__ bool range_gated_off(const RangeGuard& rg) {
  if (rg.gate && *(volatile const int*)rg.gate != rg.epoch) return true;
  if (rg.trips && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(rg.trips, 1);  // a re-run starts
  return false;
}

// The chained re-run's tile queue (fp32_chain_kernel): the block takes its next tile of a
// stage with one block-uniform atomicAdd, so tiles go only to blocks that are running -- the
// chain needs no co-resident grid (a block that starts late finds the stage's queue empty).
__device__ __forceinline__ int chain_take(int* q) {
  __shared__ int s_job;
  __syncthreads();  // the previous tile's LDS use is done; s_job is free
  if (threadIdx.x == 0) s_job = atomicAdd(q, 1);
  __syncthreads();
  return s_job;
}

// ((t0*k0 + t1*k1) + t2*k2), every op rounded (utils.py:64-68)
__device__ __forceinline__ float project(const float* k, float t0, float t1, float t2) {
  return __fadd_rn(__fadd_rn(__fmul_rn(t0, k[0]), __fmul_rn(t1, k[1])), __fmul_rn(t2, k[2]));
}

// ------------------------------------------------------------------------------------
// Generic implicit-GEMM convolution on fp32 MFMA.
//
// Block = 4 waves (256 threads).  Output tile TH x TW pixels (forward conv) or TH x TW
// coarse positions x 4 phases (stride-2 transposed conv).  Waves are arranged WM x WN x WK
// over (M tiles, N tiles, taps); WK > 1 splits the taps and reduces through LDS.
//
// MFMA 32x32x2 f32 operand maps (cdna_hip_programming.md §3): lane l holds A[i=l&31][k=l>>5],
// B[k=l>>5][j=l&31]; D register r of lane l is row (r&3)+8*(r>>2)+4*(l>>5), column l&31.
// K ordering inside one tap: for ci-group q (8 channels) and r = 0..3 the k-pair of one MFMA
// is (ci = 8q + r for lane half 0, ci = 8q + 4 + r for lane half 1).  A lane therefore reads
// 4 consecutive channels of one pixel with a single ds_read_b128, and the host repacks the
// weights as W[model][tap][q][h][co][r] so its B fragment is one 16-B global load.
// ------------------------------------------------------------------------------------

template <int CIN, int COUT, int KS, int S, bool TR, int TH, int TW, int WM, int WN, int WK>
struct ConvGeom {
  static_assert(WM * WN * WK == 4, "4 waves per block");
  static_assert(CIN % 8 == 0 && COUT % 32 == 0, "channel tiling");
  static_assert((TH * TW) % 32 == 0, "M tile is 32 pixels");
  static constexpr int MT = TH * TW / 32;
  static constexpr int NT = COUT / 32;
  static_assert(MT % WM == 0 && NT % WN == 0, "wave split");
  static constexpr int MTW = MT / WM;
  static constexpr int NTW = NT / WN;
  static constexpr int HH = TR ? TH + 2 : (TH - 1) * S + KS;
  static constexpr int HW = TR ? TW + 2 : (TW - 1) * S + KS;
  static constexpr int PS = CIN + 4;  // LDS pixel stride (floats), 16-B aligned, bank skew
  static constexpr int NQ = CIN / 8;
  static constexpr int NTAPS = KS * KS;
  static constexpr int HALO_FLOATS = HH * HW * PS;
  static constexpr int RED_FLOATS = (WK > 1) ? (WK - 1) * WM * WN * MTW * NTW * 16 * 64 : 0;
  static constexpr int LDS_FLOATS = HALO_FLOATS > RED_FLOATS ? HALO_FLOATS : RED_FLOATS;
};

template <int IN_MODE, int CIN>
__device__ __forceinline__ void stage_halo(float* lds, const ConvArgs& a, int p, int gy0, int gx0,
                                           int HH, int HW, int PS) {
  if constexpr (IN_MODE == IN_F32) {
    const float* inp = a.in + (size_t)p * a.H * a.W * CIN;
    constexpr int C4 = CIN / 4;
    const int total = HH * HW * C4;
    for (int idx = threadIdx.x; idx < total; idx += 256) {
      const int pix = idx / C4, c4 = idx - pix * C4;
      const int hy = pix / HW, hx = pix - hy * HW;
      const int gy = gy0 + hy, gx = gx0 + hx;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)
        v = *(const f32x4*)(inp + ((size_t)gy * a.W + gx) * CIN + c4 * 4);
      *(f32x4*)(lds + pix * PS + c4 * 4) = v;
    }
  } else {
    // u8 latent (N, h, w, 96): plane p = (type, n), channels type*32 .. type*32+31,
    // dequantised as x.astype(f32)/255 (decoder.py:40-41).
    static_assert(CIN == 32, "latent planes carry 32 channels");
    const int n = p % a.nimg, type = p / a.nimg;
    const uint8_t* inp = a.in_u8 + (size_t)n * a.H * a.W * 96 + type * 32;
    const int total = HH * HW * 8;  // 8 groups of 4 channels
    for (int idx = threadIdx.x; idx < total; idx += 256) {
      const int pix = idx >> 3, c4 = idx & 7;
      const int hy = pix / HW, hx = pix - hy * HW;
      const int gy = gy0 + hy, gx = gx0 + hx;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
        const uint32_t q = *(const uint32_t*)(inp + ((size_t)gy * a.W + gx) * 96 + c4 * 4);
        v[0] = c_u8_to_unit[q & 255];
        v[1] = c_u8_to_unit[(q >> 8) & 255];
        v[2] = c_u8_to_unit[(q >> 16) & 255];
        v[3] = c_u8_to_unit[q >> 24];
      }
      *(f32x4*)(lds + pix * PS + c4 * 4) = v;
    }
  }
}

// Epilogue for one 32x32 accumulator tile: bias, leaky, optional residual add, optional
// clip + quantise to the latent layout.  (oy_of, ox_of) map the tile row to output coords.
template <int COUT, int OUT_MODE, bool RESID>
__device__ __forceinline__ void store_tile(const ConvArgs& a, int p, int model, int nt, const f32x16& acc,
                                           const int* oy_of, const int* ox_of, float scale = 1.0f) {
  const int lane = threadIdx.x & 63;
  const int co = nt * 32 + (lane & 31);
  const float b = a.bias[model * COUT + co];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int oy = oy_of[r], ox = ox_of[r];
    if (oy < a.OH && ox < a.OW) {
      // scale is an exact power of two (1 on the fp32 path), then Conv -> BiasAdd -> leaky_relu
      float v = leaky02(__fadd_rn(__fmul_rn(acc[r], scale), b));
      const size_t o = (((size_t)p * a.OH + oy) * a.OW + ox) * COUT + co;
      if constexpr (RESID) v = __fadd_rn(v, a.res[o]);  // x = x + res (encoder.py:25, decoder.py:29)
      if constexpr (OUT_MODE == OUT_F32) {
        a.out[o] = v;
      } else {
        // final layer: tf.clip_by_value(x, 0, 1) (encoder.py:32); concat planes on the
        // channel axis (encoder.py:45); round(x*255) -> u8 (encoder.py:47)
        v = clip01(v);
        const int n = p % a.nimg, type = p / a.nimg;
        const size_t lo = (((size_t)n * a.OH + oy) * a.OW + ox) * 96 + type * 32 + co;
        a.out_u8[lo] = quant255(v);
        if (a.out_f32_latent) a.out_f32_latent[lo] = v;
      }
    }
  }
}

// Body of one block (b0 of nb) over its (plane, tile) jobs, grid-stride -- or, with a queue
// q (the chained gated re-run, fp32_chain_kernel), the tiles it takes from q; `lds` holds
// G::LDS_FLOATS floats.  Returns the number of tiles the block ran.
template <int CIN, int COUT, int KS, int S, bool TR, int TH, int TW, int WM, int WN, int WK, int IN_MODE,
          int OUT_MODE, bool RESID>
__device__ __forceinline__ int conv_mfma_body(const ConvArgs& a, float* lds, int b0, int nb, int* q = nullptr) {
  using G = ConvGeom<CIN, COUT, KS, S, TR, TH, TW, WM, WN, WK>;
  const int per_plane = a.tiles_y * a.tiles_x;
  int ran = 0;
  for (int job = q ? chain_take(q) : b0; job < per_plane * a.P; job = q ? chain_take(q) : job + nb, ++ran) {
  __syncthreads();  // every wave is done with the previous job's LDS
  const int p = job / per_plane;
  const int tile = job - p * per_plane;
  const int tyi = tile / a.tiles_x;
  const int t0y = tyi * TH, t0x = (tile - tyi * a.tiles_x) * TW;
  const int model = p >= a.nimg ? 1 : 0;

  int gy0, gx0;
  if constexpr (TR) {
    gy0 = t0y - 1;
    gx0 = t0x - 1;
  } else {
    gy0 = t0y * S - a.pad_y;
    gx0 = t0x * S - a.pad_x;
  }
  stage_halo<IN_MODE, CIN>(lds, a, p, gy0, gx0, G::HH, G::HW, G::PS);
  __syncthreads();

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5;
  const int wm = wave % WM, wn = (wave / WM) % WN, wk = wave / (WM * WN);

  // Per-lane A base offsets (floats) for each of this wave's M tiles.
  int a_off[G::MTW];
#pragma unroll
  for (int i = 0; i < G::MTW; ++i) {
    const int m = (wm * G::MTW + i) * 32 + (lane & 31);
    const int ty = m / TW, tx = m - (m / TW) * TW;
    a_off[i] = TR ? (ty * G::HW + tx) * G::PS : (ty * S * G::HW + tx * S) * G::PS;
    a_off[i] += half * 4;
  }
  const float* wbase = a.w + (size_t)model * G::NTAPS * CIN * COUT;
  const int wlane = (half * COUT + (lane & 31)) * 4;

  if constexpr (!TR) {
    f32x16 acc[G::MTW][G::NTW];
#pragma unroll
    for (int i = 0; i < G::MTW; ++i)
#pragma unroll
      for (int j = 0; j < G::NTW; ++j) acc[i][j] = (f32x16){};

    const int t_begin = wk * G::NTAPS / WK, t_end = (wk + 1) * G::NTAPS / WK;
    for (int t = t_begin; t < t_end; ++t) {
      const int kh = t / KS, kw = t - (t / KS) * KS;
      const int toff = (kh * G::HW + kw) * G::PS;
      const float* wt = wbase + (size_t)t * CIN * COUT + wlane;
      f32x4 bq[G::NQ][G::NTW];
#pragma unroll
      for (int q = 0; q < G::NQ; ++q)
#pragma unroll
        for (int j = 0; j < G::NTW; ++j)
          bq[q][j] = *(const f32x4*)(wt + q * 8 * COUT + (wn * G::NTW + j) * 128);
#pragma unroll
      for (int q = 0; q < G::NQ; ++q) {
        f32x4 av[G::MTW];
#pragma unroll
        for (int i = 0; i < G::MTW; ++i) av[i] = *(const f32x4*)(lds + a_off[i] + toff + q * 8);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int i = 0; i < G::MTW; ++i)
#pragma unroll
            for (int j = 0; j < G::NTW; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][r], bq[q][j][r], acc[i][j], 0, 0, 0);
      }
    }

    if constexpr (WK > 1) {
      // split-K: waves wk>0 park their partial sums in LDS (after every wave is done
      // reading the halo), wave group 0 adds them in wk order and stores.
      __syncthreads();
      const int grp = wm + WM * wn;
      if (wk > 0) {
#pragma unroll
        for (int i = 0; i < G::MTW; ++i)
#pragma unroll
          for (int j = 0; j < G::NTW; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              lds[((((wk - 1) * WM * WN + grp) * G::MTW + i) * G::NTW + j) * 1024 + r * 64 + lane] = acc[i][j][r];
      }
      __syncthreads();
      if (wk > 0) continue;  // to the next job's barrier
#pragma unroll
      for (int k = 1; k < WK; ++k)
#pragma unroll
        for (int i = 0; i < G::MTW; ++i)
#pragma unroll
          for (int j = 0; j < G::NTW; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              acc[i][j][r] = __fadd_rn(
                  acc[i][j][r], lds[((((k - 1) * WM * WN + grp) * G::MTW + i) * G::NTW + j) * 1024 + r * 64 + lane]);
    }

#pragma unroll
    for (int i = 0; i < G::MTW; ++i) {
      int oy[16], ox[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = (wm * G::MTW + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        oy[r] = t0y + m / TW;
        ox[r] = t0x + m % TW;
      }
#pragma unroll
      for (int j = 0; j < G::NTW; ++j)
        store_tile<COUT, OUT_MODE, RESID>(a, p, model, wn * G::NTW + j, acc[i][j], oy, ox);
    }
  } else {
    static_assert(!TR || (S == 2 && KS == 5 && WK == 1), "transposed path: k5 s2 phases");
    // Phase (py, px) of output (2m+py, 2n+px) gathers input (m+dy, n+dx) for dy in
    // {-1,0} (py=0) or {-1,0,1} (py=1), kernel tap t = py + 3 - 2*(dy+1).  Weights are
    // stored phase-major in the same tap order.
    int tap_base = 0;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int py = ph >> 1, px = ph & 1;
      const int ny = py ? 3 : 2, nx = px ? 3 : 2;
      f32x16 acc[G::MTW][G::NTW];
#pragma unroll
      for (int i = 0; i < G::MTW; ++i)
#pragma unroll
        for (int j = 0; j < G::NTW; ++j) acc[i][j] = (f32x16){};
      for (int iy = 0; iy < ny; ++iy) {
        for (int ix = 0; ix < nx; ++ix) {
          const int t = tap_base + iy * nx + ix;
          // halo origin is (m0-1, n0-1): input (m+dy) sits at halo row m-m0+dy+1 = ty+iy
          const int toff = (iy * G::HW + ix) * G::PS;
          const float* wt = wbase + (size_t)t * CIN * COUT + wlane;
          f32x4 bq[G::NQ][G::NTW];
#pragma unroll
          for (int q = 0; q < G::NQ; ++q)
#pragma unroll
            for (int j = 0; j < G::NTW; ++j)
              bq[q][j] = *(const f32x4*)(wt + q * 8 * COUT + (wn * G::NTW + j) * 128);
#pragma unroll
          for (int q = 0; q < G::NQ; ++q) {
            f32x4 av[G::MTW];
#pragma unroll
            for (int i = 0; i < G::MTW; ++i) av[i] = *(const f32x4*)(lds + a_off[i] + toff + q * 8);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int i = 0; i < G::MTW; ++i)
#pragma unroll
                for (int j = 0; j < G::NTW; ++j)
                  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][r], bq[q][j][r], acc[i][j], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < G::MTW; ++i) {
        int oy[16], ox[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = (wm * G::MTW + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
          oy[r] = 2 * (t0y + m / TW) + py;
          ox[r] = 2 * (t0x + m % TW) + px;
        }
#pragma unroll
        for (int j = 0; j < G::NTW; ++j)
          store_tile<COUT, OUT_MODE, RESID>(a, p, model, wn * G::NTW + j, acc[i][j], oy, ox);
      }
      tap_base += ny * nx;
    }
  }
  }  // job
  return ran;
}

template <int CIN, int COUT, int KS, int S, bool TR, int TH, int TW, int WM, int WN, int WK, int IN_MODE,
          int OUT_MODE, bool RESID>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs a) {
  using G = ConvGeom<CIN, COUT, KS, S, TR, TH, TW, WM, WN, WK>;
  __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
  // per-layer gated re-run (NIC_CHAIN=0): exit unless the split pass of this epoch tripped
  // (the chained re-run checks the gate once in fp32_chain_kernel, not in the body)
  if (range_gated_off(a.rg)) return;
  conv_mfma_body<CIN, COUT, KS, S, TR, TH, TW, WM, WN, WK, IN_MODE, OUT_MODE, RESID>(a, lds, blockIdx.x, gridDim.x);
}


// ------------------------------------------------------------------------------------
// Split-f16 ("f16x3") implicit-GEMM convolution on v_mfma_f32_32x32x16_f16.
//
// Every fp32 operand x is split as x = hi + lo, hi = f16(x), lo = f16(x - hi) (RNE; lo may
// be subnormal, which gfx950 keeps: float_denorm_mode_16_64 = 3).  Weights are first scaled
// by an exact power of two 2^k per model so that max|w*2^k| <= 2^15 keeps hi and lo normal.
// The product is a*w ~= a_hi*w_hi + a_hi*w_lo + a_lo*w_hi (three MFMAs into ONE fp32
// accumulator; f16 x f16 products are exact in fp32, the dropped a_lo*w_lo term and the
// rounding of lo are ~2^-22 relative), so the result matches an fp32 FMA chain to within a
// few fp32 ulps of the sum while running on the f16 matrix pipe (16x the f32 MFMA rate).
//
// MFMA 32x32x16 operand maps: lane l holds A[row l&31][k = 8*(l>>5) + j] and
// B[k = 8*(l>>5) + j][col l&31], j = 0..7.  K order inside one tap: k16 step s covers input
// channels 16s .. 16s+15, so a lane reads 8 consecutive channels of one pixel (16 B) from
// the hi image and 16 B from the lo image.  LDS halo: per pixel [hi: Cin f16][lo: Cin f16]
// [16 B pad].  Weights: [model][tap][s][hi,lo][h][co][j] f16, one 16-B load per fragment.
//
// Waves: WM x WN x WK, each wave owns MTW M tiles (32 pixels) x NTW N tiles (32 channels);
// its B fragments for one tap stay in registers (prefetched one tap ahead from L2) while it
// walks its M tiles, so weight traffic is 1/MTW of the MFMA operand traffic.
// ------------------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));


#ifndef NIC_MIX_SPLIT
#define NIC_MIX_SPLIT 1
#endif
__device__ __forceinline__ void split4(const f32x4& v, f16x4& hi, f16x4& lo) {
#if NIC_MIX_SPLIT
  // per pair: hi = cvt_pk_f16 (RNE); the exact differences v - f32(hi) by v_fma_mix_f32 with
  // hi read as an f16 half (one op each instead of cvt back + subtract); lo = cvt_pk_f16 of
  // them.  v - f32(hi) is exact in fp32 (Sterbenz; hi within 2x of v or both tiny), so this
  // is bit-identical to (_Float16)(v - (float)(_Float16)v) (checked over 16M values,
  // tools/mixcheck.hip).
  // One asm block for the 8 instructions, each result read at least one instruction after it
  // is written: as separate statements the compiler cannot see that none of them is a
  // transcendental op and pads every dependent pair with an s_nop (2-3 per call).
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  u32x2 H, L;
  float d0, d1, d2, d3;
  asm("v_cvt_pk_f16_f32 %0, %6, %7\n\t"
      "v_cvt_pk_f16_f32 %1, %8, %9\n\t"
      "v_fma_mix_f32 %2, -%0, 1.0, %6 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %3, -%0, 1.0, %7 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %4, -%1, 1.0, %8 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %5, -%1, 1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(H[0]), "=&v"(H[1]), "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
  asm("v_cvt_pk_f16_f32 %0, %2, %3\n\t"
      "v_cvt_pk_f16_f32 %1, %4, %5"
      : "=&v"(L[0]), "=&v"(L[1])
      : "v"(d0), "v"(d1), "v"(d2), "v"(d3));
  hi = __builtin_bit_cast(f16x4, H);
  lo = __builtin_bit_cast(f16x4, L);
#else
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const _Float16 h = (_Float16)v[r];
    hi[r] = h;
    lo[r] = (_Float16)(v[r] - (float)h);  // exact difference, then RNE to f16
  }
#endif
}

// Stage the input halo of one block into LDS as f16 hi / lo images.  Loads are issued in
// unrolled batches of 16 from clamped (always valid) addresses and zeroed afterwards when
// outside the image, so a batch's loads are all in flight before the first is consumed (a
// per-element guarded load would make the compiler wait for each load separately).
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) const char* lds_cptr_t;
// LDS byte offset of a generic pointer into __shared__ memory, and back as an LDS pointer
__device__ __forceinline__ unsigned lds_off(const void* p) { return (unsigned)(size_t)(lds_ptr_t)p; }
__device__ __forceinline__ lds_cptr_t lds_at(unsigned off) { return (lds_cptr_t)(size_t)off; }
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

// One 16-B direct-to-LDS load per lane (global_load_lds_dwordx4): lane l of the wave writes
// LDS bytes [wave_base + 16*l, +16).  No VGPR destination, counted in vmcnt.
__device__ __forceinline__ void dma16(const char* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)lds_wave_base, 16, 0, 0);
}
// vmcnt(0) through the builtin (simm16 0x0F70: vmcnt 0, expcnt 7, lgkmcnt 15) so hipcc's
// counter model sees the LDS-DMA drained; behind inline asm it would keep treating the DMA
// as pending and wait vmcnt(0) before every later LDS read, draining the B prefetches.
__device__ __forceinline__ void dma_wait_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Split-format 16-B stores from a transposed accumulator: per register group g a lane
// owns channels 8g + 4*half .. +3 of its pixel.  permlane32_swap exchanges group pairs
// (g, g+1) between the lane halves so that lanes 0..31 hold channels 8g..8g+7 and lanes
// 32..63 channels 8g+8..8g+15 (cdna_hip_programming.md T21); the inverse map is the same
// swap.  a, b: this lane's two dwords of groups g and g+1 (f16x4 each).
__device__ __forceinline__ void swap_pair(f16x4& a, f16x4& b) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  u32x2 ua = __builtin_bit_cast(u32x2, a), ub = __builtin_bit_cast(u32x2, b);
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const auto r = __builtin_amdgcn_permlane32_swap(ua[d], ub[d], false, false);
    ua[d] = r[0];
    ub[d] = r[1];
  }
  a = __builtin_bit_cast(f16x4, ua);
  b = __builtin_bit_cast(f16x4, ub);
}


typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));


// ------------------------------------------------------------------------------------
// Persistent-kernel helpers: a tile barrier that is not a memory fence, and LDS-DMA halo
// pieces (HaloPieces) shared by the weight-stationary kernels.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void stage_barrier() {
  asm volatile("" ::: "memory");  // no LDS access moves across (s_barrier itself is not a fence)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// lgkmcnt(0) (vmcnt 63, expcnt 7): this wave's LDS reads of the stage buffer have returned
__device__ __forceinline__ void lds_reads_done() { __builtin_amdgcn_s_waitcnt(0xC07F); }

template <class G, int CIN, int CCH, int NPW>
struct HaloPieces {
  static constexpr int PSS = G::PSB / 16, RPS = G::RPB / 16, HS = CCH / 8;
  static constexpr int TOTAL = G::HH * RPS;
  static constexpr int NPIECE = (TOTAL + 63) / 64;
  static constexpr int NPP = (NPIECE + NPW - 1) / NPW;  // pieces per loader wave (upper bound)
  int code[NPP];
  __device__ __forceinline__ void init(int pw, int lane) {
#pragma unroll
    for (int i = 0; i < NPP; ++i) {
      const int q = (pw + i * NPW) * 64 + lane;
      const int row = q / RPS, r = q - row * RPS;
      const int sp = r / PSS, k = r - sp * PSS;
      const int hx = G::S2 ? (sp < G::HE ? 2 * sp : 2 * (sp - G::HE) + 1) : sp;
      // data slots (the rest is pad); swizzled records (G::SWZ) hold chunk k ^ swz(hx) in slot k
      const bool read = q < TOTAL && sp < G::HW && (G::SWZ || k < 2 * HS);
      const int slot = G::SWZ ? G::chunk_at(k, hx) : k < HS ? k : CIN / 8 + (k - HS);  // + c*HS per stage
      code[i] = read ? (row | hx << 8 | slot << 16 | 1 << 24) : 0;
    }
  }
  // DMA channel slice c of plane base `base` (halo origin gy0, gx0) into buf.  OPAQUE
  // keeps the compiler from hoisting the decoded pieces out of the tile loop (64-bit
  // offsets per piece: spills in register-tight kernels).
  template <bool OPAQUE = false>
  __device__ __forceinline__ void issue(char* buf, const char* base, const char* zero16, int H, int W, int gy0,
                                        int gx0, int c, int pw) const {
#pragma unroll
    for (int i = 0; i < NPP; ++i) {
      const int piece = pw + i * NPW;
      if (NPP * NPW > NPIECE && piece >= NPIECE) break;  // wave-uniform
      int e = code[i];
      if constexpr (OPAQUE) asm volatile("" : "+v"(e));
      const int gy = gy0 + (e & 255), gx = gx0 + ((e >> 8) & 255);
      const bool ok = (e >> 24) && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      const size_t off = ((size_t)(unsigned)(gy * W + gx) * CIN + (size_t)(((e >> 16) & 255) + c * HS) * 4) * 4;
      dma16(ok ? base + off : zero16, buf + piece * 1024);
    }
  }
};

// LDS-DMA halo pieces through a buffer resource (buffer_load_dwordx4 ... lds): the
// resource spans one plane, so every halo slot above, below or outside the plane is out of
// range and the DMA writes zeros (TF's SAME padding) with no per-piece address select.
// Per lane and piece the 32-bit byte offset from the halo origin is precomputed once; a
// tile adds its origin (one v_add per piece) and, only on the tiles whose halo crosses the
// left or right image edge, retargets the slots of out-of-image columns out of range.
constexpr unsigned kDmaOOR = 0x80000000u;  // an offset past any plane: the DMA writes zeros
constexpr int kBufWord3 = 0x00020000;      // gfx9 raw-buffer resource word 3
#ifdef NIC_DIAG_KTIME  // diagnostic build only: first-wave start / last-wave exit of each kernel (100 MHz clock)
__device__ unsigned long long g_ktime[16][2];
#define KT_BEGIN(sl)                                                                         \
  do {                                                                                       \
    if ((threadIdx.x & 63) == 0) atomicMin(&g_ktime[sl][0], __builtin_amdgcn_s_memrealtime()); \
  } while (0)
#define KT_END(sl)                                                                           \
  do {                                                                                       \
    if ((threadIdx.x & 63) == 0) atomicMax(&g_ktime[sl][1], __builtin_amdgcn_s_memrealtime()); \
  } while (0)
struct KtGuard {
  int sl;
  __device__ explicit KtGuard(int s) : sl(s) { KT_BEGIN(s); }
  __device__ ~KtGuard() { KT_END(sl); }
};
#define KT_SCOPE(sl) KtGuard kt_guard_(sl)
extern "C" int nic_diag_ktime(unsigned long long* out, int reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ktime), sizeof(g_ktime)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long init[16][2];
    for (int k = 0; k < 16; ++k) init[k][0] = ~0ull, init[k][1] = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_ktime), init, sizeof(init)) != hipSuccess) return -1;
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
#else
#define KT_BEGIN(sl) do { } while (0)
#define KT_END(sl) do { } while (0)
#define KT_SCOPE(sl) do { } while (0)
#endif

__device__ __forceinline__ void dma16_buf(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)lds_wave_base, 16, (int)voff, 0, 0, 0);
}

template <class G, int CIN, int NPW>
struct HaloDma {
  static_assert(G::HW <= 15, "halo column packed into the low 4 bits of a 16-B aligned offset");
  static constexpr int PSS = G::PSB / 16, RPS = G::RPB / 16;
  static constexpr int TOTAL = G::HH * RPS;
  static constexpr int NPIECE = (TOTAL + 63) / 64;
  static constexpr int NPP = (NPIECE + NPW - 1) / NPW;  // pieces per loader wave (upper bound)
  // per lane and piece: byte offset of the slot from the halo origin pixel (16-B aligned)
  // | its halo column in bits 0..3; kDmaOOR for pad slots
  unsigned off[NPP];
  __device__ __forceinline__ void init(int pw, int lane, int W) {
#pragma unroll
    for (int i = 0; i < NPP; ++i) {
      const int q = (pw + i * NPW) * 64 + lane;
      const int row = q / RPS, r = q - row * RPS;
      const int sp = r / PSS, k = r - sp * PSS;
      const int x = G::S2 ? (sp < G::HE ? 2 * sp : 2 * (sp - G::HE) + 1) : sp;
      // data slots (the rest is pad); swizzled records (G::SWZ) hold chunk k ^ swz(x) in slot k
      const bool read = q < TOTAL && sp < G::HW && (G::SWZ || k < CIN / 4);
      const int slot = G::SWZ ? G::chunk_at(k, x) : k;
      off[i] = read ? (unsigned)((row * W + x) * CIN * 4 + slot * 16) | (unsigned)x : kDmaOOR;
    }
  }
  // DMA the halo with origin (gy0, gx0) of the plane at `plane` (plane_bytes long) into buf
  __device__ __forceinline__ void issue(char* buf, const char* plane, unsigned plane_bytes, int W, int gy0, int gx0,
                                        int pw) const {
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)plane, (short)0, (int)plane_bytes,
                                                                          kBufWord3);
    const unsigned org = (unsigned)((gy0 * W + gx0) * CIN * 4);  // may wrap: then out of range
    const bool edge = gx0 < 0 || gx0 + G::HW > W;                // wave-uniform
#pragma unroll
    for (int i = 0; i < NPP; ++i) {
      const int piece = pw + i * NPW;
      if (NPP * NPW > NPIECE && piece >= NPIECE) break;  // wave-uniform
      const unsigned o = off[i];
      unsigned v = (o & ~15u) + org;
      if (edge && ((unsigned)(gx0 + (int)(o & 15u)) >= (unsigned)W || o == kDmaOOR)) v = kDmaOOR;
      dma16_buf(rsrc, v, buf + piece * 1024);
    }
  }
};

// fl(h + l) for the f16 halves `S` of dwords H and L: one v_fma_mix_f32 (l * 1 + h, exact
// product and sum, one rounding) instead of two conversions and an add -- bit-identical to
// __fadd_rn((float)h, (float)l)
template <int S>
__device__ __forceinline__ float add_f16_pair(unsigned H, unsigned L) {
  float t;
  if constexpr (S == 0)
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(L), "v"(H));
  else
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(t) : "v"(L), "v"(H));
  return t;
}

// ------------------------------------------------------------------------------------
// Weight-stationary persistent conv (split-f16 on v_mfma_f32_16x16x32_f16) over a
// stride-1 window of KH x KW taps: the k3 s1 layers (KH = KW = 3), and each of the four
// sub-pixel phases of the k5 s2 Conv2DTranspose dconv7 (2x2, 2x3, 3x2, 3x3 taps, TRP).
// Wave w owns output channels 16w .. 16w+15 and keeps their weights for every tap of its
// window and every input channel in VGPRs (the MFMA A operand: w_hi and w_lo, at most
// 9 x 2 k32-steps x 2 = 36 fragments = 144 VGPRs), loaded once per block.  A launch is cut
// into block groups, one per (tap set, model); a group's blocks loop over that model's
// tiles, so no weight byte is re-read per tile (the one-tile-per-block kernels move ~8 KB
// of weight fragments per wave and tap through L2).  The halo of tile i+1 is DMA'd into
// the other LDS buffer by all waves while tile i's MFMAs run; the epilogue of tile i runs
// after the next barrier so its stores overlap tile i+1.
// D[co][pixel] per 16-pixel tile (two 8-pixel rows): lane (g, l16) holds channels
// 16w + 4g .. +3 of pixel l16.  Phase (py, px) of a transposed layer writes fine pixel
// (2y + py, 2x + px) for coarse position (y, x), from halo taps (iy, ix) < (KH, KW) at
// origin (y - 1, x - 1) with weight tap tb + iy * KW + ix (host phase-major repack).
// ------------------------------------------------------------------------------------
// 16x16 D layout -> 16-B split stores.  Lane (g, l16) holds hi and lo of 4 channels
// (4g..4g+3 of its wave's 16); v_permlane16_swap (odd 16-lane rows of the first operand <->
// even rows of the second) leaves even-g lanes with the hi of 8 channels [own | g+1's] and
// odd-g lanes with the lo of the same 8 [g-1's | own]: one dwordx4 store per lane instead
// of two dwordx2.  The swap is its own inverse (unswap16 restores a residual read in the
// store layout to this lane's hi / lo).  Every lane must take part (EXEC full).
__device__ __forceinline__ u32x4 swap16_pair(const f16x4& hi, const f16x4& lo) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  u32x2 x = __builtin_bit_cast(u32x2, hi), y = __builtin_bit_cast(u32x2, lo);
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const auto r = __builtin_amdgcn_permlane16_swap(x[d], y[d], false, false);
    x[d] = r[0];
    y[d] = r[1];
  }
  return (u32x4){x[0], x[1], y[0], y[1]};
}
__device__ __forceinline__ void unswap16(const u32x4& q, f16x4& hi, f16x4& lo) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  u32x2 x = {q[0], q[1]}, y = {q[2], q[3]};
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const auto r = __builtin_amdgcn_permlane16_swap(x[d], y[d], false, false);
    x[d] = r[0];
    y[d] = r[1];
  }
  hi = __builtin_bit_cast(f16x4, x);
  lo = __builtin_bit_cast(f16x4, y);
}

// LDS halo image of the weight-stationary kernels (3x3 window, stride 1): unpadded 256-B
// pixel records (16 slots: [hi 64 ch | lo 64 ch] in 16-B chunks), rows of HW records, and
// chunk c of halo column hx stored in slot c ^ (2 hx mod 16).  The B fragment of
// v_mfma_f32_16x16x32_f16 has lane (g, l16) read chunk c = 4 ks + 8 hl + g of pixel l16 (two
// 8-pixel rows); every ds_read_b128 16-lane group ({0-3, 12-15, 20-27}, ...) then hits 16
// distinct slots for every tap shift (exhaustive search over x-linear / XOR swizzles), and
// the image is whole 1-KB DMA pieces with no pad slots (25 instead of 32 for 10 x 10).
// Tile coordinates of a persistent block's tiles bi, bi + nb, bi + 2 nb, ... of a plane
// group (per_plane = tiles_y x tiles_x tiles per plane), walked in order without an integer
// division per tile (each call sequence -- DMA issue, conv1, epilogue -- keeps its own walk).
struct TileWalk {
  int pl, ty, tx, d_pl, d_ty, d_tx, tiles_x, tiles_y;
  __device__ __forceinline__ void init(int bi, int nb, int tiles_y_, int tiles_x_) {
    tiles_x = tiles_x_;
    tiles_y = tiles_y_;
    const int per_plane = tiles_y * tiles_x;
    pl = bi / per_plane;
    const int r = bi - pl * per_plane;
    ty = r / tiles_x;
    tx = r - ty * tiles_x;
    d_pl = nb / per_plane;
    const int dr = nb - d_pl * per_plane;
    d_ty = dr / tiles_x;
    d_tx = dr - d_ty * tiles_x;
  }
  // plane index (within the group), tile row, tile column of the current tile; then advance
  __device__ __forceinline__ void take(int& pl_, int& ty_, int& tx_) {
    pl_ = pl;
    ty_ = ty;
    tx_ = tx;
    tx += d_tx;
    if (tx >= tiles_x) {
      tx -= tiles_x;
      ++ty;
    }
    ty += d_ty;
    if (ty >= tiles_y) {
      ty -= tiles_y;
      ++pl;
    }
    pl += d_pl;
  }
};

template <int CIN, int TH, int TW>
struct GeomWS {
  static_assert(CIN == 64, "record geometry searched for Cin 64");
  static constexpr int HH = TH + 2, HW = TW + 2;
  static constexpr bool S2 = false, SWZ = true;
  static constexpr int HE = HW;
  static constexpr int PSB = CIN * 4;
  static constexpr int RPB = HW * PSB;
  static constexpr int HALO_BYTES = HH * RPB;
  static_assert(HALO_BYTES % 1024 == 0, "whole DMA pieces");
  static __device__ __forceinline__ int chunk_at(int slot, int hx) { return slot ^ ((2 * hx) & 15); }
};

// PROJ (dconv7 in front of dconv8): instead of storing the 64 channels of a pixel, the
// epilogue parks the tile's split output in LDS (hproj, 64 px x [hi 64 | lo 64] f16, 16-B
// chunks XOR-swizzled by pixel) and wave w projects pixels 16w..16w+15 onto dconv8's 25 phase taps: D[px][tap] =
// sum_ci h[px][ci] w8[tap][ci] on the same split-f16 MFMA (2 tap blocks x 2 k32-steps x 3,
// B fragments from an LDS copy of w8), scaled by 2^-k8 and stored tile-major (a.proj).
// One extra barrier per tile (hproj complete); the next tile's barrier orders its reuse.
// residual of the k3 layers: LDS-DMA per wave (NIC_RES_DMA=1, default) or VGPR loads
#ifndef NIC_RES_DMA
#define NIC_RES_DMA 1
#endif
constexpr bool kResDma = NIC_RES_DMA != 0;
template <int CIN, int COUT, int TH, int TW, bool RESID, int KH, int KW, bool TRP, bool PROJ = false>
__device__ __forceinline__ void ws_body(const ConvArgs& a, char* lds, int model, int bi, int nb, int tb, int py,
                                        int px, bool copy_w8 = true) {
  constexpr int NTAPS = KH * KW, NW = COUT / 16, KST = CIN / 32, MT = TH * TW / 16;
  static_assert(TW == 8 && CIN % 32 == 0 && COUT % 16 == 0, "16-pixel tiles = two 8-pixel rows");
  static_assert(!(TRP && RESID), "no residual on the transposed phases");
  static_assert(!PROJ || (TRP && COUT == 64 && TH * TW == 64), "projection: dconv7 8x8 tiles");
  using G = GeomWS<CIN, TH, TW>;
  // halo DMA: buffer-resource pieces (HaloDma) for the plain and projection variants; the
  // residual variant keeps the global_load_lds pieces (HaloPieces), measured 6 % faster there
  // (same-box A/B: with HaloDma its stream carries ~8x the s_waitcnt instructions -- exact
  // lgkmcnt counts instead of lgkmcnt(0) drains -- which the residual epilogue's partner
  // wave cannot absorb), while HaloDma saves 2-3 % on conv3 / dconv5 / dconv7
  constexpr bool kBufHalo = !RESID || kResDma;
  using HP = std::conditional_t<kBufHalo, HaloDma<G, CIN, NW>, HaloPieces<G, CIN, CIN, NW>>;
  constexpr int TAP_BYTES = CIN * COUT * 4;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  const int co0 = wave * 16 + 4 * g;  // this lane's 4 output channels
  // this group's tiles: the planes of `model` ([0, nimg) Y, [nimg, P) CbCr), block bi of nb
  const int per_plane = a.tiles_y * a.tiles_x;
  const int p0 = model ? a.nimg : 0, np = model ? a.P - a.nimg : a.nimg;
  const int ntot = np * per_plane;
  const int ntile = bi < ntot ? (ntot - bi + nb - 1) / nb : 0;

  // resident weights: A fragment (row co = 16w + l16, k = 8g + j of k32-step ks) is the
  // f16x3 repack's 16-B chunk (k16-step 2ks + g/2, half g%2) of channel 16w + l16
  f16x8 wr[NTAPS][KST][2];
  {
    const char* wsrc = (const char*)a.wx + ((size_t)model * a.ws_taps + tb) * TAP_BYTES;
#pragma unroll
    for (int t = 0; t < NTAPS; ++t)
#pragma unroll
      for (int ks = 0; ks < KST; ++ks)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
          wr[t][ks][hl] = *(const f16x8*)(wsrc + (size_t)t * TAP_BYTES +
                                          ((((2 * ks + (g >> 1)) * 2 + hl) * 2 + (g & 1)) * COUT + wave * 16 + l16) * 16);
  }
  const float scale = a.wscale[model];
  const f32x4 bias = *(const f32x4*)(a.bias + model * COUT + co0);
  // PROJ: dconv8 B fragments (k = channel 32ks + 8g + j, column = phase tap 16nt + l16)
  // copied to LDS once (8 KB; resident in VGPRs they would spill the main loop), published
  // by the first tile barrier
  constexpr int W8F = 2 * KST * 2;  // fragments per lane
  const f16x8* w8lds = (const f16x8*)(lds + 2 * G::HALO_BYTES) + lane;
  const float scale8 = PROJ ? a.proj_scale[model] : 0.f;
  char* hproj = lds + 2 * G::HALO_BYTES + W8F * 64 * 16;
  if constexpr (PROJ)
    if (copy_w8) {
      const f16x8* src = (const f16x8*)a.proj_w + (size_t)model * W8F * 64;
      for (int q = threadIdx.x; q < W8F * 64; q += 64 * NW) ((f16x8*)(lds + 2 * G::HALO_BYTES))[q] = src[q];
    }

  // B fragments: pixel (2m + l16/8 + kh, l16%8 + kw), chunk c = 8 hl + 4 ks + g in slot
  // c ^ swz(l16%8 + kw).  bx[kw] = record address (m = kh = 0) | slot of chunk g; chunk
  // 8 hl + 4 ks then XORs bits 6..7, and (2m + kh) rows add an immediate offset.
  int bx[KW];
#pragma unroll
  for (int kw = 0; kw < KW; ++kw) {
    const int hx = (l16 & 7) + kw;
    bx[kw] = (l16 >> 3) * G::RPB + hx * G::PSB + (G::chunk_at(g, hx) << 4);
  }

  HP hp;
  const unsigned plane_bytes = (unsigned)((size_t)a.H * a.W * CIN * 4);
  if constexpr (kBufHalo)
    hp.init(wave, lane, a.W);
  else
    hp.init(wave, lane);
  TileWalk it_issue, it_ep;  // the DMA issue and the epilogue each visit the tiles in order
  it_issue.init(bi, nb, a.tiles_y, a.tiles_x);
  it_ep = it_issue;
  auto tile_take = [&](TileWalk& w, int& p, int& t0y, int& t0x) {
    int pl, ty, tx;
    w.take(pl, ty, tx);
    p = p0 + pl;
    t0y = ty * TH;
    t0x = tx * TW;
  };
  auto issue = [&](int i) {  // called for i = 0, 1, 2, ... in order
    int p, t0y, t0x;
    tile_take(it_issue, p, t0y, t0x);
#ifdef NIC_DIAG_ONETILE  // diagnostic build only: every tile reads the halo of tile (1,1) of its
                         // model's first plane (input from L2; wrong results)
    p = p0;
    t0y = TH;
    t0x = TW;
#endif
    if constexpr (kBufHalo)
      hp.issue(lds + (i & 1) * G::HALO_BYTES, (const char*)a.in_s + (size_t)p * plane_bytes, plane_bytes, a.W,
               t0y - a.pad_y, t0x - a.pad_x, wave);
    else
      hp.template issue<true>(lds + (i & 1) * G::HALO_BYTES, (const char*)a.in_s + (size_t)p * plane_bytes, a.zero16,
                              a.H, a.W, t0y - a.pad_y, t0x - a.pad_x, 0, wave);
  };

  f32x4 acc[MT];
  u32x4 rq[MT];  // split residual of the tile in flight (RESID), in the 16-B store layout
  // kResDma: the residual tile DMA'd into this wave's LDS region (MT pieces of 1 KB, lane l
  // at 16 l: the granule it reads back) instead of into VGPRs
  char* res_lds = lds + 2 * G::HALO_BYTES + wave * MT * 1024;
  // 16-B output granule of this lane after swap16_pair: [hi | lo] half (g & 1), channels
  // 16w + 8 (g >> 1) .. +7
  const int st_off = (g & 1) * COUT + wave * 16 + 8 * (g >> 1);
  // output / residual granules through per-plane buffer resources: per lane and pixel tile m
  // the byte offset of its granule from the tile origin's, resolved once (32-bit; a granule
  // outside the image gets kDmaOOR: the store is dropped, the residual DMA writes zeros)
  constexpr int PXB = COUT * 4;  // bytes per split pixel record
  const unsigned out_plane = (unsigned)((size_t)a.OH * a.OW * PXB);
  unsigned g_off[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int dy = 2 * m + (l16 >> 3), dx = l16 & 7;
    g_off[m] = TRP ? (unsigned)(((2 * dy) * a.OW + 2 * dx) * PXB + st_off * 2)
                   : (unsigned)((dy * a.OW + dx) * PXB + st_off * 2);
  }
  int ep_p = 0, ep_y = 0, ep_x = 0;  // tile whose epilogue is pending
  float rmax = 0.f;                  // range guard of the split output
  // PROJ: tile i-1's projection, 4 chunks (tap block nt, k32-step ks) of 3 MFMAs, runs
  // between the projection barrier and tile i's stream.  (Interleaving the chunks into tile
  // i's MFMA stream, stores deferred past the next barrier, measured 2 % slower.)
  f32x4 pd[2];  // projections (tap block nt)
  // one k32-step of A fragments (tile pixels) and one chunk of w8 live at a time
  f16x8 pah, pal, pwh, pwl;
  const int ppx = 16 * wave + l16;  // projected pixel of this lane's A rows
  auto proj_load_a = [&](int ks) {
    pah = *(const f16x8*)(hproj + ppx * 256 + (((4 * ks + g) ^ (ppx & 15)) << 4));
    pal = *(const f16x8*)(hproj + ppx * 256 + (((8 + 4 * ks + g) ^ (ppx & 15)) << 4));
  };
  auto proj_load_w = [&](int j) {  // chunk j: nt = j & 1, ks = j >> 1
    pwh = w8lds[(((j & 1) * KST + (j >> 1)) * 2 + 0) * 64];
    pwl = w8lds[(((j & 1) * KST + (j >> 1)) * 2 + 1) * 64];
  };
  auto proj_mfma = [&](int j) {
    f32x4& d = pd[j & 1];
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(pal, pwh, d, 0, 0, 0);  // a_lo*w_hi
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(pah, pwl, d, 0, 0, 0);  // a_hi*w_lo
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(pah, pwh, d, 0, 0, 0);  // a_hi*w_hi
  };
  // chunks in the order (nt, ks) = (0,0), (1,0), (0,1), (1,1); after chunk j the next one's
  // fragments are read (its A at the k32-step change)
  auto proj_chunk = [&](int j) {
    proj_mfma(j);
    if (j == 1) proj_load_a(1);
    if (j + 1 < 4) proj_load_w(j + 1);
  };
  auto proj_store = [&](float* dst) {  // lane (g, l16): pixels 16w + 4g .. +3 of tap 16nt + l16
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int tap = 16 * nt + l16;
      if (tap < 25) *(f32x4*)(dst + tap * 64) = pd[nt] * scale8;
    }
  };
  auto proj_dst = [&] {  // a.proj block of the tile whose epilogue just ran (ep_*)
#ifdef NIC_DIAG_ONEPROJ  // diagnostic build only: every tile writes the same projection block
    return a.proj + (size_t)(blockIdx.x & 7) * (25 * 64) + 16 * wave + 4 * g;
#endif
    return a.proj + ((((size_t)ep_p * 4 + 2 * py + px) * a.tiles_y + ep_y / TH) * a.tiles_x + ep_x / TW) * (25 * 64) +
           16 * wave + 4 * g;
  };
#ifdef NIC_STAMPS
  unsigned long long s_wait = 0, s_epi = 0, s_mfma = 0, s_t0, s_t1, s_t2;
  const unsigned long long s_rt0 = __builtin_amdgcn_s_memrealtime(), s_c0 = __builtin_amdgcn_s_memtime();
  NIC_PNOW(s_t2);
#endif
  if (ntile > 0) issue(0);
  for (int i = 0; i <= ntile; ++i) {
#ifdef NIC_STAMPS
    NIC_PNOW(s_t0);
    if (i > 0) s_mfma += s_t0 - s_t2;
#endif
    dma_wait_all();  // this wave's DMAs of tile i (and the residual loads of tile i-1)
    lds_reads_done();
    stage_barrier();  // tile i's halo complete; everyone is done reading tile i-1's buffer
#ifdef NIC_STAMPS
    NIC_PNOW(s_t1);
    s_wait += s_t1 - s_t0;
#endif
    if (i > 0) {  // epilogue of tile i-1: *2^-k, bias, leaky (+ residual), split, 8-B stores
      __amdgpu_buffer_rsrc_t out_rs;
      unsigned out_org = 0;
      if constexpr (!PROJ) {
        out_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.out_s + (size_t)ep_p * out_plane / 2), (short)0,
                                                   (int)out_plane, kBufWord3);
        out_org = TRP ? (unsigned)(((2 * ep_y + py) * a.OW + 2 * ep_x + px) * PXB)
                      : (unsigned)((ep_y * a.OW + ep_x) * PXB);
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int y = ep_y + 2 * m + (l16 >> 3), x = ep_x + (l16 & 7);
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = leaky02(scale_bias(acc[m][r], scale, bias[r]));
        if constexpr (RESID) {
          f16x4 rh, rl;
          if constexpr (kResDma) rq[m] = *(const u32x4*)(res_lds + m * 1024 + lane * 16);
          unswap16(rq[m], rh, rl);
          typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
          const u32x2 H = __builtin_bit_cast(u32x2, rh), L = __builtin_bit_cast(u32x2, rl);
          static_for<4>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            v[r] = __fadd_rn(v[r], add_f16_pair<r & 1>(H[r >> 1], L[r >> 1]));
          });
        }
        if (y < a.H && x < a.W) range_track(rmax, v);
        f16x4 hi, lo;
        split4(v, hi, lo);
        u32x4 q = swap16_pair(hi, lo);  // even g: hi of 8 channels, odd g: lo of the same 8
        if constexpr (PROJ) {  // chunk (g & 1) * 8 + 2w + g / 2 of pixel 16m + l16
          const int pp = 16 * m + l16, ch = (g & 1) * 8 + 2 * wave + (g >> 1);
          *(u32x4*)(hproj + pp * 256 + ((ch ^ (pp & 15)) << 4)) = q;
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(q, out_rs, y < a.H && x < a.W ? out_org + g_off[m] : kDmaOOR, 0, 0);
        }
      }
    }
    // PROJ: the next halo's DMA issue runs before the projection barrier, where it overlaps
    // the other waves finishing their epilogues (buffer (i+1)&1 was last read by tile i-1's
    // stream, which every wave finished before the top barrier)
    if constexpr (PROJ)
      if (i + 1 < ntile) issue(i + 1);
    if constexpr (PROJ)
      if (i > 0) {
        lds_reads_done();  // lgkmcnt(0): this wave's hproj writes have landed
        stage_barrier();   // the whole tile's channels are in hproj
      }
    if constexpr (!PROJ)
      if (i + 1 < ntile) issue(i + 1);  // into the buffer tile i-1 used
    if constexpr (PROJ)
      if (i > 0) {  // tile i-1's projection (4 chunks of 3 MFMAs) and its stores
        proj_load_a(0);
        proj_load_w(0);
        pd[0] = pd[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) proj_chunk(j);
        proj_store(proj_dst());
      }
    if (i == ntile) break;
    tile_take(it_ep, ep_p, ep_y, ep_x);
    if constexpr (RESID) {  // consumed by this tile's epilogue, after the next vmcnt(0)
      if constexpr (kResDma) {  // this wave's own LDS region: its reads came first
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(a.res_s + (size_t)ep_p * out_plane / 2), (short)0, (int)out_plane, kBufWord3);
        const unsigned org = (unsigned)((ep_y * a.OW + ep_x) * PXB);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const bool in = ep_y + 2 * m + (l16 >> 3) < a.OH && ep_x + (l16 & 7) < a.OW;
          dma16_buf(rs, in ? org + g_off[m] : kDmaOOR, res_lds + m * 1024);
        }
      } else {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int oy = min(ep_y + 2 * m + (l16 >> 3), a.OH - 1), ox = min(ep_x + (l16 & 7), a.OW - 1);
          rq[m] = *(const u32x4*)(a.res_s + (((size_t)ep_p * a.OH + oy) * a.OW + ox) * COUT * 2 + st_off);
        }
      }
    }
    const char* buf = lds + (i & 1) * G::HALO_BYTES;
#ifdef NIC_STAMPS
    NIC_PNOW(s_t2);
    s_epi += s_t2 - s_t1;
#endif
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // bx in this buffer (HALO_BYTES is a multiple of 256: the XOR bits are untouched)
    unsigned bb[KW];
#pragma unroll
    for (int kw = 0; kw < KW; ++kw) bb[kw] = lds_off(buf) + bx[kw];
    // NTAPS x KST k32-steps, fully unrolled (the weight registers are indexed statically).
    // Rolling fragment buffer: once pixel tile m's three MFMAs of step s are issued, its
    // registers receive step s+1's fragment, (MT-1)*3 MFMAs before they are needed.
    constexpr int NSTEP = NTAPS * KST;
    f16x8 fb[MT][2];
    // fragment (hi or lo) of pixel tile m at step st: chunk variant 2 hl + ks (bits 6..7 =
    // 8 hl + 4 ks), row 2m + kh
    auto frag = [&](int m, int st, int hl) {
      const int t = st / KST, ks = st - t * KST, kh = t / KW, kw = t - kh * KW;
      return *(const __attribute__((address_space(3))) f16x8*)(lds_at(bb[kw] ^ ((2 * hl + ks) << 6)) +
                                                               (2 * m + kh) * G::RPB);
    };
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      fb[m][0] = frag(m, 0, 0);
      fb[m][1] = frag(m, 0, 1);
    }
    __builtin_amdgcn_s_setprio(1);  // the MFMA stream outranks the partner wave's epilogue / DMA issue
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
      const int t = st / KST, ks = st - t * KST;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][ks][1], fb[m][0], acc[m], 0, 0, 0);  // w_lo*a_hi
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][ks][0], fb[m][1], acc[m], 0, 0, 0);  // w_hi*a_lo
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][ks][0], fb[m][0], acc[m], 0, 0, 0);  // w_hi*a_hi
        if (st + 1 < NSTEP) {
          fb[m][0] = frag(m, st + 1, 0);
          fb[m][1] = frag(m, st + 1, 1);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the rolling order (no hoisted reads)
      }
    }
    __builtin_amdgcn_s_setprio(0);
  }
  range_report(a.rg, rmax);
#ifdef NIC_STAMPS
  if (threadIdx.x == 0) {
    unsigned long long* o = g_stamps + blockIdx.x * 8;
    o[0] = s_wait;
    o[1] = s_epi;
    o[2] = s_mfma;
    o[3] = ntile;
    o[4] = __builtin_amdgcn_s_memtime() - s_c0;
    o[5] = __builtin_amdgcn_s_memrealtime() - s_rt0;
    o[6] = NTAPS;
    o[7] = model;
  }
#endif
}

// ------------------------------------------------------------------------------------
// Weight-stationary persistent conv for the k5 s2 forward layers (conv2 32->64, conv8
// 64->32 -> u8 latent), split-f16 on v_mfma_f32_16x16x32_f16.  25 taps of resident
// weights do not fit one wave's registers, so a block of 8 waves (two per SIMD, one block
// per CU) splits them: wave w = (cg = w % NCG: output channels 16cg..16cg+15, ts = w / NCG:
// taps [25 ts / NTS, 25 (ts+1) / NTS)).  Waves ts > 0 leave their partial sums of a tile
// in LDS (double-buffered by tile parity); the ts = 0 waves add them in the deferred
// epilogue at the start of the next tile, while the others already run its MFMAs.
// Halo: (2 TH + 3) x (2 TW + 3) input pixels, columns stored even-first then odd (so the
// 8 output columns of a 16-pixel B fragment read consecutive records), records of
// Cin / 4 + 2 slots and a row pitch of 0 mod 8 slots: conflict-free ds_read_b128.
// ------------------------------------------------------------------------------------
template <int CIN, int TH, int TW>
struct GeomS2 {
  static constexpr int HH = (TH - 1) * 2 + 5, HW = (TW - 1) * 2 + 5, HE = (HW + 1) / 2;
  static constexpr int PSS = CIN / 4 + 2, PSB = PSS * 16;  // data slots + 2 pad
  static constexpr int RPS = (HW * PSS + 7) / 8 * 8, RPB = RPS * 16;
  static constexpr int HTOT = HH * RPS;  // slots
  static constexpr int NPIECE = (HTOT + 63) / 64;
  static constexpr int HALO_BYTES = NPIECE * 1024;
  static __device__ __forceinline__ int col(int hx) { return (hx & 1) * HE + (hx >> 1); }
};


constexpr int C12_PH = 41;  // conv12's colour patch rows / cols: (19 - 1) * 2 + 5

// HIST (conv8 in nic_encode_entropy): the latent histogram counted inside conv8.  The ts = 0
// epilogue stores each tile's packed codes in LDS; the ts = 1 waves (idle ~1,700 cycles per
// tile at the top barrier, tools/c8_stamps.cpp) count them one tile later into a per-block LDS
// histogram [256][HIST_R replicas] (code 0 counted per lane in a register: trained latents are
// mostly zeros).  The block keeps the default strided walk (tiles bi, bi + nb, ...: the XCD-
// contiguous strips of xcd_pos), whose planes are visited in order, one after the other, so two
// LDS histograms alternate by plane parity: when the counted plane changes, the finished one is
// written out as the block's partial counts of that plane one tile later and cleared
// (hist_fold_kernel adds the blocks' partials per plane).  Needs >= 2 tiles per plane per block
// (nb <= tiles per plane / 2: large frames, config 5; hist_fold_supported).
// Measured against other forms (4K frames, conv8 alone 0.891-0.900 ms): counting in the ts = 0
// epilogue lengthened the critical pair of waves, and walks that give a block fewer planes
// (a contiguous range per block: 1.069 ms; per XCD: 0.952 ms) lose the strip locality.
#ifndef NIC_WS2_PRIO
#define NIC_WS2_PRIO 1  // 0 (A/B build): the tap-split streams at the default priority
#endif
constexpr int HIST_R = 2;
constexpr int HIST_LDS = 2 * 256 * HIST_R * 4 + 2 * 2 * 2 * 64 * 4;  // + codes [2][NCG][MT][64] (conv8)
template <int CIN, int COUT, int NTS, int TH, int OUT_MODE, int TS, bool HIST = false>
__device__ __forceinline__ void ws2_wave(const ConvArgs& a, char* lds, int model, int bi, int nb) {
  constexpr int TW = 8, MT = TH * TW / 16, NCG = COUT / 16, KST = CIN / 32, NW = NCG * NTS;
  static_assert(!HIST || OUT_MODE == OUT_U8_LATENT, "histogram fold: conv8 only");
  constexpr int T0 = 25 * TS / NTS, T1 = 25 * (TS + 1) / NTS, NT = T1 - T0;
  using G = GeomS2<CIN, TH, TW>;
  constexpr int TAP_BYTES = CIN * COUT * 4;
  // every wave issues its share of the halo DMA pieces.  Round-6 A/B (profiles/r6_ab_logs.txt
  // r6o): leaving the ts = 0 waves (which carry the epilogue) out of the issue moves their
  // 1,400 cycles of pieces into the other tap groups' chains; the tile period stays ~4,600
  // cycles and conv8 is 1 % slower, so the pieces stay spread over all waves
  constexpr int NPP = (G::NPIECE + NW - 1) / NW;
  constexpr int PART = MT * 1024;  // one wave's partial tile: MT x 64 lanes x 16 B
  char* part = lds + 2 * G::HALO_BYTES;  // [parity][NTS-1][NCG] partial tiles

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cg = wave % NCG;
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  const int per_plane = a.tiles_y * a.tiles_x;
  const int p0 = model ? a.nimg : 0, np = model ? a.P - a.nimg : a.nimg;
  const int ntot = np * per_plane;
  const int ntile = bi < ntot ? (ntot - bi + nb - 1) / nb : 0;
  uint32_t* hist = (uint32_t*)(part + 2 * (NTS - 1) * NCG * PART);  // HIST: [2 parities][256][HIST_R]
  uint32_t* codes = hist + 2 * 256 * HIST_R;                         // HIST: [2][NCG][MT][64]
  // HIST, ts = 1 waves: the plane (group-local) being counted, its code-0 count in this lane,
  // the plane whose histogram waits to be written out (-1: none), the tile to count next
  int hcur = 0, hpend = -1;
  uint32_t hz = 0;
  int h1_p = 0, h1_y = 0, h1_x = 0, h2_p = 0, h2_y = 0, h2_x = 0;  // tiles i-1, i-2 (after tile_take)
  auto hist_flush = [&](int q) __attribute__((always_inline)) {  // both ts = 1 waves, 128 bins each
    uint32_t* hb = hist + (q & 1) * (256 * HIST_R);
    const int t = cg * 64 + lane;  // cg 0, 1 of the ts = 1 waves (NCG = 2)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int bin = t + 128 * h;
      uint32_t c = 0;
#pragma unroll
      for (int r = 0; r < HIST_R; ++r) {
        c += hb[bin * HIST_R + r];
        hb[bin * HIST_R + r] = 0;
      }
      if (c) atomicAdd(a.hist_part + (size_t)(p0 + q) * 256 + bin, c);  // device scope, no return
    }
  };
  auto hist_close = [&] __attribute__((always_inline)) {  // this wave's code-0 count of hcur into bin 0
    uint32_t z = hz;
    for (int o = 32; o > 0; o >>= 1) z += __shfl_xor(z, o);
    if (lane == 0 && z) atomicAdd(hist + (hcur & 1) * (256 * HIST_R), z);
    hz = 0;
  };
  // count the codes the ts = 0 wave of this cg stored for tile (p, y, x) (code buffer par)
  auto hist_count = [&](int p, int ty0, int tx0, int par) __attribute__((always_inline)) {
    const int q = p - p0;  // wave-uniform; planes come in order
    if (q != hcur) {
      hist_close();
      hpend = hcur;
      hcur = q;
    }
    uint32_t* hs = hist + (q & 1) * (256 * HIST_R) + (lane & (HIST_R - 1));
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int oy = ty0 + 2 * m + (l16 >> 3), ox = tx0 + (l16 & 7);
      if (oy < a.OH && ox < a.OW) {
        const uint32_t w = codes[((par * NCG + cg) * MT + m) * 64 + lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t code = (w >> (8 * r)) & 255;
          if (code == 0)
            ++hz;
          else
            atomicAdd(hs + code * HIST_R, 1u);
        }
      }
    }
  };

  f16x8 wr[NT][KST][2];
  {
    const char* wsrc = (const char*)a.wx + ((size_t)model * 25 + T0) * TAP_BYTES;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int ks = 0; ks < KST; ++ks)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
          wr[t][ks][hl] = *(const f16x8*)(wsrc + (size_t)t * TAP_BYTES +
                                          ((((2 * ks + (g >> 1)) * 2 + hl) * 2 + (g & 1)) * COUT + cg * 16 + l16) * 16);
  }
  const float scale = a.wscale[model];
  const int co0 = cg * 16 + 4 * g;
  const f32x4 bias = *(const f32x4*)(a.bias + model * COUT + co0);
  // B fragment of pixel tile m: output pixel (2m + l16/8, l16%8) -> halo row 2 (2m + l16/8),
  // stored column l16%8 (tap (0,0)); channels 8g..8g+7
  int boff[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) boff[m] = 2 * (2 * m + (l16 >> 3)) * G::RPB + (l16 & 7) * G::PSB + g * 16;
  // tiles walked in order by each call sequence (DMA issue, epilogue)
  TileWalk w_issue, w_ep;
  w_issue.init(bi, nb, a.tiles_y, a.tiles_x);
  w_ep = w_issue;
  if constexpr (HIST)
    for (int q = threadIdx.x; q < 2 * 256 * HIST_R; q += 64 * NW) hist[q] = 0;  // published by the first barrier
  auto tile_take = [&](TileWalk& w, int& p, int& t0y, int& t0x) {
    int pl, ty, tx;
    w.take(pl, ty, tx);
    p = p0 + pl;
    t0y = ty * TH;
    t0x = tx * TW;
  };
  // this wave's DMA pieces of a halo: slot q -> (row, stored pixel sp, slot k), resolved once:
  // per piece the byte offset from the halo origin pixel and (row << 8 | column) for the
  // image-bounds test (kDmaOOR: pad slot, the buffer DMA writes zeros)
  unsigned doff[NPP];
  int drc[NPP];
#pragma unroll
  for (int j = 0; j < NPP; ++j) {
    const int piece = wave + j * NW;
    const int q = piece * 64 + lane;
    const int row = q / G::RPS, r = q - row * G::RPS;
    const int sp = r / G::PSS, k = r - sp * G::PSS;
    const int hx = sp < G::HE ? 2 * sp : 2 * (sp - G::HE) + 1;
    const bool ok = piece < G::NPIECE && q < G::HTOT && sp < G::HW && k < CIN / 4;
    doff[j] = ok ? (unsigned)((row * a.W + hx) * CIN * 4 + k * 16) : kDmaOOR;
    drc[j] = row << 8 | hx;
  }
  const unsigned plane_bytes = (unsigned)((size_t)a.H * a.W * CIN * 4);
  auto issue = [&](int i) {  // called for i = 0, 1, 2, ... in order
    int p, t0y, t0x;
    tile_take(w_issue, p, t0y, t0x);
#ifdef NIC_DIAG_C8NODMA  // diagnostic build only: conv8 fetches the first two halos only (wrong results)
    if (OUT_MODE == OUT_U8_LATENT && i > 1) return;
#endif
    const int gy0 = 2 * t0y - a.pad_y, gx0 = 2 * t0x - a.pad_x;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)a.in_s + (size_t)p * plane_bytes), (short)0, (int)plane_bytes, kBufWord3);
    const unsigned org = (unsigned)((gy0 * a.W + gx0) * CIN * 4);
    char* buf = lds + (i & 1) * G::HALO_BYTES;
#pragma unroll
    for (int j = 0; j < NPP; ++j) {
      const int piece = wave + j * NW;
      if (NPP * NW > G::NPIECE && piece >= G::NPIECE) break;  // wave-uniform
      const bool in = (unsigned)(gy0 + (drc[j] >> 8)) < (unsigned)a.H && (unsigned)(gx0 + (drc[j] & 255)) < (unsigned)a.W;
      dma16_buf(rsrc, doff[j] != kDmaOOR && in ? doff[j] + org : kDmaOOR, buf + piece * 1024);
    }
  };


  f32x4 acc[MT];
  const int st_off = (g & 1) * COUT + cg * 16 + 8 * (g >> 1);  // split store granule (swap16_pair)
  int ep_p = 0, ep_y = 0, ep_x = 0;
  float rmax = 0.f;  // range guard of the split outputs
  if (ntile > 0) issue(0);
#ifdef NIC_STAMPS
  unsigned long long sx[8] = {}, sa, sb;
  NIC_PNOW(sa);
#define WS2_MARK(kk)      \
  do {                    \
    NIC_PNOW(sb);         \
    sx[kk] += sb - sa;    \
    sa = sb;              \
  } while (0)
#else
#define WS2_MARK(kk) \
  do {               \
  } while (0)
#endif
  for (int i = 0; i <= ntile; ++i) {
    WS2_MARK(6);  // (the previous iteration's tail)
    dma_wait_all();
    lds_reads_done();
    WS2_MARK(5);      // DMA / LDS drain
    stage_barrier();  // halo of tile i complete; partials of tile i-1 written
    WS2_MARK(0);      // top barrier
    if constexpr (TS == 0) {
      if (i > 0) {  // epilogue of tile i-1: own sums + the other tap groups' partials
        const char* pp = part + (((i - 1) & 1) * (NTS - 1) * NCG + cg) * PART + lane * 16;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
#pragma unroll
          for (int s = 1; s < NTS; ++s) {
            const f32x4 q = *(const f32x4*)(pp + ((s - 1) * NCG) * PART + m * 1024);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[m][r] = __fadd_rn(acc[m][r], q[r]);
          }
          const int oy = ep_y + 2 * m + (l16 >> 3), ox = ep_x + (l16 & 7);
          f32x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = leaky02(scale_bias(acc[m][r], scale, bias[r]));
          if constexpr (OUT_MODE == OUT_SPLIT) {
            if (oy < a.OH && ox < a.OW) range_track(rmax, v);
            f16x4 hi, lo;
            split4(v, hi, lo);
            const u32x4 q = swap16_pair(hi, lo);
            if (oy < a.OH && ox < a.OW)
              *(u32x4*)(a.out_s + (((size_t)ep_p * a.OH + oy) * a.OW + ox) * COUT * 2 + st_off) = q;
          } else {  // clip, round(x*255) into the latent layout (N, h, w, 96)
            if (oy < a.OH && ox < a.OW) {
              const int n = ep_p % a.nimg, type = ep_p / a.nimg;
              const size_t lo = (((size_t)n * a.OH + oy) * a.OW + ox) * 96 + type * 32 + co0;
              uint32_t packed = 0;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                v[r] = clip01(v[r]);
                packed |= (uint32_t)quant255(v[r]) << (8 * r);
              }
              *(uint32_t*)(a.out_u8 + lo) = packed;
              if (a.out_f32_latent) *(f32x4*)(a.out_f32_latent + lo) = v;
              if constexpr (HIST) codes[((((i - 1) & 1) * NCG + cg) * MT + m) * 64 + lane] = packed;
            }
          }
        }
      }
    }
    WS2_MARK(1);  // epilogue (ts 0)
    if (i == ntile) break;
    // the next tile's halo into the buffer of tile i-1.  (Its pieces spread through the MFMA
    // stream below instead, one per 2 / 3 groups, took conv8 from 0.0635 to 0.0665 / 0.0701 ms:
    // a piece waiting for the texture path stalls the in-order wave's MFMAs behind it.)
    if (i + 1 < ntile) issue(i + 1);
    WS2_MARK(2);  // halo DMA issue
    if constexpr (HIST) {
      h2_p = h1_p;
      h2_y = h1_y;
      h2_x = h1_x;
      h1_p = ep_p;
      h1_y = ep_y;
      h1_x = ep_x;
    }
    tile_take(w_ep, ep_p, ep_y, ep_x);
    const char* buf = lds + (i & 1) * G::HALO_BYTES;
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // NT taps x KST k32-steps x MT pixel tiles, B fragments read DEPTH groups ahead
    constexpr int NG = NT * KST * MT, DEPTH = 3;
    auto grp_off = [&](int gq) {
      const int st = gq / MT, m = gq - st * MT;
      const int t = T0 + st / KST, ks = st % KST, kh = t / 5, kw = t - kh * 5;
      return boff[m] + kh * G::RPB + G::col(kw) * G::PSB + ks * 64;
    };
    f16x8 fb[DEPTH][2];
#pragma unroll
    for (int gq = 0; gq < DEPTH; ++gq) {
      fb[gq][0] = *(const f16x8*)(buf + grp_off(gq));
      fb[gq][1] = *(const f16x8*)(buf + grp_off(gq) + CIN * 2);
    }
    // NIC_WS2_PRIO: the MFMA streams at priority 1, the last tap group's (7 taps in conv8, the
    // most per SIMD pair; its partner ts 1 waits ~1,740 cycles per tile) at 2: conv8 0.0620-0.0624
    // vs 0.0637-0.0640 ms (3 alternating rounds, profiles/r4_ab_logs.txt).  Not with HIST: the
    // ts 1 waves count the codes after their stream, and behind the priority that took conv8 on
    // 4K frames from 0.925 to 1.047 ms.
    if constexpr (NIC_WS2_PRIO && !HIST) __builtin_amdgcn_s_setprio(TS == NTS - 1 ? 2 : 1);
    static_for<NG>([&](auto gqc) {
      constexpr int gq = decltype(gqc)::value;
      constexpr int st = gq / MT, m = gq - st * MT, t = st / KST, ks = st % KST;
      f16x8(&cur)[2] = fb[gq % DEPTH];
      acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][ks][1], cur[0], acc[m], 0, 0, 0);  // w_lo*a_hi
      acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][ks][0], cur[1], acc[m], 0, 0, 0);  // w_hi*a_lo
      acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][ks][0], cur[0], acc[m], 0, 0, 0);  // w_hi*a_hi
      if constexpr (gq + DEPTH < NG) {
        cur[0] = *(const f16x8*)(buf + grp_off(gq + DEPTH));
        cur[1] = *(const f16x8*)(buf + grp_off(gq + DEPTH) + CIN * 2);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the stream order
    });
    if constexpr (NIC_WS2_PRIO && !HIST) __builtin_amdgcn_s_setprio(0);
    WS2_MARK(3);  // MFMA stream
    if constexpr (TS > 0) {  // partial sums of tile i for the ts = 0 wave of this cg
      char* pp = part + (((i & 1) * (NTS - 1) + TS - 1) * NCG + cg) * PART + lane * 16;
#pragma unroll
      for (int m = 0; m < MT; ++m) *(f32x4*)(pp + m * 1024) = acc[m];
    }
    WS2_MARK(4);  // partials
    // HIST: the ts = 1 waves count after their own MFMA stream, where they would wait at the
    // next barrier: tile i-2's codes (stored by ts = 0 at the top of iteration i-1)
    if constexpr (HIST && TS == 1) {
      if (hpend >= 0) {  // both ts = 1 waves closed it before this iteration's barrier
        hist_flush(hpend);
        hpend = -1;
      }
      if (i >= 2) hist_count(h2_p, h2_y, h2_x, i & 1);
    }
  }
  range_report(a.rg, rmax);
  if constexpr (HIST) {  // the last tile's codes, then the last planes' partial counts
    __syncthreads();
    if constexpr (TS == 1) {
      if (hpend >= 0) {
        hist_flush(hpend);
        hpend = -1;
      }
      if (ntile > 1) hist_count(h1_p, h1_y, h1_x, (ntile - 2) & 1);  // tile ntile-2
      if (ntile > 0) hist_count(ep_p, ep_y, ep_x, (ntile - 1) & 1);  // tile ntile-1
      hist_close();
    }
    __syncthreads();
    if constexpr (TS == 1) {
      if (hpend >= 0) hist_flush(hpend);
      if (ntile > 0) hist_flush(hcur);
    }
  }
#ifdef NIC_STAMPS
  if (lane == 0) {
    unsigned long long* o = g_stamps + ((size_t)blockIdx.x * 8 + wave) * 8;
#pragma unroll
    for (int q = 0; q < 7; ++q) o[q] = sx[q];
    o[7] = ntile;
  }
#endif
#undef WS2_MARK
}

// conv1 + conv2 fused and software-pipelined (split-f16; encoder.py:10-11, 20-21 with the
// colour front end utils.py:74-77): conv2 weight-stationary on 8 x 8 output tiles, conv1
// computed per tile into conv2's LDS halo (its 19 x 19 outputs), two halo buffers so that conv1
// of tile i+1 runs beside conv2 of tile i (c12r_wave below).
//
// The colour planes come from a pre-pass (colour_split_kernel): every RGB pixel's Y, Cb, Cr
// (x/255, ((r k0 + g k1) + b k2) + off, every op rounded) split once into f16 hi / lo
// planes with a zero border wide enough for every tile's 41 x 42 patch (conv1's SAME
// padding), so a tile's patch is a plain LDS-DMA of 2 x 41 rows and conv1 reads its
// im2col B fragments (tap pairs = 2 consecutive f16) straight from LDS with no split.
// (Computing the patch per tile from the RGB bytes -- each colour value 6.6 times over,
// plus the split per im2col element -- made the kernel VALU-issue bound.)
//
// patch row pitch in dwords (2 x C12_PPW f16 columns, the first 41 used).  A multiple of 4: rows
// of whole 16-B chunks, DMA'd 1 KB per piece (10 pieces per tile; pitch 21 took 28 one-dword
// pieces), and the im2col ds_read_b32 groups meet 746 LDS
// cycles per tile instead of 866 (tools/c12_lds_banks.py)
constexpr int C12_PPW = 28;
constexpr int C12_PDW = C12_PPW % 4 == 0 ? 4 : 1;  // dwords per lane of one DMA piece
constexpr int C12_PPIECE = (C12_PH * C12_PPW + 64 * C12_PDW - 1) / (64 * C12_PDW);  // DMA pieces per plane
constexpr int C12_PLANE = C12_PPIECE * 64 * 4 * C12_PDW;  // bytes per patch plane in LDS (hi or lo)
constexpr int C12_NPD = (2 * C12_PPIECE + 3) / 4;         // pieces per issuing wave (4 waves)

// The colour-patch DMA of conv12 (tile -> patch buffer), issued by 4 waves (index cg): piece
// k = cg + 4 j of the tile's 2 x C12_PPIECE pieces.  Per lane and piece the byte offset from the
// patch origin in a colour plane, resolved once.
struct C12PatchDma {
  unsigned doff[C12_NPD];
  __device__ __forceinline__ void init(int cg, int lane, int cp_w) {
#pragma unroll
    for (int j = 0; j < C12_NPD; ++j) {
      const int k = cg + 4 * j, q = (k % C12_PPIECE) * 64 * C12_PDW + lane * C12_PDW;  // dword in the plane
      const int row = q / C12_PPW, dc = q - row * C12_PPW;
      doff[j] = k < 2 * C12_PPIECE && q < C12_PH * C12_PPW ? (unsigned)((row * cp_w + 2 * dc) * 2) : kDmaOOR;
    }
  }
  __device__ __forceinline__ void issue(const ConvArgs& a, int cg, int p, int t0y, int t0x, char* dst) const {
    const size_t cp_plane = (size_t)a.cp_h * a.cp_w;  // f16 elements per colour plane
    const unsigned org = (unsigned)((4 * t0y * a.cp_w + 4 * t0x) * 2);
#pragma unroll
    for (int j = 0; j < C12_NPD; ++j) {
      const int k = cg + 4 * j;  // wave-uniform
      if (k >= 2 * C12_PPIECE) break;
      const int hl = k / C12_PPIECE;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.cplane + ((size_t)hl * a.P + p) * cp_plane), (short)0, (int)(cp_plane * 2), kBufWord3);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + hl * C12_PLANE + (k % C12_PPIECE) * 256 * C12_PDW),
                                               4 * C12_PDW, (int)(doff[j] == kDmaOOR ? kDmaOOR : doff[j] + org), 0, 0, 0);
    }
  }
};

// Padded colour planes of the fused conv1 (ConvArgs::cplane): origin offsets and sizes in
// f16 elements for conv2's tile grid, so that tile (ty, tx)'s patch starts at row 32 ty,
// column 32 tx (dword aligned) and every patch element lies inside the plane.
void c12_plane_geom(int OH, int OW, int pad_y, int pad_x, int p1y, int p1x, int* oy, int* ox, int* hp, int* wp) {
  const int ty = (OH + 7) / 8, tx = (OW + 7) / 8;
  *oy = 2 * pad_y + p1y;
  *ox = 2 * pad_x + p1x;
  *hp = 32 * (ty - 1) + C12_PH;
  *wp = (32 * (tx - 1) + 2 * C12_PPW + 3) & ~3;  // a multiple of 4: colour_split_kernel's 8-B quads
}


// One thread per (image, padded row, 4 columns): the three colour planes of four pixels, split
// into hi / lo f16 (zero outside the image), one 8-B store per plane and half (the plane width
// is a multiple of 4).  The 12 RGB bytes of 4 interior pixels are read as 4 aligned dwords of
// the image row (a buffer resource over the row) and re-aligned by v_alignbyte; border quads
// read pixel by pixel.  A dword that straddles the row's end is not guaranteed to return its
// in-range bytes, so a quad takes the dword path only when every dword it uses lies inside the
// row (d[3] is used iff the byte shift is non-zero).  With conv1 / conv2's SAME offsets
// (ox = 3, 4, 5, 6 for W = 0, 3, 2, 1 mod 4) the last interior quad never needs a straddling
// dword, so the byte path only ever takes the true borders.  Grid (ceil(hp * wp / 4 / 256), N): the image is blockIdx.y.
// (Two columns per thread with byte loads: 20.9 vs 20.1 us per launch, profiles/r5w_*.)
__global__ __launch_bounds__(256) void colour_split_kernel(const uint8_t* __restrict__ rgb, uint16_t* __restrict__ cp,
                                                            int N, int H, int W, int oy, int ox, int hp, int wp) {
  KT_SCOPE(0);
  const int quads = wp >> 2;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= hp * quads) return;
  const int n = blockIdx.y;
  const int yp = t / quads, q4 = t - yp * quads;
  const size_t plane = (size_t)hp * wp, P = 3 * (size_t)N;
  const int y = yp - oy, x0 = 4 * q4 - ox;
  const bool row_in = (unsigned)y < (unsigned)H;
  float v[3][4];
  auto colour = [&](int e, unsigned r, unsigned g, unsigned b) {
    const float r8 = u8_unit(r), g8 = u8_unit(g), b8 = u8_unit(b);
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k][e] = __fadd_rn(project(c_ycbcr + 3 * k, r8, g8, b8), c_ycbcr_off[k]);
  };
  const unsigned b0 = 3u * (unsigned)x0, a0 = b0 & ~3u, sh = b0 & 3u;
  if (row_in && x0 >= 0 && x0 + 3 < W && (sh == 0 || a0 + 16u <= 3u * (unsigned)W)) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(rgb + ((size_t)n * H + y) * W * 3), (short)0, W * 3, kBufWord3);
    unsigned d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, a0 + 4u * i, 0, 0);
    const unsigned w0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh), w1 = __builtin_amdgcn_alignbyte(d[2], d[1], sh),
                   w2 = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
    colour(0, w0 & 255, (w0 >> 8) & 255, (w0 >> 16) & 255);
    colour(1, w0 >> 24, w1 & 255, (w1 >> 8) & 255);
    colour(2, (w1 >> 16) & 255, w1 >> 24, w2 & 255);
    colour(3, (w2 >> 8) & 255, (w2 >> 16) & 255, w2 >> 24);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int x = x0 + e;
      const bool in = row_in && (unsigned)x < (unsigned)W;
      const uint8_t* px = rgb + (((size_t)n * H + (in ? y : 0)) * W + (in ? x : 0)) * 3;
      colour(e, px[0], px[1], px[2]);
      if (!in)
#pragma unroll
        for (int k = 0; k < 3; ++k) v[k][e] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    unsigned hw[2], lw[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const _Float16 h0 = (_Float16)v[k][2 * h], h1 = (_Float16)v[k][2 * h + 1];
      const _Float16 l0 = (_Float16)(v[k][2 * h] - (float)h0), l1 = (_Float16)(v[k][2 * h + 1] - (float)h1);
      hw[h] = (unsigned)__builtin_bit_cast(uint16_t, h0) | (unsigned)__builtin_bit_cast(uint16_t, h1) << 16;
      lw[h] = (unsigned)__builtin_bit_cast(uint16_t, l0) | (unsigned)__builtin_bit_cast(uint16_t, l1) << 16;
    }
    const size_t o = ((size_t)k * N + n) * plane + (size_t)yp * wp + 4 * q4;  // 8-B aligned
    typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
    // nontemporal: 20.4 vs 21.6 us per launch, conv12 unchanged (profiles/r6_ab_logs.txt r6cs)
    __builtin_nontemporal_store((u32x2v){hw[0], hw[1]}, (u32x2v*)(cp + o));
    __builtin_nontemporal_store((u32x2v){lw[0], lw[1]}, (u32x2v*)(cp + P * plane + o));
  }
}


// conv1 + conv2 with specialised roles: each SIMD holds one conv2 wave (R2: all 25
// taps of 16 output channels resident, 200 VGPRs of w_hi / w_lo; a bare MFMA stream per tile)
// and one "vector" wave (R1: the conv2 epilogue of those 16 channels, a quarter of conv1, the
// colour-patch DMA).  In the tap-split form both waves of a SIMD carry a stream and vector
// work, and the ts 0 wave's chain (epilogue, conv1 share, stream) sets the tile period while
// its conv1 MFMAs wait behind the partner's stream; here the vector wave's MFMAs (conv1) run
// at priority over the bare stream, whose only other work is 4 accumulator stores per tile.
// One block barrier per tile.  After B_top(i): halo i (conv1(i), written in period i-1) and
// patch i+1 are complete, and acc(i-1) (stored by R2 before B_top(i)) is in LDS.
//   R2: stream(i) on halo i&1 -> (flag: acc(i-1) read) -> acc(i) to LDS
//   R1: acc(i-1) from LDS -> flag -> patch DMA(i+2) -> epilogue(i-1) -> conv1(i+1) into halo
//       (i+1)&1 -> vmcnt: patch(i+2) landed
// The accumulator tile passes between the two waves of a SIMD only (one per channel group),
// so the LDS flag orders its reuse.  Different summation order from the tap-split form (one
// 75-MFMA chain per output instead of two 36 / 39 chains added in fp32): a different fp32
// rounding of the same sums, within the oracle contract.
#ifndef NIC_C12_REUSE
#define NIC_C12_REUSE 1  // 0 (A/B build): tiles bi, bi + nb, ... and every conv1 halo computed in full
#endif
template <int ROLE>
__device__ __forceinline__ void c12r_wave(const ConvArgs& a, char* lds, int model, int bi, int nb) {
  constexpr int CIN = 32, COUT = 64, MT = 4, NCG = 4;
  using G = GeomS2<CIN, 8, 8>;
  constexpr int TAP_BYTES = CIN * COUT * 4;
  constexpr int PART = MT * 1024;                 // one accumulator tile: MT x 64 lanes x 16 B
  char* accs = lds + 2 * G::HALO_BYTES;           // [NCG] accumulator tiles
  char* patches = accs + NCG * PART;              // [2 parities][hi, lo] patch planes
  int* pflag = (int*)(patches + 4 * C12_PLANE);   // [NCG] last tile whose acc R1 has read
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cg = wave & 3;
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  const int per_plane = a.tiles_y * a.tiles_x;
  const int p0 = model ? a.nimg : 0, np = model ? a.P - a.nimg : a.nimg;
  const int ntot = np * per_plane;
  // the block's tiles: a contiguous raster range (its successive tiles are row neighbours, so
  // conv1's halo columns shared with the previous tile are copied, not recomputed).  Same box
  // (profiles/r6_ab_logs.txt r6r): 4K conv12 3.397 -> 3.333 ms, config 2 equal (its rows are 8
  // tiles); the contiguous walk alone 3.414
  constexpr bool CONTIG = NIC_C12_REUSE != 0;
  const int t_first = CONTIG ? (int)((long long)bi * ntot / nb) : bi;
  const int ntile = CONTIG ? (int)((long long)(bi + 1) * ntot / nb) - t_first : bi < ntot ? (ntot - bi + nb - 1) / nb : 0;
  const int t_step = CONTIG ? 1 : nb;
  float rmax = 0.f;
  if (threadIdx.x < NCG) pflag[threadIdx.x] = 0;
#ifdef NIC_STAMPS  // per wave cycle sums (tools/c12_stamps.cpp)
  unsigned long long sx[8] = {}, sa, sb;
  const unsigned long long s_rt0 = __builtin_amdgcn_s_memrealtime(), s_c0 = __builtin_amdgcn_s_memtime();
  NIC_PNOW(sa);
#define C12R_MARK(kk)  \
  do {                 \
    NIC_PNOW(sb);      \
    sx[kk] += sb - sa; \
    sa = sb;           \
  } while (0)
#else
#define C12R_MARK(kk) \
  do {                \
  } while (0)
#endif

  if constexpr (ROLE == 2) {
    f16x8 wr[25][2];
    {
      const char* wsrc = (const char*)a.wx + (size_t)model * 25 * TAP_BYTES;
#pragma unroll
      for (int t = 0; t < 25; ++t)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
          wr[t][hl] = *(const f16x8*)(wsrc + (size_t)t * TAP_BYTES + ((((g >> 1) * 2 + hl) * 2 + (g & 1)) * COUT + cg * 16 + l16) * 16);
    }
    // B fragment of pixel tile m at tap (0, 0): halo row 2 (2m + l16/8), column l16 % 8
    const int boff = 2 * (l16 >> 3) * G::RPB + (l16 & 7) * G::PSB + g * 16;
    lds_reads_done();
    stage_barrier();  // prologue barrier 1 (patches 0, 1)
    stage_barrier();  // prologue barrier 2 (halo 0)
    C12R_MARK(6);
    for (int i = 0; i < ntile; ++i) {
      const char* buf = lds + (i & 1) * G::HALO_BYTES + boff;
      f32x4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = (f32x4){0.f, 0.f, 0.f, 0.f};
      constexpr int NG = 25 * MT, DEPTH = 2;  // B-fragment groups read ahead (3: no faster)
      auto grp_off = [](int gq) {
        const int t = gq / MT, m = gq - t * MT, kh = t / 5, kw = t - kh * 5;
        return 4 * m * G::RPB + kh * G::RPB + G::col(kw) * G::PSB;
      };
      f16x8 fb[DEPTH][2];
#pragma unroll
      for (int gq = 0; gq < DEPTH; ++gq) {
        fb[gq][0] = *(const f16x8*)(buf + grp_off(gq));
        fb[gq][1] = *(const f16x8*)(buf + grp_off(gq) + CIN * 2);
      }
#if defined(NIC_DIAG_C12R) && NIC_DIAG_C12R == 2  // diagnostic: no R2 stream at all (R1 alone)
      if (false)
#endif
      static_for<NG>([&](auto gqc) {
        constexpr int gq = decltype(gqc)::value;
        constexpr int t = gq / MT, m = gq - t * MT;
        f16x8(&cur)[2] = fb[gq % DEPTH];
#if defined(NIC_DIAG_C12R) && NIC_DIAG_C12R == 1  // diagnostic: the stream's LDS reads, no MFMAs
        asm volatile("" ::"v"(cur[0]), "v"(cur[1]), "v"(wr[t][0]), "v"(wr[t][1]));
#else
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][1], cur[0], acc[m], 0, 0, 0);  // w_lo*a_hi
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][0], cur[1], acc[m], 0, 0, 0);  // w_hi*a_lo
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][0], cur[0], acc[m], 0, 0, 0);  // w_hi*a_hi
#endif
        if constexpr (gq + DEPTH < NG) {
          cur[0] = *(const f16x8*)(buf + grp_off(gq + DEPTH));
          cur[1] = *(const f16x8*)(buf + grp_off(gq + DEPTH) + CIN * 2);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the stream order
      });
      C12R_MARK(5);
      if (i > 0)
        while (__hip_atomic_load(pflag + cg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < i)
          __builtin_amdgcn_s_sleep(1);
      char* pp = accs + cg * PART + lane * 16;
#pragma unroll
      for (int m = 0; m < MT; ++m) *(f32x4*)(pp + m * 1024) = acc[m];
      lds_reads_done();  // (lgkmcnt 0: the acc stores too) before the barrier publishes them
      C12R_MARK(2);
      stage_barrier();   // B_top(i+1)
      C12R_MARK(0);
    }
  } else {
    __builtin_amdgcn_s_setprio(1);  // the vector wave's MFMAs and VALU ahead of the bare stream
    TileWalk w_patch, w_c1, w_ep;
    w_patch.init(t_first, t_step, a.tiles_y, a.tiles_x);
    w_c1 = w_ep = w_patch;
    auto tile_take = [&](TileWalk& w, int& p, int& t0y, int& t0x) {
      int pl, ty, tx;
      w.take(pl, ty, tx);
      p = p0 + pl;
      t0y = ty * 8;
      t0x = tx * 8;
    };
    f16x8 A1[2][2];
    f32x4 b1[2];
    {
      const f16x8* wa = (const f16x8*)a.wx1 + (size_t)model * 2 * 2 * 64 + lane;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) A1[ct][hl] = wa[(ct * 2 + hl) * 64];
        b1[ct] = *(const f32x4*)(a.bias1 + model * 32 + 16 * ct + 4 * g);
      }
    }
    const float scale1 = a.wscale1[model];
    const float scale = a.wscale[model];
    const int co0 = cg * 16 + 4 * g;
    const f32x4 bias = *(const f32x4*)(a.bias + model * COUT + co0);
    int poff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pr = 4 * g + j;
      poff[j] = pr < 15 ? ((pr / 3) * C12_PPW + pr % 3) * 4 : 0;
    }
    // the patch DMA stays with R1: issued by R2 instead (its stream has ~1,000 cycles of slack
    // per tile) conv12 measured 1 % slower
    C12PatchDma pdma;
    pdma.init(cg, lane, a.cp_w);
    auto patch_dma = [&](int i) {  // tile i's patch into patch buffer i & 1 (called in order)
      int p, t0y, t0x;
      tile_take(w_patch, p, t0y, t0x);
      pdma.issue(a, cg, p, t0y, t0x, patches + (i & 1) * 2 * C12_PLANE);
    };
    // conv1 of tile i on this wave's pixel tiles cg + 4u (patch buffer i & 1 -> halo buffer
    // i & 1), software-pipelined: all fragment reads, then the MFMA chains, then the epilogues.
    // Full: the 19 x 19 halo in 23 pixel tiles of 16 (raster order).  REUSE (tile i-1 is the left
    // neighbour): halo columns 0-2 are columns 16-18 of tile i-1's halo (buffer (i-1) & 1, which
    // R2 only reads now), copied; conv1 computes columns 3-18, one halo row per pixel tile (19).
    auto conv1_tiles = [&](auto reuse_c, int i, int t0y, int t0x) {
      constexpr bool REUSE = decltype(reuse_c)::value;
      constexpr int NPT = REUSE ? G::HH : (G::HH * G::HW + 15) / 16, PTW = (NPT + 3) / 4;
      char* halo = lds + (i & 1) * G::HALO_BYTES;
      const char* ph = patches + (i & 1) * 2 * C12_PLANE;
      const int c1y0 = 2 * t0y - a.pad_y, c1x0 = 2 * t0x - a.pad_x;
      if constexpr (REUSE) {  // 19 rows x 3 records x 8 16-B chunks over the 4 R1 waves
        const char* prev = lds + ((i - 1) & 1) * G::HALO_BYTES;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int c = (cg + 4 * k) * 64 + lane;
          if (c < G::HH * 3 * 8) {
            const int rec = c >> 3, ch = c & 7, hy = rec / 3, j = rec - hy * 3;
            const u32x4 v = *(const u32x4*)(prev + hy * G::RPB + G::col(16 + j) * G::PSB + ch * 16);
            *(u32x4*)(halo + hy * G::RPB + G::col(j) * G::PSB + ch * 16) = v;
          }
        }
      }
      auto pix = [&](int pt, int& hy, int& hx) {  // pixel tile pt, lane l16 -> halo (hy, hx)
        if constexpr (REUSE) {
          hy = pt;
          hx = 3 + l16;
        } else {
          const int q = 16 * pt + l16;
          hy = q / G::HW;
          hx = q - hy * G::HW;
        }
      };
      f16x8 bh[PTW], bl[PTW];
#pragma unroll
      for (int u = 0; u < PTW; ++u) {
        int hy, hx;
        pix(cg + 4 * u, hy, hx);
        if (hy >= G::HH) hy = hx = 0;  // past the last pixel tile (not stored)
        const char* pb = ph + (2 * hy * C12_PPW + hx) * 4;
        u32x4 H, L;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          H[j] = *(const uint32_t*)(pb + poff[j]);
          L[j] = *(const uint32_t*)(pb + C12_PLANE + poff[j]);
        }
        bh[u] = __builtin_bit_cast(f16x8, H);
        bl[u] = __builtin_bit_cast(f16x8, L);
      }
      f32x4 c1[PTW][2];
#pragma unroll
      for (int u = 0; u < PTW; ++u)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          c1[u][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1[ct][1], bh[u], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          c1[u][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1[ct][0], bl[u], c1[u][ct], 0, 0, 0);
          c1[u][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1[ct][0], bh[u], c1[u][ct], 0, 0, 0);
        }
#pragma unroll
      for (int u = 0; u < PTW; ++u) {
        const int pt = cg + 4 * u;
        if (pt >= NPT) break;  // wave-uniform
        int hy, hx;
        pix(pt, hy, hx);
        const bool qv = hy < G::HH;
        const bool in1 = qv && (unsigned)(c1y0 + hy) < (unsigned)a.H && (unsigned)(c1x0 + hx) < (unsigned)a.W;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          f32x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = in1 ? leaky02(scale_bias(c1[u][ct][r], scale1, b1[ct][r])) : 0.f;
          range_track(rmax, v);
          f16x4 hi, lo;
          split4(v, hi, lo);
          const u32x4 q16 = swap16_pair(hi, lo);
          if (qv)
            *(u32x4*)(halo + hy * G::RPB + G::col(hx) * G::PSB + (g & 1) * CIN * 2 + (16 * ct + 4 * (g & ~1)) * 2) = q16;
        }
      }
    };
    auto conv1 = [&](int i) {
      int p, t0y, t0x;
      tile_take(w_c1, p, t0y, t0x);
      if (CONTIG && i > 0 && t0x > 0)
        conv1_tiles(std::integral_constant<bool, true>{}, i, t0y, t0x);
      else
        conv1_tiles(std::integral_constant<bool, false>{}, i, t0y, t0x);
    };
    const int st_off = (g & 1) * COUT + cg * 16 + 8 * (g >> 1);  // split store granule (swap16_pair)
    // prologue: patches 0, 1 -> barrier -> conv1(0) -> barrier
    if (ntile > 0) patch_dma(0);
    if (ntile > 1) patch_dma(1);
    dma_wait_all();
    stage_barrier();
    if (ntile > 0) conv1(0);
    lds_reads_done();
    stage_barrier();
    C12R_MARK(6);
    for (int i = 0; i <= ntile; ++i) {
      if (i > 0) {
        // acc(i-1) of this channel group, then the flag that frees the buffer for R2
        const char* pp = accs + cg * PART + lane * 16;
        f32x4 acc[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = *(const f32x4*)(pp + m * 1024);
        lds_reads_done();
        __hip_atomic_store(pflag + cg, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (i + 2 < ntile) patch_dma(i + 2);  // into buffer i&1, which conv1(i) read in period i-1
        int p, t0y, t0x;
        tile_take(w_ep, p, t0y, t0x);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int oy = t0y + 2 * m + (l16 >> 3), ox = t0x + (l16 & 7);
          f32x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = leaky02(scale_bias(acc[m][r], scale, bias[r]));
          const bool inside = oy < a.OH && ox < a.OW;
          if (inside) range_track(rmax, v);
          f16x4 hi, lo;
          split4(v, hi, lo);
          const u32x4 qv = swap16_pair(hi, lo);
          if (inside) *(u32x4*)(a.out_s + (((size_t)p * a.OH + oy) * a.OW + ox) * COUT * 2 + st_off) = qv;
        }
      }
      C12R_MARK(1);
      if (i == ntile) break;
      if (i == 0 && ntile > 2) patch_dma(2);
#if defined(NIC_DIAG_C12R) && NIC_DIAG_C12R == 3  // diagnostic: no conv1 (R2 alone, stale halos)
      if (false)
#endif
      if (i + 1 < ntile) conv1(i + 1);
      C12R_MARK(3);
      dma_wait_all();   // patch(i+2) landed (the epilogue's stores too)
      lds_reads_done();
      C12R_MARK(4);
      stage_barrier();  // B_top(i+1)
      C12R_MARK(0);
    }
  }
#ifdef NIC_STAMPS
  if (lane == 0) {
    unsigned long long* o = g_stamps + ((size_t)blockIdx.x * 8 + wave) * 8;
#pragma unroll
    for (int q = 0; q < 7; ++q) o[q] = sx[q];
    o[7] = ntile;
    if (wave == 0) {
      g_stamps[256 * 64 + 2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - s_c0;
      g_stamps[256 * 64 + 2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - s_rt0;
    }
  }
#endif
#undef C12R_MARK
  range_report(a.rg, rmax);
}

// XCD-contiguous tile positions: block b of a group of nb runs on XCD
// (base + b) % 8, so give the blocks of one XCD consecutive positions in each round of nb
// tiles -- neighbouring tiles, whose halos overlap, are then fetched into one L2.
__device__ __forceinline__ int xcd_pos(int b, int nb) {
  const int x = b & 7, q = nb >> 3, r = nb & 7;
  return x * q + (x < r ? x : r) + (b >> 3);  // prefix of the XCD classes before x, then rank
}

__global__ __launch_bounds__(512) void conv12_kernel(ConvArgs a) {
  KT_SCOPE(1);
  using G = GeomS2<32, 8, 8>;
  __shared__ __attribute__((aligned(16)))
  char lds[2 * G::HALO_BYTES + 4 * 4 * 1024 + 4 * C12_PLANE + 16];
  int gi = 0;
  while (gi + 1 < a.ws_ngrp && (int)blockIdx.x >= a.ws_blk[gi + 1]) ++gi;
  const int nb = a.ws_blk[gi + 1] - a.ws_blk[gi];
  const int bi = xcd_pos(blockIdx.x - a.ws_blk[gi], nb);
  if (__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) < 4)
    c12r_wave<2>(a, lds, gi, bi, nb);
  else
    c12r_wave<1>(a, lds, gi, bi, nb);
}

template <int CIN, int COUT, int NTS, int TH, int OUT_MODE, bool HIST = false>
__global__ __launch_bounds__(64 * (COUT / 16) * NTS) void conv_ws2_kernel(ConvArgs a) {
  KT_SCOPE(3);
  using G = GeomS2<CIN, TH, 8>;
  constexpr int NCG = COUT / 16;
  static_assert(NCG * NTS == 8, "8 waves per block");
  constexpr int PARTS = 2 * (NTS - 1) * NCG * (TH / 2) * 1024;
  __shared__ __attribute__((aligned(16)))
  char lds[2 * G::HALO_BYTES + PARTS + (HIST ? HIST_LDS : 0)];
  int gi = 0;
  while (gi + 1 < a.ws_ngrp && (int)blockIdx.x >= a.ws_blk[gi + 1]) ++gi;
  const int nb = a.ws_blk[gi + 1] - a.ws_blk[gi];
  const int bi = xcd_pos(blockIdx.x - a.ws_blk[gi], nb);
  const int ts = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) / NCG;
  static_for<NTS>([&](auto tsc) {
    constexpr int TS = decltype(tsc)::value;
    if (ts == TS) ws2_wave<CIN, COUT, NTS, TH, OUT_MODE, TS, HIST>(a, lds, gi, bi, nb);
  });
}

// Block groups: group gi = blocks [ws_blk[gi], ws_blk[gi + 1]), model gi & 1, tap set gi >> 1
// (the phase of a transposed layer).
template <int CIN, int COUT, int TH, int TW, bool RESID, bool TRP, bool PROJ = false>
__global__ __launch_bounds__(64 * (COUT / 16), 2) void conv_ws_kernel(ConvArgs a) {
  KT_SCOPE(6);
  using G = GeomWS<CIN, TH, TW>;
  __shared__ __attribute__((aligned(16)))
  char lds[2 * G::HALO_BYTES + (PROJ ? 2 * (CIN / 32) * 2 * 64 * 16 + TH * TW * COUT * 4 : 0) +
           (RESID && kResDma ? (COUT / 16) * (TH * TW / 16) * 1024 : 0)];
  // ws_xcd: block b runs on XCD b % 8; the logical block x * (G / 8) + min(x, G % 8) + b / 8
  // (x = b % 8, a bijection onto [0, G)) gives each XCD a contiguous range of the groups'
  // blocks, so the tiles its blocks take at one time are neighbours whose shared halo rows /
  // columns hit that XCD's L2
  const int xcd = blockIdx.x & 7, ng = gridDim.x;
  const int lb = a.ws_xcd ? xcd * (ng >> 3) + min(xcd, ng & 7) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  int gi = 0;
  while (gi + 1 < a.ws_ngrp && lb >= a.ws_blk[gi + 1]) ++gi;
  const int bi = lb - a.ws_blk[gi], nb = a.ws_blk[gi + 1] - a.ws_blk[gi];
  const int model = gi & 1;
  if constexpr (!TRP) {
    ws_body<CIN, COUT, TH, TW, RESID, 3, 3, false>(a, lds, model, bi, nb, 0, 0, 0);
  } else if (a.ws_ngrp == 2) {
    // every block runs all four sub-pixel phases over its share of the model's tiles, one
    // after the other (weights reloaded per phase; dconv8's w8 copied to LDS once): equal
    // work per block whatever the per-tile overheads of the phases
    ws_body<CIN, COUT, TH, TW, false, 3, 3, true, PROJ>(a, lds, model, bi, nb, 16, 1, 1);
    ws_body<CIN, COUT, TH, TW, false, 2, 3, true, PROJ>(a, lds, model, bi, nb, 4, 0, 1, false);
    ws_body<CIN, COUT, TH, TW, false, 3, 2, true, PROJ>(a, lds, model, bi, nb, 10, 1, 0, false);
    ws_body<CIN, COUT, TH, TW, false, 2, 2, true, PROJ>(a, lds, model, bi, nb, 0, 0, 0, false);
  } else {
    switch (gi >> 1) {  // phase-major tap bases 0, 4, 10, 16 (for_each_phase_tap)
      case 0: ws_body<CIN, COUT, TH, TW, false, 2, 2, true, PROJ>(a, lds, model, bi, nb, 0, 0, 0); break;
      case 1: ws_body<CIN, COUT, TH, TW, false, 2, 3, true, PROJ>(a, lds, model, bi, nb, 4, 0, 1); break;
      case 2: ws_body<CIN, COUT, TH, TW, false, 3, 2, true, PROJ>(a, lds, model, bi, nb, 10, 1, 0); break;
      default: ws_body<CIN, COUT, TH, TW, false, 3, 3, true, PROJ>(a, lds, model, bi, nb, 16, 1, 1); break;
    }
  }
}

// ------------------------------------------------------------------------------------
// dconv1 (Conv2DTranspose 32 -> 64, k5 s2 on the dequantised latent, decoder.py:10,20,40-41)
// as a persistent weight-stationary kernel on the u8 codes (codes 0..255 are exact in f16:
// they are the B operand, 2 MFMAs per MAC, 1/255 folded into the epilogue scale, one
// rounding), all four sub-pixel phases per staged tile.  A block of 8 waves (one per CU)
// stages a tile's codes once and runs all 25 taps on it: wave w < 4 holds phases (1,1) and
// (0,0) (9 + 4 taps), wave w + 4 phases (0,1) and (1,0) (6 + 6 taps) of output channels
// 16 (w & 3) .. + 15 -- 13 and 12 taps of resident A fragments (w_hi, w_lo of 32 input
// channels: 8 VGPRs per tap), so the two SIMD partners carry nearly equal MFMA work on one
// halo and each phase's epilogue overlaps its partner's MFMAs.  Halo: 10 x 10 coarse pixels
// of 32 codes, loaded to registers two tiles ahead and written to LDS as f16 records of 64 B
// (4 slots) in rows of 800 B (50 slots): for every tap column, each of ds_read_b128's four
// lane groups ({0-3,12-15,20-27}, ...; lane (g, l16) reads slot g of pixel (l16 / 8,
// l16 % 8 + kw)) hits 16 distinct 16-B bank slots (exhaustive search over record / row
// pitches and chunk swizzles; 80-B records in 896-B rows had 50 % bank-conflict cycles).
// Earlier forms, measured slower and removed (DESIGN sections 5, 5b): one tile per block
// (all 25 taps of weights re-read from L2 per block, latency-bound: PMC issue stall 0.60,
// MFMA busy 0.23) and a per-phase walk (each tile's codes staged four times, 32-72 MFMAs per
// wave between two barriers).
// ------------------------------------------------------------------------------------
constexpr int D1_PSB = 64;           // LDS bytes per halo pixel: 32 f16 codes, unpadded
constexpr int D1_RPB = 800;          // halo row pitch (10 pixels + 160 B): 50 slots = 2 mod 16
constexpr int D1_HB = 10 * D1_RPB;   // one halo buffer
constexpr int D1A_LD = 2;  // code dwords per thread per tile (800 over 512 threads)
#ifndef NIC_D1A_PF
#define NIC_D1A_PF 2  // code prefetch distance in tiles (1: A/B build)
#endif

template <int KH1, int KW1, int TB1, int PY1, int PX1, int KH2, int KW2, int TB2, int PY2, int PX2>
__device__ __forceinline__ void d1all_wave(const ConvArgs& a, char* lds, int model, int bi, int nb) {
  constexpr int COUT = 64, MT = 4, TAP_BYTES = 32 * COUT * 4, PXB = COUT * 4;
  constexpr int NT1 = KH1 * KW1, NT2 = KH2 * KW2;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), cg = wave & 3;
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  const int per_plane = a.tiles_y * a.tiles_x;
  // (one group walking both models' planes with the weights reloaded at the switch -- 12 tiles
  // for every block at config 2 instead of 13 for a few Y blocks -- measured slower, round 4:
  // dconv1 0.0604-0.0608 vs 0.0555-0.0567 ms, the mid-walk reload costs more than the tail)
  const int p0 = model ? a.nimg : 0, np = model ? a.P - a.nimg : a.nimg;
  const int ntot = np * per_plane;
  const int ntile = bi < ntot ? (ntot - bi + nb - 1) / nb : 0;
  if (ntile == 0) return;  // block-uniform

  f16x8 w1[NT1][2], w2[NT2][2];
  float scale;
  f32x4 bias;
  auto load_weights = [&](int m) __attribute__((always_inline)) {
    const char* wsrc = (const char*)a.wx + (size_t)m * 25 * TAP_BYTES;
    auto frag_w = [&](int tap, int hl) {
      return *(const f16x8*)(wsrc + (size_t)tap * TAP_BYTES + ((((g >> 1) * 2 + hl) * 2 + (g & 1)) * COUT + cg * 16 + l16) * 16);
    };
#pragma unroll
    for (int t = 0; t < NT1; ++t)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) w1[t][hl] = frag_w(TB1 + t, hl);
#pragma unroll
    for (int t = 0; t < NT2; ++t)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) w2[t][hl] = frag_w(TB2 + t, hl);
    scale = a.wscale[m] * 0.0039215688593685627f;  // 2^-k and the dequantiser's 1/255
    bias = *(const f32x4*)(a.bias + m * COUT + cg * 16 + 4 * g);
  };
  load_weights(model);

  // code staging: thread q = threadIdx.x + 512 j loads dword q & 7 of halo pixel q >> 3
  int st_lds[D1A_LD], st_hy[D1A_LD], st_hx[D1A_LD];
#pragma unroll
  for (int j = 0; j < D1A_LD; ++j) {
    const int q = threadIdx.x + 512 * j, pix = q >> 3;
    st_hy[j] = q < 800 ? pix / 10 : -1000;
    st_hx[j] = pix - (pix / 10) * 10;
    st_lds[j] = (pix / 10) * D1_RPB + st_hx[j] * D1_PSB + (q & 7) * 8;
  }
  // codes of the next two tiles in registers (cqa: even tiles, cqb: odd), loaded two tiles
  // ahead: one tile of MFMAs (~3.3k cycles per SIMD) did not cover the HBM latency of the next
  // tile's code loads
  uint32_t cqa[D1A_LD], cqb[D1A_LD];
  TileWalk it_ld, it_run;
  it_ld.init(bi, nb, a.tiles_y, a.tiles_x);
  it_run = it_ld;
  // Buffer loads with an out-of-range offset (0) for pad pixels, issued unconditionally (a tile
  // past the walk: an empty resource): with no branch around them the compiler counts them
  // exactly and waits for a tile's codes with vmcnt(N), past the stores issued since, instead of
  // vmcnt(0), which drained the previous tile's stores first (0.0555 vs 0.0568-0.0572 ms,
  // profiles/r5n_d1_ab; the stores themselves cost ~13 us: 0.043 ms with them dropped,
  // diagnostic build NIC_DIAG_D1NOST)
  const size_t img_bytes = (size_t)a.H * a.W * 96;
  auto load_codes = [&](uint32_t (&cq)[D1A_LD], bool live) __attribute__((always_inline)) {
    int pl, ty, tx;
    it_ld.take(pl, ty, tx);
    const int p = p0 + pl, type = p / a.nimg;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.in_u8 + (live ? (size_t)(p % a.nimg) * img_bytes + type * 32 : 0)), (short)0,
        live ? (int)(img_bytes - type * 32) : 0, kBufWord3);
#pragma unroll
    for (int j = 0; j < D1A_LD; ++j) {
      const int gy = ty * 8 - 1 + st_hy[j], gx = tx * 8 - 1 + st_hx[j];
      const bool ok = (unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W;
      cq[j] = __builtin_amdgcn_raw_buffer_load_b32(
          rs, ok ? (unsigned)(((gy * a.W + gx) * 96) + (threadIdx.x & 7) * 4) : kDmaOOR, 0, 0);
    }
  };
  const int st_off = (g & 1) * COUT + cg * 16 + 8 * (g >> 1);
  const unsigned out_plane = (unsigned)((size_t)a.OH * a.OW * PXB);
  unsigned g_off[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int dy = 2 * m + (l16 >> 3), dx = l16 & 7;
    g_off[m] = (unsigned)(((2 * dy) * a.OW + 2 * dx) * PXB + st_off * 2);
  }
  float rmax = 0.f;
  // one phase of the staged tile: MFMA chains over its taps, then bias + leaky + split stores
  auto phase = [&](const char* buf, const f16x8* wr, auto shape_c, int py, int px, int p, int ty0, int tx0) {
    constexpr int KH = decltype(shape_c)::value / 4, KW = decltype(shape_c)::value % 4, NTAPS = KH * KW;
    int bx[KW];
#pragma unroll
    for (int kw = 0; kw < KW; ++kw) bx[kw] = (l16 >> 3) * D1_RPB + ((l16 & 7) + kw) * D1_PSB + g * 16;  // halo origin (y - 1, x - 1)
    const unsigned bb = lds_off(buf);
    auto frag = [&](int m, int t) {
      const int kh = t / KW, kw = t - kh * KW;
      return *(const __attribute__((address_space(3))) f16x8*)(lds_at(bb + bx[kw]) + (2 * m + kh) * D1_RPB);
    };
    f32x4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = (f32x4){0.f, 0.f, 0.f, 0.f};
#ifndef NIC_D1_LA
#define NIC_D1_LA 1  // B-fragment read-ahead in taps (A/B build: 2)
#endif
    f16x8 fb[NIC_D1_LA][MT];
#pragma unroll
    for (int u = 0; u < NIC_D1_LA; ++u)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        if (u < NTAPS) fb[u][m] = frag(m, u);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = 0; t < NTAPS; ++t) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        f16x8& cur = fb[t % NIC_D1_LA][m];
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[2 * t + 1], cur, acc[m], 0, 0, 0);  // w_lo*c
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[2 * t], cur, acc[m], 0, 0, 0);      // w_hi*c
        if (t + NIC_D1_LA < NTAPS) cur = frag(m, t + NIC_D1_LA);
        __builtin_amdgcn_sched_barrier(0);  // keep the rolling order
      }
    }
    __builtin_amdgcn_s_setprio(0);
    const __amdgpu_buffer_rsrc_t out_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.out_s + (size_t)p * out_plane / 2), (short)0, (int)out_plane, kBufWord3);
    const unsigned out_org = (unsigned)(((2 * ty0 + py) * a.OW + 2 * tx0 + px) * PXB);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int y = ty0 + 2 * m + (l16 >> 3), x = tx0 + (l16 & 7);
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = leaky02(scale_bias(acc[m][r], scale, bias[r]));
      const bool in = y < a.H && x < a.W;
      if (in) range_track(rmax, v);
      f16x4 hi, lo;
      split4(v, hi, lo);
#ifdef NIC_DIAG_D1NOST  // diagnostic build only: every store dropped (out of range; wrong results)
      __builtin_amdgcn_raw_buffer_store_b128(swap16_pair(hi, lo), out_rs, kDmaOOR, 0, 0);
#elif defined(NIC_DIAG_D1LIN)  // diagnostic build only: the same bytes as 1-KB contiguous stores (wrong layout)
      {
        const unsigned tq = (unsigned)(((ty0 >> 3) * a.tiles_x + (tx0 >> 3)) * 4 + py * 2 + px) * 4 + cg;
        __builtin_amdgcn_raw_buffer_store_b128(swap16_pair(hi, lo), out_rs, tq * 4096u + (unsigned)(m * 64 + lane) * 16u, 0, 0);
      }
#else
      __builtin_amdgcn_raw_buffer_store_b128(swap16_pair(hi, lo), out_rs, in ? out_org + g_off[m] : kDmaOOR, 0, 0);
#endif
    }
  };
  auto step = [&](int i, uint32_t (&cq)[D1A_LD]) __attribute__((always_inline)) {
    char* buf = lds + (i & 1) * D1_HB;
#pragma unroll
    for (int j = 0; j < D1A_LD; ++j) {  // codes -> f16 (exact) in LDS
      if (st_hy[j] < 0) continue;
      const uint32_t q = cq[j];
      const f16x4 c = {(_Float16)(float)(q & 255), (_Float16)(float)((q >> 8) & 255),
                       (_Float16)(float)((q >> 16) & 255), (_Float16)(float)(q >> 24)};
      *(f16x4*)(buf + st_lds[j]) = c;
    }
    lds_reads_done();
    stage_barrier();  // tile i's halo complete; tile i-2's reads of this buffer done everywhere
    int pl, ty, tx;
    it_run.take(pl, ty, tx);
    if constexpr (NIC_D1A_PF == 2) {
      load_codes(cq, i + 2 < ntile);  // tile i+2: lands during this tile's and the next's MFMAs
    } else {  // A/B build: one tile ahead
      load_codes(cq, i + 1 < ntile);
    }
    phase(buf, &w1[0][0], std::integral_constant<int, KH1 * 4 + KW1>{}, PY1, PX1, p0 + pl, ty * 8, tx * 8);
    phase(buf, &w2[0][0], std::integral_constant<int, KH2 * 4 + KW2>{}, PY2, PX2, p0 + pl, ty * 8, tx * 8);
  };
  load_codes(cqa, true);
  if constexpr (NIC_D1A_PF == 2) {
    load_codes(cqb, ntile > 1);
    // 16 dropped stores (empty resource): the loop header then sees as many memory operations
    // younger than cqa / cqb on entry as on the back edge (a tile's 8 stores, the next codes, the
    // next tile's 8 stores), so the compiler's merged counter waits stay at vmcnt(18) instead of
    // the prologue's vmcnt(2), which drained the last tile's stores before every other tile
    {
      const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc((void*)a.out_s, (short)0, 0, kBufWord3);
#pragma unroll
      for (int k = 0; k < 16; ++k) __builtin_amdgcn_raw_buffer_store_b32(0u, none, kDmaOOR + 256u * k, 0, 0);
    }
    int i = 0;
    for (; i + 1 < ntile; i += 2) {  // no branch inside: the back edge's counter state is exact
      step(i, cqa);
      step(i + 1, cqb);
    }
    if (i < ntile) step(i, cqa);
  } else {
    for (int i = 0; i < ntile; ++i) step(i, cqa);
  }
  range_report(a.rg, rmax);
}

__global__ __launch_bounds__(512, 1) void dconv1_all_kernel(ConvArgs a) {
  KT_SCOPE(5);
  __shared__ __attribute__((aligned(16))) char lds[2 * D1_HB];
  const int gi = (int)blockIdx.x >= a.ws_blk[1] ? 1 : 0;
  const int bi = blockIdx.x - a.ws_blk[gi], nb = a.ws_blk[gi + 1] - a.ws_blk[gi];
  if (threadIdx.x < 256)  // phases (1,1) 3x3 taps (tap base 16) and (0,0) 2x2 (base 0)
    d1all_wave<3, 3, 16, 1, 1, 2, 2, 0, 0, 0>(a, lds, gi, bi, nb);
  else  // phases (0,1) 2x3 (base 4) and (1,0) 3x2 (base 10)
    d1all_wave<2, 3, 4, 0, 1, 3, 2, 10, 1, 0>(a, lds, gi, bi, nb);
}

// ------------------------------------------------------------------------------------
// Fused residual pair of the k3 s1 layers: out = leaky(conv_b(leaky(conv_a(x) + b_a)) + b_b) + x
// (encoder.py:22-25 conv3 -> conv4 -> + res; decoder.py:26-29 dconv5 -> dconv6 -> + res, the
// Conv2DTranspose k3 s1 layers repacked as flipped convs).  Split-f16 in and out.
//
// The two separate weight-stationary launches move, per pixel, the input with its tile halo
// (256 B x 1.56), conv_a's output out and back in with its halo, the residual, and the
// output: ~1.6 KB per pixel for 147 kFLOP -- at the f16x3 ridge point (833 TFLOP/s / 8 TB/s).
// Here a block owns whole rows (planes up to K3P_MAX_W = 64 columns: the 256^2 images of
// BASELINE config 2) -- a contiguous range of the stream of all planes' rows, one block per
// CU -- and streams down each plane's part of it:
//   * the input rows arrive by LDS-DMA into a 5-row ring (row y+2 lands while row y+1 is
//     being convolved), read once from HBM (+2 rows per segment);
//   * waves 0-3 (conv_a, 16 output channels each, weights resident in VGPRs) convolve input
//     rows y-1..y+1 into row y of a 4-row ring of conv_a outputs in LDS (split records);
//   * waves 4-7 (conv_b) convolve rows y-3..y-1 of that ring into output row y-2, add the
//     residual from the input ring (still resident) and store the split row to HBM.
// One block barrier per row step.  conv_a's row never leaves the chip, the residual is not
// re-read, and the only halo is one recomputed conv_a row on each side of a range boundary
// inside a plane (config 2: 48 rows per block, +4 % conv_a work).  LDS rows are 66 pixel records (the image's columns plus zero
// records for columns -1 and W, conv SAME padding), chunk c of record r in slot c ^ (2r & 15):
// every B-fragment ds_read_b128 (16 consecutive pixels per lane group) is conflict-free
// (the GeomWS swizzle, checked for the row layout against MI355X_MICROARCH.md's lane groups).
// ------------------------------------------------------------------------------------
constexpr int K3P_MAX_W = 64;
constexpr int K3P_SW = 62;                          // strip mode: output columns per strip
constexpr int K3P_REC = 256;                        // split record: 64 ch x [hi | lo] f16
constexpr int K3P_RW = K3P_MAX_W + 4;               // records per LDS row (66 used, whole DMA pieces)
constexpr int K3P_ROWB = K3P_RW * K3P_REC;          // 17,408 B
constexpr int K3P_NI = 5, K3P_NC = 4;               // input / conv_a ring rows
// skewed pair: the next input row's DMA issued by conv_b after its deferred epilogue
// (NIC_K3P_DMAB=1) instead of by conv_a at the step start, whose stream then starts at once
#ifndef NIC_K3P_DMAB
#define NIC_K3P_DMAB 1
#endif
constexpr bool kK3pDmaB = NIC_K3P_DMAB != 0;
constexpr int K3P_LDS = (K3P_NI + K3P_NC) * K3P_ROWB;  // 156,672 B

__device__ __forceinline__ int k3p_off(int rec, int chunk) { return rec * K3P_REC + ((chunk ^ ((2 * rec) & 15)) << 4); }

// STRIP (planes wider than 64 columns, MT = 4): the plane is cut into strips of 62 output
// columns (a.tiles_x of them); per strip the input rows carry 66 columns (2 each side), conv_a
// computes 64 (the strip's 62 plus the column either side conv_b needs, zeros outside the
// plane) and conv_b the strip's 62 (3 % of its lanes and 3 % of conv_a's work are the seams).
// Row ranges of the pair's blocks balanced by pipeline steps (launch_k3pair_x3): block b takes
// rows [start[b], start[b + 1]) of the stream; start[0] < 0: the plain equal-rows split
constexpr int K3P_MAX_GRID = 320;
struct K3Ranges {
  int start[K3P_MAX_GRID + 1];
};
template <int MT, bool SKEW, bool STRIP>
__global__ __launch_bounds__(512, 1) void conv_k3pair_kernel(ConvArgs a, K3Ranges rng) {
  KT_SCOPE(2);
  constexpr int COUT = 64, KST = 2;
  __shared__ __attribute__((aligned(16))) char lds[K3P_LDS];
  char* in_ring = lds;
  char* c3_ring = lds + K3P_NI * K3P_ROWB;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int role = wave >> 2, w = wave & 3;  // role 0: conv_a, 1: conv_b; w: 16-channel group
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  const int H = a.H, W = a.W;
  // this block's contiguous range of output rows in the stream of all planes' rows (p * H + y),
  // cut into one segment per plane it touches: the ring pipeline fills and drains once per
  // segment, and only a segment boundary inside a plane recomputes a conv_a row
  static_assert(!STRIP || MT == 4, "strips are 4 M tiles wide");
  const int nstrips = STRIP ? a.tiles_x : 1;
  const long long total_rows = (long long)a.P * nstrips * H;
  long long g0, g1;
  if (rng.start[0] >= 0) {
    g0 = rng.start[blockIdx.x];
    g1 = rng.start[blockIdx.x + 1];
  } else {
    const long long per_block = (total_rows + gridDim.x - 1) / gridDim.x;
    g0 = (long long)blockIdx.x * per_block;
    g1 = min(g0 + per_block, total_rows);
  }
  const unsigned plane_bytes = (unsigned)(H * W) * K3P_REC;

  // zero records: columns -1 and W.. of every ring row (never written afterwards)
  for (int q = threadIdx.x; q < (K3P_NI + K3P_NC) * K3P_RW * 16; q += 512) {
    const int row = q / (K3P_RW * 16), r = q - row * (K3P_RW * 16), rec = r >> 4;
    if (rec == 0 || rec > W) *(u32x4*)(lds + row * K3P_ROWB + r * 16) = (u32x4){0u, 0u, 0u, 0u};
  }

  // B fragments: pixel 16 m + l16 of an LDS row at tap column kw -> record 16 m + l16 + kw;
  // lane group g reads chunk 8 hl + 4 ks + g (the XOR with (2 hl + ks) << 6 selects hl, ks)
  int bx[3];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) bx[kw] = k3p_off(l16 + kw, g);
  const int chunk_st = (g & 1) * 8 + 2 * w + (g >> 1);  // this lane's 16-B granule after swap16_pair
  const int chunk_rh = 2 * w + (g >> 1), rsub = 8 * (g & 1);  // residual: hi / lo of channels 16 w + 4 g ..

  f16x8 wr[9][KST][2];
  int model = -1;
  float scale = 0.f;
  f32x4 bias = {};
  float rmax = 0.f;
  auto load_weights = [&](int m) {
    const uint16_t* wx = role == 0 ? a.wx : a.wx2;
    constexpr int TAP_BYTES = 64 * COUT * 4;
    const char* wsrc = (const char*)wx + (size_t)m * 9 * TAP_BYTES;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int ks = 0; ks < KST; ++ks)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
          wr[t][ks][hl] = *(const f16x8*)(wsrc + (size_t)t * TAP_BYTES +
                                          ((((2 * ks + (g >> 1)) * 2 + hl) * 2 + (g & 1)) * COUT + w * 16 + l16) * 16);
    scale = role == 0 ? a.wscale[m] : a.wscale2[m];
    bias = *(const f32x4*)((role == 0 ? a.bias : a.bias2) + m * COUT + 16 * w + 4 * g);
  };

  // Column geometry of a segment (strip origin sx0): input record r holds column xi0 + r,
  // conv_a's pixel i is column xa0 + i (its output record i + ca_off), conv_b's pixel j column
  // sx0 + j (valid below jmax), whose residual is input record j + rb_off.
  constexpr int ca_off = STRIP ? 0 : 1, rb_off = STRIP ? 2 : 1, jmax = STRIP ? K3P_SW : 64;
  constexpr int rec0 = STRIP ? 0 : 1;  // first DMA'd input record (single strip: record 0 is column -1, zero)
  int sx0 = 0;
  // input row y (zeros outside the plane) into ring slot `slot`: 1-KB DMA pieces over the 8
  // waves; LDS slot k of record rec holds chunk k ^ (2 rec & 15) of column xi0 + rec
  // SKEW: the conv_a waves issue every piece (conv_b's step then starts with its epilogue)
  auto dma_row = [&](const __amdgpu_buffer_rsrc_t& rs, int y, int slot) {
    const int npiece = STRIP ? K3P_RW / 4 : (W * 16 + 63) / 64;
    const int xi0 = STRIP ? sx0 - 2 : -1;
    char* dst = in_ring + slot * K3P_ROWB + rec0 * K3P_REC;
    if (SKEW && role == (kK3pDmaB ? 0 : 1)) return;
    for (int k = SKEW ? w : wave; k < npiece; k += SKEW ? 4 : 8) {
      const int q = 64 * k + lane, rec = rec0 + (q >> 4), x = xi0 + rec, ch = (q & 15) ^ ((2 * rec) & 15);
      const bool ok = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W && rec < K3P_MAX_W + 2;
      dma16_buf(rs, ok ? (unsigned)((y * W + x) * K3P_REC + ch * 16) : kDmaOOR, dst + k * 1024);
    }
  };

  // one output row of this wave's layer: taps (kh, kw) over LDS rows r_kh (byte offsets), then
  // `epi(m)` for each M tile (a no-op for conv_b in SKEW mode: its epilogue runs next step)
  f32x4 acc[MT];
#ifdef NIC_STAMPS  // tools/k3p_stamps.cpp: per role, cycles waiting at the step barrier, in the
                   // MFMA stream, in the epilogue, and in the DMA issue
  unsigned long long s_wait = 0, s_mfma = 0, s_epi = 0, s_dma = 0, s_t0, s_t1, s_steps = 0;
  const unsigned long long s_rt0 = __builtin_amdgcn_s_memrealtime(), s_c0 = __builtin_amdgcn_s_memtime();
#endif
  auto conv_row = [&](unsigned r0b, unsigned r1b, unsigned r2b, auto&& epi) {
#ifdef NIC_STAMPS
    NIC_PNOW(s_t0);
#endif
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = (f32x4){0.f, 0.f, 0.f, 0.f};
    constexpr int NSTEP = 9 * KST;
    // per (kh, kw): row base + this lane's record / slot (row bases are multiples of 256 B, so
    // the (hl, ks) XOR below leaves them intact): one v_xor per fragment read, the M tile in
    // the ds_read immediate
    unsigned xb[3][3];
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      xb[0][kw] = r0b + (unsigned)bx[kw];
      xb[1][kw] = r1b + (unsigned)bx[kw];
      xb[2][kw] = r2b + (unsigned)bx[kw];
    }
    auto frag = [&](int m, int st, int hl) {
      const int t = st / KST, ks = st - t * KST, kh = t / 3, kw = t - kh * 3;
      return *(const __attribute__((address_space(3))) f16x8*)(lds_at(xb[kh][kw] ^ (unsigned)((2 * hl + ks) << 6)) +
                                                               m * 16 * K3P_REC);
    };
    f16x8 fb[MT][2];
    static_for<MT>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      fb[m][0] = frag(m, 0, 0);
      fb[m][1] = frag(m, 0, 1);
    });
    // (conv_b's stream at priority 2 over conv_a's measured 1 % slower: conv_a's stream, and with
    // it the epilogue writing the rows conv_b needs next step, then finishes later; round 4)
    __builtin_amdgcn_s_setprio(1);
    static_for<NSTEP>([&](auto stc) {
      constexpr int st = decltype(stc)::value, t = st / KST, ks = st % KST;
      static_for<MT>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][ks][1], fb[m][0], acc[m], 0, 0, 0);  // w_lo*a_hi
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][ks][0], fb[m][1], acc[m], 0, 0, 0);  // w_hi*a_lo
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[t][ks][0], fb[m][0], acc[m], 0, 0, 0);  // w_hi*a_hi
        if constexpr (st + 1 < NSTEP) {
          fb[m][0] = frag(m, st + 1, 0);
          fb[m][1] = frag(m, st + 1, 1);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the rolling order
      });
    });
    __builtin_amdgcn_s_setprio(0);
#ifdef NIC_STAMPS
    NIC_PNOW(s_t1);
    s_mfma += s_t1 - s_t0;
#endif
    static_for<MT>([&](auto mc) { epi(decltype(mc)::value); });
#ifdef NIC_STAMPS
    NIC_PNOW(s_t0);
    s_epi += s_t0 - s_t1;
#endif
  };

  const unsigned in_base = lds_off(in_ring), c3_base = lds_off(c3_ring);
  // conv_b: the residual (input row y4, split) of this lane's 4 channels per M tile, read from
  // the input ring into registers; epilogue of output row y4 from acc and those registers
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  u32x2 rr[MT][2];
  auto load_res = [&](const char* res) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int jx = 16 * m + l16;
      rr[m][0] = *(const u32x2*)(res + k3p_off(jx + rb_off, chunk_rh) + rsub);
      rr[m][1] = *(const u32x2*)(res + k3p_off(jx + rb_off, 8 + chunk_rh) + rsub);
    }
  };
  auto epi_b = [&](int m, int y4, const __amdgpu_buffer_rsrc_t& rs_out) {
    const int jx = 16 * m + l16, x = sx0 + jx;
    const bool valid = jx < jmax && x < W;
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = leaky02(scale_bias(acc[m][r], scale, bias[r]));
    static_for<4>([&](auto rc) {  // x = x + res (encoder.py:25, decoder.py:29)
      constexpr int r = decltype(rc)::value;
      v[r] = __fadd_rn(v[r], add_f16_pair<r & 1>(rr[m][0][r >> 1], rr[m][1][r >> 1]));
    });
    if (valid) range_track(rmax, v);
    f16x4 hi, lo;
    split4(v, hi, lo);
    const u32x4 q = swap16_pair(hi, lo);
    const unsigned orow = (unsigned)(y4 * W) * K3P_REC + (unsigned)chunk_st * 16;
    __builtin_amdgcn_raw_buffer_store_b128(q, rs_out, valid ? orow + (unsigned)(x * K3P_REC) : kDmaOOR, 0, 0);
  };
  // the step loop per role, compiled separately: values one role keeps across the step
  // barrier (conv_b's accumulators and residual in SKEW mode) are not live in the other's code
  auto run = [&](auto role_c) {
    constexpr int ROLE = decltype(role_c)::value;
    for (long long gs = g0; gs < g1;) {
      const long long col = gs / H;  // (plane, strip) column of rows
      const int p = (int)(col / nstrips);
      sx0 = (int)(col - (long long)p * nstrips) * K3P_SW;
      const int r0 = (int)(gs - col * H), r1 = (int)min((long long)H, g1 - col * H), nrow = r1 - r0;
      gs = col * H + r1;
      const int m_item = p >= a.nimg ? 1 : 0;
      if (m_item != model) {  // wave-uniform: items of one model are consecutive
        model = m_item;
        load_weights(model);
      }
      const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((const char*)a.in_s + (size_t)p * plane_bytes), (short)0, (int)plane_bytes, kBufWord3);
      const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((char*)a.out_s + (size_t)p * plane_bytes), (short)0, (int)plane_bytes, kBufWord3);
      // input rows r0 - 2 .. r0 (ring slot of row y: (y - r0 + 2) % 5)
#pragma unroll
      for (int k = 0; k < 3; ++k) dma_row(rs_in, r0 - 2 + k, k);
      dma_wait_all();
      lds_reads_done();  // (first item) the zero records are written
      stage_barrier();
      for (int j = 0; j <= nrow + 2; ++j) {
#ifdef NIC_STAMPS
        unsigned long long s_a, s_b;
        NIC_PNOW(s_a);
#endif
        // the next input row lands during this step.  (SKEW: issuing conv_a's pieces inside its
        // MFMA stream instead measured no faster -- 4 LDS-DMA issues cost ~700 cycles either way)
        // kK3pDmaB: conv_b issues it, after its deferred epilogue once it has rows (j >= 3)
        if (j <= nrow && !(SKEW && kK3pDmaB && ROLE == 1 && j >= 3)) dma_row(rs_in, r0 + j + 1, (j + 3) % K3P_NI);
#ifdef NIC_STAMPS
        NIC_PNOW(s_b);
        s_dma += s_b - s_a;
        ++s_steps;
#endif
        if constexpr (ROLE == 0) {
          if (j <= nrow + 1) {  // conv_a row y3 = r0 - 1 + j into conv_a ring slot j % 4
            const int y3 = r0 - 1 + j;
            char* dst = c3_ring + (j % K3P_NC) * K3P_ROWB;
            const int xa0 = STRIP ? sx0 - 1 : 0;
            auto epi = [&](int m) {
              const int i = 16 * m + l16, x = xa0 + i;
              const bool in = (unsigned)x < (unsigned)W;  // outside the plane: zero (conv_b's padding)
              f32x4 v;
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = in ? leaky02(scale_bias(acc[m][r], scale, bias[r])) : 0.f;
              if (in) range_track(rmax, v);
              f16x4 hi, lo;
              split4(v, hi, lo);
              const u32x4 q = swap16_pair(hi, lo);
              *(u32x4*)(dst + k3p_off(i + ca_off, chunk_st)) = q;
            };
            if ((unsigned)y3 < (unsigned)H) {
              conv_row(in_base + (unsigned)((j % K3P_NI) * K3P_ROWB), in_base + (unsigned)(((j + 1) % K3P_NI) * K3P_ROWB),
                       in_base + (unsigned)(((j + 2) % K3P_NI) * K3P_ROWB), epi);
            } else {  // rows outside the plane: zeros (conv_b's SAME padding)
#pragma unroll
              for (int m = 0; m < MT; ++m) *(u32x4*)(dst + k3p_off(16 * m + l16 + ca_off, chunk_st)) = (u32x4){0u, 0u, 0u, 0u};
            }
          }
        } else if (j >= 3) {  // conv_b row y4 = r0 + j - 3 from conv_a rows y4 - 1 .. y4 + 1
          const int y4 = r0 + j - 3;
          const char* res = in_ring + ((j + 4) % K3P_NI) * K3P_ROWB;  // input row y4 (the residual)
          const unsigned cb0 = c3_base + (unsigned)(((j + 1) % K3P_NC) * K3P_ROWB),
                         cb1 = c3_base + (unsigned)(((j + 2) % K3P_NC) * K3P_ROWB),
                         cb2 = c3_base + (unsigned)(((j + 3) % K3P_NC) * K3P_ROWB);
          if constexpr (SKEW) {
            if (j >= 4) {  // row y4 - 1: its accumulators and residual are still in registers
#ifdef NIC_STAMPS
              unsigned long long s_e0, s_e1;
              NIC_PNOW(s_e0);
#endif
              static_for<MT>([&](auto mc) { epi_b(decltype(mc)::value, y4 - 1, rs_out); });
#ifdef NIC_STAMPS
              NIC_PNOW(s_e1);
              s_epi += s_e1 - s_e0;
#endif
            }
            // slot (j + 3) % 5 held row y4 - 1's residual, in registers since the last step
            if constexpr (kK3pDmaB)
              if (j <= nrow) dma_row(rs_in, r0 + j + 1, (j + 3) % K3P_NI);
            conv_row(cb0, cb1, cb2, [](int) {});
            load_res(res);  // row y4's residual, read before the next step's DMA reuses its slot
          } else {
            conv_row(cb0, cb1, cb2, [&](int m) {
              if (m == 0) load_res(res);
              epi_b(m, y4, rs_out);
            });
          }
        }
        // this wave's DMA of the next input row landed; conv_b's MT output stores, issued after
        // it, may stay in flight (vector memory operations complete in issue order on gfx9).
        // SKEW: conv_b issues no DMA -- only its LDS reads must be done
#ifdef NIC_STAMPS
        NIC_PNOW(s_a);
#endif
        if (ROLE == 1 && (SKEW || j >= 3)) {
          if constexpr (!SKEW)
            __builtin_amdgcn_s_waitcnt(0x0F70 | MT);  // vmcnt(MT), expcnt 7, lgkmcnt 15
          else if constexpr (kK3pDmaB)
            dma_wait_all();  // conv_b's pieces of the next row (and its older output stores)
        } else if (!(SKEW && kK3pDmaB)) {
          dma_wait_all();
        }
        lds_reads_done();  // and its LDS reads / conv_a writes are done
        stage_barrier();
#ifdef NIC_STAMPS
        NIC_PNOW(s_b);
        s_wait += s_b - s_a;
#endif
      }
      if constexpr (SKEW)  // the segment's last conv_b row
        if (ROLE == 1 && nrow > 0) static_for<MT>([&](auto mc) { epi_b(decltype(mc)::value, r0 + nrow - 1, rs_out); });
    }
  };
  if (role == 0)
    run(std::integral_constant<int, 0>{});
  else
    run(std::integral_constant<int, 1>{});
  range_report(a.rg, rmax);
#ifdef NIC_STAMPS
  if (lane == 0 && (wave == 0 || wave == 4)) {
    unsigned long long* o = g_stamps + (size_t)blockIdx.x * 16 + role * 8;
    o[0] = s_wait;
    o[1] = s_mfma;
    o[2] = s_epi;
    o[3] = s_dma;
    o[4] = s_steps;
    o[5] = __builtin_amdgcn_s_memtime() - s_c0;
    o[6] = __builtin_amdgcn_s_memrealtime() - s_rt0;
    o[7] = 1;
  }
#endif
}

// strips for a plane of W columns (0: the fused pair does not take it): one for W <= 64, else
// 62-column strips when their lanes waste at most 10 % (4K frames: 16 strips over 960 columns)
// (Config 4's 192-column planes would take 4 strips with 23 % of the lanes idle: the pair then
// takes 0.72 / 0.70 ms against 0.31 + 0.35 / 0.30 + 0.34 ms for the two launches, step 3.18 vs
// 3.14 ms on one box, 3 rounds -- so those planes keep the two launches)
static int k3pair_strips(int W) {
  if (W <= K3P_MAX_W) return 1;
  const int n = (W + K3P_SW - 1) / K3P_SW;
  return 10LL * n * 64 <= 11LL * W ? n : 0;
}
bool k3pair_supported(int H, int W) {
  return H > 0 && W > 0 && k3pair_strips(W) > 0 && (long long)H * W * K3P_REC < (1LL << 31);
}

// (Round 4 built the pair on Winograd F(2,3) along y -- 2/3 of the products, both layers' U
// kernels resident in one wave per SIMD -- and measured it 16 % slower than this direct pair:
// with one wave per SIMD nothing hides the transform VALU; removed in round 5,
// see DESIGN section 9 for why a two-wave form does not fit the 160 KB of LDS either.)

// ------------------------------------------------------------------------------------
// conv1 (1 -> 32, k5 s2) with the RGB -> YCbCr front end fused (encoder.py:39-41,
// utils.py:74-77).  Block: 16x16 output pixels of one plane, 4 waves x 2 M tiles x 32 co.
// K = 25 taps padded to 26 (13 MFMAs); lane half h supplies tap 2s+h of step s.
// ------------------------------------------------------------------------------------
constexpr int C1_T = 16;
constexpr int C1_HH = (C1_T - 1) * 2 + 5;  // 35
constexpr int C1_HE = (C1_HH + 1) / 2;     // 18 even columns, then 17 odd ones
// row pitch 40 dwords: the two halo rows an M tile (2 x 16 pixels, stride 2) reads per tap
// are 80 = 16 mod 32 banks apart, and even/odd-split columns make each row's 16 reads
// consecutive -- conflict-free ds_read_b32 for all 32 lanes of a half
constexpr int C1_PS = 40;

constexpr int C1_LDS_FLOATS = C1_HH * C1_PS;
__device__ __forceinline__ int conv1_colour_body(const Conv1Args& a, float* plane, int b0, int nb, int* q = nullptr) {
  float rmax = 0.f;  // range guard of the split output
  const int per_plane = a.tiles_y * a.tiles_x;
  int ran = 0;  // grid-stride or queued, as conv_mfma_body
  for (int job = q ? chain_take(q) : b0; job < per_plane * a.P; job = q ? chain_take(q) : job + nb, ++ran) {
  __syncthreads();  // the previous job's plane reads are done
  const int p = job / per_plane, tile = job - p * per_plane;
  const int n = p % a.nimg, type = p / a.nimg;
  const int model = type > 0 ? 1 : 0;
  const int tyi = tile / a.tiles_x;
  const int t0y = tyi * C1_T, t0x = (tile - tyi * a.tiles_x) * C1_T;
  const int gy0 = t0y * 2 - a.pad_y, gx0 = t0x * 2 - a.pad_x;
  const uint8_t* img = a.rgb + (size_t)n * a.H * a.W * 3;
  const float* k = c_ycbcr + type * 3;
  const float off = c_ycbcr_off[type];
  constexpr int C1_ITER = (C1_HH * C1_HH + 255) / 256;
  uint8_t rgbv[C1_ITER][3];
#pragma unroll
  for (int it = 0; it < C1_ITER; ++it) {  // all byte loads in flight before any is used
    const int idx = min((int)threadIdx.x + it * 256, C1_HH * C1_HH - 1);
    const int hy = idx / C1_HH, hx = idx - hy * C1_HH;
    const int cy = min(max(gy0 + hy, 0), a.H - 1), cx = min(max(gx0 + hx, 0), a.W - 1);
    const uint8_t* px = img + ((size_t)cy * a.W + cx) * 3;
    rgbv[it][0] = px[0];
    rgbv[it][1] = px[1];
    rgbv[it][2] = px[2];
  }
#pragma unroll
  for (int it = 0; it < C1_ITER; ++it) {
    const int idx = threadIdx.x + it * 256;
    if (idx < C1_HH * C1_HH) {
      const int hy = idx / C1_HH, hx = idx - hy * C1_HH;
      const int gy = gy0 + hy, gx = gx0 + hx;
      float v = 0.f;  // SAME zero padding of the colour plane
      if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
        const float r = c_u8_to_unit[rgbv[it][0]], g = c_u8_to_unit[rgbv[it][1]], b = c_u8_to_unit[rgbv[it][2]];
        v = __fadd_rn(project(k, r, g, b), off);
      }
      plane[hy * C1_PS + (hx & 1) * C1_HE + (hx >> 1)] = v;
    }
  }
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5;
  // Weights are the MFMA A operand (rows = output channels), the plane values the B operand
  // (columns = pixels): lane half h supplies tap 2s+h of step s; D[co][pixel] then gives
  // each lane one pixel and four consecutive channels per register group (16-B stores).
  float bw[13];
  const float* w = a.w + model * 26 * 32 + (lane & 31);
#pragma unroll
  for (int s = 0; s < 13; ++s) bw[s] = w[(2 * s + half) * 32];

#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int mt = wave * 2 + i;
    const int m = mt * 32 + (lane & 31);
    const int ty = m / C1_T, tx = m % C1_T;
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < 13; ++s) {
      int tap = 2 * s + half;
      if (tap > 24) tap = 24;  // weight is zero; any finite operand
      const int kh = tap / 5, kw = tap % 5;
      const float av = plane[(ty * 2 + kh) * C1_PS + (kw & 1) * C1_HE + tx + (kw >> 1)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[s], av, acc, 0, 0, 0);
    }
    const int oy = t0y + ty, ox = t0x + tx;
    const bool inside = oy < a.OH && ox < a.OW;
    const size_t pix = inside ? ((size_t)p * a.OH + oy) * a.OW + ox : 0;
    f32x4 v[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 b = *(const f32x4*)(a.bias + model * 32 + 8 * g + 4 * half);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[g][q] = leaky02(__fadd_rn(acc[4 * g + q], b[q]));
    }
    if (a.out_s) {  // split format for the f16x3 conv2: 16-B stores after lane-half swaps
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
        if (inside) {
          range_track(rmax, v[g]);
          range_track(rmax, v[g + 1]);
        }
        f16x4 h0, l0, h1, l1;
        split4(v[g], h0, l0);
        split4(v[g + 1], h1, l1);
        swap_pair(h0, h1);
        swap_pair(l0, l1);
        const int co = 8 * g + 8 * half;
        if (inside) {
          *(f16x8*)(a.out_s + pix * 64 + co) = (f16x8){h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
          *(f16x8*)(a.out_s + pix * 64 + 32 + co) = (f16x8){l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
        }
      }
    } else if (inside) {
#pragma unroll
      for (int g = 0; g < 4; ++g) *(f32x4*)(a.out + pix * 32 + 8 * g + 4 * half) = v[g];
    }
  }
  }  // job
  range_report(a.rg, rmax);
  return ran;
}

__global__ __launch_bounds__(256) void conv1_colour_kernel(Conv1Args a) {
  __shared__ float plane[C1_LDS_FLOATS];
  if (range_gated_off(a.rg)) return;
  conv1_colour_body(a, plane, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------------------------
// dconv8 (64 -> 1, transposed k5 s2) fused with the inverse colour transform and output
// quantiser (decoder.py:31-32, 45-48; utils.py:70-72).  HBM-bound: it streams the 64-ch
// dconv7 output once (P x 4h x 4w x 256 B) and writes 3 B per output pixel.
// Block = 256 threads = 8 x 32 coarse positions of one image, one thread per position;
// for each of the Y, Cb, Cr planes the 10 x 34 halo is staged 32 channels at a time
// (128-B contiguous pieces per pixel, 144-B LDS pixel stride: conflict-free ds_read_b128 for
// 16 consecutive positions).  A thread keeps its 4 output phases of each plane in
// registers, then converts to RGB.  Weights are block-uniform (scalar loads).
// ------------------------------------------------------------------------------------
constexpr int D8_TH = 8, D8_TW = 32;
constexpr int D8_HH = D8_TH + 2, D8_HW = D8_TW + 2;  // 10 x 34
constexpr int D8_CC = 32;                            // channels per LDS chunk
constexpr int D8_PS = D8_CC + 4;                     // pixel stride in LDS (floats)

constexpr int D8_C4 = D8_CC / 4;
constexpr int D8_LOADS = (D8_HH * D8_HW * D8_C4 + 255) / 256;  // 16-B loads per thread per chunk

// Issue the global loads of one (plane, channel chunk) halo into registers.
__device__ __forceinline__ void d8_load(f32x4 (&r)[D8_LOADS], const Dconv8Args& a, int p, int c0, int t0y, int t0x) {
  const float* inp = a.in + (size_t)p * a.H * a.W * 64 + c0;
#pragma unroll
  for (int k = 0; k < D8_LOADS; ++k) {
    const int idx = threadIdx.x + k * 256;
    const int pix = idx / D8_C4, c4 = idx % D8_C4;
    const int hy = pix / D8_HW, hx = pix - hy * D8_HW;
    const int gy = t0y - 1 + hy, gx = t0x - 1 + hx;
    const int cy = min(max(gy, 0), a.H - 1), cx = min(max(gx, 0), a.W - 1);
    r[k] = *(const f32x4*)(inp + ((size_t)cy * a.W + cx) * 64 + c4 * 4);  // clamped: always valid
    if (!(gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)) r[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
}

// Inverse colour transform, clip and quantiser of the four output pixels (2my + py, 2mx + px)
// of image n (decoder.py:45-48, utils.py:70-72): convert_to_rgb (Y - 0, Cb - .5, Cr - .5)
// projected by fp32(inv kernel), clipped; 6-B stores (two pixels per output row).
__device__ __forceinline__ void d8_store_rgb(const Dconv8Args& a, int n, int my, int mx, const float (&outv)[3][4]) {
  const int OW = a.W * 2;
#pragma unroll
  for (int py = 0; py < 2; ++py) {
    uint8_t rgb[6];
    float rgbf[6];
#pragma unroll
    for (int px = 0; px < 2; ++px) {
      const int ph = py * 2 + px;
      const float t0 = __fsub_rn(outv[0][ph], c_ycbcr_off[0]);
      const float t1 = __fsub_rn(outv[1][ph], c_ycbcr_off[1]);
      const float t2 = __fsub_rn(outv[2][ph], c_ycbcr_off[2]);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v = clip01(project(c_ycbcr_inv + 3 * c, t0, t1, t2));
        rgbf[px * 3 + c] = v;
        rgb[px * 3 + c] = quant255(v);
      }
    }
    const size_t o = (((size_t)n * a.H * 2 + 2 * my + py) * OW + 2 * mx) * 3;
    uint16_t* d16 = (uint16_t*)(a.out_u8 + o);  // o is even: 2-byte aligned
    d16[0] = rgb[0] | (rgb[1] << 8);
    d16[1] = rgb[2] | (rgb[3] << 8);
    d16[2] = rgb[4] | (rgb[5] << 8);
    if (a.out_f32) {
#pragma unroll
      for (int k = 0; k < 6; ++k) a.out_f32[o + k] = rgbf[k];
    }
  }
}

constexpr int D8_LDS_FLOATS = D8_HH * D8_HW * D8_PS;
// UNR: channel-quad unroll (2 in the standalone kernel; 1 inside fp32_chain_kernel, whose
// register budget is that of two resident blocks per CU)
template <int UNR = 2>
__device__ __forceinline__ int dconv8_colour_body(const Dconv8Args& a, float* halo, int b0, int nb, int* q = nullptr) {
  const int per_img = a.tiles_y * a.tiles_x;
  int ran = 0;  // grid-stride or queued, as conv_mfma_body
  for (int job = q ? chain_take(q) : b0; job < per_img * a.nimg; job = q ? chain_take(q) : job + nb, ++ran) {
  const int n = job / per_img, tile = job - n * per_img;
  const int tyi = tile / a.tiles_x;
  const int t0y = tyi * D8_TH, t0x = (tile - tyi * a.tiles_x) * D8_TW;
  const int ty = threadIdx.x / D8_TW, tx = threadIdx.x % D8_TW;
  float outv[3][4];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};

  // 6 steps = 3 planes (Y, Cb, Cr) x 2 channel chunks; the next step's halo is loaded
  // into registers while this step computes (issue early, write to LDS after the barrier)
  f32x4 pre[D8_LOADS];
  d8_load(pre, a, n, 0, t0y, t0x);
#pragma unroll 1
  for (int step = 0; step < 6; ++step) {
    const int type = step >> 1, c0 = (step & 1) * D8_CC;
    const int model = type > 0 ? 1 : 0;
    __syncthreads();  // everyone is done reading the previous chunk
#pragma unroll
    for (int k = 0; k < D8_LOADS; ++k) {
      const int idx = threadIdx.x + k * 256;
      if (idx < D8_HH * D8_HW * D8_C4) *(f32x4*)(halo + (idx / D8_C4) * D8_PS + (idx % D8_C4) * 4) = pre[k];
    }
    __syncthreads();
    if (step + 1 < 6) {
      const int nt = (step + 1) >> 1;
      d8_load(pre, a, nt * a.nimg + n, ((step + 1) & 1) * D8_CC, t0y, t0x);
    }
    const float* __restrict__ w = a.w + model * 25 * 64 + c0;  // [phase-tap][ci]
#pragma unroll UNR
    for (int c4 = 0; c4 < D8_C4; ++c4) {
      f32x4 x[3][3];
#pragma unroll
      for (int iy = 0; iy < 3; ++iy)
#pragma unroll
        for (int ix = 0; ix < 3; ++ix)
          x[iy][ix] = *(const f32x4*)(halo + ((ty + iy) * D8_HW + tx + ix) * D8_PS + c4 * 4);
      int tb = 0;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int py = ph >> 1, px = ph & 1;
        const int ny = py ? 3 : 2, nx = px ? 3 : 2;
#pragma unroll
        for (int iy = 0; iy < ny; ++iy)
#pragma unroll
          for (int ix = 0; ix < nx; ++ix) {
            const float* wt = w + (tb + iy * nx + ix) * 64 + c4 * 4;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[ph] = fmaf(x[iy][ix][r], wt[r], acc[ph]);
          }
        tb += ny * nx;
      }
    }
    if (step & 1) {
      const float b = a.bias[model];
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        outv[type][ph] = clip01(leaky02(__fadd_rn(acc[ph], b)));
        acc[ph] = 0.f;
      }
    }
  }

  const int my = t0y + ty, mx = t0x + tx;
  if (my < a.H && mx < a.W) d8_store_rgb(a, n, my, mx, outv);
  }  // job (the next job's first step barrier orders the halo reuse)
  return ran;
}

__global__ __launch_bounds__(256) void dconv8_colour_kernel(Dconv8Args a) {
  __shared__ __attribute__((aligned(16))) float halo[D8_LDS_FLOATS];
  if (range_gated_off(a.rg)) return;
  dconv8_colour_body(a, halo, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------------------------
// dconv8 as a gather of dconv7's projections (f16x3 decoder tail, see ws_body PROJ):
// output pixel (2m + (py, px)) of plane p = bias + sum over the phase's window (iy, ix) of
// proj[m - 1 + (iy, ix)][tb(py, px) + iy (2 + px) + ix], then leaky, clip and the colour
// epilogue.  One thread per coarse position m, all three planes; every (pixel, tap)
// projection feeds exactly one output, so the 25 floats per pixel are read once.  Block =
// 16 x 16 positions; wave w takes the positions of parity (w / 2, w % 2), 8 x 8 at stride
// 2, so for every (iy, ix) its 64 neighbours share one dconv7 phase and form an 8 x 8
// window of that phase's coarse grid: each load reads whole 32-B rows of the tile-major
// projection planes.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dconv8_gather_kernel(Dconv8Args a) {
  KT_SCOPE(7);
  // XCD-aware order: blocks are dealt round-robin to the 8 XCDs, so block L runs on XCD
  // L % 8; give each XCD a contiguous raster range of (image, tile) instead, so neighbouring
  // tiles -- which read each other's edge projections -- share that XCD's L2
  const int gx = gridDim.x, total = gx * gridDim.y, L = blockIdx.y * gx + blockIdx.x;
  const int T = (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);
  const int n = T / gx, tb = T - n * gx;
  const int tyi = tb / a.tiles_x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int my = tyi * 16 + 2 * (lane >> 3) + (wave >> 1);
  const int mx = (tb - tyi * a.tiles_x) * 16 + 2 * (lane & 7) + (wave & 1);
  if (my >= a.H || mx >= a.W) return;
  constexpr int TB[4] = {0, 4, 10, 16};  // phase-major tap bases (for_each_phase_tap)
  // the 9 neighbours' tap-0 byte offsets inside one plane's projection block (the same for
  // the three planes), resolved once; neighbours outside the image get an offset past the
  // buffer, whose loads return 0.  Buffer loads from a per-plane resource keep every address
  // 32-bit and the tap offsets in the instruction's immediate.
  const unsigned plane_floats = 4u * a.tiles_y7 * a.tiles_x7 * (25u * 64u);
  unsigned off[3][3];
#pragma unroll
  for (int iy = 0; iy < 3; ++iy)
#pragma unroll
    for (int ix = 0; ix < 3; ++ix) {
      const int ny = my - 1 + iy, nx = mx - 1 + ix;
      const bool ok = (unsigned)ny < (unsigned)a.H && (unsigned)nx < (unsigned)a.W;
      const int cy = ny >> 1, cx = nx >> 1, ph7 = (ny & 1) * 2 + (nx & 1);
      off[iy][ix] = ok ? (((unsigned)((ph7 * a.tiles_y7 + (cy >> 3)) * a.tiles_x7 + (cx >> 3)) * (25u * 64u) +
                           (unsigned)((cy & 7) * 8 + (cx & 7))) * 4u)
                       : kDmaOOR;
    }
  float outv[3][4];
#pragma unroll
  for (int type = 0; type < 3; ++type) {
    const int p = type * a.nimg + n;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.proj + (size_t)p * plane_floats), (short)0, (int)(plane_floats * 4u), kBufWord3);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int iy = 0; iy < 3; ++iy)
#pragma unroll
      for (int ix = 0; ix < 3; ++ix) {
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {
          const int py = ph >> 1, px = ph & 1;
          if (iy < 2 + py && ix < 2 + px) {
            const float v = __builtin_bit_cast(
                float, __builtin_amdgcn_raw_buffer_load_b32(rs, off[iy][ix] + (TB[ph] + iy * (2 + px) + ix) * 256, 0, 0));
            acc[ph] = __fadd_rn(acc[ph], v);
          }
        }
      }
    const float b = a.bias[type > 0 ? 1 : 0];
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) outv[type][ph] = clip01(leaky02(__fadd_rn(acc[ph], b)));
  }
  d8_store_rgb(a, n, my, mx, outv);
}


// ------------------------------------------------------------------------------------
// Histogram entropy (tf1_13/src/training.py:66-71) and bitstream pack/unpack
// (utils.py:35-40).
// ------------------------------------------------------------------------------------
// One block reads a contiguous byte range of one image's latent (h, w, 96) with 16-B loads
// (every pixel = 6 vectors: vectors 0-1 Y, 2-3 Cb, 4-5 Cr) and counts all three planes
// into LDS histograms replicated R times, replica-minor ([plane][bin][r], r = lane % R),
// so lanes that hit the same bin (skewed latents: ~40 % zeros) spread over R banks.  Each
// block writes its 3 x 256 partial counts (no atomics, no memset); hist_entropy_kernel
// reduces them.  HBM-bound: 1 B read per code.
constexpr int HIST_UNR_DEFAULT = 4;  // 16-B loads in flight per thread
template <int R, bool ZB, int NT, int HIST_UNR = HIST_UNR_DEFAULT>
__global__ __launch_bounds__(NT) void latent_hist_kernel(const uint8_t* __restrict__ z, int nimg, int plane_px,
                                                          uint32_t* __restrict__ counts, int chunk_vec) {
  __shared__ uint32_t h[3 * 256 * R];
  for (int i = threadIdx.x; i < 3 * 256 * R; i += NT) h[i] = 0;
  __syncthreads();
  const int n = blockIdx.y;
  const int nvec = plane_px * 6;
  const u32x4* __restrict__ base = (const u32x4*)(z + (size_t)n * plane_px * 96);
  const int v0 = blockIdx.x * chunk_vec;
  const int v1 = min(v0 + chunk_vec, nvec);
  const int lane = threadIdx.x & 63;
  uint32_t* hr = h + (threadIdx.x & (R - 1));
  uint32_t zeros[3] = {0, 0, 0};  // ZB: per-lane count of code 0, per plane
  for (int v = v0 + threadIdx.x; v < v1; v += NT * HIST_UNR) {
    u32x4 q[HIST_UNR];
#pragma unroll
    for (int u = 0; u < HIST_UNR; ++u)
      q[u] = v + u * NT < v1 ? __builtin_nontemporal_load(base + v + u * NT) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < HIST_UNR; ++u) {
      if (v + u * NT >= v1) break;
      const int plane = ((v + u * NT) % 6) >> 1;
      uint32_t* hp = hr + plane * (256 * R);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t w = q[u][k];
#pragma unroll
        for (int by = 0; by < 4; ++by) {
          const uint32_t b = (w >> (8 * by)) & 255;
          if (ZB) {
            if (b == 0) {
              zeros[0] += plane == 0;
              zeros[1] += plane == 1;
              zeros[2] += plane == 2;
            } else {
              atomicAdd(&hp[b * R], 1u);
            }
          } else {
            atomicAdd(&hp[b * R], 1u);
          }
        }
      }
    }
  }
  if (ZB) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      uint32_t c = zeros[pl];
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
      if (lane == 0 && c) atomicAdd(&h[pl * 256 * R], c);
    }
  }
  __syncthreads();
  // partial counts of this block: part[type][n][chunk][bin] (reduced by hist_entropy_kernel)
  for (int i = threadIdx.x; i < 3 * 256; i += NT) {
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) c += h[i * R + r];
    const int type = i >> 8, bin = i & 255;
    counts[(((size_t)type * nimg + n) * gridDim.x + blockIdx.x) * 256 + bin] = c;
  }
}

// Plane p's entropy from its 256 counts (thread `bin` < 256 holds count c; threads 0-255 are
// waves 0-3): p_i = c_i / N (fp32), term = p_i * (-log(clip(p_i, 1e-5, 1)) / log 2), summed in
// double in a fixed order (64-lane butterflies, then the 4 waves) -- shared by both reduces so
// their bits agree exactly.  Ends with a block barrier; thread 0 writes bits[p].
__device__ __forceinline__ void plane_entropy(uint32_t c, int bin, int p, float n_sym, uint32_t* __restrict__ counts,
                                              float* __restrict__ bits, double* red) {
  double s = 0.0;
  if (bin < 256) {
    if (counts) counts[(size_t)p * 256 + bin] = c;
    const float pr = __fdiv_rn((float)c, n_sym);
    const float lg = logf(fminf(fmaxf(pr, 1e-5f), 1.0f));
    s = (double)__fmul_rn(pr, __fdiv_rn(-lg, 0.693147182464599609375f));
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((bin & 63) == 0) red[bin >> 6] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0 && bits) bits[p] = (float)(((red[0] + red[1]) + red[2]) + red[3]);
}

__global__ __launch_bounds__(1024) void hist_entropy_kernel(const uint32_t* __restrict__ part, int chunks, float n_sym,
                                                            uint32_t* __restrict__ counts, float* __restrict__ bits) {
  // one block per plane p; thread (g, q) sums bins 4q..4q+3 (one 16-B load) of every 16th
  // partial of the plane (exact integers, 16 loads in flight: one round covers 256 partials),
  // the 16 groups meet in LDS; then plane_entropy
  __shared__ u32x4 grp[16][64];
  __shared__ double red[4];
  const int p = blockIdx.x;
  const int q = threadIdx.x & 63, g = threadIdx.x >> 6;
  const u32x4* src = (const u32x4*)(part + (size_t)p * chunks * 256) + q;
  u32x4 acc[4] = {};
  for (int k0 = g; k0 < chunks; k0 += 256) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int k = k0 + 16 * u;
      acc[u & 3] += k < chunks ? src[(size_t)k * 64] : u32x4{0, 0, 0, 0};
    }
  }
  grp[g][q] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  const int bin = threadIdx.x;
  uint32_t c = 0;
  if (bin < 256) {
#pragma unroll
    for (int j = 0; j < 16; ++j) c += ((const uint32_t*)grp[j])[bin];
  }
  plane_entropy(c, bin, p, n_sym, counts, bits, red);
}

// The folded histogram's reduce: conv8's blocks added their partial counts into acc (device-
// scope atomics, one per non-zero bin per block and plane); one 256-thread block per plane
// reads its 256 counts, clears them for the next call and computes the plane's entropy.
// (Partial rows per block reduced here instead -- 85-171 x 1 KB per plane -- took 23 us, as
// long as the two-call histogram.)  A tripped range guard: the latent was rewritten by the
// exact-fp32 re-run after conv8 counted, so the plane is recounted from z.
__global__ __launch_bounds__(256) void hist_fold_kernel(uint32_t* __restrict__ acc, int nimg,
                                                        const uint8_t* __restrict__ z, int plane_px, RangeGuard trip,
                                                        float n_sym, uint32_t* __restrict__ counts,
                                                        float* __restrict__ bits) {
  __shared__ uint32_t h[256];
  __shared__ double red[4];
  const int p = blockIdx.x, bin = threadIdx.x;
  const bool tripped = trip.flag && *(volatile const int*)trip.flag == trip.epoch;
  uint32_t c = acc[(size_t)p * 256 + bin];
  acc[(size_t)p * 256 + bin] = 0u;  // ready for the next fold
  if (tripped) {
    h[bin] = 0;
    __syncthreads();
    const int n = p % nimg, type = p / nimg;
    const uint8_t* src = z + (size_t)n * plane_px * 96 + type * 32;
    for (long long i = bin; i < (long long)plane_px * 8; i += 256) {
      const uint32_t w = *(const uint32_t*)(src + (i >> 3) * 96 + (i & 7) * 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) atomicAdd(&h[(w >> (8 * k)) & 255], 1u);
    }
    __syncthreads();
    c = h[bin];
  }
  plane_entropy(c, bin, p, n_sym, counts, bits, red);
}

__global__ __launch_bounds__(256) void pack_latent_kernel(const uint8_t* __restrict__ z, uint8_t* __restrict__ out,
                                                          size_t plane_elems, int nimg) {
  // packed[n][f / (8w)][f % (8w)][p] = z[n][(f/32) / w][(f/32) % w][32p + f % 32],
  // i.e. flat index f of plane p in (n, 4h, 8w) equals flat index f of (n, h, w, 32).
  const size_t total = (size_t)nimg * plane_elems;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t n = i / plane_elems, f = i - n * plane_elems;
    const size_t src = n * plane_elems * 3 + (f >> 5) * 96 + (f & 31);
    uint8_t* dst = out + (n * plane_elems + f) * 3;
    dst[0] = z[src];
    dst[1] = z[src + 32];
    dst[2] = z[src + 64];
  }
}

__global__ __launch_bounds__(256) void unpack_latent_kernel(const uint8_t* __restrict__ img, uint8_t* __restrict__ z,
                                                            size_t plane_elems, int nimg) {
  const size_t total = (size_t)nimg * plane_elems;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t n = i / plane_elems, f = i - n * plane_elems;
    const size_t dst = n * plane_elems * 3 + (f >> 5) * 96 + (f & 31);
    const uint8_t* src = img + (n * plane_elems + f) * 3;
    z[dst] = src[0];
    z[dst + 32] = src[1];
    z[dst + 64] = src[2];
  }
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
// Grid of a grid-stride fp32 kernel: 8 blocks per CU, but one per CU for the gated re-run of
// the range-guard fallback, which exits at once unless its pass tripped (the usual case: a
// smaller grid drains faster; a tripped pass re-runs on fewer, longer-lived blocks)
// ------------------------------------------------------------------------------------
// The gated exact-fp32 re-run of a split-f16 pass as ONE launch: every stage of the pass
// (conv1 / conv_mfma layers / dconv8) in sequence.  When the split pass stayed in range every
// block exits at the gate, so the pass costs one dispatch instead of one per layer (each
// dispatch, even of an empty kernel, holds the queue for ~5 us: measured 4.7-5.3 us for 1 to
// 256 blocks).
//
// No grid barrier, so no co-residency requirement: the tiles of stage s are handed out by a
// queue word (chain_take); a block that has run its share adds its tile count to the stage's
// done word (release) and, before taking tiles of stage s+1, waits for done == the stage's
// tile total (acquire).  Every tile taken is held by a running block that never waits while it
// holds one, so the totals are always reached: blocks that start late (other streams' kernels
// on the CUs, a grid larger than fits) find the queues drained and pass through.  The last
// block to leave zeroes the words for the next chain on the ctx (stream-ordered).
// ------------------------------------------------------------------------------------
template <class... Gs>
constexpr int max_lds_floats() {
  int m = 0;
  ((m = Gs::LDS_FLOATS > m ? Gs::LDS_FLOATS : m), ...);
  return m;
}
using G_c2 = ConvGeom<32, 64, 5, 2, false, 8, 8, 2, 2, 1>;
using G_k3 = ConvGeom<64, 64, 3, 1, false, 8, 16, 4, 1, 1>;
using G_c8 = ConvGeom<64, 32, 5, 2, false, 4, 8, 1, 1, 4>;
using G_d1 = ConvGeom<32, 64, 5, 2, true, 8, 8, 2, 2, 1>;
using G_d7 = ConvGeom<64, 64, 5, 2, true, 8, 16, 4, 1, 1>;
constexpr int kChainLds = std::max({max_lds_floats<G_c2, G_k3, G_c8, G_d1, G_d7>(), C1_LDS_FLOATS, D8_LDS_FLOATS});

// stage s's words: q[s] = next tile, q[kChainMax + s] = tiles done, q[2 kChainMax] = blocks out
__device__ __forceinline__ void chain_stage_done(int* done, int ran) {
  __syncthreads();  // every wave's stores of the stage are issued and waited for
  if (threadIdx.x == 0) {
    __threadfence();  // release them device-wide (every XCD)
    if (ran) atomicAdd(done, ran);
  }
}
__device__ __forceinline__ void chain_stage_wait(const int* done, int total) {
  if (threadIdx.x == 0) {
    while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < total) __builtin_amdgcn_s_sleep(2);
    __threadfence();  // acquire the other blocks' stage outputs
  }
  __syncthreads();
}

__global__ __launch_bounds__(256, 2) void fp32_chain_kernel(Fp32Chain ch) {
  KT_SCOPE(4);
  __shared__ __attribute__((aligned(16))) float lds[kChainLds];
  if (range_gated_off(ch.gate)) return;  // whole grid: the gate word is the same for every block
  const int b0 = blockIdx.x, nb = gridDim.x;
  int* q = ch.q;
  if (ch.diag_late && b0 == 0) {  // diagnostic: block 0 starts ~1 ms late
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100000ull) __builtin_amdgcn_s_sleep(8);
  }
  for (int s = 0; s < ch.nstage; ++s) {
    if (s > 0) chain_stage_wait(q + kChainMax + s - 1, ch.total[s - 1]);
    const ConvArgs& a = ch.c[s];
    int* qs = q + s;
    int ran = 0;
    switch (ch.kind[s]) {
      case L_CONV1: ran = conv1_colour_body(ch.c1, lds, b0, nb, qs); break;
      case L_DCONV8: ran = dconv8_colour_body<1>(ch.d8, lds, b0, nb, qs); break;
      case L_CONV2: ran = conv_mfma_body<32, 64, 5, 2, false, 8, 8, 2, 2, 1, IN_F32, OUT_F32, false>(a, lds, b0, nb, qs); break;
      case L_CONV3:
      case L_DCONV5: ran = conv_mfma_body<64, 64, 3, 1, false, 8, 16, 4, 1, 1, IN_F32, OUT_F32, false>(a, lds, b0, nb, qs); break;
      case L_CONV4:
      case L_DCONV6: ran = conv_mfma_body<64, 64, 3, 1, false, 8, 16, 4, 1, 1, IN_F32, OUT_F32, true>(a, lds, b0, nb, qs); break;
      case L_CONV8: ran = conv_mfma_body<64, 32, 5, 2, false, 4, 8, 1, 1, 4, IN_F32, OUT_U8_LATENT, false>(a, lds, b0, nb, qs); break;
      case L_DCONV1: ran = conv_mfma_body<32, 64, 5, 2, true, 8, 8, 2, 2, 1, IN_U8_LATENT, OUT_F32, false>(a, lds, b0, nb, qs); break;
      case L_DCONV7: ran = conv_mfma_body<64, 64, 5, 2, true, 8, 16, 4, 1, 1, IN_F32, OUT_F32, false>(a, lds, b0, nb, qs); break;
      default: break;
    }
    chain_stage_done(q + kChainMax + s, ran);
  }
  if (threadIdx.x == 0 && atomicAdd(q + 2 * kChainMax, 1) == nb - 1) {  // the last block out: reset
    for (int s = 0; s < ch.nstage; ++s) {
      __hip_atomic_store(q + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(q + kChainMax + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(q + 2 * kChainMax, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static void conv_tiles(LayerId id, ConvArgs& a) {  // launch_conv's tile grid for layer id
  const bool tr = id == L_DCONV1 || id == L_DCONV7;
  int th = 8, tw = 16;
  if (id == L_CONV2 || id == L_DCONV1) tw = 8;
  if (id == L_CONV8) th = 4, tw = 8;
  const int gy = tr ? a.H : a.OH, gx = tr ? a.W : a.OW;
  a.tiles_y = (gy + th - 1) / th;
  a.tiles_x = (gx + tw - 1) / tw;
}

hipError_t chain_add_layer(Fp32Chain& ch, LayerId id, ConvArgs a) {
  if (ch.nstage >= kChainMax || id == L_CONV1 || id == L_DCONV8 || id >= L_COUNT) return hipErrorInvalidValue;
  conv_tiles(id, a);
  // < INT32_MAX - grid: the queue word counts past the total by at most one take per block
  if ((long long)a.tiles_y * a.tiles_x * a.P > INT32_MAX / 2) return hipErrorInvalidValue;
  ch.total[ch.nstage] = a.tiles_y * a.tiles_x * a.P;
  ch.kind[ch.nstage] = id;
  ch.c[ch.nstage++] = a;
  return hipSuccess;
}

hipError_t chain_add_conv1(Fp32Chain& ch, Conv1Args a) {
  if (ch.nstage >= kChainMax) return hipErrorInvalidValue;
  a.tiles_y = (a.OH + C1_T - 1) / C1_T;
  a.tiles_x = (a.OW + C1_T - 1) / C1_T;
  if ((long long)a.tiles_y * a.tiles_x * a.P > INT32_MAX / 2) return hipErrorInvalidValue;
  ch.total[ch.nstage] = a.tiles_y * a.tiles_x * a.P;
  ch.kind[ch.nstage++] = L_CONV1;
  ch.c1 = a;
  return hipSuccess;
}

hipError_t chain_add_dconv8(Fp32Chain& ch, Dconv8Args a) {
  if (ch.nstage >= kChainMax) return hipErrorInvalidValue;
  a.tiles_y = (a.H + D8_TH - 1) / D8_TH;
  a.tiles_x = (a.W + D8_TW - 1) / D8_TW;
  if ((long long)a.tiles_y * a.tiles_x * a.nimg > INT32_MAX / 2) return hipErrorInvalidValue;
  ch.total[ch.nstage] = a.tiles_y * a.tiles_x * a.nimg;
  ch.kind[ch.nstage++] = L_DCONV8;
  ch.d8 = a;
  return hipSuccess;
}

// Blocks of fp32_chain_kernel resident per CU (its LDS / VGPRs), per device (informational:
// the queued chain runs on any number of resident blocks).
static int chain_occupancy() {
  static int cache[64] = {};
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return 0;
  if (!cache[d]) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fp32_chain_kernel, 256, 0) != hipSuccess) n = 0;
    cache[d] = n > 0 ? n : -1;
  }
  return cache[d];
}

// NIC_DIAG_CHAIN=N (GPU test only): the chain's grid is N blocks per CU -- far more than fit at
// once, so most blocks start only after others have left -- and block 0 starts ~1 ms late
static int chain_diag_grid() {
  static const int v = [] {
    const char* e = getenv("NIC_DIAG_CHAIN");
    return e ? std::max(1, std::min(64, atoi(e))) : 0;
  }();
  return v;
}

void fp32_chain_launch_info(int* blocks_per_cu, int* grid, int* cooperative) {
  *blocks_per_cu = chain_occupancy();
  *grid = device_cus() * std::max(1, chain_diag_grid());
  *cooperative = 0;
}

hipError_t launch_fp32_chain(const Fp32Chain& chain, hipStream_t st) {
  if (chain.nstage == 0) return hipSuccess;
  if (!chain.q || !chain.gate.gate) return hipErrorInvalidValue;
  if (chain_occupancy() < 1) return hipErrorInvalidConfiguration;
  Fp32Chain ch = chain;
  const int diag = chain_diag_grid();
  ch.diag_late = diag ? 1 : 0;
  // one 256-thread block per CU; nothing requires them resident together
  hipLaunchKernelGGL(fp32_chain_kernel, dim3(device_cus() * std::max(1, diag)), dim3(256), 0, st, ch);
  return hipGetLastError();
}

// grid of the fp32 one-tile-per-block launches: 8 blocks per CU, 1 for a gated re-run (NIC_CHAIN=0),
// which exits at its gate unless the split pass tripped (a smaller grid drains faster)
static int fp32_grid(const RangeGuard& rg, long long jobs) {
  return (int)std::min<long long>(jobs, (long long)(rg.gate ? 1 : 8) * device_cus());
}

template <int CIN, int COUT, int KS, int S, bool TR, int TH, int TW, int WM, int WN, int WK, int IN_MODE,
          int OUT_MODE, bool RESID>
static hipError_t launch_conv(ConvArgs a, hipStream_t st) {
  const int gy = TR ? a.H : a.OH, gx = TR ? a.W : a.OW;  // tile grid over coarse / output coords
  a.tiles_y = (gy + TH - 1) / TH;
  a.tiles_x = (gx + TW - 1) / TW;
  const long long jobs = (long long)a.tiles_y * a.tiles_x * a.P;
  if (jobs == 0) return hipSuccess;
  if (jobs > INT32_MAX) return hipErrorInvalidValue;
  const int grid = fp32_grid(a.rg, jobs);
  hipLaunchKernelGGL((conv_mfma_kernel<CIN, COUT, KS, S, TR, TH, TW, WM, WN, WK, IN_MODE, OUT_MODE, RESID>),
                     dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t upload_constants(const float* u8_to_unit, const float* ycbcr, const float* ycbcr_inv, const float* off) {
  hipError_t e;
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_u8_to_unit), u8_to_unit, 256 * sizeof(float))) != hipSuccess) return e;
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_ycbcr), ycbcr, 9 * sizeof(float))) != hipSuccess) return e;
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_ycbcr_inv), ycbcr_inv, 9 * sizeof(float))) != hipSuccess) return e;
  return hipMemcpyToSymbol(HIP_SYMBOL(c_ycbcr_off), off, 3 * sizeof(float));
}

hipError_t launch_layer(LayerId id, const ConvArgs& a, hipStream_t st) {
  switch (id) {
    // encoder (conv1 has its own kernel)
    case L_CONV2:  // 32->64 k5 s2: 8x8 tile, 4 waves = 2(M) x 2(N)
      return launch_conv<32, 64, 5, 2, false, 8, 8, 2, 2, 1, IN_F32, OUT_F32, false>(a, st);
    case L_CONV3:  // 64->64 k3 s1: 8x16 tile, 4 waves along M, each 32 px x 64 co
      return launch_conv<64, 64, 3, 1, false, 8, 16, 4, 1, 1, IN_F32, OUT_F32, false>(a, st);
    case L_CONV4:  // + residual
      return launch_conv<64, 64, 3, 1, false, 8, 16, 4, 1, 1, IN_F32, OUT_F32, true>(a, st);
    case L_CONV8:  // 64->32 k5 s2 -> u8 latent: 4x8 tile, taps split over the 4 waves
      return launch_conv<64, 32, 5, 2, false, 4, 8, 1, 1, 4, IN_F32, OUT_U8_LATENT, false>(a, st);
    // decoder (dconv8 has its own kernel)
    case L_DCONV1:  // latent u8 -> 64, transposed k5 s2: 8x8 coarse tile, 2(M) x 2(N)
      return launch_conv<32, 64, 5, 2, true, 8, 8, 2, 2, 1, IN_U8_LATENT, OUT_F32, false>(a, st);
    case L_DCONV5:  // transposed k3 s1 == conv k3 s1 with flipped kernel
      return launch_conv<64, 64, 3, 1, false, 8, 16, 4, 1, 1, IN_F32, OUT_F32, false>(a, st);
    case L_DCONV6:
      return launch_conv<64, 64, 3, 1, false, 8, 16, 4, 1, 1, IN_F32, OUT_F32, true>(a, st);
    case L_DCONV7:  // 64->64 transposed k5 s2: 8x16 coarse tile, 4 waves along M
      return launch_conv<64, 64, 5, 2, true, 8, 16, 4, 1, 1, IN_F32, OUT_F32, false>(a, st);
    default:
      return hipErrorInvalidValue;
  }
}


static int device_cus() {
  static int cache[64] = {};
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return 256;
  if (!cache[d]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n <= 0) n = 256;
    cache[d] = n;
  }
  return cache[d];
}

// Weight-stationary launch: 2 resident blocks per CU, split into groups (tap set, model)
// in proportion to each group's MFMA work (planes x taps).
template <int CIN, int COUT, int TH, int TW, bool RESID, bool TRP, bool PROJ = false>
static hipError_t launch_ws(ConvArgs a, hipStream_t st) {
  a.tiles_y = (a.H + TH - 1) / TH;
  a.tiles_x = (a.W + TW - 1) / TW;
  const long long per_plane = (long long)a.tiles_y * a.tiles_x;
  const long long nt = per_plane * a.P;
  if (nt == 0) return hipSuccess;
  if (nt > INT32_MAX || a.P != 3 * a.nimg) return hipErrorInvalidValue;
  // HaloDma: 32-bit plane offsets, out-of-range slots past the plane (kDmaOOR)
  if ((long long)a.H * a.W * CIN * 4 >= (1LL << 30)) return hipErrorInvalidValue;
  a.ntiles = (int)nt;
  // one block group per model (transposed layers: every block runs the four phases over its
  // tiles; per-phase groups measured 6 % slower)
  a.ws_taps = TRP ? 25 : 9;
  a.ws_ngrp = 2;
  long long work[2], total = 0;
  for (int gi = 0; gi < 2; ++gi) {
    work[gi] = ((gi & 1) ? a.P - a.nimg : a.nimg) * per_plane;
    total += work[gi];
  }
  const int target = 2 * device_cus();  // 2 resident blocks per CU
  a.ws_blk[0] = 0;
  for (int gi = 0; gi < a.ws_ngrp; ++gi) {
    const long long tiles = ((gi & 1) ? a.P - a.nimg : a.nimg) * per_plane;
    long long b = (work[gi] * target + total / 2) / total;
    b = b < 1 ? 1 : b > tiles ? tiles : b;
    a.ws_blk[gi + 1] = a.ws_blk[gi] + (int)b;
  }
  a.ws_xcd = 1;
  hipLaunchKernelGGL((conv_ws_kernel<CIN, COUT, TH, TW, RESID, TRP, PROJ>), dim3(a.ws_blk[a.ws_ngrp]),
                     dim3(64 * (COUT / 16)), 0, st, a);
  return hipGetLastError();
}

// Block row ranges of the fused pair by pipeline steps.  A block pays ~3 fill steps per segment
// (the part of its range inside one (plane, strip) column of H rows) on top of one step per row:
// equal-row ranges give the blocks that straddle a plane boundary 2 segments (config 2: 48 rows
// = 54 steps against 51 for a one-segment block).  Greedy ranges under a step budget T, the
// smallest T that fits the grid (binary search), even that out.  F = the per-segment cost the
// budget charges, in steps (2: pair 0.2379-0.2385 ms vs 0.2388-0.2402 at 3, 0.2392-0.2404 at 4
// and 0.2415-0.2423 for the equal-rows split; same box, profiles/r4_ab_logs.txt).
static void k3pair_balance(long long total, int H, int G, K3Ranges& r) {
  constexpr int F = 2;
  if (G <= 0 || G > K3P_MAX_GRID || total >= (1LL << 31) || H <= 0) return;
  // blocks the greedy needs under budget T (stops counting past G); fills r when `write`
  auto fill = [&](long long T, bool write) {
    long long s = 0;
    int b = 0;
    while (s < total) {
      if (b == G) return G + 1;
      if (write) r.start[b] = (int)s;
      ++b;
      long long budget = T;
      while (s < total && budget > F) {
        const long long left = H - s % H, take = std::min(left, budget - F);
        s += take;
        budget -= take + F;
        if (take < left) break;
      }
    }
    if (write)
      for (int k = b; k <= G; ++k) r.start[k] = (int)total;
    return b;
  };
  const long long per = (total + G - 1) / G;
  long long lo = F + 1, hi = per + F * (per / H + 2);  // the equal split fits hi
  if (fill(hi, false) > G) return;
  while (lo < hi) {
    const long long mid = (lo + hi) / 2;
    if (fill(mid, false) <= G)
      hi = mid;
    else
      lo = mid + 1;
  }
  fill(hi, true);
}

hipError_t launch_k3pair_x3(const ConvArgs& a0, hipStream_t st) {
  ConvArgs a = a0;
  if (!k3pair_supported(a.H, a.W) || a.OH != a.H || a.OW != a.W || !a.wx2 || !a.bias2 || a.P != 3 * a.nimg)
    return hipErrorInvalidValue;
  a.tiles_x = k3pair_strips(a.W);
  const long long rows = (long long)a.P * a.tiles_x * a.H;
  if (rows == 0) return hipSuccess;
  // at most one block per CU, at least 4 rows per block: a block's fixed cost is 3 pipeline fill
  // steps and 2 recomputed conv_a rows, so small batches (the host surface's chunks: 11-21
  // images) are faster spread over every CU with few rows each than on fewer CUs with more (16
  // rows per block left 124 of 256 CUs idle at 11 images)
  constexpr int sr = 4;
  const int grid = (int)std::max(1LL, std::min<long long>((rows + sr - 1) / sr, device_cus()));
  const int mt = (a.W + 15) / 16;
  // SKEW: conv_b runs each row's epilogue at the start of the next step, beside conv_a's MFMA
  // stream, instead of after its own stream (the lockstep order measured 1.3 % slower)
  K3Ranges rng;
  rng.start[0] = -1;
  k3pair_balance(rows, a.H, grid, rng);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, st, a, rng); };
  auto pick = [&](auto skc) {
    constexpr bool SK = decltype(skc)::value;
    if (a.tiles_x > 1) {
      go(conv_k3pair_kernel<4, SK, true>);
    } else {
      switch (mt) {
        case 1: go(conv_k3pair_kernel<1, SK, false>); break;
        case 2: go(conv_k3pair_kernel<2, SK, false>); break;
        case 3: go(conv_k3pair_kernel<3, SK, false>); break;
        default: go(conv_k3pair_kernel<4, SK, false>); break;
      }
    }
  };
  pick(std::true_type{});
  return hipGetLastError();
}

// k5 s2 forward convs: one 8-wave block per CU, split into a Y and a CbCr group in
// proportion to their planes.
static void ws2_groups(int nimg, long long per_plane, int* by, int* bc) {
  const int target = device_cus();
  const long long ty = per_plane * nimg, tc = per_plane * 2 * nimg;
  long long y = std::max(1LL, std::min((long long)(target + 1) / 3, ty));
  *by = (int)y;
  *bc = (int)std::max(1LL, std::min((long long)target - y, tc));
}

// conv8's tile grid (4 x 8 output tiles) and the fold's condition: every block meets each plane
// of its group in >= 2 consecutive tiles (group blocks <= tiles per plane / 2) -- large frames
// (config 5); batches of small images run the two-call form
bool hist_fold_supported(int nimg, int h8, int w8) {
  if (nimg <= 0 || h8 <= 0 || w8 <= 0) return false;
  const long long pp = (long long)((h8 + 3) / 4) * ((w8 + 7) / 8);
  int by, bc;
  ws2_groups(nimg, pp, &by, &bc);
  return 2LL * by <= pp && 2LL * bc <= pp;
}

size_t hist_fold_scratch_bytes(int nimg, int h8, int w8) {  // the counts [3 nimg][256]
  (void)h8;
  (void)w8;
  return (size_t)3 * nimg * 256 * sizeof(uint32_t);
}

// k5 s2 forward convs on the tap-split weight-stationary kernel (conv2 of conv12 with PIPE12,
// conv8 with the latent histogram fold when a.hist_part is set)
template <int CIN, int COUT, int NTS, int TH, int OUT_MODE, bool PIPE12 = false>
static hipError_t launch_ws2(ConvArgs a, hipStream_t st) {
  a.tiles_y = (a.OH + TH - 1) / TH;
  a.tiles_x = (a.OW + 7) / 8;
  const long long per_plane = (long long)a.tiles_y * a.tiles_x;
  const long long nt = per_plane * a.P;
  if (nt == 0) return hipSuccess;
  if (nt > INT32_MAX || a.P != 3 * a.nimg) return hipErrorInvalidValue;
  a.ntiles = (int)nt;
  a.ws_taps = 25;
  a.ws_ngrp = 2;
  int by, bc;
  ws2_groups(a.nimg, per_plane, &by, &bc);
  a.ws_blk[0] = 0;
  a.ws_blk[1] = by;
  a.ws_blk[2] = by + bc;
  if constexpr (PIPE12) {
    hipLaunchKernelGGL(conv12_kernel, dim3(a.ws_blk[2]), dim3(512), 0, st, a);
  } else if constexpr (OUT_MODE == OUT_U8_LATENT) {
    if (a.hist_part) {
      if (!hist_fold_supported(a.nimg, a.OH, a.OW)) return hipErrorInvalidValue;
      hipLaunchKernelGGL((conv_ws2_kernel<CIN, COUT, NTS, TH, OUT_MODE, true>), dim3(a.ws_blk[2]), dim3(512), 0, st, a);
    } else {
      hipLaunchKernelGGL((conv_ws2_kernel<CIN, COUT, NTS, TH, OUT_MODE>), dim3(a.ws_blk[2]), dim3(512), 0, st, a);
    }
  } else {
    hipLaunchKernelGGL((conv_ws2_kernel<CIN, COUT, NTS, TH, OUT_MODE>), dim3(a.ws_blk[2]), dim3(512), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t launch_conv12_x3(const ConvArgs& a0, hipStream_t st) {
  ConvArgs a = a0;
  if (!a.rgb || !a.wx1 || !a.bias1 || a.H0 <= 0 || a.W0 <= 0) return hipErrorInvalidValue;
  if (!a.cplane || a.OH <= 0 || a.OW <= 0) return hipErrorInvalidValue;
  int oy, ox;
  c12_plane_geom(a.OH, a.OW, a.pad_y, a.pad_x, a.p1y, a.p1x, &oy, &ox, &a.cp_h, &a.cp_w);
  // 32-bit byte offsets inside one plane (buffer resources of the patch DMA)
  if ((long long)a.cp_h * a.cp_w * 2 >= (1LL << 31)) return hipErrorInvalidValue;
  const long long per_img = (long long)a.cp_h * (a.cp_w / 4);  // < 2^31 (checked above)
  if (per_img == 0 || a.nimg == 0) return hipSuccess;
  if (a.nimg > 65535 || (long long)a.W0 * 3 >= (1LL << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(colour_split_kernel, dim3((unsigned)((per_img + 255) / 256), a.nimg),
                     dim3(256), 0, st, a.rgb, a.cplane, a.nimg, a.H0, a.W0, oy, ox, a.cp_h, a.cp_w);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_ws2<32, 64, 2, 8, OUT_SPLIT, true>(a, st);
}

// all phases per staged tile: one 8-wave block per CU, blocks split between the models in
// proportion to their tiles (Y : CbCr = 1 : 2)
static hipError_t launch_dconv1_all(ConvArgs a, hipStream_t st) {
  a.tiles_y = (a.H + 7) / 8;
  a.tiles_x = (a.W + 7) / 8;
  const long long per_plane = (long long)a.tiles_y * a.tiles_x, nt = per_plane * a.P;
  if (nt == 0) return hipSuccess;
  if (nt > INT32_MAX || a.P != 3 * a.nimg || a.OH != 2 * a.H || a.OW != 2 * a.W || !a.in_u8) return hipErrorInvalidValue;
  if ((long long)a.OH * a.OW * 256 >= (1LL << 31)) return hipErrorInvalidValue;  // 32-bit granule offsets
  const long long target = device_cus();
  const long long ty = (long long)a.nimg * per_plane, tc = 2LL * a.nimg * per_plane;
  const int by = (int)std::max(1LL, std::min(ty, (target + 1) / 3)), bc = (int)std::max(1LL, std::min(tc, target - by));
  a.ws_ngrp = 2;
  a.ws_blk[0] = 0;
  a.ws_blk[1] = by;
  a.ws_blk[2] = by + bc;
  hipLaunchKernelGGL(dconv1_all_kernel, dim3(a.ws_blk[2]), dim3(512), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_layer_x3(LayerId id, const ConvArgs& a, hipStream_t st) {
  switch (id) {
    case L_CONV2:  // 32->64 k5 s2 (conv12_kernel runs it fused with conv1; this form is unused there)
      return launch_ws2<32, 64, 2, 8, OUT_SPLIT>(a, st);
    case L_CONV3:  // 64->64 k3 s1 weight-stationary (the fused pair takes planes it supports)
    case L_DCONV5:
      return launch_ws<64, 64, 8, 8, false, false>(a, st);
    case L_CONV4:
    case L_DCONV6:
      return launch_ws<64, 64, 8, 8, true, false>(a, st);
    case L_CONV8:  // 64->32 k5 s2 -> latent: tap-split weight-stationary (2 channel groups x 4 tap
                   // quarters, 4x8 tiles)
      return launch_ws2<64, 32, 4, 4, OUT_U8_LATENT>(a, st);
    case L_DCONV1:  // latent -> 64, transposed k5 s2: all four phases per staged 8x8 code tile
      return launch_dconv1_all(a, st);
    default:  // dconv7 runs with dconv8's projections (launch_dconv7_proj_x3)
      return hipErrorInvalidValue;
  }
}

hipError_t launch_dconv7_proj_x3(const ConvArgs& a, hipStream_t st) {
  if (!a.proj || !a.proj_w || a.OH != 2 * a.H || a.OW != 2 * a.W) return hipErrorInvalidValue;
  return launch_ws<64, 64, 8, 8, false, true, true>(a, st);
}

hipError_t launch_conv1(Conv1Args a, hipStream_t st) {
  a.tiles_y = (a.OH + C1_T - 1) / C1_T;
  a.tiles_x = (a.OW + C1_T - 1) / C1_T;
  const long long jobs = (long long)a.tiles_y * a.tiles_x * a.P;
  if (jobs == 0) return hipSuccess;
  if (jobs > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv1_colour_kernel, dim3(fp32_grid(a.rg, jobs)), dim3(256), 0,
                     st, a);
  return hipGetLastError();
}

hipError_t launch_dconv8(Dconv8Args a, hipStream_t st) {
  a.tiles_y = (a.H + D8_TH - 1) / D8_TH;
  a.tiles_x = (a.W + D8_TW - 1) / D8_TW;
  const long long jobs = (long long)a.tiles_y * a.tiles_x * a.nimg;
  if (jobs == 0) return hipSuccess;
  if (jobs > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dconv8_colour_kernel, dim3(fp32_grid(a.rg, jobs)), dim3(256), 0,
                     st, a);
  return hipGetLastError();
}

hipError_t launch_dconv8_gather(Dconv8Args a, hipStream_t st) {
  if (!a.proj || (a.H & 1) || (a.W & 1)) return hipErrorInvalidValue;
  if (a.tiles_y7 != (a.H / 2 + 7) / 8 || a.tiles_x7 != (a.W / 2 + 7) / 8) return hipErrorInvalidValue;
  const int tiles_y = (a.H + 15) / 16;
  a.tiles_x = (a.W + 15) / 16;
  hipLaunchKernelGGL(dconv8_gather_kernel, dim3(tiles_y * a.tiles_x, a.nimg), dim3(256), 0, st, a);
  return hipGetLastError();
}

int hist_chunks(int nimg, int plane_px, int* chunk_vec, int blocks) {
  // `blocks` over the whole batch (one full wave of blocks, no tail round: 6 resident
  // 256-thread blocks or 2 1024-thread blocks per CU x 256 CUs), 4 KB .. 256 KB of latent each
  const long long nvec = (long long)plane_px * 6;
  long long cv = ((nvec * nimg + blocks - 1) / blocks + 255) / 256 * 256;
  cv = cv < 256 ? 256 : (cv > 16384 ? 16384 : cv);
  *chunk_vec = (int)cv;
  return (int)((nvec + cv - 1) / cv);
}

size_t hist_scratch_bytes(int nimg, int plane_px) {
  int cv;  // sized for the most partials any variant writes
  return (size_t)3 * nimg * hist_chunks(nimg, plane_px, &cv, 1536) * 256 * sizeof(uint32_t);
}

hipError_t launch_hist(const uint8_t* z, int nimg, int plane_px, uint32_t* part, uint32_t* counts, float* bits,
                       hipStream_t st) {
  // 1024-thread blocks, 512 of them (2 per CU) with 16 LDS replicas per bin from 24 MB of latent
  // up, else 256-thread blocks with 8 (>= 48 KB per block: the per-block LDS clear and 768
  // partial stores amortised).  Measured on 4K x 8 latents (tools/hist_ab.py, round 2):
  // 16 replicas 21.6 us, 8 25.4, 32 (98 KB, one block per CU) 27.2; a packed-u16 32-replica
  // layout 15 % slower.  NIC_HIST=big / small forces either form (read per call: the GPU test
  // runs both on one latent).
  const char* hv = getenv("NIC_HIST");
  const int force = !hv ? 0 : hv[0] == 'b' ? 1 : hv[0] == 's' ? 2 : 0;
  const long long total = (long long)plane_px * 96 * nimg;
  const bool big = force ? force == 1 : total >= (24ll << 20);
  int chunk_vec;
  const int chunks = hist_chunks(nimg, plane_px, &chunk_vec, big ? 512 : 1536);
  if (big)
    hipLaunchKernelGGL((latent_hist_kernel<16, false, 1024>), dim3(chunks, nimg), dim3(1024), 0, st, z, nimg, plane_px, part,
                       chunk_vec);
  else
    hipLaunchKernelGGL((latent_hist_kernel<8, false, 256>), dim3(chunks, nimg), dim3(256), 0, st, z, nimg, plane_px, part,
                       chunk_vec);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(hist_entropy_kernel, dim3(3 * nimg), dim3(1024), 0, st, part, chunks, (float)plane_px * 32.0f,
                     counts, bits);
  return hipGetLastError();
}

hipError_t launch_hist_fold(uint32_t* part, const uint8_t* z, int nimg, int h8, int w8, RangeGuard trip,
                            uint32_t* counts, float* bits, hipStream_t st) {
  if (!hist_fold_supported(nimg, h8, w8)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(hist_fold_kernel, dim3(3 * nimg), dim3(256), 0, st, part, nimg, z, h8 * w8, trip,
                     (float)h8 * w8 * 32.0f, counts, bits);
  return hipGetLastError();
}

hipError_t launch_pack(const uint8_t* z, uint8_t* out, int nimg, int h8, int w8, bool unpack, hipStream_t st) {
  const size_t plane_elems = (size_t)h8 * w8 * 32;
  const size_t total = plane_elems * nimg;
  const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  if (unpack)
    hipLaunchKernelGGL(unpack_latent_kernel, dim3(blocks), dim3(256), 0, st, z, out, plane_elems, nimg);
  else
    hipLaunchKernelGGL(pack_latent_kernel, dim3(blocks), dim3(256), 0, st, z, out, plane_elems, nimg);
  return hipGetLastError();
}

}  // namespace nic
