// Quality metrics on the device: MS-SSIM (tf.image.ssim_multiscale, as called by
// tf2_0/tests/calc_ssim.py:13 with max_val=255) and per-image squared error (PSNR).
//
// MS-SSIM per scale k (5 scales): one block per (32x32 output tile, plane) stages the
// 42x42 input window of both images in LDS (shifted by -0.5: covariances are
// shift-invariant and the smaller magnitudes keep more fp32 bits), runs the separable
// 11-tap Gaussian (sigma 1.5) horizontally into 4 LDS maps (x, y, x^2+y^2, x*y) and
// vertically per output pixel, forms luminance * cs and cs and writes the tile's two sums
// (fp64) -- no atomics, so the result is deterministic.  Between scales a 2x2 average
// pool (odd sizes padded SYMMETRIC, i.e. the last row/column repeated) writes planar fp32
// images for the next scale.  A final block per image reduces the tile sums to means,
// relu's them and forms the weighted geometric mean over scales, averaged over channels.
// HBM-bound and tiny next to the codec: scale 0 reads 2 x 3 B per pixel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nic_kernels.h"

namespace nic {

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kSsimTile = 32;                    // output tile edge
constexpr int kSsimTaps = 11;                    // Gaussian window (TF filter_size)
constexpr int kSsimIn = kSsimTile + kSsimTaps - 1;  // 42: input window edge

__constant__ float c_gauss[kSsimTaps];
__constant__ double c_msssim_w[kSsimScales];

__device__ inline float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One (tile, plane) of one scale.  U8: the scale-0 images, u8 NHWC (N,H,W,3); otherwise
// planar fp32 (P,H,W) written by pool_kernel.
template <bool U8>
__global__ __launch_bounds__(256) void ssim_tile_kernel(SsimScaleArgs a) {
  __shared__ float sx[kSsimIn][kSsimIn + 1];
  __shared__ float sy[kSsimIn][kSsimIn + 1];
  __shared__ float hm[4][kSsimIn][kSsimTile];
  __shared__ float red[2][4];
  const int tid = threadIdx.x;
  const int p = blockIdx.y;
  const int tx = blockIdx.x % a.tiles_x, ty = blockIdx.x / a.tiles_x;
  const int y0 = ty * kSsimTile, x0 = tx * kSsimTile;
  const int OH = a.H - kSsimTaps + 1, OW = a.W - kSsimTaps + 1;

  // window load: every element's global load issued before any is used (one latency
  // round per block instead of one per 256 elements)
  constexpr int kLoads = (kSsimIn * kSsimIn + 255) / 256;
  float lx[kLoads], ly[kLoads];
#pragma unroll
  for (int k = 0; k < kLoads; ++k) {
    const int i = tid + 256 * k;
    const int r = i / kSsimIn, c = i % kSsimIn;
    const int y = y0 + r, x = x0 + c;
    lx[k] = 0.f;
    ly[k] = 0.f;
    if (i < kSsimIn * kSsimIn && y < a.H && x < a.W) {
      if constexpr (U8) {
        const int img = p / 3, ch = p % 3;
        const size_t o = ((size_t)(img * a.H + y) * a.W + x) * 3 + ch;
        lx[k] = (float)a.a8[o];
        ly[k] = (float)a.b8[o];
      } else {
        const size_t o = ((size_t)p * a.H + y) * a.W + x;
        lx[k] = a.af[o];
        ly[k] = a.bf[o];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kLoads; ++k) {
    const int i = tid + 256 * k;
    if (i < kSsimIn * kSsimIn) {
      const int r = i / kSsimIn, c = i % kSsimIn;
      const bool in = y0 + r < a.H && x0 + c < a.W;
      // convert_image_dtype: u8 * (1/255) in fp32; shifted by -0.5 (0 outside the image)
      sx[r][c] = in ? (U8 ? lx[k] * (1.0f / 255.0f) : lx[k]) - 0.5f : 0.f;
      sy[r][c] = in ? (U8 ? ly[k] * (1.0f / 255.0f) : ly[k]) - 0.5f : 0.f;
    }
  }
  __syncthreads();

  // horizontal pass: an item is 4 consecutive outputs of one row (register window of 14
  // inputs, the products x^2 + y^2 and xy formed once per input)
  constexpr int kSeg = 4, kSegs = kSsimTile / kSeg;
  for (int i = tid; i < kSsimIn * kSegs; i += 256) {
    const int r = i / kSegs, c0 = (i % kSegs) * kSeg;
    constexpr int kWin = kSeg + kSsimTaps - 1;
    // (x, y) and (x^2 + y^2, xy) pairs: the four sums run as two packed fp32 FMA streams
    f32x2 wxy[kWin], wqp[kWin];
#pragma unroll
    for (int j = 0; j < kWin; ++j) {
      const float vx = sx[r][c0 + j], vy = sy[r][c0 + j];
      wxy[j] = (f32x2){vx, vy};
      wqp[j] = (f32x2){fmaf(vx, vx, vy * vy), vx * vy};
    }
#pragma unroll
    for (int o = 0; o < kSeg; ++o) {
      f32x2 s01 = {0.f, 0.f}, s23 = {0.f, 0.f};
#pragma unroll
      for (int j = 0; j < kSsimTaps; ++j) {
        const f32x2 g = {c_gauss[j], c_gauss[j]};
        s01 = __builtin_elementwise_fma(g, wxy[o + j], s01);
        s23 = __builtin_elementwise_fma(g, wqp[o + j], s23);
      }
      hm[0][r][c0 + o] = s01[0];
      hm[1][r][c0 + o] = s01[1];
      hm[2][r][c0 + o] = s23[0];
      hm[3][r][c0 + o] = s23[1];
    }
  }
  __syncthreads();

  // vertical pass: an item is 4 consecutive rows of one column (window of 14 rows)
  const float c1 = 0.01f * 0.01f, c2 = 0.03f * 0.03f;  // (k1 * max_val)^2, (k2 * max_val)^2, max_val = 1
  float ssum = 0.f, csum = 0.f;
  for (int i = tid; i < kSsimTile * kSegs; i += 256) {
    const int c = i % kSsimTile, r0 = (i / kSsimTile) * kSeg;
    f32x2 a01[kSeg], a23[kSeg];
#pragma unroll
    for (int o = 0; o < kSeg; ++o) {
      a01[o] = (f32x2){0.f, 0.f};
      a23[o] = (f32x2){0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < kSeg + kSsimTaps - 1; ++j) {
      const f32x2 v01 = {hm[0][r0 + j][c], hm[1][r0 + j][c]}, v23 = {hm[2][r0 + j][c], hm[3][r0 + j][c]};
#pragma unroll
      for (int o = 0; o < kSeg; ++o) {
        const int t = j - o;  // tap of input row r0 + j for output row r0 + o
        if (t >= 0 && t < kSsimTaps) {
          const f32x2 g = {c_gauss[t], c_gauss[t]};
          a01[o] = __builtin_elementwise_fma(g, v01, a01[o]);
          a23[o] = __builtin_elementwise_fma(g, v23, a23[o]);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < kSeg; ++o) {
      if (y0 + r0 + o >= OH || x0 + c >= OW) continue;
      const float m0 = a01[o][0], m1 = a01[o][1], e2 = a23[o][0], e3 = a23[o][1];
      const float mx = m0 + 0.5f, my = m1 + 0.5f;
      // v_rcp_f32 (1 ulp) instead of the IEEE division sequence
      const float lum = (2.f * mx * my + c1) * __builtin_amdgcn_rcpf(mx * mx + my * my + c1);
      const float cs = (2.f * (e3 - m0 * m1) + c2) * __builtin_amdgcn_rcpf(e2 - (m0 * m0 + m1 * m1) + c2);
      ssum += lum * cs;
      csum += cs;
    }
  }
  ssum = wave_sum(ssum);
  csum = wave_sum(csum);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = ssum;
    red[1][tid >> 6] = csum;
  }
  __syncthreads();
  if (tid == 0) {
    double s = 0.0, cc = 0.0;
    for (int w = 0; w < 4; ++w) {
      s += red[0][w];
      cc += red[1][w];
    }
    a.part[(size_t)p * a.tiles + blockIdx.x] = make_double2(s, cc);
  }
}

// 2x2 VALID average pool after SYMMETRIC padding of odd sizes (pad 1 at the end repeats
// the last row / column): (P,H,W) -> (P,ceil(H/2),ceil(W/2)) fp32, both images.
template <bool U8>
__global__ __launch_bounds__(256) void ssim_pool_kernel(SsimScaleArgs a, float* __restrict__ oa,
                                                        float* __restrict__ ob) {
  const int OH = (a.H + 1) / 2, OW = (a.W + 1) / 2;
  const size_t total = (size_t)a.P * OH * OW;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int ox = (int)(i % OW);
    const size_t t = i / OW;
    const int oy = (int)(t % OH), p = (int)(t / OH);
    const int ya = 2 * oy, yb = min(2 * oy + 1, a.H - 1), xa = 2 * ox, xb = min(2 * ox + 1, a.W - 1);
    float v[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int yy[4] = {ya, yb, ya, yb}, xx[4] = {xa, xa, xb, xb};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (U8) {
          const int img = p / 3, ch = p % 3;
          const uint8_t* src = s ? a.b8 : a.a8;
          v[s][q] = (float)src[((size_t)(img * a.H + yy[q]) * a.W + xx[q]) * 3 + ch] * (1.0f / 255.0f);
        } else {
          const float* src = s ? a.bf : a.af;
          v[s][q] = src[((size_t)p * a.H + yy[q]) * a.W + xx[q]];
        }
      }
    }
    oa[i] = 0.25f * (((v[0][0] + v[0][1]) + v[0][2]) + v[0][3]);
    ob[i] = 0.25f * (((v[1][0] + v[1][1]) + v[1][2]) + v[1][3]);
  }
}

// One block per image, one wave per (channel, scale): tile sums -> means (all 15 waves
// load at once), then thread 0 forms the weighted geometric mean.
constexpr int kCombineWaves = 3 * kSsimScales;
__global__ __launch_bounds__(64 * kCombineWaves) void msssim_combine_kernel(SsimCombineArgs a) {
  __shared__ double mean[3][kSsimScales][2];
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  {
    const int ch = w / kSsimScales, k = w % kSsimScales;
    const double2* part = a.part + a.offset[k] + (size_t)(img * 3 + ch) * a.tiles[k];
    double s = 0.0, c = 0.0;
    for (int t = lane; t < a.tiles[k]; t += 64) {
      s += part[t].x;
      c += part[t].y;
    }
    for (int o = 32; o > 0; o >>= 1) {
      s += __shfl_xor(s, o, 64);
      c += __shfl_xor(c, o, 64);
    }
    if (lane == 0) {
      mean[ch][k][0] = s / (double)a.valid[k];
      mean[ch][k][1] = c / (double)a.valid[k];
    }
  }
  __syncthreads();
  if (tid == 0) {
    double acc = 0.0;
    for (int ch = 0; ch < 3; ++ch) {
      double prod = 1.0;
      for (int k = 0; k < kSsimScales; ++k) {
        // cs of scales 0..3, full SSIM of the last scale, each relu'd
        const double v = k < kSsimScales - 1 ? mean[ch][k][1] : mean[ch][k][0];
        prod *= pow(fmax(v, 0.0), c_msssim_w[k]);
        if (a.per_scale) {
          a.per_scale[((img * 3 + ch) * kSsimScales + k) * 2 + 0] = (float)mean[ch][k][0];
          a.per_scale[((img * 3 + ch) * kSsimScales + k) * 2 + 1] = (float)mean[ch][k][1];
        }
      }
      acc += prod;
    }
    a.out[img] = (float)(acc / 3.0);
  }
}

// Sum of squared u8 differences per image: grid (chunks, n); 4-byte words when every
// image starts 4-byte aligned, bytes otherwise.  Integer atomics: exact and order-free.
__global__ __launch_bounds__(256) void sq_err_kernel(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                                     int64_t bytes, int words, unsigned long long* __restrict__ sse) {
  const int img = blockIdx.y;
  const uint8_t* pa = a + (size_t)img * bytes;
  const uint8_t* pb = b + (size_t)img * bytes;
  unsigned long long acc = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  if (words) {
    const uint32_t* wa = reinterpret_cast<const uint32_t*>(pa);
    const uint32_t* wb = reinterpret_cast<const uint32_t*>(pb);
    const int64_t nw = bytes >> 2;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += stride) {
      const uint32_t u = wa[i], v = wb[i];
      uint32_t s = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = (int)((u >> (8 * q)) & 255u) - (int)((v >> (8 * q)) & 255u);
        s += (uint32_t)(d * d);
      }
      acc += s;
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < bytes; i += stride) {
      const int d = (int)pa[i] - (int)pb[i];
      acc += (unsigned long long)(d * d);
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(sse + img, acc);
}

}  // namespace

hipError_t upload_ssim_constants() {
  // _fspecial_gauss(11, 1.5): exp(-(i^2 + j^2) / (2 sigma^2)) normalised; separable as
  // the outer product of the normalised 1-D window
  double g[kSsimTaps], sum = 0.0;
  for (int i = 0; i < kSsimTaps; ++i) {
    const double d = i - (kSsimTaps - 1) / 2.0;
    g[i] = exp(-0.5 * d * d / (1.5 * 1.5));
    sum += g[i];
  }
  float gf[kSsimTaps];
  for (int i = 0; i < kSsimTaps; ++i) gf[i] = (float)(g[i] / sum);
  const double w[kSsimScales] = {0.0448, 0.2856, 0.3001, 0.2363, 0.1333};
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_gauss), gf, sizeof(gf));
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_msssim_w), w, sizeof(w));
  return e;
}

void ssim_plan(int nimg, int H, int W, SsimPlan* plan) {
  const int P = 3 * nimg;
  size_t off = 0, img_bytes = 0;
  int h = H, w = W;
  for (int k = 0; k < kSsimScales; ++k) {
    if (k > 0) {
      h = (h + 1) / 2;
      w = (w + 1) / 2;
      plan->img_off[k] = img_bytes;
      img_bytes += 2 * (size_t)P * h * w * sizeof(float);
    }
    plan->h[k] = h;
    plan->w[k] = w;
    const int oh = h - kSsimTaps + 1, ow = w - kSsimTaps + 1;
    plan->tiles_x[k] = (ow + kSsimTile - 1) / kSsimTile;
    plan->tiles[k] = plan->tiles_x[k] * ((oh + kSsimTile - 1) / kSsimTile);
    plan->valid[k] = (int64_t)oh * ow;
    plan->part_off[k] = off;
    off += (size_t)P * plan->tiles[k];
  }
  plan->img_off[0] = 0;
  plan->img_bytes = (img_bytes + 255) & ~(size_t)255;
  plan->bytes = plan->img_bytes + off * sizeof(double2);
}

hipError_t launch_ms_ssim(const uint8_t* a, const uint8_t* b, int nimg, int H, int W, void* scratch, float* out,
                          float* per_scale, hipStream_t st) {
  hipError_t e;
  SsimPlan pl;
  ssim_plan(nimg, H, W, &pl);
  char* base = static_cast<char*>(scratch);
  double2* part = reinterpret_cast<double2*>(base + pl.img_bytes);
  const int P = 3 * nimg;
  const float* cur_a = nullptr;
  const float* cur_b = nullptr;
  for (int k = 0; k < kSsimScales; ++k) {
    SsimScaleArgs s{};
    s.a8 = a;
    s.b8 = b;
    s.af = cur_a;
    s.bf = cur_b;
    s.P = P;
    s.H = pl.h[k];
    s.W = pl.w[k];
    s.tiles_x = pl.tiles_x[k];
    s.tiles = pl.tiles[k];
    s.part = part + pl.part_off[k];
    if (k == 0)
      hipLaunchKernelGGL(ssim_tile_kernel<true>, dim3(pl.tiles[k], P), dim3(256), 0, st, s);
    else
      hipLaunchKernelGGL(ssim_tile_kernel<false>, dim3(pl.tiles[k], P), dim3(256), 0, st, s);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (k + 1 < kSsimScales) {
      float* na = reinterpret_cast<float*>(base + pl.img_off[k + 1]);
      float* nb = na + (size_t)P * pl.h[k + 1] * pl.w[k + 1];
      const size_t total = (size_t)P * pl.h[k + 1] * pl.w[k + 1];
      const int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
      if (k == 0)
        hipLaunchKernelGGL(ssim_pool_kernel<true>, dim3(blocks), dim3(256), 0, st, s, na, nb);
      else
        hipLaunchKernelGGL(ssim_pool_kernel<false>, dim3(blocks), dim3(256), 0, st, s, na, nb);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      cur_a = na;
      cur_b = nb;
    }
  }
  SsimCombineArgs c{};
  c.part = part;
  for (int k = 0; k < kSsimScales; ++k) {
    c.offset[k] = pl.part_off[k];
    c.tiles[k] = pl.tiles[k];
    c.valid[k] = pl.valid[k];
  }
  c.out = out;
  c.per_scale = per_scale;
  hipLaunchKernelGGL(msssim_combine_kernel, dim3(nimg), dim3(64 * kCombineWaves), 0, st, c);
  return hipGetLastError();
}

hipError_t launch_sq_err(const uint8_t* a, const uint8_t* b, int nimg, int64_t bytes, unsigned long long* sse,
                         hipStream_t st) {
  hipError_t e = hipMemsetAsync(sse, 0, (size_t)nimg * sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  const bool words = (bytes % 4 == 0) && ((uintptr_t)a % 4 == 0) && ((uintptr_t)b % 4 == 0);
  const int64_t units = words ? bytes / 4 : bytes;
  const int chunks = (int)std::max<int64_t>(1, std::min<int64_t>((units + 255) / 256, std::max(1, 2048 / nimg)));
  hipLaunchKernelGGL(sq_err_kernel, dim3(chunks, nimg), dim3(256), 0, st, a, b, bytes, words ? 1 : 0, sse);
  return hipGetLastError();
}

}  // namespace nic
