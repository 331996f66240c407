// Training side path on the matrix cores (tf2_0/src/training.py:74-151):
// the convolutions of the Training step's forward and backward passes -- the codec's
// BaseEncoder / BaseDecoder (encoder.py:7-32, decoder.py:7-32) and the Entropynet's convs
// (training.py:25-42) -- as split-f16 ("f16x3") MFMA GEMMs over NHWC fp32 tensors.
//
// Every convolution of the step is one of two GEMM shapes:
//
//  * gather GEMM  y[m][co] = bias[co] + sum_{tap, ci} x[src(m, tap)][ci] * W(tap, ci, co)
//      m = output pixel (n, oy, ox).  Forward conv (Keras Conv2D, SAME): src = s*o + k - pad.
//      "Transposed" gather: src = (o + pad - k) / s where divisible -- the forward of
//      Conv2DTranspose (SAME) and the input gradient of Conv2D.  The input gradient of
//      Conv2DTranspose is a forward-conv gather.  W(tap, ci, co) reads the stored kernel
//      [tap][ci][co] (wt_layout 0) or [tap][co][ci] (wt_layout 1), so no transposed copy of a
//      kernel is ever made.
//  * weight-gradient GEMM  dW[tap][a][b] = sum_u gat[s*u + k - pad][a] * dir[u][b]
//      (Conv2D: gat = x, dir = dy; Conv2DTranspose: gat = dy, dir = x), K = every pixel of
//      the batch, split into slices whose partial sums a second kernel adds in a fixed order
//      (deterministic, no atomics).
//
// Arithmetic: each operand tile is scaled by an exact power of two (per tensor, from
// nic_absmax_scale: max |x| * scale in [2^13, 2^14), so gradients of 1e-9 keep every bit)
// and split hi = f16(x), lo = f16(x - hi) while it is staged into LDS; three
// v_mfma_f32_16x16x32_f16 per fragment pair (hi*hi + hi*lo + lo*hi) accumulate in fp32;
// the epilogue multiplies by the exact inverse scales.  Error ~2^-22 relative per product,
// fp32-class (tests/test_gpu_train.py: vs torch fp32 autograd).
//
// Tiles: 256-thread blocks, K in chunks of 32 staged through LDS (row pitch 40 f16 = 80 B:
// the 16-B fragment reads of a 16-lane group hit distinct banks); the next chunk's global
// loads are issued before the current chunk's MFMAs (register double buffer).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nic_kernels.h"

namespace nic {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int TK = 32;  // K per chunk
constexpr int LP = 40;  // LDS row pitch (f16)
constexpr int GM = 64;  // gather GEMM: output pixels per block (4 waves x 16)

__device__ __forceinline__ void split1(float v, _Float16& hi, _Float16& lo) {
  hi = (_Float16)v;
  lo = (_Float16)(v - (float)hi);
}

__device__ __forceinline__ float ld_scale(const float* s) { return s ? *s : 1.0f; }

// ---- gather GEMM -------------------------------------------------------------------------
struct GatherArgs {
  const float* x;      // [n][h][w][cin]
  const f16x8* wp;     // packed split weights (pack_w_kernel): [K/32 chunk][NT/16 co tile][hi, lo][64 lanes]
  const float* bias;   // [cout] or null
  const float* sx;     // device scale of x (power of two) or null
  const float* sw;     // device scale of the weights or null (already applied in wp)
  float* y;            // [n][oh][ow][cout]
  int n, h, w, cin, oh, ow, cout, kh, kw, stride, pad_y, pad_x, transposed;
  int act;             // 1: leaky_relu(0.2) of the biased sum (Keras activation=tf.nn.leaky_relu)
  int K;               // kh * kw * cin
  long long M;         // n * oh * ow
  int ph_blk[5];       // phase mode: first block of output phase (py, px) = (p >> 1, p & 1), then the grid
};

// Output pixel m of the block's set -> (b, oy, ox).  Phase mode: the pixels of one output
// phase (oy % 2, ox % 2) = (py, px) only, so every pixel of the block uses the same taps.
__device__ __forceinline__ bool pixel_of(const GatherArgs& a, bool ph, int py, int px, long long m, int& b, int& oy,
                                         int& ox) {
  if (!ph) {
    if (m >= a.M) return false;
    const long long per = (long long)a.oh * a.ow;
    b = (int)(m / per);
    const int r = (int)(m - (long long)b * per);
    oy = r / a.ow;
    ox = r - oy * a.ow;
    return true;
  }
  const int qh = (a.oh - py + 1) >> 1, qw = (a.ow - px + 1) >> 1;
  const long long per = (long long)qh * qw;
  if (per == 0 || m >= (long long)a.n * per) return false;
  b = (int)(m / per);
  const int r = (int)(m - (long long)b * per), qy = r / qw;
  oy = 2 * qy + py;
  ox = 2 * (r - qy * qw) + px;
  return true;
}

// source pixel of output pixel (b, oy, ox) at tap (ky, kx); -1 when outside / not on the grid
__device__ __forceinline__ long long gather_src(const GatherArgs& a, int b, int oy, int ox, int ky, int kx) {
  int iy, ix;
  if (a.transposed) {
    const int ty = oy + a.pad_y - ky, tx = ox + a.pad_x - kx;
    if (ty < 0 || tx < 0) return -1;
    if (a.stride == 1) {  // (uniform branches: no integer division for the strides in use)
      iy = ty;
      ix = tx;
    } else if (a.stride == 2) {
      if ((ty | tx) & 1) return -1;
      iy = ty >> 1;
      ix = tx >> 1;
    } else {
      if (ty % a.stride || tx % a.stride) return -1;
      iy = ty / a.stride;
      ix = tx / a.stride;
    }
  } else {
    iy = a.stride * oy + ky - a.pad_y;
    ix = a.stride * ox + kx - a.pad_x;
  }
  if ((unsigned)iy >= (unsigned)a.h || (unsigned)ix >= (unsigned)a.w) return -1;
  return ((long long)b * a.h + iy) * a.w + ix;
}

// Weights -> split-f16 MFMA A fragments, once per call: fragment (chunk c, co tile t, hi|lo,
// lane) holds rows co = 16 t + (lane & 15), k = 32 c + 8 (lane >> 4) + j of w * scale, where
// k = tap * cin + ci and W(tap, ci, co) reads layout 0 [tap][ci][co] or 1 [tap][co][ci].
__global__ __launch_bounds__(256) void pack_w_kernel(const float* __restrict__ wt, int layout, int cin, int cout, int K,
                                                     int ntt, int nchunk, const float* __restrict__ sw,
                                                     f16x8* __restrict__ wp) {
  const int total = nchunk * ntt * 64;
  const float s = ld_scale(sw);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int lane = i & 63, ct = i >> 6, t = ct % ntt, c = ct / ntt;
    const int co = 16 * t + (lane & 15);
    f16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * c + 8 * (lane >> 4) + j;
      float v = 0.f;
      if (co < cout && k < K) {
        const int tap = k / cin, ci = k - tap * cin;
        v = layout ? wt[((size_t)tap * cout + co) * cin + ci] : wt[((size_t)tap * cin + ci) * cout + co];
      }
      _Float16 h, l;
      split1(v * s, h, l);
      hi[j] = h;
      lo[j] = l;
    }
    wp[(size_t)(ct * 2 + 0) * 64 + lane] = hi;
    wp[(size_t)(ct * 2 + 1) * 64 + lane] = lo;
  }
}

// NT = output channels per block (16, 32 or 64); VEC: cin % 32 == 0 (a K chunk is 32
// consecutive channels of one tap: two float4 per thread, stored as f16x4 hi / lo), else one
// element per (pixel, k); PH (VEC, transposed, stride 2): the block's pixels share one output
// phase and the K loop visits only that phase's taps (a quarter of them).  The weights'
// A fragments come straight from the packed buffer (one chunk ahead in registers); only the
// gathered activations go through LDS.
template <int NT, bool VEC, bool PH>
__global__ __launch_bounds__(256) void conv_gather_kernel(GatherArgs a) {
  __shared__ __attribute__((aligned(16))) _Float16 xs[2][GM * LP];  // [hi, lo][pixel][k]
  constexpr int NTT = NT / 16;
  constexpr int XN = VEC ? 2 : 8;  // x elements (float4s when VEC) per thread per chunk
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l16 = lane & 15;
  int phase = 0, blk = blockIdx.x;
  if constexpr (PH) {
    while (phase < 3 && blk >= a.ph_blk[phase + 1]) ++phase;
    blk -= a.ph_blk[phase];
  }
  const int py = phase >> 1, px = phase & 1;
  const long long m0 = (long long)blk * GM;
  const float sx = ld_scale(a.sx), sw = ld_scale(a.sw);
  // K chunks: all of them, or (PH) the phase's taps ky = ky0 + 2 i, kx = kx0 + 2 j
  const int cc_n = VEC ? a.cin / TK : 1;
  const int ky0 = (py + a.pad_y) & 1, kx0 = (px + a.pad_x) & 1;
  const int tny = (a.kh - ky0 + 1) >> 1, tnx = (a.kw - kx0 + 1) >> 1;
  const int nchunk = PH ? tny * tnx * cc_n : (a.K + TK - 1) / TK;
  auto chunk_tap = [&](int c, int& ky, int& kx, int& ci0, int& gc) {  // VEC: tap and channel block of chunk c
    if constexpr (PH) {
      const int tt = c / cc_n, cc = c - tt * cc_n, iy = tt / tnx;
      ky = ky0 + 2 * iy;
      kx = kx0 + 2 * (tt - iy * tnx);
      ci0 = cc * TK;
      gc = (ky * a.kw + kx) * cc_n + cc;
    } else {
      const int k0 = c * TK, tap = k0 / a.cin;
      ky = tap / a.kw;
      kx = tap - ky * a.kw;
      ci0 = k0 - tap * a.cin;
      gc = c;
    }
  };

  // this thread's staging pixels: VEC px = tid/8 + 32 r; scalar px = tid/32 + 8 e
  int pb[XN], pyy[XN], pxx[XN];
#pragma unroll
  for (int e = 0; e < XN; ++e) {
    const int sp = VEC ? (tid >> 3) + 32 * e : (tid >> 5) + 8 * e;
    if (!pixel_of(a, PH, py, px, m0 + sp, pb[e], pyy[e], pxx[e])) pb[e] = -1;
  }

  f32x4 xv[VEC ? XN : 1];
  float xsv[VEC ? 1 : XN];
  f16x8 wc[NTT][2], wn[NTT][2];  // A fragments of the current / next chunk (static indices: no scratch)
  auto load = [&](int c, f16x8 (&w)[NTT][2]) {
    int ky, kx, ci0, gc;
    if constexpr (VEC) {
      chunk_tap(c, ky, kx, ci0, gc);
#pragma unroll
      for (int e = 0; e < XN; ++e) {
        const long long s = pb[e] >= 0 ? gather_src(a, pb[e], pyy[e], pxx[e], ky, kx) : -1;
        xv[e] = s >= 0 ? *(const f32x4*)(a.x + s * a.cin + ci0 + 4 * (tid & 7)) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    } else {
      gc = c;
      const int k = c * TK + (tid & 31);
      const int tap = k / a.cin, ci = k - tap * a.cin;
      ky = tap / a.kw;
      kx = tap - ky * a.kw;
#pragma unroll
      for (int e = 0; e < XN; ++e) {
        const long long s = (pb[e] >= 0 && k < a.K) ? gather_src(a, pb[e], pyy[e], pxx[e], ky, kx) : -1;
        xsv[e] = s >= 0 ? a.x[s * a.cin + ci] : 0.f;
      }
    }
#pragma unroll
    for (int t = 0; t < NTT; ++t)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) w[t][hl] = a.wp[((size_t)(gc * NTT + t) * 2 + hl) * 64 + lane];
  };
  auto stage = [&]() {
    if constexpr (VEC) {
      typedef _Float16 f16x4v __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int e = 0; e < XN; ++e) {
        const int sp = (tid >> 3) + 32 * e, k = 4 * (tid & 7);
        f16x4v hi, lo;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          _Float16 h, l;
          split1(xv[e][r] * sx, h, l);
          hi[r] = h;
          lo[r] = l;
        }
        *(f16x4v*)&xs[0][sp * LP + k] = hi;
        *(f16x4v*)&xs[1][sp * LP + k] = lo;
      }
    } else {
#pragma unroll
      for (int e = 0; e < XN; ++e) {
        const int sp = (tid >> 5) + 8 * e, k = tid & 31;
        split1(xsv[e] * sx, xs[0][sp * LP + k], xs[1][sp * LP + k]);
      }
    }
  };

  f32x4 acc[NTT];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (nchunk > 0) load(0, wc);
  for (int c = 0; c < nchunk; ++c) {
    __syncthreads();  // every wave is done with the previous chunk's tile
    stage();
    __syncthreads();
    if (c + 1 < nchunk) load(c + 1, wn);  // in flight during this chunk's MFMAs
    const int bo = (wave * 16 + l16) * LP + 8 * g;
    const f16x8 bh = *(const f16x8*)&xs[0][bo], bl = *(const f16x8*)&xs[1][bo];
#pragma unroll
    for (int t = 0; t < NTT; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wc[t][1], bh, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wc[t][0], bl, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wc[t][0], bh, acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < NTT; ++t) {
      wc[t][0] = wn[t][0];
      wc[t][1] = wn[t][1];
    }
  }
  // D[co = 16t + 4g + r][pixel 16 wave + l16]
  int b, oy, ox;
  if (!pixel_of(a, PH, py, px, m0 + wave * 16 + l16, b, oy, ox)) return;
  const float isx = 1.0f / sx, isw = 1.0f / sw;  // exact: powers of two (applied one at a time)
  float* yp = a.y + (((long long)b * a.oh + oy) * a.ow + ox) * a.cout;
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    const int co = t * 16 + 4 * g;
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (acc[t][r] * isx) * isw + (a.bias && co + r < a.cout ? a.bias[co + r] : 0.f);
    if (a.act)  // tf.nn.leaky_relu(z, 0.2) = max(0.2 z, z): z for z > 0, else 0.2 z (one rounding)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(__fmul_rn(v[r], 0.2f), v[r]);
    if ((a.cout & 3) == 0 && co + 4 <= a.cout) {
      *(f32x4*)(yp + co) = v;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (co + r < a.cout) yp[co + r] = v[r];
    }
  }
}

// ---- activation + bias gradient of a layer ------------------------------------------------
// dz = dy * (act && !(y > 0) ? 0.2 : 1): tf.nn.leaky_relu's gradient (z > 0 ? dy : 0.2 dy),
// read from the layer's output y (y > 0 iff z > 0); db[c] = sum over rows of dz[row][c]
// (BiasAddGrad); and the power-of-two operand scale of dz (nic_absmax_scale's, from the same
// pass).  A block takes kAbgRows rows; thread t owns V consecutive columns (V = 4: 16-B loads
// when cols % 4 == 0) of row lane t / (cols / V), summed per thread in row order, then over
// the row lanes in order into part[block][c] (max |dz| into part[nblk * cols + block]);
// abg_reduce_kernel adds the blocks' partials of a column in a fixed order (deterministic).
constexpr int kAbgRows = 256;
template <int V>
__global__ __launch_bounds__(256) void act_bias_grad_kernel(const float* __restrict__ y, const float* __restrict__ dy,
                                                            long long rows, int cols, int act, float* __restrict__ dz,
                                                            float* __restrict__ part) {
  typedef float fv __attribute__((ext_vector_type(V)));
  __shared__ float red[256 * V];
  __shared__ float wm[4];
  const int cg = cols / V, nrl = 256 / cg, t = threadIdx.x, c0 = (t % cg) * V, rl = t / cg;
  const long long r0 = (long long)blockIdx.x * kAbgRows;
  const long long r1 = r0 + kAbgRows < rows ? r0 + kAbgRows : rows;
  fv s = {};
  float m = 0.f;
  if (rl < nrl) {
#pragma unroll 4
    for (long long r = r0 + rl; r < r1; r += nrl) {
      const long long e = r * cols + c0;
      fv g = *(const fv*)(dy + e);
      if (act) {
        const fv yv = *(const fv*)(y + e);
#pragma unroll
        for (int k = 0; k < V; ++k)
          if (!(yv[k] > 0.f)) g[k] = __fmul_rn(g[k], 0.2f);
      }
      if (dz) *(fv*)(dz + e) = g;
#pragma unroll
      for (int k = 0; k < V; ++k) {
        s[k] = __fadd_rn(s[k], g[k]);
        m = fmaxf(m, fabsf(g[k]));
      }
    }
  }
#pragma unroll
  for (int k = 0; k < V; ++k) red[t * V + k] = s[k];
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((t & 63) == 0) wm[t >> 6] = m;
  __syncthreads();
  if (t < cols) {  // column t: lane group t / V of every row lane, in row-lane order
    float b = 0.f;
    for (int k = 0; k < nrl; ++k) b = __fadd_rn(b, red[(k * cg + t / V) * V + t % V]);
    part[(long long)blockIdx.x * cols + t] = b;
  }
  if (t == 0) part[(long long)gridDim.x * cols + blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

// Block c < cols: db[c] = sum of the blocks' partials of column c (thread k adds partials k,
// k + 256, ... in order, then a fixed pairwise tree over the threads); block cols: the scale
// of the blocks' max |dz| (nic_absmax_scale's formula)
__global__ __launch_bounds__(256) void abg_reduce_kernel(const float* __restrict__ part, int nblk, int cols,
                                                         float* __restrict__ db, float* __restrict__ scale) {
  __shared__ float red[256];
  const int c = blockIdx.x, t = threadIdx.x;
  if (c < cols) {
    if (!db) return;
    float s = 0.f;
    for (int k = t; k < nblk; k += 256) s = __fadd_rn(s, part[(long long)k * cols + c]);
    red[t] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (t < o) red[t] = __fadd_rn(red[t], red[t + o]);
      __syncthreads();
    }
    if (t == 0) db[c] = red[0];
  } else {
    if (!scale) return;
    float m = 0.f;
    for (int k = t; k < nblk; k += 256) m = fmaxf(m, part[(long long)nblk * cols + k]);
    red[t] = m;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (t < o) red[t] = fmaxf(red[t], red[t + o]);
      __syncthreads();
    }
    if (t == 0) {
      m = red[0];
      float sc = 1.0f;
      if (m > 0.f && isfinite(m)) sc = ldexpf(1.0f, min(max(13 - ilogbf(m), -126), 126));
      *scale = sc;
    }
  }
}

// ---- SSIM map of the loss from its filtered terms (tf.image.ssim, training.py:119-121) ------
// Per pixel of the VALID map, from mx = G*x, my = G*y, sxy = G*(x y), sxx = G*(x^2 + y^2):
//   num0 = (mx my) 2, den0 = mx mx + my my, lum = (num0 + c1) / (den0 + c1),
//   cs = ((2 sxy - num0) + c2) / ((sxx - den0) + c2), v = lum cs
// in tf.image.ssim's op order, every op rounded; forward: the per-image mean of v (per-block
// partial sums in pixel order, then added in block order: deterministic); backward: the four
// terms' gradients of g[n] * mean.
constexpr int kSsimPix = 1024;  // map pixels per block
struct SsimTerms {
  float num0, den0, lum, cs, a, b, c, d;
};
__device__ __forceinline__ SsimTerms ssim_terms(float mx, float my, float sxy, float sxx, float c1, float c2) {
  SsimTerms t;
  t.num0 = __fmul_rn(__fmul_rn(mx, my), 2.0f);
  t.den0 = __fadd_rn(__fmul_rn(mx, mx), __fmul_rn(my, my));
  t.a = __fadd_rn(t.num0, c1);
  t.b = __fadd_rn(t.den0, c1);
  t.lum = __fdiv_rn(t.a, t.b);
  t.c = __fadd_rn(__fsub_rn(__fmul_rn(sxy, 2.0f), t.num0), c2);
  t.d = __fadd_rn(__fsub_rn(sxx, t.den0), c2);
  t.cs = __fdiv_rn(t.c, t.d);
  return t;
}
__global__ __launch_bounds__(256) void ssim_map_kernel(const float* __restrict__ mx, const float* __restrict__ my,
                                                       const float* __restrict__ sxy, const float* __restrict__ sxx,
                                                       long long hw, int bpi, float c1, float c2,
                                                       float* __restrict__ part) {
  __shared__ float red[256];
  const int n = blockIdx.x / bpi, bk = blockIdx.x - n * bpi, t = threadIdx.x;
  const long long base = (long long)n * hw, p0 = (long long)bk * kSsimPix;
  float s = 0.f;
  for (long long p = p0 + t; p < p0 + kSsimPix && p < hw; p += 256) {
    const long long e = base + p;
    const SsimTerms q = ssim_terms(mx[e], my[e], sxy[e], sxx[e], c1, c2);
    s = __fadd_rn(s, __fmul_rn(q.lum, q.cs));
  }
  red[t] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] = __fadd_rn(red[t], red[t + o]);
    __syncthreads();
  }
  if (t == 0) part[blockIdx.x] = red[0];
}
__global__ __launch_bounds__(64) void ssim_mean_kernel(const float* __restrict__ part, int n, int bpi, long long hw,
                                                       float* __restrict__ out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int k = 0; k < bpi; ++k) s = __fadd_rn(s, part[(long long)i * bpi + k]);
  out[i] = __fdiv_rn(s, (float)hw);
}
__global__ __launch_bounds__(256) void ssim_map_grad_kernel(const float* __restrict__ mx, const float* __restrict__ my,
                                                            const float* __restrict__ sxy, const float* __restrict__ sxx,
                                                            const float* __restrict__ g, int n, long long hw, float c1,
                                                            float c2, float* __restrict__ gmx, float* __restrict__ gmy,
                                                            float* __restrict__ gsxy, float* __restrict__ gsxx) {
  const long long total = (long long)n * hw;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const float x = mx[e], y = my[e];
    const SsimTerms q = ssim_terms(x, y, sxy[e], sxx[e], c1, c2);
    const float G = __fdiv_rn(g[e / hw], (float)hw);  // d mean / d v
    // v = (a / b) (c / d): dv/dnum0 = cs / b - lum / d, dv/dden0 = lum cs / d - lum cs / b,
    // dv/d(2 sxy) = lum / d, dv/dsxx = -lum cs / d
    const float ib = __frcp_rn(q.b), id = __frcp_rn(q.d), v = __fmul_rn(q.lum, q.cs);
    const float dnum0 = __fmul_rn(G, __fsub_rn(__fmul_rn(q.cs, ib), __fmul_rn(q.lum, id)));
    const float dden0 = __fmul_rn(G, __fsub_rn(__fmul_rn(v, id), __fmul_rn(v, ib)));
    gmx[e] = __fmul_rn(2.0f, __fadd_rn(__fmul_rn(dnum0, y), __fmul_rn(dden0, x)));
    gmy[e] = __fmul_rn(2.0f, __fadd_rn(__fmul_rn(dnum0, x), __fmul_rn(dden0, y)));
    gsxy[e] = __fmul_rn(2.0f, __fmul_rn(G, __fmul_rn(q.lum, id)));
    gsxx[e] = -__fmul_rn(G, __fmul_rn(v, id));
  }
}

// ---- separable Gaussian of the SSIM loss (tf.image.ssim's 11-tap window) --------------------
// One-channel planes (n, h, w): VALID correlation along x (vertical = 0) or y, or its adjoint
// (the input gradient: a full convolution with the same taps).
__global__ __launch_bounds__(256) void gauss1d_kernel(const float* __restrict__ in, int n, int hi, int wi,
                                                      const float* __restrict__ taps, int nt, int vertical, int adjoint,
                                                      float* __restrict__ out, int ho, int wo) {
  const long long total = (long long)n * ho * wo;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int x = (int)(i % wo);
    const long long r = i / wo;
    const int y = (int)(r % ho), b = (int)(r / ho);
    const float* src = in + (long long)b * hi * wi;
    float s = 0.f;
    for (int k = 0; k < nt; ++k) {
      const int yy = vertical ? (adjoint ? y - k : y + k) : y;
      const int xx = vertical ? x : (adjoint ? x - k : x + k);
      if ((unsigned)yy < (unsigned)hi && (unsigned)xx < (unsigned)wi) s = fmaf(taps[k], src[(long long)yy * wi + xx], s);
    }
    out[i] = s;
  }
}

// ---- weight-gradient GEMM ------------------------------------------------------------------
struct WgradArgs {
  const float* gat;   // [n][gh][gw][ca], read at s*u + k - pad
  const float* dir;   // [n][uh][uw][cb]
  const float* sg;    // device scales or null
  const float* sd;
  float* part;        // [slices][taps * ca rows][cb]
  int n, gh, gw, ca, uh, uw, cb, kh, kw, stride, pad_y, pad_x;
  int rows;           // taps * ca: the GEMM's M (row r = tap * ca + a)
  long long U;        // n * uh * uw
  int slice_len;      // pixels per slice (multiple of TK)
};

// M = (tap, a) rows flattened (r = tap * ca + a), N = b, K = the slice's pixels.  NA rows
// per block (16 ... 64: one tap of a 64-channel gat, two taps of a 32-channel one, or all
// 25 taps of a one-channel one), NB >= cb; block (row block, slice) stages the dir
// tile once for all its rows; wave w owns the 16 x 16 output tiles w, w + 4, ...
template <int NA, int NB>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int NMAX = NA > NB ? NA : NB;
  __shared__ __attribute__((aligned(16))) _Float16 gs[2][NMAX * LP];  // [hi, lo][a][u]
  __shared__ __attribute__((aligned(16))) _Float16 ds[2][NMAX * LP];  // [hi, lo][b][u]
  constexpr int NTA = NA / 16, NTB = NB / 16, NTILE = NTA * NTB, TPW = (NTILE + 3) / 4;
  // staging: thread item = (channel, 4 consecutive pixels u): 4 loads coalesced across the
  // channel-contiguous lanes, one f16x4 hi and one lo store into the [channel][u] tiles
  constexpr int GE = (TK / 4 * NA + 255) / 256, DE = (TK / 4 * NB + 255) / 256;
  typedef _Float16 f16x4v __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int r0 = blockIdx.x * NA, slice = blockIdx.y;
  const long long u0 = (long long)slice * a.slice_len;
  const long long u1 = u0 + a.slice_len < a.U ? u0 + a.slice_len : a.U;
  const float sg = ld_scale(a.sg), sd = ld_scale(a.sd);
  const long long per = (long long)a.uh * a.uw;

  f32x4 gv[GE], dv[DE];
  // pixel coordinates (b, uy, ux) of each gat item's first u, advanced by TK per chunk with
  // compares instead of the per-element integer divisions they replace
  int ib_[GE], iy_[GE], ix_[GE];
#pragma unroll
  for (int e = 0; e < GE; ++e) {
    const long long u = u0 + 4 * ((tid + 256 * e) / NA);
    ib_[e] = (int)(u / per);
    const int r = (int)(u - (long long)ib_[e] * per);
    iy_[e] = r / a.uw;
    ix_[e] = r - iy_[e] * a.uw;
  }
  auto step_pix = [&](int& b, int& y, int& x, int d) {
    x += d;
    while (x >= a.uw) {
      x -= a.uw;
      if (++y == a.uh) {
        y = 0;
        ++b;
      }
    }
  };
  auto load = [&](long long ub) {
#pragma unroll
    for (int e = 0; e < GE; ++e) {
      const int idx = tid + 256 * e, ug = idx / NA, row = r0 + idx % NA;
      const int tap = row / a.ca, ch = row - tap * a.ca, ky = tap / a.kw, kx = tap - ky * a.kw;
      int b = ib_[e], uy = iy_[e], ux = ix_[e];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long u = ub + 4 * ug + i;
        if (i) step_pix(b, uy, ux, 1);
        float v = 0.f;
        if (idx < TK / 4 * NA && row < a.rows && u < u1) {
          const int gy = a.stride * uy + ky - a.pad_y, gx = a.stride * ux + kx - a.pad_x;
          if ((unsigned)gy < (unsigned)a.gh && (unsigned)gx < (unsigned)a.gw)
            v = a.gat[(((size_t)b * a.gh + gy) * a.gw + gx) * a.ca + ch];
        }
        gv[e][i] = v;
      }
      step_pix(ib_[e], iy_[e], ix_[e], TK);  // this item's first u in the next chunk
    }
#pragma unroll
    for (int e = 0; e < DE; ++e) {
      const int idx = tid + 256 * e, ug = idx / NB, ch = idx % NB;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long u = ub + 4 * ug + i;
        dv[e][i] = (idx < TK / 4 * NB && ch < a.cb && u < u1) ? a.dir[u * a.cb + ch] : 0.f;
      }
    }
  };
  auto put = [&](_Float16 (&tile)[2][(NA > NB ? NA : NB) * LP], int row, int col, const f32x4& v, float s) {
    f16x4v hi, lo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      _Float16 h, l;
      split1(v[i] * s, h, l);
      hi[i] = h;
      lo[i] = l;
    }
    *(f16x4v*)&tile[0][row * LP + col] = hi;
    *(f16x4v*)&tile[1][row * LP + col] = lo;
  };
  auto stage = [&]() {
#pragma unroll
    for (int e = 0; e < GE; ++e) {
      const int idx = tid + 256 * e;
      if (idx < TK / 4 * NA) put(gs, idx % NA, 4 * (idx / NA), gv[e], sg);
    }
#pragma unroll
    for (int e = 0; e < DE; ++e) {
      const int idx = tid + 256 * e;
      if (idx < TK / 4 * NB) put(ds, idx % NB, 4 * (idx / NB), dv[e], sd);
    }
  };

  f32x4 acc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (u0 < u1) load(u0);
  for (long long ub = u0; ub < u1; ub += TK) {
    __syncthreads();
    stage();
    __syncthreads();
    if (ub + TK < u1) load(ub + TK);
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int t = wave + 4 * j;
      if (t >= NTILE) break;  // wave-uniform
      const int ta = t / NTB, tb = t - ta * NTB;
      const int ao = (ta * 16 + l16) * LP + 8 * g, bo = (tb * 16 + l16) * LP + 8 * g;
      const f16x8 ah = *(const f16x8*)&gs[0][ao], al = *(const f16x8*)&gs[1][ao];
      const f16x8 bh = *(const f16x8*)&ds[0][bo], bl = *(const f16x8*)&ds[1][bo];
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[j], 0, 0, 0);
    }
  }
  const float isg = 1.0f / sg, isd = 1.0f / sd;
  float* out = a.part + ((size_t)slice * a.rows + r0) * a.cb;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + 4 * j;
    if (t >= NTILE) break;
    const int ta = t / NTB, tb = t - ta * NTB, bcol = tb * 16 + l16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int arow = ta * 16 + 4 * g + r;
      if (r0 + arow < a.rows && bcol < a.cb) out[(size_t)arow * a.cb + bcol] = (acc[j][r] * isg) * isd;
    }
  }
}

// dw[i] = sum over slices of part[s][i]: 8 independent loads in flight per thread, summed
// in a fixed order (deterministic)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int slices, long long nw,
                                                           float* __restrict__ dw) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nw; i += (long long)gridDim.x * 256) {
    float s = 0.f;
    int k = 0;
    for (; k + 8 <= slices; k += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(size_t)(k + j) * nw + i];
      s += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    }
    for (; k < slices; ++k) s += part[(size_t)k * nw + i];
    dw[i] = s;
  }
}

// ---- power-of-two operand scales -------------------------------------------------------------
constexpr int kScaleBlocks = 512;

__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, long long n, float* __restrict__ part) {
  float m = 0.f;
  const long long n4 = ((reinterpret_cast<uintptr_t>(x) & 15) == 0) ? n / 4 : 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const f32x4 v = ((const f32x4*)x)[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  for (long long i = 4 * n4 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    m = fmaxf(m, fabsf(x[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

// scale = 2^(13 - floor(log2 max)): max * scale in [2^13, 2^14) (1 for zero / non-finite)
__global__ __launch_bounds__(256) void scale_finish_kernel(const float* __restrict__ part, int nb, float* __restrict__ scale) {
  float m = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) m = fmaxf(m, part[i]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
    float s = 1.0f;
    if (m > 0.f && isfinite(m)) s = ldexpf(1.0f, min(max(13 - ilogbf(m), -126), 126));
    *scale = s;
  }
}

template <int NT, bool VEC, bool PH>
hipError_t launch_gather_t(const GatherArgs& a, hipStream_t st) {
  const long long blocks = PH ? a.ph_blk[4] : (a.M + GM - 1) / GM;
  hipLaunchKernelGGL((conv_gather_kernel<NT, VEC, PH>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <int NA, int NB>
hipError_t launch_wgrad_t(const WgradArgs& a, int slices, hipStream_t st) {
  hipLaunchKernelGGL((conv_wgrad_kernel<NA, NB>), dim3((a.rows + NA - 1) / NA, slices), dim3(256), 0, st, a);
  return hipGetLastError();
}

int tile16(int c) { return c <= 16 ? 16 : c <= 32 ? 32 : 64; }

}  // namespace

size_t train_scale_work_floats() { return kScaleBlocks; }

hipError_t launch_absmax_scale(const float* x, long long n, float* scale, float* work, hipStream_t st) {
  const long long want = (n / 4 + 255) / 256;
  const int nb = (int)(want < 1 ? 1 : want > kScaleBlocks ? kScaleBlocks : want);
  hipLaunchKernelGGL(absmax_kernel, dim3(nb), dim3(256), 0, st, x, n, work);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(scale_finish_kernel, dim3(1), dim3(256), 0, st, work, nb, scale);
  return hipGetLastError();
}

size_t train_gather_work_bytes(int kh, int kw, int cin, int cout) {
  return (size_t)((kh * kw * cin + TK - 1) / TK) * (tile16(cout) / 16) * 2 * 64 * sizeof(f16x8);
}

size_t train_abg_work_floats(long long rows, int cols) {
  return (size_t)((rows + kAbgRows - 1) / kAbgRows) * (cols + 1);
}

hipError_t launch_act_bias_grad(const float* y, const float* dy, long long rows, int cols, int act, float* dz, float* db,
                                float* dz_scale, float* work, hipStream_t st) {
  const long long nblk = (rows + kAbgRows - 1) / kAbgRows;
  if (nblk > INT32_MAX) return hipErrorInvalidValue;
  if (nblk == 0 && db) {
    const hipError_t e = hipMemsetAsync(db, 0, (size_t)cols * sizeof(float), st);
    if (e != hipSuccess) return e;
  }
  if (nblk > 0) {
    const bool vec = cols % 4 == 0 && (((uintptr_t)dy | (uintptr_t)y | (uintptr_t)dz) & 15) == 0;
    if (vec)
      hipLaunchKernelGGL(act_bias_grad_kernel<4>, dim3((unsigned)nblk), dim3(256), 0, st, y, dy, rows, cols, act, dz, work);
    else
      hipLaunchKernelGGL(act_bias_grad_kernel<1>, dim3((unsigned)nblk), dim3(256), 0, st, y, dy, rows, cols, act, dz, work);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if ((db && nblk > 0) || dz_scale) {  // (an empty tensor's scale: 1)
    hipLaunchKernelGGL(abg_reduce_kernel, dim3((unsigned)cols + 1), dim3(256), 0, st, work, (int)nblk, cols,
                       nblk > 0 ? db : nullptr, dz_scale);
    return hipGetLastError();
  }
  return hipSuccess;
}

hipError_t launch_conv_gather(const float* x, int n, int h, int w, int cin, const float* wt, int kh, int kw, int layout,
                              int stride, int pad_y, int pad_x, int transposed, const float* bias, const float* x_scale,
                              const float* w_scale, float* y, int oh, int ow, int cout, int act, void* work,
                              hipStream_t st) {
  GatherArgs a{};
  a.act = act;
  a.x = x; a.wp = (const f16x8*)work; a.bias = bias; a.y = y;
  a.sx = x_scale; a.sw = w_scale;
  a.n = n; a.h = h; a.w = w; a.cin = cin; a.oh = oh; a.ow = ow; a.cout = cout; a.kh = kh; a.kw = kw;
  a.stride = stride; a.pad_y = pad_y; a.pad_x = pad_x; a.transposed = transposed;
  a.K = kh * kw * cin;
  a.M = (long long)n * oh * ow;
  if (a.M == 0) return hipSuccess;
  const int ntt = tile16(cout) / 16, nchunk = (a.K + TK - 1) / TK;
  {
    const int total = nchunk * ntt * 64;
    hipLaunchKernelGGL(pack_w_kernel, dim3((total + 255) / 256), dim3(256), 0, st, wt, layout, cin, cout, a.K, ntt,
                       nchunk, w_scale, (f16x8*)work);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const bool vec = cin % TK == 0 && ((uintptr_t)x & 15) == 0;
  const bool ph = vec && transposed && stride == 2;
  if (ph) {  // blocks per output phase
    a.ph_blk[0] = 0;
    for (int p = 0; p < 4; ++p) {
      const long long qh = (oh - (p >> 1) + 1) / 2, qw = (ow - (p & 1) + 1) / 2;
      a.ph_blk[p + 1] = a.ph_blk[p] + (int)((n * qh * qw + GM - 1) / GM);
    }
    if (a.ph_blk[4] == 0) return hipSuccess;
  }
  switch (tile16(cout) | (vec ? 1 : 0) | (ph ? 2 : 0)) {
    case 16: return launch_gather_t<16, false, false>(a, st);
    case 17: return launch_gather_t<16, true, false>(a, st);
    case 19: return launch_gather_t<16, true, true>(a, st);
    case 32: return launch_gather_t<32, false, false>(a, st);
    case 33: return launch_gather_t<32, true, false>(a, st);
    case 35: return launch_gather_t<32, true, true>(a, st);
    case 64: return launch_gather_t<64, false, false>(a, st);
    case 65: return launch_gather_t<64, true, false>(a, st);
    default: return launch_gather_t<64, true, true>(a, st);
  }
}

size_t train_ssim_work_floats(int n, long long hw) { return (size_t)n * ((hw + kSsimPix - 1) / kSsimPix); }

hipError_t launch_ssim_map(const float* mx, const float* my, const float* sxy, const float* sxx, int n, long long hw,
                           float c1, float c2, float* out, float* work, hipStream_t st) {
  const long long bpi = (hw + kSsimPix - 1) / kSsimPix;
  if (n == 0) return hipSuccess;
  if (bpi * n > INT32_MAX || bpi > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ssim_map_kernel, dim3((unsigned)(bpi * n)), dim3(256), 0, st, mx, my, sxy, sxx, hw, (int)bpi, c1,
                     c2, work);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ssim_mean_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, work, n, (int)bpi, hw, out);
  return hipGetLastError();
}

hipError_t launch_ssim_map_grad(const float* mx, const float* my, const float* sxy, const float* sxx, const float* g,
                                int n, long long hw, float c1, float c2, float* gmx, float* gmy, float* gsxy,
                                float* gsxx, hipStream_t st) {
  const long long total = (long long)n * hw;
  if (total == 0) return hipSuccess;
  const long long blocks = (total + 255) / 256;
  hipLaunchKernelGGL(ssim_map_grad_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, st, mx, my,
                     sxy, sxx, g, n, hw, c1, c2, gmx, gmy, gsxy, gsxx);
  return hipGetLastError();
}

hipError_t launch_gauss1d(const float* in, int n, int hi, int wi, const float* taps, int nt, int vertical, int adjoint,
                          float* out, int ho, int wo, hipStream_t st) {
  const long long total = (long long)n * ho * wo;
  if (total == 0) return hipSuccess;
  const long long blocks = (total + 255) / 256;
  hipLaunchKernelGGL(gauss1d_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, st, in, n, hi,
                     wi, taps, nt, vertical, adjoint, out, ho, wo);
  return hipGetLastError();
}

// rows per block: 64 (one tap of a 64-channel gat, two of a 32-channel one) / 32 / 16 rows
// (all 25 taps of a one-channel gat)
static int wgrad_na(int taps, int ca) {
  const int rows = taps * ca;
  (void)taps;
  return rows > 32 ? 64 : rows > 16 ? 32 : 16;  // (two taps of 64 channels per block, NA 128: measured 35 % slower)
}

// slices so that row blocks x slices fills the chip about eight times over, each slice
// >= 4 chunks
static int wgrad_slices(long long U, int rowblocks) {
  long long want = (2048 + rowblocks - 1) / rowblocks;
  const long long maxs = (U + 4 * TK - 1) / (4 * TK);
  if (want > maxs) want = maxs;
  return (int)(want < 1 ? 1 : want);
}

size_t train_wgrad_work_floats(int n, int uh, int uw, int kh, int kw, int ca, int cb) {
  const long long U = (long long)n * uh * uw;
  const int rows = kh * kw * ca, na = wgrad_na(kh * kw, ca);
  return (size_t)wgrad_slices(U, (rows + na - 1) / na) * rows * cb;
}

hipError_t launch_conv_wgrad(const float* gat, int n, int gh, int gw, int ca, const float* dir, int uh, int uw, int cb,
                             int kh, int kw, int stride, int pad_y, int pad_x, const float* gat_scale,
                             const float* dir_scale, float* dw, float* work, hipStream_t st) {
  WgradArgs a{};
  a.gat = gat; a.dir = dir; a.sg = gat_scale; a.sd = dir_scale;
  a.part = work;
  a.n = n; a.gh = gh; a.gw = gw; a.ca = ca; a.uh = uh; a.uw = uw; a.cb = cb; a.kh = kh; a.kw = kw;
  a.stride = stride; a.pad_y = pad_y; a.pad_x = pad_x;
  a.U = (long long)n * uh * uw;
  const int taps = kh * kw;
  const long long nw = (long long)taps * ca * cb;
  if (nw == 0) return hipSuccess;
  if (a.U == 0) return hipMemsetAsync(dw, 0, nw * sizeof(float), st);
  a.rows = taps * ca;
  const int na = wgrad_na(taps, ca);
  const int slices = wgrad_slices(a.U, (a.rows + na - 1) / na);
  a.slice_len = (int)(((a.U + slices - 1) / slices + TK - 1) / TK * TK);
  hipError_t e;
  switch (na * 1000 + tile16(cb)) {
    case 16016: e = launch_wgrad_t<16, 16>(a, slices, st); break;
    case 16032: e = launch_wgrad_t<16, 32>(a, slices, st); break;
    case 16064: e = launch_wgrad_t<16, 64>(a, slices, st); break;
    case 32016: e = launch_wgrad_t<32, 16>(a, slices, st); break;
    case 32032: e = launch_wgrad_t<32, 32>(a, slices, st); break;
    case 32064: e = launch_wgrad_t<32, 64>(a, slices, st); break;
    case 64016: e = launch_wgrad_t<64, 16>(a, slices, st); break;
    case 64032: e = launch_wgrad_t<64, 32>(a, slices, st); break;
    default: e = launch_wgrad_t<64, 64>(a, slices, st); break;
  }
  if (e != hipSuccess) return e;
  const long long rb = (nw + 255) / 256;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(rb < 1024 ? rb : 1024)), dim3(256), 0, st, work, slices, nw, dw);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// tf.keras Adam (training.py:147-149 `optimizer.apply_gradients`; Keras' OptimizerV2 Adam calls
// TensorFlow's ResourceApplyAdam with use_nesterov = false) over many tensors in one launch.
// TF's ApplyAdam functor (training_ops, published algorithm; TF is not in the reference tree):
//   alpha = lr * sqrt(1 - beta2^t) / (1 - beta1^t)     (host, fp32, as Keras' iteration powers)
//   m += (g - m) * (1 - beta1);  v += (g * g - v) * (1 - beta2)
//   var -= (m * alpha) / (sqrt(v) + epsilon)
// every op an fp32 rounding in that order (no contraction: -ffp-contract=off; sqrt and the
// division correctly rounded, as NumPy's fp32 ops: the GPU test is bit-exact against them).  Block (x, k) updates elements [1024 x, 1024 x + 1024) of
// tensor k, then the same range one grid-width further on (n > max_n is covered), k's {var, m, v, grad, n} record is table[5k .. 5k+4].
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adam_keras_kernel(const long long* __restrict__ table, float alpha, float b1c,
                                                         float b2c, float eps) {
  const long long* r = table + 5 * blockIdx.y;
  float* var = (float*)r[0];
  float* m = (float*)r[1];
  float* v = (float*)r[2];
  const float* g = (const float*)r[3];
  const long long n = r[4];
  // grid-stride over the record: a record longer than the max_n that sized the grid is
  // still updated whole
  for (long long base = (long long)blockIdx.x * 1024; base < n; base += (long long)gridDim.x * 1024)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long i = base + k * 256 + threadIdx.x;
    if (i >= n) break;
    const float gi = g[i];
    const float mi = __fadd_rn(m[i], __fmul_rn(__fsub_rn(gi, m[i]), b1c));
    const float vi = __fadd_rn(v[i], __fmul_rn(__fsub_rn(__fmul_rn(gi, gi), v[i]), b2c));
    m[i] = mi;
    v[i] = vi;
    // sqrt correctly rounded: the f64 square root rounded to f32 (double rounding is exact for
    // sqrt at 53 >= 2 x 24 + 2 bits; v_sqrt_f32 alone is within 1 ulp, not correctly rounded)
    const float sv = (float)__dsqrt_rn((double)vi);
    var[i] = __fsub_rn(var[i], __fdiv_rn(__fmul_rn(mi, alpha), __fadd_rn(sv, eps)));
  }
}

hipError_t launch_adam_keras(const long long* table, int count, long long max_n, float alpha, float beta1,
                             float beta2, float eps, hipStream_t st) {
  if (count <= 0 || max_n <= 0) return hipSuccess;
  const long long bx = (max_n + 1023) / 1024;
  if (bx > INT32_MAX || count > 65535) return hipErrorInvalidValue;
  const float b1c = 1.0f - beta1, b2c = 1.0f - beta2;  // fp32, as T(1) - beta
  hipLaunchKernelGGL(adam_keras_kernel, dim3((unsigned)bx, (unsigned)count), dim3(256), 0, st, table, alpha, b1c, b2c,
                     eps);
  return hipGetLastError();
}

}  // namespace nic
