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
  const float* wt;     // [kh*kw][cin][cout] (layout 0) or [kh*kw][cout][cin] (layout 1)
  const float* bias;   // [cout] or null
  const float* sx;     // device scale of x (power of two) or null
  const float* sw;     // device scale of wt or null
  float* y;            // [n][oh][ow][cout]
  int n, h, w, cin, oh, ow, cout, kh, kw, stride, pad_y, pad_x, transposed, layout;
  int K;               // kh * kw * cin
  long long M;         // n * oh * ow
};

// source pixel of output pixel (b, oy, ox) at tap (ky, kx); -1 when outside / not on the grid
__device__ __forceinline__ long long gather_src(const GatherArgs& a, int b, int oy, int ox, int ky, int kx) {
  int iy, ix;
  if (a.transposed) {
    const int ty = oy + a.pad_y - ky, tx = ox + a.pad_x - kx;
    if (ty < 0 || tx < 0 || ty % a.stride || tx % a.stride) return -1;
    iy = ty / a.stride;
    ix = tx / a.stride;
  } else {
    iy = a.stride * oy + ky - a.pad_y;
    ix = a.stride * ox + kx - a.pad_x;
  }
  if ((unsigned)iy >= (unsigned)a.h || (unsigned)ix >= (unsigned)a.w) return -1;
  return ((long long)b * a.h + iy) * a.w + ix;
}

// NT = output channels per block (16, 32 or 64); VEC: cin % 32 == 0 (a K chunk is 32
// consecutive channels of one tap: two float4 per thread), else one element per (pixel, k)
template <int NT, bool VEC>
__global__ __launch_bounds__(256) void conv_gather_kernel(GatherArgs a) {
  __shared__ __attribute__((aligned(16))) _Float16 xs[2][GM * LP];  // [hi, lo][pixel][k]
  __shared__ __attribute__((aligned(16))) _Float16 ws[2][NT * LP];  // [hi, lo][co][k]
  constexpr int NTT = NT / 16;
  constexpr int XN = VEC ? 2 : 8;               // x elements (float4s when VEC) per thread per chunk
  constexpr int WN = NT * TK / 256;             // weight elements per thread per chunk
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const long long m0 = (long long)blockIdx.x * GM;
  const float sx = ld_scale(a.sx), sw = ld_scale(a.sw);
  const int nchunk = (a.K + TK - 1) / TK;
  // this thread's staging pixels: VEC px = tid/8 + 32 r; scalar px = tid/32 + 8 e
  int pb[XN], py[XN], pxx[XN];
#pragma unroll
  for (int e = 0; e < XN; ++e) {
    const int px = VEC ? (tid >> 3) + 32 * e : (tid >> 5) + 8 * e;
    const long long m = m0 + px;
    if (m < a.M) {
      const long long per = (long long)a.oh * a.ow;
      pb[e] = (int)(m / per);
      const int r = (int)(m - (long long)pb[e] * per);
      py[e] = r / a.ow;
      pxx[e] = r - py[e] * a.ow;
    } else {
      pb[e] = -1;
      py[e] = pxx[e] = 0;
    }
  }

  f32x4 xv[VEC ? XN : 1];
  float xsv[VEC ? 1 : XN];
  float wv[WN];
  auto load = [&](int c) {
    const int k0 = c * TK;
    if constexpr (VEC) {
      const int tap = k0 / a.cin, ci0 = k0 - tap * a.cin, ky = tap / a.kw, kx = tap - ky * a.kw;
#pragma unroll
      for (int e = 0; e < XN; ++e) {
        const long long s = pb[e] >= 0 ? gather_src(a, pb[e], py[e], pxx[e], ky, kx) : -1;
        xv[e] = s >= 0 ? *(const f32x4*)(a.x + s * a.cin + ci0 + 4 * (tid & 7)) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    } else {
      const int k = k0 + (tid & 31);
      const int tap = k / a.cin, ci = k - tap * a.cin, ky = tap / a.kw, kx = tap - ky * a.kw;
#pragma unroll
      for (int e = 0; e < XN; ++e) {
        const long long s = (pb[e] >= 0 && k < a.K) ? gather_src(a, pb[e], py[e], pxx[e], ky, kx) : -1;
        xsv[e] = s >= 0 ? a.x[s * a.cin + ci] : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < WN; ++e) {
      const int idx = tid + 256 * e;
      // layout 0: co fastest (contiguous in [tap][ci][co]); layout 1: k fastest ([tap][co][ci])
      const int co = a.layout ? idx / TK : idx % NT, kk = a.layout ? idx % TK : idx / NT;
      const int k = k0 + kk;
      float v = 0.f;
      if (co < a.cout && k < a.K) {
        const int tap = k / a.cin, ci = k - tap * a.cin;
        v = a.layout ? a.wt[((size_t)tap * a.cout + co) * a.cin + ci] : a.wt[((size_t)tap * a.cin + ci) * a.cout + co];
      }
      wv[e] = v;
    }
  };
  auto stage = [&]() {
    if constexpr (VEC) {
#pragma unroll
      for (int e = 0; e < XN; ++e) {
        const int px = (tid >> 3) + 32 * e, k = 4 * (tid & 7);
#pragma unroll
        for (int r = 0; r < 4; ++r) split1(xv[e][r] * sx, xs[0][px * LP + k + r], xs[1][px * LP + k + r]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < XN; ++e) {
        const int px = (tid >> 5) + 8 * e, k = tid & 31;
        split1(xsv[e] * sx, xs[0][px * LP + k], xs[1][px * LP + k]);
      }
    }
#pragma unroll
    for (int e = 0; e < WN; ++e) {
      const int idx = tid + 256 * e;
      const int co = a.layout ? idx / TK : idx % NT, kk = a.layout ? idx % TK : idx / NT;
      split1(wv[e] * sw, ws[0][co * LP + kk], ws[1][co * LP + kk]);
    }
  };

  f32x4 acc[NTT];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int c = 0; c < nchunk; ++c) {
    __syncthreads();  // every wave is done with the previous chunk's tiles
    stage();
    __syncthreads();
    if (c + 1 < nchunk) load(c + 1);  // in flight during this chunk's MFMAs
    const int bo = (wave * 16 + l16) * LP + 8 * g;
    const f16x8 bh = *(const f16x8*)&xs[0][bo], bl = *(const f16x8*)&xs[1][bo];
#pragma unroll
    for (int t = 0; t < NTT; ++t) {
      const int ao = (t * 16 + l16) * LP + 8 * g;
      const f16x8 ah = *(const f16x8*)&ws[0][ao], al = *(const f16x8*)&ws[1][ao];
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[t], 0, 0, 0);
    }
  }
  // D[co = 16t + 4g + r][pixel 16 wave + l16]
  const long long m = m0 + wave * 16 + l16;
  if (m >= a.M) return;
  const float isx = 1.0f / sx, isw = 1.0f / sw;  // exact: powers of two (applied one at a time)
  float* yp = a.y + m * a.cout;
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    const int co = t * 16 + 4 * g;
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (acc[t][r] * isx) * isw + (a.bias && co + r < a.cout ? a.bias[co + r] : 0.f);
    if ((a.cout & 3) == 0 && co + 4 <= a.cout) {
      *(f32x4*)(yp + co) = v;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (co + r < a.cout) yp[co + r] = v[r];
    }
  }
}

// ---- weight-gradient GEMM ------------------------------------------------------------------
struct WgradArgs {
  const float* gat;   // [n][gh][gw][ca], read at s*u + k - pad
  const float* dir;   // [n][uh][uw][cb]
  const float* sg;    // device scales or null
  const float* sd;
  float* part;        // [slices][taps][ca][cb]
  int n, gh, gw, ca, uh, uw, cb, kh, kw, stride, pad_y, pad_x;
  long long U;        // n * uh * uw
  int slice_len;      // pixels per slice (multiple of TK)
};

// NA, NB = channel tiles (16, 32, 64) >= ca, cb.  Block (tap, slice); wave w owns the
// (a, b) 16 x 16 output tiles w, w + 4, ...
template <int NA, int NB>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) _Float16 gs[2][NA * LP];  // [hi, lo][a][u]
  __shared__ __attribute__((aligned(16))) _Float16 ds[2][NB * LP];  // [hi, lo][b][u]
  constexpr int NTA = NA / 16, NTB = NB / 16, NTILE = NTA * NTB, TPW = (NTILE + 3) / 4;
  constexpr int GE = (TK * NA + 255) / 256, DE = (TK * NB + 255) / 256;  // elements per thread
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int tap = blockIdx.x, slice = blockIdx.y, ky = tap / a.kw, kx = tap - ky * a.kw;
  const long long u0 = (long long)slice * a.slice_len;
  const long long u1 = u0 + a.slice_len < a.U ? u0 + a.slice_len : a.U;
  const float sg = ld_scale(a.sg), sd = ld_scale(a.sd);
  const long long per = (long long)a.uh * a.uw;

  float gv[GE], dv[DE];
  auto load = [&](long long ub) {
#pragma unroll
    for (int e = 0; e < GE; ++e) {  // element (u = idx / NA, channel idx % NA): channels fastest
      const int idx = tid + 256 * e, ul = idx / NA, ch = idx % NA;
      const long long u = ub + ul;
      float v = 0.f;
      if (idx < TK * NA && ch < a.ca && u < u1) {
        const int b = (int)(u / per), r = (int)(u - (long long)b * per), uy = r / a.uw, ux = r - uy * a.uw;
        const int iy = a.stride * uy + ky - a.pad_y, ix = a.stride * ux + kx - a.pad_x;
        if ((unsigned)iy < (unsigned)a.gh && (unsigned)ix < (unsigned)a.gw)
          v = a.gat[(((size_t)b * a.gh + iy) * a.gw + ix) * a.ca + ch];
      }
      gv[e] = v;
    }
#pragma unroll
    for (int e = 0; e < DE; ++e) {
      const int idx = tid + 256 * e, ul = idx / NB, ch = idx % NB;
      const long long u = ub + ul;
      dv[e] = (idx < TK * NB && ch < a.cb && u < u1) ? a.dir[u * a.cb + ch] : 0.f;
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int e = 0; e < GE; ++e) {
      const int idx = tid + 256 * e;
      if (idx < TK * NA) split1(gv[e] * sg, gs[0][(idx % NA) * LP + idx / NA], gs[1][(idx % NA) * LP + idx / NA]);
    }
#pragma unroll
    for (int e = 0; e < DE; ++e) {
      const int idx = tid + 256 * e;
      if (idx < TK * NB) split1(dv[e] * sd, ds[0][(idx % NB) * LP + idx / NB], ds[1][(idx % NB) * LP + idx / NB]);
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
  const int taps = a.kh * a.kw;
  float* out = a.part + ((size_t)slice * taps + tap) * a.ca * a.cb;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + 4 * j;
    if (t >= NTILE) break;
    const int ta = t / NTB, tb = t - ta * NTB, bcol = tb * 16 + l16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int arow = ta * 16 + 4 * g + r;
      if (arow < a.ca && bcol < a.cb) out[(size_t)arow * a.cb + bcol] = (acc[j][r] * isg) * isd;
    }
  }
}

// dw[i] = sum over slices of part[s][i], in slice order
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int slices, long long nw,
                                                           float* __restrict__ dw) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nw; i += (long long)gridDim.x * 256) {
    float s = 0.f;
    for (int k = 0; k < slices; ++k) s += part[(size_t)k * nw + i];
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

template <int NT, bool VEC>
hipError_t launch_gather_t(const GatherArgs& a, hipStream_t st) {
  const long long blocks = (a.M + GM - 1) / GM;
  hipLaunchKernelGGL((conv_gather_kernel<NT, VEC>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <int NA, int NB>
hipError_t launch_wgrad_t(const WgradArgs& a, int slices, hipStream_t st) {
  hipLaunchKernelGGL((conv_wgrad_kernel<NA, NB>), dim3(a.kh * a.kw, slices), dim3(256), 0, st, a);
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

hipError_t launch_conv_gather(const float* x, int n, int h, int w, int cin, const float* wt, int kh, int kw, int layout,
                              int stride, int pad_y, int pad_x, int transposed, const float* bias, const float* scales,
                              float* y, int oh, int ow, int cout, hipStream_t st) {
  GatherArgs a{};
  a.x = x; a.wt = wt; a.bias = bias; a.y = y;
  a.sx = scales; a.sw = scales ? scales + 1 : nullptr;
  a.n = n; a.h = h; a.w = w; a.cin = cin; a.oh = oh; a.ow = ow; a.cout = cout; a.kh = kh; a.kw = kw;
  a.stride = stride; a.pad_y = pad_y; a.pad_x = pad_x; a.transposed = transposed; a.layout = layout;
  a.K = kh * kw * cin;
  a.M = (long long)n * oh * ow;
  if (a.M == 0) return hipSuccess;
  const bool vec = cin % TK == 0 && ((uintptr_t)x & 15) == 0;
  switch (tile16(cout) | (vec ? 1 : 0)) {
    case 16: return launch_gather_t<16, false>(a, st);
    case 17: return launch_gather_t<16, true>(a, st);
    case 32: return launch_gather_t<32, false>(a, st);
    case 33: return launch_gather_t<32, true>(a, st);
    case 64: return launch_gather_t<64, false>(a, st);
    default: return launch_gather_t<64, true>(a, st);
  }
}

// slices so that taps x slices fills the chip several times over, each slice >= 4 chunks
static int wgrad_slices(long long U, int taps) {
  long long want = (2048 + taps - 1) / taps;
  const long long maxs = (U + 4 * TK - 1) / (4 * TK);
  if (want > maxs) want = maxs;
  return (int)(want < 1 ? 1 : want);
}

size_t train_wgrad_work_floats(int n, int uh, int uw, int kh, int kw, int ca, int cb) {
  const long long U = (long long)n * uh * uw;
  return (size_t)wgrad_slices(U, kh * kw) * kh * kw * ca * cb;
}

hipError_t launch_conv_wgrad(const float* gat, int n, int gh, int gw, int ca, const float* dir, int uh, int uw, int cb,
                             int kh, int kw, int stride, int pad_y, int pad_x, const float* scales, float* dw,
                             float* work, hipStream_t st) {
  WgradArgs a{};
  a.gat = gat; a.dir = dir; a.sg = scales; a.sd = scales ? scales + 1 : nullptr;
  a.part = work;
  a.n = n; a.gh = gh; a.gw = gw; a.ca = ca; a.uh = uh; a.uw = uw; a.cb = cb; a.kh = kh; a.kw = kw;
  a.stride = stride; a.pad_y = pad_y; a.pad_x = pad_x;
  a.U = (long long)n * uh * uw;
  const int taps = kh * kw;
  const long long nw = (long long)taps * ca * cb;
  if (nw == 0) return hipSuccess;
  if (a.U == 0) return hipMemsetAsync(dw, 0, nw * sizeof(float), st);
  const int slices = wgrad_slices(a.U, taps);
  a.slice_len = (int)(((a.U + slices - 1) / slices + TK - 1) / TK * TK);
  hipError_t e;
  switch (tile16(ca) * 100 + tile16(cb)) {
    case 1616: e = launch_wgrad_t<16, 16>(a, slices, st); break;
    case 1632: e = launch_wgrad_t<16, 32>(a, slices, st); break;
    case 1664: e = launch_wgrad_t<16, 64>(a, slices, st); break;
    case 3216: e = launch_wgrad_t<32, 16>(a, slices, st); break;
    case 3232: e = launch_wgrad_t<32, 32>(a, slices, st); break;
    case 3264: e = launch_wgrad_t<32, 64>(a, slices, st); break;
    case 6416: e = launch_wgrad_t<64, 16>(a, slices, st); break;
    case 6432: e = launch_wgrad_t<64, 32>(a, slices, st); break;
    default: e = launch_wgrad_t<64, 64>(a, slices, st); break;
  }
  if (e != hipSuccess) return e;
  const long long rb = (nw + 255) / 256;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(rb < 1024 ? rb : 1024)), dim3(256), 0, st, work, slices, nw, dw);
  return hipGetLastError();
}

}  // namespace nic
