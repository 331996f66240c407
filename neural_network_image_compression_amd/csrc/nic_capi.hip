// C-ABI of the codec hot path (declared in include/nic.h): context, Keras-layout weight
// upload + repack to the kernels' fragment layouts, and the encode / decode pipelines.
//
// Pipeline per call (P = 3N planes, Y planes first, then Cb, then Cr):
//   encode: conv1+colour (rgb u8 -> R0) -> conv2 (R0 -> R1) -> conv3 (R1 -> R2)
//           -> conv4 + res (R2, R1 -> R3) -> conv8 + clip + quantise (R3 -> latent u8)
//   decode: dconv1 + dequantise (latent u8 -> R1) -> dconv5 (R1 -> R2)
//           -> dconv6 + res (R2, R1 -> R3) -> dconv7 (R3 -> R0)
//           -> dconv8 + inverse colour + quantise (R0 -> rgb u8)
// mirroring BaseEncoder.call (encoder.py:19-32) / BaseDecoder.call (decoder.py:19-32).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nic.h"
#include "nic_kernels.h"

using namespace nic;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace

// the thread's error message for the C-ABI entry points outside this file (nic_png.cpp)
int nic::set_error(int code, const char* msg) { return fail(code, "%s", msg); }

namespace {

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) return fail(NIC_EHIP, "%s: %s", #expr, hipGetErrorString(_e));     \
  } while (0)

struct LayerSpec {
  const char* name;
  int k, s, cin, cout;
  bool transposed;
  LayerId id;
};

// encoder.py:10-17, decoder.py:10-17
const LayerSpec kEnc[5] = {
    {"conv1", 5, 2, 1, 32, false, L_CONV1},  {"conv2", 5, 2, 32, 64, false, L_CONV2},
    {"conv3", 3, 1, 64, 64, false, L_CONV3}, {"conv4", 3, 1, 64, 64, false, L_CONV4},
    {"conv8", 5, 2, 64, 32, false, L_CONV8},
};
const LayerSpec kDec[5] = {
    {"dconv1", 5, 2, 32, 64, true, L_DCONV1}, {"dconv5", 3, 1, 64, 64, true, L_DCONV5},
    {"dconv6", 3, 1, 64, 64, true, L_DCONV6}, {"dconv7", 5, 2, 64, 64, true, L_DCONV7},
    {"dconv8", 5, 2, 64, 1, true, L_DCONV8},
};

// device floats per model for a layer's repacked kernel
size_t packed_kernel_floats(const LayerSpec& L) {
  if (L.id == L_CONV1) return 26 * 32;
  if (L.id == L_DCONV8) return 25 * 64;
  return (size_t)L.k * L.k * L.cin * L.cout;
}

// Forward-conv fragment order: Wr[tap][q][h][co][r] with ci = 8q + 4h + r.
// get(tap, ci, co) returns the weight multiplying input channel ci for output co at tap.
template <class F>
void repack_fragments(std::vector<float>& out, int taps, int cin, int cout, F get) {
  out.assign((size_t)taps * cin * cout, 0.f);
  for (int t = 0; t < taps; ++t)
    for (int q = 0; q < cin / 8; ++q)
      for (int h = 0; h < 2; ++h)
        for (int co = 0; co < cout; ++co)
          for (int r = 0; r < 4; ++r) {
            const int ci = 8 * q + 4 * h + r;
            out[((((size_t)t * (cin / 8) + q) * 2 + h) * cout + co) * 4 + r] = get(t, ci, co);
          }
}

// Split-f16 fragment order: Wx[tap][s][hl][h][co][j] with ci = 16s + 8h + j, holding
// hi = f16(w*2^k) (hl = 0) and lo = f16(w*2^k - hi) (hl = 1).  2^k is chosen per model so
// that max|w*2^k| < 2^15: hi and lo stay normal f16 numbers.  Returns k.
template <class F>
int repack_x3(std::vector<uint16_t>& out, int taps, int cin, int cout, F get) {
  float maxabs = 0.f;
  for (int t = 0; t < taps; ++t)
    for (int ci = 0; ci < cin; ++ci)
      for (int co = 0; co < cout; ++co) maxabs = std::max(maxabs, std::fabs(get(t, ci, co)));
  int k = 0;
  if (maxabs > 0.f && std::isfinite(maxabs)) {
    int e = 0;
    std::frexp(maxabs, &e);  // maxabs = m * 2^e, m in [0.5, 1)
    k = std::min(std::max(15 - e, -100), 100);
  }
  out.assign((size_t)taps * cin * cout * 2, 0);
  for (int t = 0; t < taps; ++t)
    for (int s = 0; s < cin / 16; ++s)
      for (int h = 0; h < 2; ++h)
        for (int co = 0; co < cout; ++co)
          for (int j = 0; j < 8; ++j) {
            const int ci = 16 * s + 8 * h + j;
            const float w = std::ldexp(get(t, ci, co), k);
            const _Float16 hi = (_Float16)w;
            const _Float16 lo = (_Float16)(w - (float)hi);
            const size_t base = ((((size_t)t * (cin / 16) + s) * 2) * 2 + h) * cout * 8;
            std::memcpy(&out[base + (size_t)co * 8 + j], &hi, 2);
            std::memcpy(&out[base + (size_t)2 * cout * 8 + (size_t)co * 8 + j], &lo, 2);
          }
  return k;
}

// Phase-major tap enumeration of a k5 s2 Conv2DTranspose: for phase (py, px) and
// halo offsets (iy, ix), the kernel tap is (py + 3 - 2*iy, px + 3 - 2*ix).
template <class F>
void for_each_phase_tap(F f) {
  int t = 0;
  for (int ph = 0; ph < 4; ++ph) {
    const int py = ph >> 1, px = ph & 1, ny = py ? 3 : 2, nx = px ? 3 : 2;
    for (int iy = 0; iy < ny; ++iy)
      for (int ix = 0; ix < nx; ++ix) f(t++, py + 3 - 2 * iy, px + 3 - 2 * ix);
  }
}

// Repack a Keras-layout kernel for the fp32 path (out) and, for the MFMA layers with
// Cin >= 32, the split-f16 path (outx, returns the scale exponent k; -1000 if none).
int repack_kernel(const LayerSpec& L, const float* K, std::vector<float>& out, std::vector<uint16_t>& outx) {
  const int k = L.k, cin = L.cin, cout = L.cout;
  outx.clear();
  if (L.id == L_CONV1) {  // HWIO (5,5,1,32) -> [26][32], tap 25 = 0
    out.assign(26 * 32, 0.f);
    for (int t = 0; t < 25; ++t)
      for (int co = 0; co < 32; ++co) out[t * 32 + co] = K[t * 32 + co];
    // split-f16 MFMA A fragments of the fused conv1 (v_mfma_f32_16x16x32_f16): [co tile ct]
    // [hi,lo][lane][j], lane l holds row co = 16ct + (l & 15) and k = 8 (l >> 4) + j, where
    // k = 2 * pair + e, pair = kh * 3 + kw / 2, kw = 2 (pair % 3) + e (zero for kw = 5 and
    // pair >= 15: 25 taps in 32 slots), scaled by 2^k so every value is a normal f16 pair
    float maxabs = 0.f;
    for (int i = 0; i < 25 * 32; ++i) maxabs = std::max(maxabs, std::fabs(K[i]));
    int kexp = 0;
    if (maxabs > 0.f && std::isfinite(maxabs)) {
      int e = 0;
      std::frexp(maxabs, &e);
      kexp = std::min(std::max(15 - e, -100), 100);
    }
    outx.assign((size_t)2 * 2 * 64 * 8, 0);
    for (int ct = 0; ct < 2; ++ct)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int kk = 8 * (lane >> 4) + j, pr = kk >> 1, kh = pr / 3, kw = 2 * (pr % 3) + (kk & 1);
          const int co = 16 * ct + (lane & 15);
          if (pr >= 15 || kw >= 5) continue;
          const float w = std::ldexp(K[(kh * 5 + kw) * 32 + co], kexp);
          const _Float16 hi = (_Float16)w;
          const _Float16 lo = (_Float16)(w - (float)hi);
          std::memcpy(&outx[(((size_t)ct * 2 + 0) * 64 + lane) * 8 + j], &hi, 2);
          std::memcpy(&outx[(((size_t)ct * 2 + 1) * 64 + lane) * 8 + j], &lo, 2);
        }
    return kexp;
  }
  if (L.id == L_DCONV8) {  // (5,5,1,64) (kh,kw,Cout,Cin) -> [25 phase taps][64]
    out.assign(25 * 64, 0.f);
    for_each_phase_tap([&](int t, int ky, int kx) {
      for (int ci = 0; ci < 64; ++ci) out[t * 64 + ci] = K[((size_t)(ky * 5 + kx) * 1 + 0) * 64 + ci];
    });
    // split-f16 MFMA A fragments [nbr d=(iy,ix)][chunk c][hi,lo][lane][j]: lane l holds row
    // l&15 (= phase (py,px) when < 4) and channels 32c + 8*(l>>4) + j.  Phase (py,px) uses
    // halo row offset iy iff iy < 2 + py (kernel row py + 3 - 2*iy), likewise ix.
    float maxabs = 0.f;
    for (int i = 0; i < 25 * 64; ++i) maxabs = std::max(maxabs, std::fabs(K[i]));
    int kexp = 0;
    if (maxabs > 0.f && std::isfinite(maxabs)) {
      int e = 0;
      std::frexp(maxabs, &e);
      kexp = std::min(std::max(15 - e, -100), 100);
    }
    outx.assign((size_t)9 * 2 * 2 * 64 * 8, 0);
    for (int d = 0; d < 9; ++d) {
      const int iy = d / 3, ix = d % 3;
      for (int c = 0; c < 2; ++c)
        for (int lane = 0; lane < 64; ++lane) {
          const int row = lane & 15, kg = lane >> 4;
          if (row >= 4) continue;
          const int py = row >> 1, px = row & 1;
          if (iy >= 2 + py || ix >= 2 + px) continue;
          const int ky = py + 3 - 2 * iy, kx = px + 3 - 2 * ix;
          for (int j = 0; j < 8; ++j) {
            const int ci = 32 * c + 8 * kg + j;
            const float w = std::ldexp(K[(size_t)(ky * 5 + kx) * 64 + ci], kexp);
            const _Float16 hi = (_Float16)w;
            const _Float16 lo = (_Float16)(w - (float)hi);
            std::memcpy(&outx[((((size_t)d * 2 + c) * 2 + 0) * 64 + lane) * 8 + j], &hi, 2);
            std::memcpy(&outx[((((size_t)d * 2 + c) * 2 + 1) * 64 + lane) * 8 + j], &lo, 2);
          }
        }
    }
    return kexp;
  }
  if (!L.transposed) {  // HWIO
    auto get = [&](int t, int ci, int co) { return K[((size_t)t * cin + ci) * cout + co]; };
    repack_fragments(out, k * k, cin, cout, get);
    return repack_x3(outx, k * k, cin, cout, get);
  }
  if (L.s == 1) {  // transposed k3 s1 == conv with flipped taps, swapped channels
    auto get = [&](int t, int ci, int co) {
      const int u = t / k, v = t % k;
      const int ky = k - 1 - u, kx = k - 1 - v;
      return K[(((size_t)ky * k + kx) * cout + co) * cin + ci];
    };
    repack_fragments(out, k * k, cin, cout, get);
    return repack_x3(outx, k * k, cin, cout, get);
  }
  // transposed k5 s2, phase-major taps
  std::vector<int> tap_ky(25), tap_kx(25);
  for_each_phase_tap([&](int t, int ky, int kx) {
    tap_ky[t] = ky;
    tap_kx[t] = kx;
  });
  auto get = [&](int t, int ci, int co) { return K[(((size_t)tap_ky[t] * 5 + tap_kx[t]) * cout + co) * cin + ci]; };
  repack_fragments(out, 25, cin, cout, get);
  return repack_x3(outx, 25, cin, cout, get);
}

struct SamePad {
  int out, lo;
};
SamePad same_pad(int n, int k, int s) {
  const int out = (n + s - 1) / s;
  const int pad = std::max((out - 1) * s + k - n, 0);
  return {out, pad / 2};
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

constexpr int kHostMaxChunks = 16;

struct nic_ctx {
  int device = 0;
  float* wk[L_COUNT] = {};  // [2 models][packed kernel]
  float* wb[L_COUNT] = {};  // [2 models][cout]
  uint16_t* wx[L_COUNT] = {};  // split-f16 kernels [2 models][taps*cin*cout*2]
  float wscale[L_COUNT][2] = {};  // 2^-k per model for the split-f16 kernels
  // dconv8 as the B operand of dconv7's fused projection: [2 models][2 tap blocks][2 k32][hi,lo][64][8]
  uint16_t* wproj = nullptr;
  int precision = NIC_PRECISION_F16X3;
  // f16 range guard (nic.h NIC_RANGE_*): device words [flag, re-run count, the chained
  // re-run's grid barrier (arrivals, generation, timeout flag)], the epoch of the
  // latest split-f16 pass, the policy, a pinned host word for the ERROR policy's check
  int* range = nullptr;
  int* range_host = nullptr;
  int epoch = 0;
  int range_policy = NIC_RANGE_FALLBACK;
  long long error_trips = 0;
  char* zero16 = nullptr;  // 256 zero bytes: DMA source for halo padding
  bool have_k[4][5] = {};
  bool have_b[4][5] = {};
  char* ws = nullptr;
  size_t ws_bytes = 0;
  uint32_t* counts = nullptr;
  size_t counts_bytes = 0;
  // set only inside nic_encode_entropy: conv8's folded-histogram counts (fold_acc, [3n][256],
  // zero between calls: the reduce clears what it reads)
  uint32_t* fold_part = nullptr;
  uint32_t* fold_acc = nullptr;
  size_t fold_acc_bytes = 0;
  char* qs = nullptr;  // MS-SSIM scratch (pooled scales + tile sums), grown on demand
  size_t qs_bytes = 0;
  // optional per-layer HIP-event timing (nic_set_timing): one event pair per layer and
  // call, read back and accumulated by nic_layer_times
  // host-array surface (nic_encode_host / nic_decode_host): its own copy-in, compute and
  // copy-out streams, per-chunk events, pinned staging and device buffers, grown on demand
  hipStream_t hs[3] = {};  // H2D, compute, D2H
  hipEvent_t hev[3][kHostMaxChunks] = {};
  hipEvent_t hev_caller = nullptr;
  uint8_t* pin_in = nullptr;
  uint8_t* pin_out = nullptr;
  size_t pin_in_bytes = 0, pin_out_bytes = 0;
  uint8_t* hdev = nullptr;
  size_t hdev_bytes = 0;
  bool timing = false;
  hipEvent_t ev[L_COUNT][2] = {};
  bool ev_pending[L_COUNT] = {};
  double ms_sum[L_COUNT] = {};
  long launches[L_COUNT] = {};
};

namespace {

const LayerSpec* find_layer(int model_id, const char* name, int* index) {
  const LayerSpec* tab = model_id < 2 ? kEnc : kDec;
  for (int i = 0; i < 5; ++i)
    if (std::strcmp(tab[i].name, name) == 0) {
      *index = i;
      return &tab[i];
    }
  return nullptr;
}

int ensure_ws(nic_ctx* c, size_t bytes) {
  if (bytes <= c->ws_bytes) return NIC_OK;
  if (c->ws) HIP_TRY(hipFree(c->ws));
  c->ws = nullptr;
  c->ws_bytes = 0;
  if (hipMalloc(&c->ws, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return fail(NIC_ENOMEM, "workspace allocation of %zu bytes failed", bytes);
  }
  c->ws_bytes = bytes;
  return NIC_OK;
}

struct EncGeom {
  SamePad c1y, c1x, c2y, c2x, c8y, c8x;
  size_t r0, r123;  // floats per region
};
EncGeom enc_geom(int n, int h, int w) {
  EncGeom g;
  g.c1y = same_pad(h, 5, 2);
  g.c1x = same_pad(w, 5, 2);
  g.c2y = same_pad(g.c1y.out, 5, 2);
  g.c2x = same_pad(g.c1x.out, 5, 2);
  g.c8y = same_pad(g.c2y.out, 5, 2);
  g.c8x = same_pad(g.c2x.out, 5, 2);
  const size_t P = 3 * (size_t)n;
  // R0: conv1's output, or (conv1 fused into conv2) the padded split colour planes
  int oy, ox, hp, wp;
  c12_plane_geom(g.c2y.out, g.c2x.out, g.c2y.lo, g.c2x.lo, g.c1y.lo, g.c1x.lo, &oy, &ox, &hp, &wp);
  g.r0 = std::max(P * g.c1y.out * g.c1x.out * 32, (2 * P * (size_t)hp * wp + 1) / 2);
  g.r123 = P * g.c2y.out * g.c2x.out * 64;
  return g;
}
struct DecGeom {
  size_t r0, r123;
};
DecGeom dec_geom(int n, int h8, int w8) {
  const size_t P = 3 * (size_t)n;
  // R0: dconv7's output, or its dconv8 projections ([P][4 phases][8x8 tiles of the
  // 2h8 x 2w8 coarse grid][25][64] floats, launch_dconv7_proj_x3)
  const size_t t7 = (size_t)((2 * h8 + 7) / 8) * ((2 * w8 + 7) / 8);
  const size_t r0 = std::max(P * (4 * (size_t)h8) * (4 * (size_t)w8) * 64, P * 4 * t7 * 25 * 64);
  return {r0, P * (2 * (size_t)h8) * (2 * (size_t)w8) * 64};
}
constexpr size_t kProjFrag = 2 * 2 * 2 * 64 * 8;  // u16 per model in nic_ctx::wproj

// dconv8's phase-tap kernel [25][64] (fp32 repack) as split-f16 B fragments of the
// projection MFMA: lane l of (tap block nt, k32-step ks) holds column tap 16 nt + (l & 15)
// and rows ci = 32 ks + 8 (l >> 4) + j, scaled by 2^kexp (zero for taps >= 25)
std::vector<uint16_t> proj_fragments(const std::vector<float>& w25, int kexp) {
  std::vector<uint16_t> f(kProjFrag, 0);
  for (int nt = 0; nt < 2; ++nt)
    for (int ks = 0; ks < 2; ++ks)
      for (int lane = 0; lane < 64; ++lane) {
        const int tap = 16 * nt + (lane & 15);
        if (tap >= 25) continue;
        for (int j = 0; j < 8; ++j) {
          const float w = std::ldexp(w25[(size_t)tap * 64 + 32 * ks + 8 * (lane >> 4) + j], kexp);
          const _Float16 hi = (_Float16)w;
          const _Float16 lo = (_Float16)(w - (float)hi);
          std::memcpy(&f[((((size_t)nt * 2 + ks) * 2 + 0) * 64 + lane) * 8 + j], &hi, 2);
          std::memcpy(&f[((((size_t)nt * 2 + ks) * 2 + 1) * 64 + lane) * 8 + j], &lo, 2);
        }
      }
  return f;
}
size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

int ensure_regions(nic_ctx* c, size_t r0, size_t r123, float** R) {
  const size_t b0 = align_up(r0 * 4), b1 = align_up(r123 * 4);
  int rc = ensure_ws(c, b0 + 3 * b1);
  if (rc) return rc;
  R[0] = (float*)c->ws;
  R[1] = (float*)(c->ws + b0);
  R[2] = (float*)(c->ws + b0 + b1);
  R[3] = (float*)(c->ws + b0 + 2 * b1);
  return NIC_OK;
}

// Collect a finished event pair of layer id into the running sums.
int collect_layer(nic_ctx* c, int id) {
  if (!c->ev_pending[id]) return NIC_OK;
  HIP_TRY(hipEventSynchronize(c->ev[id][1]));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, c->ev[id][0], c->ev[id][1]));
  c->ms_sum[id] += ms;
  c->launches[id] += 1;
  c->ev_pending[id] = false;
  return NIC_OK;
}

// Bracket one launch with the layer's event pair when timing is on.
struct LayerTimer {
  nic_ctx* c;
  int id;
  hipStream_t st;
  int rc = NIC_OK;
  LayerTimer(nic_ctx* c_, int id_, hipStream_t st_) : c(c_), id(id_), st(st_) {
    if (!c->timing) return;
    rc = collect_layer(c, id);  // previous call's pair must be read before reuse
    if (rc == NIC_OK && hipEventRecord(c->ev[id][0], st) != hipSuccess) rc = fail(NIC_EHIP, "hipEventRecord");
  }
  int done() {
    if (!c->timing || rc) return rc;
    if (hipEventRecord(c->ev[id][1], st) != hipSuccess) return fail(NIC_EHIP, "hipEventRecord");
    c->ev_pending[id] = true;
    return NIC_OK;
  }
};

#define TIMED(layer, launch_expr)                  \
  do {                                             \
    LayerTimer _t(c, layer, st);                   \
    if (_t.rc) return _t.rc;                       \
    HIP_TRY(launch_expr);                          \
    int _rc = _t.done();                           \
    if (_rc) return _rc;                           \
  } while (0)

bool models_ready(const nic_ctx* c, int m0) {
  for (int m = m0; m < m0 + 2; ++m)
    for (int i = 0; i < 5; ++i)
      if (!c->have_k[m][i] || !c->have_b[m][i]) return false;
  return true;
}

}  // namespace

extern "C" {

int nic_version(void) { return 200; }

int nic_constants(float* ycbcr9, float* ycbcr_inv9, float* off3) {
  // host copy of what nic_create uploads; lets tests compare with np.linalg.inv (utils.py:8)
  const double K[9] = {0.299, 0.587, 0.114, -0.16874, -0.33126, 0.5, 0.5, -0.41869, -0.08131};
  const double det = K[0] * (K[4] * K[8] - K[5] * K[7]) - K[1] * (K[3] * K[8] - K[5] * K[6]) +
                     K[2] * (K[3] * K[7] - K[4] * K[6]);
  const double inv[9] = {(K[4] * K[8] - K[5] * K[7]) / det, (K[2] * K[7] - K[1] * K[8]) / det,
                         (K[1] * K[5] - K[2] * K[4]) / det, (K[5] * K[6] - K[3] * K[8]) / det,
                         (K[0] * K[8] - K[2] * K[6]) / det, (K[2] * K[3] - K[0] * K[5]) / det,
                         (K[3] * K[7] - K[4] * K[6]) / det, (K[1] * K[6] - K[0] * K[7]) / det,
                         (K[0] * K[4] - K[1] * K[3]) / det};
  for (int i = 0; i < 9; ++i) {
    if (ycbcr9) ycbcr9[i] = (float)K[i];
    if (ycbcr_inv9) ycbcr_inv9[i] = (float)inv[i];
  }
  if (off3) {
    off3[0] = 0.0f;
    off3[1] = 0.5f;
    off3[2] = 0.5f;
  }
  return NIC_OK;
}

const char* nic_last_error(void) { return g_err.c_str(); }

int nic_create(int device, nic_ctx** out) {
  if (!out) return fail(NIC_EINVAL, "nic_create: out is NULL");
  *out = nullptr;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(NIC_EINVAL, "nic_create: device %d out of range [0,%d)", device, ndev);
  DeviceGuard guard(device);
  nic_ctx* c = new nic_ctx();
  c->device = device;
  for (int half = 0; half < 2; ++half) {
    const LayerSpec* tab = half ? kDec : kEnc;
    for (int i = 0; i < 5; ++i) {
      const LayerSpec& L = tab[i];
      const size_t kb = 2 * packed_kernel_floats(L) * sizeof(float), bb = 2 * L.cout * sizeof(float);
      // split-f16 fragments: dconv8 [2][9][2][2][64][8], conv1 [2][2][2][64][8], else as wk
      const size_t xb = L.id == L_DCONV8 ? 2 * 9 * 2 * 2 * 64 * 16 : L.id == L_CONV1 ? 2 * 2 * 2 * 64 * 16 : kb;
      if (hipMalloc(&c->wk[L.id], kb) != hipSuccess || hipMalloc(&c->wb[L.id], bb) != hipSuccess ||
          hipMalloc(&c->wx[L.id], xb) != hipSuccess) {
        nic_destroy(c);
        return fail(NIC_ENOMEM, "nic_create: weight allocation failed");
      }
      (void)hipMemset(c->wk[L.id], 0, kb);
      (void)hipMemset(c->wb[L.id], 0, bb);
      (void)hipMemset(c->wx[L.id], 0, xb);
      c->wscale[L.id][0] = c->wscale[L.id][1] = 1.0f;
    }
  }
  if (hipMalloc(&c->wproj, 2 * kProjFrag * 2) != hipSuccess || hipMemset(c->wproj, 0, 2 * kProjFrag * 2) != hipSuccess) {
    nic_destroy(c);
    return fail(NIC_ENOMEM, "nic_create: weight allocation failed");
  }
  // range words: [0] split pass epoch that tripped, [1] re-runs, [2..] the chained re-run's queue
  static_assert(2 + kChainQWords <= 32, "range words");
  if (hipMalloc(&c->range, 32 * sizeof(int)) != hipSuccess || hipMemset(c->range, 0, 32 * sizeof(int)) != hipSuccess ||
      hipHostMalloc(&c->range_host, 8 * sizeof(int), hipHostMallocDefault) != hipSuccess) {
    nic_destroy(c);
    return fail(NIC_ENOMEM, "nic_create: range-guard allocation failed");
  }
  if (hipMalloc(&c->zero16, 256) != hipSuccess || hipMemset(c->zero16, 0, 256) != hipSuccess) {
    nic_destroy(c);
    return fail(NIC_ENOMEM, "nic_create: zero buffer allocation failed");
  }
  // constants: u8 -> fp32 /255 (correctly rounded on the host), colour matrices
  // (utils.py:7-9; the inverse is np.linalg.inv in float64, then rounded to fp32)
  float lut[256];
  for (int i = 0; i < 256; ++i) lut[i] = (float)i / 255.0f;
  float kf[9], kinv[9], off[3];
  nic_constants(kf, kinv, off);
  hipError_t e = upload_constants(lut, kf, kinv, off);
  if (e == hipSuccess) e = upload_ssim_constants();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    nic_destroy(c);
    return fail(NIC_EHIP, "nic_create: constant upload: %s", hipGetErrorString(e));
  }
  *out = c;
  return NIC_OK;
}

int nic_destroy(nic_ctx* c) {
  if (!c) return NIC_OK;
  DeviceGuard guard(c->device);
  for (int i = 0; i < L_COUNT; ++i) {
    if (c->wk[i]) (void)hipFree(c->wk[i]);
    if (c->wb[i]) (void)hipFree(c->wb[i]);
    if (c->wx[i]) (void)hipFree(c->wx[i]);
  }
  if (c->ws) (void)hipFree(c->ws);
  if (c->counts) (void)hipFree(c->counts);
  if (c->fold_acc) (void)hipFree(c->fold_acc);
  if (c->qs) (void)hipFree(c->qs);
  if (c->zero16) (void)hipFree(c->zero16);
  if (c->wproj) (void)hipFree(c->wproj);
  if (c->range) (void)hipFree(c->range);
  if (c->range_host) (void)hipHostFree(c->range_host);
  for (int i = 0; i < L_COUNT; ++i)
    for (int j = 0; j < 2; ++j)
      if (c->ev[i][j]) (void)hipEventDestroy(c->ev[i][j]);
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < kHostMaxChunks; ++k)
      if (c->hev[i][k]) (void)hipEventDestroy(c->hev[i][k]);
  for (int i = 0; i < 3; ++i)
    if (c->hs[i]) (void)hipStreamDestroy(c->hs[i]);
  if (c->hev_caller) (void)hipEventDestroy(c->hev_caller);
  if (c->pin_in) (void)hipHostFree(c->pin_in);
  if (c->pin_out) (void)hipHostFree(c->pin_out);
  if (c->hdev) (void)hipFree(c->hdev);
  delete c;
  return NIC_OK;
}

int nic_set_weights(nic_ctx* c, int model_id, const char* layer, const float* host, const int64_t* shape,
                    int ndim) {
  if (!c || !layer || !host || !shape) return fail(NIC_EINVAL, "nic_set_weights: NULL argument");
  if (model_id < 0 || model_id > 3) return fail(NIC_EINVAL, "nic_set_weights: model_id %d not in 0..3", model_id);
  const char* slash = std::strchr(layer, '/');
  if (!slash) return fail(NIC_EINVAL, "nic_set_weights: layer '%s' must be '<name>/kernel' or '<name>/bias'", layer);
  const std::string lname(layer, slash - layer), kind(slash + 1);
  int idx = -1;
  const LayerSpec* L = find_layer(model_id, lname.c_str(), &idx);
  if (!L) return fail(NIC_EINVAL, "nic_set_weights: model %d has no layer '%s'", model_id, lname.c_str());
  const int m = model_id & 1;  // slot within the encoder / decoder pair
  DeviceGuard guard(c->device);
  if (kind == "kernel") {
    const int64_t want[4] = {L->k, L->k, L->transposed ? L->cout : L->cin, L->transposed ? L->cin : L->cout};
    if (ndim != 4 || shape[0] != want[0] || shape[1] != want[1] || shape[2] != want[2] || shape[3] != want[3])
      return fail(NIC_ESHAPE, "nic_set_weights: %s/kernel expects shape (%lld,%lld,%lld,%lld)", lname.c_str(),
                  (long long)want[0], (long long)want[1], (long long)want[2], (long long)want[3]);
    std::vector<float> packed;
    std::vector<uint16_t> packedx;
    const int kexp = repack_kernel(*L, host, packed, packedx);
    HIP_TRY(hipMemcpy(c->wk[L->id] + m * packed.size(), packed.data(), packed.size() * sizeof(float),
                      hipMemcpyHostToDevice));
    if (!packedx.empty()) {
      HIP_TRY(hipMemcpy(c->wx[L->id] + m * packedx.size(), packedx.data(), packedx.size() * sizeof(uint16_t),
                        hipMemcpyHostToDevice));
      c->wscale[L->id][m] = std::ldexp(1.0f, -kexp);
    }
    if (L->id == L_DCONV8) {
      const std::vector<uint16_t> f = proj_fragments(packed, kexp);
      HIP_TRY(hipMemcpy(c->wproj + m * kProjFrag, f.data(), f.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    }
    c->have_k[model_id][idx] = true;
  } else if (kind == "bias") {
    if (ndim != 1 || shape[0] != L->cout)
      return fail(NIC_ESHAPE, "nic_set_weights: %s/bias expects shape (%d,)", lname.c_str(), L->cout);
    HIP_TRY(hipMemcpy(c->wb[L->id] + m * L->cout, host, L->cout * sizeof(float), hipMemcpyHostToDevice));
    c->have_b[model_id][idx] = true;
  } else {
    return fail(NIC_EINVAL, "nic_set_weights: '%s' is neither kernel nor bias", kind.c_str());
  }
  return NIC_OK;
}

int nic_weights_ready(nic_ctx* c, int* enc, int* dec) {
  if (!c) return fail(NIC_EINVAL, "nic_weights_ready: NULL ctx");
  if (enc) *enc = models_ready(c, 0);
  if (dec) *dec = models_ready(c, 2);
  return NIC_OK;
}

int nic_latent_shape(int h, int w, int* h8, int* w8) {
  if (h <= 0 || w <= 0) return fail(NIC_ESHAPE, "nic_latent_shape: h=%d w=%d must be positive", h, w);
  const SamePad a = same_pad(same_pad(same_pad(h, 5, 2).out, 5, 2).out, 5, 2);
  const SamePad b = same_pad(same_pad(same_pad(w, 5, 2).out, 5, 2).out, 5, 2);
  if (h8) *h8 = a.out;
  if (w8) *w8 = b.out;
  return NIC_OK;
}

int nic_reserve(nic_ctx* c, int n, int h, int w) {
  if (!c) return fail(NIC_EINVAL, "nic_reserve: NULL ctx");
  if (n < 0 || h <= 0 || w <= 0) return fail(NIC_ESHAPE, "nic_reserve: bad shape (%d,%d,%d)", n, h, w);
  DeviceGuard guard(c->device);
  const EncGeom e = enc_geom(n, h, w);
  const DecGeom d = dec_geom(n, e.c8y.out, e.c8x.out);
  float* R[4];
  int rc = ensure_regions(c, std::max(e.r0, d.r0), std::max(e.r123, d.r123), R);
  if (rc) return rc;
  const size_t cb = n > 0 ? hist_scratch_bytes(n, e.c8y.out * e.c8x.out) : 0;
  if (cb > c->counts_bytes) {
    if (c->counts) HIP_TRY(hipFree(c->counts));
    c->counts = nullptr;
    c->counts_bytes = 0;
    HIP_TRY(hipMalloc(&c->counts, cb));
    c->counts_bytes = cb;
  }
  return NIC_OK;
}

}  // extern "C"

namespace {

// NIC_K3P=0: the k3 residual pairs as two weight-stationary launches instead of the fused one
// (A/B; the fused kernel takes planes up to 64 columns, wider ones always use two launches)
bool use_k3pair() {
  static const bool on = [] {
    const char* e = getenv("NIC_K3P");
    return !(e && e[0] == '0');
  }();
  return on;
}
// the fused k3 residual pair of one encoder / decoder pass
hipError_t launch_pair(nic_ctx* c, ConvArgs ap, LayerId lb, hipStream_t st) {
  ap.wx2 = c->wx[lb];
  ap.wscale2[0] = c->wscale[lb][0];
  ap.wscale2[1] = c->wscale[lb][1];
  ap.bias2 = c->wb[lb];
  return launch_k3pair_x3(ap, st);
}

// NIC_CHAIN=0: the gated re-run as one launch per layer (A/B)
bool use_chain() {
  static const bool on = [] {
    const char* e = getenv("NIC_CHAIN");
    return !(e && e[0] == '0');
  }();
  return on;
}

// One encode pass: split-f16 kernels (x3, producers report to rg.flag) or exact-fp32 ones
// (rg.gate set: a re-run that exits unless the split pass of the same epoch tripped).
// `timed` brackets the launches with the per-layer events (the gated re-run is not timed).
int encode_pass(nic_ctx* c, const uint8_t* rgb, int n, int h, int w, uint8_t* latent, float* prequant,
                hipStream_t st, bool x3, const RangeGuard& rg, bool timed) {
  const EncGeom g = enc_geom(n, h, w);
  float* R[4];
  int rc = ensure_regions(c, g.r0, g.r123, R);
  if (rc) return rc;
  const int P = 3 * n;
  const bool timing_on = c->timing;
  c->timing = timing_on && timed;
  struct Restore {
    nic_ctx* c;
    bool v;
    ~Restore() { c->timing = v; }
  } restore{c, timing_on};

  Conv1Args a1{};
  a1.rg = rg;
  a1.rgb = rgb;
  a1.out = R[0];
  a1.out_s = x3 ? (uint16_t*)R[0] : nullptr;
  a1.w = c->wk[L_CONV1];
  a1.bias = c->wb[L_CONV1];
  a1.P = P;
  a1.nimg = n;
  a1.H = h;
  a1.W = w;
  a1.OH = g.c1y.out;
  a1.OW = g.c1x.out;
  a1.pad_y = g.c1y.lo;
  a1.pad_x = g.c1x.lo;
  // the gated exact-fp32 re-run: all layers recorded into one launch (fp32_chain_kernel)
  Fp32Chain chain{};
  const bool chained = !x3 && rg.gate && use_chain();
  chain.gate = rg;
  chain.q = c->range + 2;
  // f16x3: conv1 runs inside the conv2 kernel (launch_conv12_x3, timed as conv2)
  const bool fuse12 = x3;
  if (!fuse12) TIMED(L_CONV1, chained ? chain_add_conv1(chain, a1) : launch_conv1(a1, st));
  // the re-run's head is conv1 (it counts the trip); later layers only gate
  RangeGuard rgl = rg;
  rgl.trips = nullptr;
  auto run = [&](LayerId id, const ConvArgs& a) {
    return chained ? chain_add_layer(chain, id, a) : x3 ? launch_layer_x3(id, a, st) : launch_layer(id, a, st);
  };

  auto conv = [&](LayerId id, const float* in, float* out, const float* res, int H, int W, int OH, int OW, int py,
                  int px) {
    ConvArgs a{};
    a.rg = rgl;
    a.in = in;
    a.out = out;
    a.res = res;
    a.in_s = (const uint16_t*)in;  // the same region read as split f16 (f16x3 kernels)
    a.out_s = (uint16_t*)out;
    a.res_s = (const uint16_t*)res;
    a.zero16 = c->zero16;
    a.w = c->wk[id];
    a.wx = c->wx[id];
    a.wscale[0] = c->wscale[id][0];
    a.wscale[1] = c->wscale[id][1];
    a.bias = c->wb[id];
    a.P = P;
    a.nimg = n;
    a.H = H;
    a.W = W;
    a.OH = OH;
    a.OW = OW;
    a.pad_y = py;
    a.pad_x = px;
    return a;
  };
  const int h1 = g.c1y.out, w1 = g.c1x.out, h2 = g.c2y.out, w2 = g.c2x.out;
  ConvArgs a2 = conv(L_CONV2, R[0], R[1], nullptr, h1, w1, h2, w2, g.c2y.lo, g.c2x.lo);
  if (fuse12) {
    a2.rgb = rgb;
    a2.wx1 = c->wx[L_CONV1];
    a2.wscale1[0] = c->wscale[L_CONV1][0];
    a2.wscale1[1] = c->wscale[L_CONV1][1];
    a2.bias1 = c->wb[L_CONV1];
    a2.H0 = h;
    a2.W0 = w;
    a2.p1y = g.c1y.lo;
    a2.p1x = g.c1x.lo;
    a2.cplane = (uint16_t*)R[0];  // colour planes (R0 is free: conv1 writes no output)
    TIMED(L_CONV2, launch_conv12_x3(a2, st));
  } else {
    TIMED(L_CONV2, run(L_CONV2, a2));
  }
  if (x3 && use_k3pair() && k3pair_supported(h2, w2)) {
    // conv3 -> conv4 -> + res as one launch (R1 -> R3, the residual read from the input
    // rows in LDS); timed as conv4
    TIMED(L_CONV4, launch_pair(c, conv(L_CONV3, R[1], R[3], nullptr, h2, w2, h2, w2, 1, 1), L_CONV4, st));
  } else {
    TIMED(L_CONV3, run(L_CONV3, conv(L_CONV3, R[1], R[2], nullptr, h2, w2, h2, w2, 1, 1)));
    TIMED(L_CONV4, run(L_CONV4, conv(L_CONV4, R[2], R[3], R[1], h2, w2, h2, w2, 1, 1)));
  }
  ConvArgs a8 = conv(L_CONV8, R[3], nullptr, nullptr, h2, w2, g.c8y.out, g.c8x.out, g.c8y.lo, g.c8x.lo);
  a8.out_u8 = latent;
  a8.out_f32_latent = prequant;
  if (x3 && c->fold_part) {  // nic_encode_entropy: the split pass's conv8 counts the codes
    a8.hist_part = c->fold_part;
  }
  TIMED(L_CONV8, run(L_CONV8, a8));
  if (chained) HIP_TRY(launch_fp32_chain(chain, st));
  return NIC_OK;
}

// One decode pass (see encode_pass).
int decode_pass(nic_ctx* c, const uint8_t* latent, int n, int h8, int w8, uint8_t* rgb, float* rgb_f32,
                hipStream_t st, bool x3, const RangeGuard& rg, bool timed) {
  const DecGeom g = dec_geom(n, h8, w8);
  float* R[4];
  int rc = ensure_regions(c, g.r0, g.r123, R);
  if (rc) return rc;
  const int P = 3 * n;
  const bool timing_on = c->timing;
  c->timing = timing_on && timed;
  struct Restore {
    nic_ctx* c;
    bool v;
    ~Restore() { c->timing = v; }
  } restore{c, timing_on};
  // the re-run's head is dconv1 (it counts the trip); later layers only gate
  RangeGuard rgl = rg;
  rgl.trips = nullptr;
  Fp32Chain chain{};  // the gated exact-fp32 re-run as one launch (see encode_pass)
  const bool chained = !x3 && rg.gate && use_chain();
  chain.gate = rg;
  chain.q = c->range + 2;
  auto run = [&](LayerId id, const ConvArgs& a) {
    return chained ? chain_add_layer(chain, id, a) : x3 ? launch_layer_x3(id, a, st) : launch_layer(id, a, st);
  };
  auto conv = [&](LayerId id, const float* in, float* out, const float* res, int H, int W, int OH, int OW) {
    ConvArgs a{};
    a.rg = rgl;
    a.in = in;
    a.out = out;
    a.res = res;
    a.in_s = (const uint16_t*)in;  // the same region read as split f16 (f16x3 kernels)
    a.out_s = (uint16_t*)out;
    a.res_s = (const uint16_t*)res;
    a.zero16 = c->zero16;
    a.w = c->wk[id];
    a.wx = c->wx[id];
    a.wscale[0] = c->wscale[id][0];
    a.wscale[1] = c->wscale[id][1];
    a.bias = c->wb[id];
    a.P = P;
    a.nimg = n;
    a.H = H;
    a.W = W;
    a.OH = OH;
    a.OW = OW;
    a.pad_y = 1;
    a.pad_x = 1;
    return a;
  };
  ConvArgs d1 = conv(L_DCONV1, nullptr, R[1], nullptr, h8, w8, 2 * h8, 2 * w8);
  d1.in_u8 = latent;
  d1.rg = rg;
  TIMED(L_DCONV1, run(L_DCONV1, d1));
  const int h2 = 2 * h8, w2 = 2 * w8;
  if (x3 && use_k3pair() && k3pair_supported(h2, w2)) {  // dconv5 -> dconv6 -> + res, timed as dconv6
    TIMED(L_DCONV6, launch_pair(c, conv(L_DCONV5, R[1], R[3], nullptr, h2, w2, h2, w2), L_DCONV6, st));
  } else {
    TIMED(L_DCONV5, run(L_DCONV5, conv(L_DCONV5, R[1], R[2], nullptr, h2, w2, h2, w2)));
    TIMED(L_DCONV6, run(L_DCONV6, conv(L_DCONV6, R[2], R[3], R[1], h2, w2, h2, w2)));
  }
  ConvArgs d7 = conv(L_DCONV7, R[3], R[0], nullptr, h2, w2, 2 * h2, 2 * w2);
  // f16x3: dconv7 writes dconv8's per-pixel tap projections (100 B / pixel instead of 256)
  const bool fuse78 = x3;
  if (fuse78) {
    d7.proj = R[0];
    d7.proj_w = c->wproj;
    d7.proj_scale[0] = c->wscale[L_DCONV8][0];
    d7.proj_scale[1] = c->wscale[L_DCONV8][1];
    TIMED(L_DCONV7, launch_dconv7_proj_x3(d7, st));
  } else {
    TIMED(L_DCONV7, run(L_DCONV7, d7));
  }
  Dconv8Args a8{};
  a8.rg = rgl;
  a8.in = R[0];
  a8.in_s = (const uint16_t*)R[0];
  a8.zero16 = c->zero16;
  a8.out_u8 = rgb;
  a8.out_f32 = rgb_f32;
  a8.w = c->wk[L_DCONV8];
  a8.wx = c->wx[L_DCONV8];
  a8.wscale[0] = c->wscale[L_DCONV8][0];
  a8.wscale[1] = c->wscale[L_DCONV8][1];
  a8.bias = c->wb[L_DCONV8];
  a8.nimg = n;
  a8.H = 2 * h2;
  a8.W = 2 * w2;
  if (fuse78) {
    a8.proj = R[0];
    a8.tiles_y7 = (h2 + 7) / 8;
    a8.tiles_x7 = (w2 + 7) / 8;
    TIMED(L_DCONV8, launch_dconv8_gather(a8, st));
  } else {
    TIMED(L_DCONV8, chained ? chain_add_dconv8(chain, a8) : launch_dconv8(a8, st));
  }
  if (chained) HIP_TRY(launch_fp32_chain(chain, st));
  return NIC_OK;
}

// The f16 range guard around a split-f16 pass (nic.h, NIC_RANGE_*): the pass's producers
// report to the ctx's flag word under a fresh epoch; then either the exact-fp32 re-run is
// queued behind it, gated on that epoch (FALLBACK: stream-ordered, no host sync), or the
// stream is synchronised and a tripped pass returns NIC_ERANGE (ERROR).
// The split-f16 kernels address one plane's 64-channel split activation (and dconv7's
// projections) with 32-bit buffer offsets: a plane of the 64-channel levels (h/4 x w/4,
// resp. 2h8 x 2w8) must stay under 2^30 bytes, i.e. about 67 MP per image.  Larger images
// run the exact-fp32 kernels (64-bit addressing) instead of failing (nic.h).
bool x3_plane_fits(long long h64, long long w64) { return h64 * w64 * 64 * 4 < (1LL << 30); }

template <class Pass>
int guarded(nic_ctx* c, hipStream_t st, const char* what, bool x3_fits, Pass pass) {
  if (c->precision != NIC_PRECISION_F16X3 || !x3_fits) return pass(false, RangeGuard{}, true);
  if (++c->epoch <= 0) c->epoch = 1;  // the flag word starts at 0: never a live epoch
  RangeGuard prod{};
  prod.flag = c->range;
  prod.epoch = c->epoch;
  int rc = pass(true, prod, true);
  if (rc) return rc;
  if (c->range_policy == NIC_RANGE_FALLBACK) {
    RangeGuard gate{};
    gate.gate = c->range;
    gate.trips = c->range + 1;
    gate.epoch = c->epoch;
    return pass(false, gate, false);
  }
  HIP_TRY(hipMemcpyAsync(c->range_host, c->range, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (*c->range_host == c->epoch) {
    ++c->error_trips;
    return fail(NIC_ERANGE, "%s: an activation reached the f16 limit of the split-f16 pass (|x| >= 65504); "
                "outputs are undefined (use NIC_RANGE_FALLBACK or NIC_PRECISION_FP32)", what);
  }
  return NIC_OK;
}

// -- host-array surface ------------------------------------------------------------------
// Chunk k of a host call: its H2D DMA on hs[0], its device pass on hs[1], its D2H DMA on hs[2],
// so chunk k+1's copy-in and chunk k-1's copy-out overlap chunk k's pass.  Chunk sizes ramp
// up and down (weights min(2^i, 2^(K-1-i))): a small first chunk starts the device early and
// a small last chunk keeps the exposed D2H tail short (edge chunks at 0.25 / 0.35 of a middle
// one and equal middles measured the same, round 4).
void host_chunk_plan(int n, int k, std::vector<int>& lo) {
  k = std::max(1, std::min({k, n, kHostMaxChunks}));
  std::vector<double> wgt(k);
  double tot = 0;
  for (int i = 0; i < k; ++i)
    tot += wgt[i] = (double)(1 << std::min(i, k - 1 - i));
  lo.assign(1, 0);
  double acc = 0;
  for (int i = 0; i < k; ++i) {
    acc += wgt[i];
    const int b = i + 1 == k ? n : std::max(lo.back() + 1, std::min(n - (k - 1 - i), (int)std::lround(n * acc / tot)));
    lo.push_back(b);
  }
}

bool host_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // plain pageable memory: not known to HIP
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

int grow_pinned(uint8_t*& p, size_t& have, size_t need) {
  if (need <= have) return NIC_OK;
  if (p) HIP_TRY(hipHostFree(p));
  p = nullptr;
  have = 0;
  if (hipHostMalloc((void**)&p, need, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return fail(NIC_ENOMEM, "pinned staging allocation of %zu bytes failed", need);
  }
  have = need;
  return NIC_OK;
}

// Staging copies of the host-array surface (pageable <-> page-locked), split over a pool of
// worker threads: one thread copies ~50 GB/s, so a 12.6 MB batch took 0.26 ms on the host
// thread -- ahead of the first chunk's DMA and between the later chunks' issues, where it
// delayed their copy-in past the previous chunk's pass.  Workers spin briefly after each copy
// (the chunks of one call come ~0.1 ms apart), then sleep on a condition variable; the pool is
// never destroyed (detached threads parked at exit).  NIC_HOST_COPY_THREADS: worker count
// (plus the calling thread).  Default 0 = plain memcpy on the calling thread: with 7 workers the
// host-plan sweep measured the encoder 0.942 -> 0.865 ms on one box, but the bench's host path
// swung between 1,809 and 2,160 MP/s with it against 2,084-2,213 without (profiles/r4_ab_logs.txt):
// a worker descheduled under the box's CPU quota stalls the caller, which waits for every part.
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool* p = new CopyPool();
    return *p;
  }
  void copy(void* dst, const void* src, size_t n) {
    if (nw_ == 0 || n < kMinParallel) {
      std::memcpy(dst, src, n);
      return;
    }
    std::lock_guard<std::mutex> call(call_mu_);
    dst_ = (char*)dst;
    src_ = (const char*)src;
    n_ = n;
    pending_.store(nw_, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(mu_);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    part(0);
    while (pending_.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
  }

 private:
  static constexpr size_t kMinParallel = 256 << 10;
  static constexpr int kSpin = 1 << 15;
  CopyPool() {
    const char* e = getenv("NIC_HOST_COPY_THREADS");
    nw_ = std::max(0, std::min(31, e ? atoi(e) : 0));
    for (int i = 0; i < nw_; ++i) std::thread([this, i] { worker(i + 1); }).detach();
  }
  void part(int id) {  // 4 KB-aligned share id of nw_ + 1
    const size_t parts = (size_t)nw_ + 1, pages = (n_ + 4095) / 4096;
    const size_t b = std::min(n_, pages * id / parts * 4096), e = std::min(n_, pages * (id + 1) / parts * 4096);
    if (e > b) std::memcpy(dst_ + b, src_ + b, e - b);
  }
  void worker(int id) {
    unsigned seen = 0;
    for (;;) {
      unsigned g;
      int spins = 0;
      while ((g = gen_.load(std::memory_order_acquire)) == seen) {
        if (++spins < kSpin) {
          __builtin_ia32_pause();
          continue;
        }
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
      }
      seen = g;
      part(id);
      pending_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  int nw_ = 0;
  char* dst_ = nullptr;
  const char* src_ = nullptr;
  size_t n_ = 0;
  std::atomic<unsigned> gen_{0};
  std::atomic<int> pending_{0};
  std::mutex mu_, call_mu_;
  std::condition_variable cv_;
};

// (A second pass slot on a second compute stream, so chunk k+1's kernels could fill chunk k's
// tails, measured slower in round 4 -- round trip 2.15-2.20 vs 1.93-1.96 ms: two chunk passes'
// persistent kernels, one block per CU each, contend for the CUs -- and was removed.)

// Host-side wait for an event: polling hipEventQuery returns as soon as the GPU signals, where
// hipEventSynchronize may sleep and pay a wake-up latency per chunk (no worse, less jitter).
hipError_t host_wait(hipEvent_t e) {
  for (;;) {
    const hipError_t r = hipEventQuery(e);
    if (r != hipErrorNotReady) return r;
    __builtin_ia32_pause();
  }
}

int host_setup(nic_ctx* c) {
  for (int i = 0; i < 3; ++i)
    if (!c->hs[i]) HIP_TRY(hipStreamCreateWithFlags(&c->hs[i], hipStreamNonBlocking));
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < kHostMaxChunks; ++k)
      if (!c->hev[i][k]) HIP_TRY(hipEventCreateWithFlags(&c->hev[i][k], hipEventDisableTiming));
  if (!c->hev_caller) HIP_TRY(hipEventCreateWithFlags(&c->hev_caller, hipEventDisableTiming));
  return NIC_OK;
}

// in (n x in_row bytes, host) -> pass(dev_in, count, dev_out, stream) per chunk -> out (host).
// Page-locked inputs / outputs are DMA'd directly; pageable ones go through the ctx's pinned
// staging (host memcpy of chunk k+1 while chunk k's DMA runs).  Ordered after the work
// queued on `caller`; returns with every chunk's output in `out`.
template <class Pass>
int host_pipeline(nic_ctx* c, const uint8_t* in, size_t in_row, uint8_t* out, size_t out_row, int n, int chunks,
                  hipStream_t caller, Pass pass) {
  int rc = host_setup(c);
  if (rc) return rc;
  const bool in_pin = host_pinned(in), out_pin = host_pinned(out);
  if (!in_pin && (rc = grow_pinned(c->pin_in, c->pin_in_bytes, n * in_row))) return rc;
  if (!out_pin && (rc = grow_pinned(c->pin_out, c->pin_out_bytes, n * out_row))) return rc;
  const size_t dev_bytes = ((n * in_row + 255) & ~(size_t)255) + n * out_row;
  if (dev_bytes > c->hdev_bytes) {
    if (c->hdev) HIP_TRY(hipFree(c->hdev));
    c->hdev = nullptr;
    c->hdev_bytes = 0;
    if (hipMalloc(&c->hdev, dev_bytes) != hipSuccess) {
      (void)hipGetLastError();
      return fail(NIC_ENOMEM, "host-surface device buffers of %zu bytes failed", dev_bytes);
    }
    c->hdev_bytes = dev_bytes;
  }
  uint8_t* d_in = c->hdev;
  uint8_t* d_out = c->hdev + ((n * in_row + 255) & ~(size_t)255);
  std::vector<int> lo;
  host_chunk_plan(n, chunks, lo);
  const int K = (int)lo.size() - 1;
  HIP_TRY(hipEventRecord(c->hev_caller, caller));
  HIP_TRY(hipStreamWaitEvent(c->hs[0], c->hev_caller, 0));
  HIP_TRY(hipStreamWaitEvent(c->hs[1], c->hev_caller, 0));
  int err = NIC_OK, issued = 0;
  for (int k = 0; k < K && !err; ++k) {
    const size_t i0 = lo[k] * in_row, ib = (lo[k + 1] - lo[k]) * in_row;
    const size_t o0 = lo[k] * out_row, ob = (lo[k + 1] - lo[k]) * out_row;
    const uint8_t* src = in + i0;
    if (!in_pin) {
      CopyPool::get().copy(c->pin_in + i0, in + i0, ib);
      src = c->pin_in + i0;
    }
    hipError_t e = hipMemcpyAsync(d_in + i0, src, ib, hipMemcpyHostToDevice, c->hs[0]);
    if (e == hipSuccess) e = hipEventRecord(c->hev[0][k], c->hs[0]);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->hs[1], c->hev[0][k], 0);
    if (e != hipSuccess) {
      err = fail(NIC_EHIP, "host surface: %s", hipGetErrorString(e));
      break;
    }
    err = pass(d_in + i0, lo[k + 1] - lo[k], d_out + o0, c->hs[1]);
    if (err) break;
    e = hipEventRecord(c->hev[1][k], c->hs[1]);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->hs[2], c->hev[1][k], 0);
    if (e == hipSuccess)
      e = hipMemcpyAsync(out_pin ? out + o0 : c->pin_out + o0, d_out + o0, ob, hipMemcpyDeviceToHost, c->hs[2]);
    if (e == hipSuccess) e = hipEventRecord(c->hev[2][k], c->hs[2]);
    if (e != hipSuccess) {
      err = fail(NIC_EHIP, "host surface: %s", hipGetErrorString(e));
      break;
    }
    ++issued;
  }
  for (int k = 0; k < issued && !err; ++k) {  // chunk k's unstaging overlaps chunk k+1's work
    hipError_t e = host_wait(c->hev[2][k]);
    if (e != hipSuccess) {
      err = fail(NIC_EHIP, "host surface: %s", hipGetErrorString(e));
      break;
    }
    if (!out_pin) CopyPool::get().copy(out + lo[k] * out_row, c->pin_out + lo[k] * out_row, (lo[k + 1] - lo[k]) * out_row);
  }
  // success: every copy-in fed a pass and every pass a copy-out, so the last copy-out's event
  // means all three streams are idle -- no stream synchronisations (~10-30 us per call); any
  // error path drains them
  if (err || issued != K)
    for (int i = 0; i < 3; ++i) (void)hipStreamSynchronize(c->hs[i]);
  return err;
}

}  // namespace

extern "C" {

int nic_encode(nic_ctx* c, const uint8_t* rgb, int n, int h, int w, uint8_t* latent, float* prequant,
               void* stream) {
  if (!c) return fail(NIC_EINVAL, "nic_encode: NULL ctx");
  if (n < 0 || h <= 0 || w <= 0) return fail(NIC_ESHAPE, "nic_encode: bad input shape (%d,%d,%d,3)", n, h, w);
  if (!models_ready(c, 0)) return fail(NIC_ENOWEIGHTS, "nic_encode: encoder weights not fully set");
  if (n == 0) return NIC_OK;  // empty batch: pointers may be NULL
  if (!rgb || !latent) return fail(NIC_EINVAL, "nic_encode: NULL buffer");
  if (3LL * n > 65535) return fail(NIC_ESHAPE, "nic_encode: batch %d exceeds 21845 images per call", n);
  DeviceGuard guard(c->device);
  hipStream_t st = (hipStream_t)stream;
  const EncGeom eg = enc_geom(n, h, w);
  return guarded(c, st, "nic_encode", x3_plane_fits(eg.c2y.out, eg.c2x.out), [&](bool x3, const RangeGuard& rg, bool timed) {
    return encode_pass(c, rgb, n, h, w, latent, prequant, st, x3, rg, timed);
  });
}

int nic_decode(nic_ctx* c, const uint8_t* latent, int n, int h8, int w8, uint8_t* rgb, float* rgb_f32,
               void* stream) {
  if (!c) return fail(NIC_EINVAL, "nic_decode: NULL ctx");
  if (n < 0 || h8 <= 0 || w8 <= 0) return fail(NIC_ESHAPE, "nic_decode: bad latent shape (%d,%d,%d,96)", n, h8, w8);
  if (!models_ready(c, 2)) return fail(NIC_ENOWEIGHTS, "nic_decode: decoder weights not fully set");
  if (n == 0) return NIC_OK;
  if (!latent || !rgb) return fail(NIC_EINVAL, "nic_decode: NULL buffer");
  if (3LL * n > 65535) return fail(NIC_ESHAPE, "nic_decode: batch %d exceeds 21845 images per call", n);
  DeviceGuard guard(c->device);
  hipStream_t st = (hipStream_t)stream;
  return guarded(c, st, "nic_decode", x3_plane_fits(2LL * h8, 2LL * w8), [&](bool x3, const RangeGuard& rg, bool timed) {
    return decode_pass(c, latent, n, h8, w8, rgb, rgb_f32, st, x3, rg, timed);
  });
}

int nic_encode_host(nic_ctx* c, const uint8_t* rgb, int n, int h, int w, uint8_t* latent, int chunks,
                    void* stream) {
  if (!c) return fail(NIC_EINVAL, "nic_encode_host: NULL ctx");
  if (n < 0 || h <= 0 || w <= 0) return fail(NIC_ESHAPE, "nic_encode_host: bad input shape (%d,%d,%d,3)", n, h, w);
  if (!models_ready(c, 0)) return fail(NIC_ENOWEIGHTS, "nic_encode_host: encoder weights not fully set");
  if (n == 0) return NIC_OK;
  if (!rgb || !latent) return fail(NIC_EINVAL, "nic_encode_host: NULL buffer");
  if (3LL * n > 65535) return fail(NIC_ESHAPE, "nic_encode_host: batch %d exceeds 21845 images per call", n);
  int h8, w8;
  nic_latent_shape(h, w, &h8, &w8);
  const EncGeom eg = enc_geom(1, h, w);
  const bool fits = x3_plane_fits(eg.c2y.out, eg.c2x.out);
  DeviceGuard guard(c->device);
  return host_pipeline(c, rgb, (size_t)h * w * 3, latent, (size_t)h8 * w8 * 96, n, chunks, (hipStream_t)stream,
                       [&](const uint8_t* x, int m, uint8_t* z, hipStream_t st) {
                         return guarded(c, st, "nic_encode_host", fits, [&](bool x3, const RangeGuard& rg, bool timed) {
                           return encode_pass(c, x, m, h, w, z, nullptr, st, x3, rg, timed);
                         });
                       });
}

int nic_decode_host(nic_ctx* c, const uint8_t* latent, int n, int h8, int w8, uint8_t* rgb, int chunks,
                    void* stream) {
  if (!c) return fail(NIC_EINVAL, "nic_decode_host: NULL ctx");
  if (n < 0 || h8 <= 0 || w8 <= 0) return fail(NIC_ESHAPE, "nic_decode_host: bad latent shape (%d,%d,%d,96)", n, h8, w8);
  if (!models_ready(c, 2)) return fail(NIC_ENOWEIGHTS, "nic_decode_host: decoder weights not fully set");
  if (n == 0) return NIC_OK;
  if (!latent || !rgb) return fail(NIC_EINVAL, "nic_decode_host: NULL buffer");
  if (3LL * n > 65535) return fail(NIC_ESHAPE, "nic_decode_host: batch %d exceeds 21845 images per call", n);
  DeviceGuard guard(c->device);
  return host_pipeline(c, latent, (size_t)h8 * w8 * 96, rgb, (size_t)64 * h8 * w8 * 3, n, chunks, (hipStream_t)stream,
                       [&](const uint8_t* z, int m, uint8_t* x, hipStream_t st) {
                         return guarded(c, st, "nic_decode_host", x3_plane_fits(2LL * h8, 2LL * w8), [&](bool x3, const RangeGuard& rg, bool timed) {
                           return decode_pass(c, z, m, h8, w8, x, nullptr, st, x3, rg, timed);
                         });
                       });
}

int nic_entropy_hist(nic_ctx* c, const uint8_t* latent, int n, int h8, int w8, uint32_t* counts, float* bits,
                     void* stream) {
  if (!c) return fail(NIC_EINVAL, "nic_entropy_hist: NULL ctx");
  if (n < 0 || h8 <= 0 || w8 <= 0) return fail(NIC_ESHAPE, "nic_entropy_hist: bad latent shape (%d,%d,%d,96)", n, h8, w8);
  if (n == 0 || (!counts && !bits)) return NIC_OK;
  if (!latent) return fail(NIC_EINVAL, "nic_entropy_hist: NULL latent");
  if (3LL * n > 65535) return fail(NIC_ESHAPE, "nic_entropy_hist: batch %d too large", n);
  if ((long long)h8 * w8 * 6 > 0x7fffffffLL) return fail(NIC_ESHAPE, "nic_entropy_hist: latent %dx%d too large", h8, w8);
  DeviceGuard guard(c->device);
  const size_t cb = hist_scratch_bytes(n, h8 * w8);
  if (cb > c->counts_bytes) {
    if (c->counts) HIP_TRY(hipFree(c->counts));
    c->counts = nullptr;
    c->counts_bytes = 0;
    HIP_TRY(hipMalloc(&c->counts, cb));
    c->counts_bytes = cb;
  }
  HIP_TRY(launch_hist(latent, n, h8 * w8, c->counts, counts, bits, (hipStream_t)stream));
  return NIC_OK;
}

// the fold needs the split-f16 pass with the tap-split conv8 and >= 2 of a plane's conv8 tiles
// per block of its group (hist_fold_supported); otherwise nic_encode_entropy runs the two calls
static bool encode_entropy_folds(const nic_ctx* c, int n, int h, int w) {
  const EncGeom eg = enc_geom(n, h, w);
  return c->precision == NIC_PRECISION_F16X3 && x3_plane_fits(eg.c2y.out, eg.c2x.out) &&
         hist_fold_supported(n, eg.c8y.out, eg.c8x.out);
}

// the shape limits nic_encode_entropy applies (shared with the fold query, so the query never
// reports a form for a shape the call refuses)
static int encode_entropy_shape(const char* fn, int n, int h, int w) {
  if (n < 0 || h <= 0 || w <= 0) return fail(NIC_ESHAPE, "%s: bad input shape (%d,%d,%d,3)", fn, n, h, w);
  if (3LL * n > 65535) return fail(NIC_ESHAPE, "%s: batch %d exceeds 21845 images per call", fn, n);
  int h8, w8;
  nic_latent_shape(h, w, &h8, &w8);
  if ((long long)h8 * w8 * 6 > 0x7fffffffLL) return fail(NIC_ESHAPE, "%s: latent %dx%d too large", fn, h8, w8);
  return NIC_OK;
}

int nic_encode_entropy_fold(nic_ctx* c, int n, int h, int w, int* folds) {
  if (!c || !folds) return fail(NIC_EINVAL, "nic_encode_entropy_fold: NULL argument");
  if (n == 0) return fail(NIC_ESHAPE, "nic_encode_entropy_fold: empty batch");
  if (int rc = encode_entropy_shape("nic_encode_entropy_fold", n, h, w)) return rc;
  DeviceGuard guard(c->device);
  *folds = encode_entropy_folds(c, n, h, w) ? 1 : 0;
  return NIC_OK;
}

int nic_encode_entropy(nic_ctx* c, const uint8_t* rgb, int n, int h, int w, uint8_t* latent, uint32_t* counts,
                       float* bits, void* stream) {
  if (!c) return fail(NIC_EINVAL, "nic_encode_entropy: NULL ctx");
  if (int rc = encode_entropy_shape("nic_encode_entropy", n, h, w)) return rc;
  if (!models_ready(c, 0)) return fail(NIC_ENOWEIGHTS, "nic_encode_entropy: encoder weights not fully set");
  if (n == 0) return NIC_OK;
  if (!rgb || !latent) return fail(NIC_EINVAL, "nic_encode_entropy: NULL buffer");
  DeviceGuard guard(c->device);
  hipStream_t st = (hipStream_t)stream;
  const EncGeom eg = enc_geom(n, h, w);
  const int h8 = eg.c8y.out, w8 = eg.c8x.out;
  const bool fits = x3_plane_fits(eg.c2y.out, eg.c2x.out);
  // the fold needs the split-f16 pass with the tap-split conv8 and block ranges within a plane;
  // otherwise (and for counts == bits == NULL) the two-step form
  const bool fold = (counts || bits) && encode_entropy_folds(c, n, h, w);
  if (!fold) {
    int rc = nic_encode(c, rgb, n, h, w, latent, nullptr, stream);
    if (rc || (!counts && !bits)) return rc;
    return nic_entropy_hist(c, latent, n, h8, w8, counts, bits, stream);
  }
  const size_t fb = hist_fold_scratch_bytes(n, h8, w8);
  if (fb > c->fold_acc_bytes) {  // zeroed once; every reduce clears what it read
    if (c->fold_acc) HIP_TRY(hipFree(c->fold_acc));
    c->fold_acc = nullptr;
    c->fold_acc_bytes = 0;
    HIP_TRY(hipMalloc(&c->fold_acc, fb));
    HIP_TRY(hipMemset(c->fold_acc, 0, fb));
    c->fold_acc_bytes = fb;
  }
  c->fold_part = c->fold_acc;
  int rc = guarded(c, st, "nic_encode_entropy", fits, [&](bool x3, const RangeGuard& rg, bool timed) {
    return encode_pass(c, rgb, n, h, w, latent, nullptr, st, x3, rg, timed);
  });
  c->fold_part = nullptr;
  if (rc) {  // conv8 may have counted: leave the accumulator clean for the next call
    (void)hipMemsetAsync(c->fold_acc, 0, fb, st);
    return rc;
  }
  RangeGuard trip{};  // the split pass's epoch: a trip means the re-run rewrote the latent
  trip.flag = c->range;
  trip.epoch = c->epoch;
  HIP_TRY(launch_hist_fold(c->fold_acc, latent, n, h8, w8, trip, counts, bits, st));
  return NIC_OK;
}

int nic_ms_ssim(nic_ctx* c, const uint8_t* a, const uint8_t* b, int n, int h, int w, float* ms_ssim,
                float* per_scale, void* stream) {
  if (!c) return fail(NIC_EINVAL, "nic_ms_ssim: NULL ctx");
  if (n < 0 || h <= 0 || w <= 0) return fail(NIC_ESHAPE, "nic_ms_ssim: bad image shape (%d,%d,%d,3)", n, h, w);
  {  // tf.image.ssim_multiscale: every scale (ceil halving) holds the 11 x 11 window
    int sh = h, sw = w;
    for (int k = 0; k < kSsimScales; ++k, sh = (sh + 1) / 2, sw = (sw + 1) / 2)
      if (sh < 11 || sw < 11)
        return fail(NIC_ESHAPE, "nic_ms_ssim: scale %d of a %dx%d image is %dx%d, smaller than the 11x11 window "
                    "(H, W >= 161)", k, h, w, sh, sw);
  }
  if (n == 0) return NIC_OK;
  if (!a || !b || !ms_ssim) return fail(NIC_EINVAL, "nic_ms_ssim: NULL argument");
  if (3LL * n > 65535) return fail(NIC_ESHAPE, "nic_ms_ssim: batch %d too large", n);
  DeviceGuard guard(c->device);
  SsimPlan pl;
  ssim_plan(n, h, w, &pl);
  if (pl.bytes > c->qs_bytes) {
    if (c->qs) HIP_TRY(hipFree(c->qs));
    c->qs = nullptr;
    c->qs_bytes = 0;
    if (hipMalloc(&c->qs, pl.bytes) != hipSuccess) {
      (void)hipGetLastError();
      return fail(NIC_ENOMEM, "nic_ms_ssim: scratch allocation of %zu bytes failed", pl.bytes);
    }
    c->qs_bytes = pl.bytes;
  }
  HIP_TRY(launch_ms_ssim(a, b, n, h, w, c->qs, ms_ssim, per_scale, (hipStream_t)stream));
  return NIC_OK;
}

int nic_sq_err(const uint8_t* a, const uint8_t* b, int n, int64_t bytes_per_image, uint64_t* sse, void* stream) {
  if (n < 0 || bytes_per_image < 0) return fail(NIC_ESHAPE, "nic_sq_err: bad shape (%d, %lld)", n, (long long)bytes_per_image);
  if (n == 0) return NIC_OK;
  if (!a || !b || !sse) return fail(NIC_EINVAL, "nic_sq_err: NULL argument");
  if (n > 65535) return fail(NIC_ESHAPE, "nic_sq_err: batch %d too large", n);
  HIP_TRY(launch_sq_err(a, b, n, bytes_per_image, reinterpret_cast<unsigned long long*>(sse), (hipStream_t)stream));
  return NIC_OK;
}

int nic_pack_latent(const uint8_t* latent, int n, int h8, int w8, uint8_t* packed, void* stream) {
  if (n < 0 || h8 <= 0 || w8 <= 0) return fail(NIC_ESHAPE, "nic_pack_latent: bad shape (%d,%d,%d)", n, h8, w8);
  if (n == 0) return NIC_OK;
  if (!latent || !packed) return fail(NIC_EINVAL, "nic_pack_latent: NULL argument");
  HIP_TRY(launch_pack(latent, packed, n, h8, w8, false, (hipStream_t)stream));
  return NIC_OK;
}

int nic_unpack_latent(const uint8_t* packed, int n, int h8, int w8, uint8_t* latent, void* stream) {
  if (n < 0 || h8 <= 0 || w8 <= 0) return fail(NIC_ESHAPE, "nic_unpack_latent: bad shape (%d,%d,%d)", n, h8, w8);
  if (n == 0) return NIC_OK;
  if (!latent || !packed) return fail(NIC_EINVAL, "nic_unpack_latent: NULL argument");
  HIP_TRY(launch_pack(packed, latent, n, h8, w8, true, (hipStream_t)stream));
  return NIC_OK;
}

// ---- training side path (nic_train.hip) ----------------------------------------------------
static bool train_dims_ok(int c) { return c >= 1 && c <= 64; }

int nic_conv_gather_work(int kh, int kw, int cin, int cout, int64_t* bytes) {
  if (!bytes) return fail(NIC_EINVAL, "nic_conv_gather_work: NULL argument");
  if (kh <= 0 || kw <= 0 || kh * kw > 64 || !train_dims_ok(cin) || !train_dims_ok(cout))
    return fail(NIC_ESHAPE, "nic_conv_gather_work: bad shape");
  *bytes = (int64_t)train_gather_work_bytes(kh, kw, cin, cout);
  return NIC_OK;
}

static int conv_gather_impl(const char* name, const float* x, int n, int h, int w, int cin, const float* wt, int kh,
                            int kw, int wt_layout, int stride, int pad_y, int pad_x, int transposed, const float* bias,
                            const float* x_scale, const float* w_scale, float* y, int oh, int ow, int cout, int act,
                            void* work, int64_t work_bytes, void* stream) {
  if (n < 0 || h <= 0 || w <= 0 || oh <= 0 || ow <= 0 || kh <= 0 || kw <= 0 || kh * kw > 64 || stride <= 0 ||
      !train_dims_ok(cin) || !train_dims_ok(cout) || pad_y < 0 || pad_x < 0)
    return fail(NIC_ESHAPE, "%s: bad shape n=%d %dx%dx%d -> %dx%dx%d k=%dx%d s=%d pad=%d,%d", name, n, h, w, cin, oh, ow,
                cout, kh, kw, stride, pad_y, pad_x);
  if ((wt_layout != 0 && wt_layout != 1) || (transposed != 0 && transposed != 1) || (act != 0 && act != 1))
    return fail(NIC_EINVAL, "%s: wt_layout / transposed / act must be 0 or 1", name);
  if (n == 0) return NIC_OK;
  if (!x || !wt || !y || !work) return fail(NIC_EINVAL, "%s: NULL argument", name);
  const int64_t need = (int64_t)train_gather_work_bytes(kh, kw, cin, cout);
  if (work_bytes < need)
    return fail(NIC_EINVAL, "%s: work holds %lld bytes, needs %lld", name, (long long)work_bytes, (long long)need);
  if (((uintptr_t)work & 15) != 0) return fail(NIC_EINVAL, "%s: work must be 16-byte aligned", name);
  HIP_TRY(launch_conv_gather(x, n, h, w, cin, wt, kh, kw, wt_layout, stride, pad_y, pad_x, transposed, bias, x_scale,
                             w_scale, y, oh, ow, cout, act, work, (hipStream_t)stream));
  return NIC_OK;
}

int nic_conv_gather(const float* x, int n, int h, int w, int cin, const float* wt, int kh, int kw, int wt_layout,
                    int stride, int pad_y, int pad_x, int transposed, const float* bias, const float* x_scale,
                    const float* w_scale, float* y, int oh, int ow, int cout, void* work, int64_t work_bytes,
                    void* stream) {
  return conv_gather_impl("nic_conv_gather", x, n, h, w, cin, wt, kh, kw, wt_layout, stride, pad_y, pad_x, transposed,
                          bias, x_scale, w_scale, y, oh, ow, cout, 0, work, work_bytes, stream);
}

int nic_conv_gather_act(const float* x, int n, int h, int w, int cin, const float* wt, int kh, int kw, int wt_layout,
                        int stride, int pad_y, int pad_x, int transposed, const float* bias, const float* x_scale,
                        const float* w_scale, float* y, int oh, int ow, int cout, int act, void* work,
                        int64_t work_bytes, void* stream) {
  return conv_gather_impl("nic_conv_gather_act", x, n, h, w, cin, wt, kh, kw, wt_layout, stride, pad_y, pad_x,
                          transposed, bias, x_scale, w_scale, y, oh, ow, cout, act, work, work_bytes, stream);
}

int nic_act_bias_grad_work(int64_t rows, int cols, int64_t* floats) {
  if (!floats) return fail(NIC_EINVAL, "nic_act_bias_grad_work: NULL argument");
  if (rows < 0 || !train_dims_ok(cols)) return fail(NIC_ESHAPE, "nic_act_bias_grad_work: bad shape");
  *floats = (int64_t)train_abg_work_floats(rows, cols);
  return NIC_OK;
}

int nic_act_bias_grad(const float* y, const float* dy, int64_t rows, int cols, int act, float* dz, float* db,
                      float* dz_scale, float* work, int64_t work_floats, void* stream) {
  if (rows < 0 || !train_dims_ok(cols) || rows > (int64_t)INT32_MAX * 256)
    return fail(NIC_ESHAPE, "nic_act_bias_grad: bad shape rows=%lld cols=%d", (long long)rows, cols);
  if (act != 0 && act != 1) return fail(NIC_EINVAL, "nic_act_bias_grad: act must be 0 or 1");
  if (!dz && !db && !dz_scale) return fail(NIC_EINVAL, "nic_act_bias_grad: no output requested");
  if (rows > 0 && (!dy || (act && !y))) return fail(NIC_EINVAL, "nic_act_bias_grad: NULL argument");
  if (!work || work_floats < (int64_t)train_abg_work_floats(rows, cols))
    return fail(NIC_EINVAL, "nic_act_bias_grad: work holds %lld floats, needs %lld", (long long)work_floats,
                (long long)train_abg_work_floats(rows, cols));
  HIP_TRY(launch_act_bias_grad(y, dy, rows, cols, act, dz, db, dz_scale, work, (hipStream_t)stream));
  return NIC_OK;
}

int nic_conv_wgrad_work(int n, int uh, int uw, int kh, int kw, int ca, int cb, int64_t* floats) {
  if (!floats) return fail(NIC_EINVAL, "nic_conv_wgrad_work: NULL argument");
  if (n < 0 || uh <= 0 || uw <= 0 || kh <= 0 || kw <= 0 || kh * kw > 64 || !train_dims_ok(ca) || !train_dims_ok(cb))
    return fail(NIC_ESHAPE, "nic_conv_wgrad_work: bad shape");
  *floats = (int64_t)train_wgrad_work_floats(n, uh, uw, kh, kw, ca, cb);
  return NIC_OK;
}

int nic_conv_wgrad(const float* gat, int n, int gh, int gw, int ca, const float* dir, int uh, int uw, int cb, int kh,
                   int kw, int stride, int pad_y, int pad_x, const float* gat_scale, const float* dir_scale, float* dw,
                   float* work, int64_t work_floats, void* stream) {
  if (n < 0 || gh <= 0 || gw <= 0 || uh <= 0 || uw <= 0 || kh <= 0 || kw <= 0 || kh * kw > 64 || stride <= 0 ||
      !train_dims_ok(ca) || !train_dims_ok(cb) || pad_y < 0 || pad_x < 0)
    return fail(NIC_ESHAPE, "nic_conv_wgrad: bad shape");
  if (!dw) return fail(NIC_EINVAL, "nic_conv_wgrad: NULL argument");
  const int64_t need = (int64_t)train_wgrad_work_floats(n, uh, uw, kh, kw, ca, cb);
  if (n > 0 && (!gat || !dir || !work)) return fail(NIC_EINVAL, "nic_conv_wgrad: NULL argument");
  if (n > 0 && work_floats < need)
    return fail(NIC_EINVAL, "nic_conv_wgrad: work holds %lld floats, needs %lld", (long long)work_floats, (long long)need);
  HIP_TRY(launch_conv_wgrad(gat, n, gh, gw, ca, dir, uh, uw, cb, kh, kw, stride, pad_y, pad_x, gat_scale, dir_scale,
                            dw, work, (hipStream_t)stream));
  return NIC_OK;
}

int nic_gauss_1d(const float* in, int n, int h_in, int w_in, const float* taps, int ntaps, int vertical, int adjoint,
                 float* out, int h_out, int w_out, void* stream) {
  if (n < 0 || h_in <= 0 || w_in <= 0 || h_out <= 0 || w_out <= 0 || ntaps <= 0 || ntaps > 64)
    return fail(NIC_ESHAPE, "nic_gauss_1d: bad shape");
  const int d = ntaps - 1;
  const bool ok = vertical ? (w_out == w_in && (adjoint ? h_out == h_in + d : h_out == h_in - d))
                           : (h_out == h_in && (adjoint ? w_out == w_in + d : w_out == w_in - d));
  if (!ok) return fail(NIC_ESHAPE, "nic_gauss_1d: output %dx%d does not match input %dx%d", h_out, w_out, h_in, w_in);
  if (n == 0) return NIC_OK;
  if (!in || !taps || !out) return fail(NIC_EINVAL, "nic_gauss_1d: NULL argument");
  HIP_TRY(launch_gauss1d(in, n, h_in, w_in, taps, ntaps, vertical ? 1 : 0, adjoint ? 1 : 0, out, h_out, w_out,
                         (hipStream_t)stream));
  return NIC_OK;
}

int nic_ssim_map_work(int n, int64_t hw, int64_t* floats) {
  if (!floats) return fail(NIC_EINVAL, "nic_ssim_map_work: NULL argument");
  if (n < 0 || hw <= 0) return fail(NIC_ESHAPE, "nic_ssim_map_work: bad shape");
  *floats = (int64_t)train_ssim_work_floats(n, hw);
  return NIC_OK;
}

int nic_ssim_map(const float* mx, const float* my, const float* sxy, const float* sxx, int n, int64_t hw, float c1,
                 float c2, float* ssim_mean, float* work, int64_t work_floats, void* stream) {
  if (n < 0 || hw <= 0 || (int64_t)n * hw > ((int64_t)1 << 40)) return fail(NIC_ESHAPE, "nic_ssim_map: bad shape");
  if (n == 0) return NIC_OK;
  if (!mx || !my || !sxy || !sxx || !ssim_mean || !work) return fail(NIC_EINVAL, "nic_ssim_map: NULL argument");
  if (work_floats < (int64_t)train_ssim_work_floats(n, hw))
    return fail(NIC_EINVAL, "nic_ssim_map: work holds %lld floats, needs %lld", (long long)work_floats,
                (long long)train_ssim_work_floats(n, hw));
  HIP_TRY(launch_ssim_map(mx, my, sxy, sxx, n, hw, c1, c2, ssim_mean, work, (hipStream_t)stream));
  return NIC_OK;
}

int nic_ssim_map_grad(const float* mx, const float* my, const float* sxy, const float* sxx, const float* g, int n,
                      int64_t hw, float c1, float c2, float* gmx, float* gmy, float* gsxy, float* gsxx, void* stream) {
  if (n < 0 || hw <= 0 || (int64_t)n * hw > ((int64_t)1 << 40)) return fail(NIC_ESHAPE, "nic_ssim_map_grad: bad shape");
  if (n == 0) return NIC_OK;
  if (!mx || !my || !sxy || !sxx || !g || !gmx || !gmy || !gsxy || !gsxx)
    return fail(NIC_EINVAL, "nic_ssim_map_grad: NULL argument");
  HIP_TRY(launch_ssim_map_grad(mx, my, sxy, sxx, g, n, hw, c1, c2, gmx, gmy, gsxy, gsxx, (hipStream_t)stream));
  return NIC_OK;
}

int nic_adam_keras(const int64_t* table, int count, int64_t max_n, float alpha, float beta1, float beta2,
                   float epsilon, void* stream) {
  if (count < 0 || count > 65535 || max_n < 0) return fail(NIC_ESHAPE, "nic_adam_keras: bad count %d / max_n %lld", count, (long long)max_n);
  if (count == 0 || max_n == 0) return NIC_OK;
  if (!table) return fail(NIC_EINVAL, "nic_adam_keras: NULL table");
  HIP_TRY(launch_adam_keras((const long long*)table, count, (long long)max_n, alpha, beta1, beta2, epsilon,
                            (hipStream_t)stream));
  return NIC_OK;
}

int nic_absmax_scale(const float* x, int64_t count, float* scale, float* work, void* stream) {
  if (count < 0) return fail(NIC_ESHAPE, "nic_absmax_scale: negative count");
  if (!scale || !work || (count > 0 && !x)) return fail(NIC_EINVAL, "nic_absmax_scale: NULL argument");
  HIP_TRY(launch_absmax_scale(x, count, scale, work, (hipStream_t)stream));
  return NIC_OK;
}

int nic_set_precision(nic_ctx* c, int mode) {
  if (!c) return fail(NIC_EINVAL, "nic_set_precision: NULL ctx");
  if (mode != NIC_PRECISION_FP32 && mode != NIC_PRECISION_F16X3)
    return fail(NIC_EINVAL, "nic_set_precision: unknown mode %d", mode);
  c->precision = mode;
  return NIC_OK;
}

int nic_get_precision(nic_ctx* c, int* mode) {
  if (!c || !mode) return fail(NIC_EINVAL, "nic_get_precision: NULL argument");
  *mode = c->precision;
  return NIC_OK;
}

int nic_set_range_policy(nic_ctx* c, int policy) {
  if (!c) return fail(NIC_EINVAL, "nic_set_range_policy: NULL ctx");
  if (policy != NIC_RANGE_FALLBACK && policy != NIC_RANGE_ERROR)
    return fail(NIC_EINVAL, "nic_set_range_policy: unknown policy %d", policy);
  c->range_policy = policy;
  return NIC_OK;
}

int nic_range_trips(nic_ctx* c, int64_t* passes) {
  if (!c || !passes) return fail(NIC_EINVAL, "nic_range_trips: NULL argument");
  DeviceGuard guard(c->device);
  HIP_TRY(hipDeviceSynchronize());
  int words[2] = {};
  HIP_TRY(hipMemcpy(words, c->range, sizeof(words), hipMemcpyDeviceToHost));
  *passes = (int64_t)words[1] + c->error_trips;
  return NIC_OK;
}

int nic_rerun_launch_info(nic_ctx* c, int* blocks_per_cu, int* grid, int* cooperative) {
  if (!c || !blocks_per_cu || !grid || !cooperative) return fail(NIC_EINVAL, "nic_rerun_launch_info: NULL argument");
  DeviceGuard guard(c->device);
  fp32_chain_launch_info(blocks_per_cu, grid, cooperative);
  return NIC_OK;
}

int nic_set_timing(nic_ctx* c, int enable) {
  if (!c) return fail(NIC_EINVAL, "nic_set_timing: NULL ctx");
  DeviceGuard guard(c->device);
  if (enable && !c->ev[0][0]) {
    for (int i = 0; i < L_COUNT; ++i)
      for (int j = 0; j < 2; ++j) HIP_TRY(hipEventCreate(&c->ev[i][j]));
  }
  for (int i = 0; i < L_COUNT; ++i) {
    int rc = collect_layer(c, i);
    if (rc) return rc;
    c->ms_sum[i] = 0.0;
    c->launches[i] = 0;
  }
  c->timing = enable != 0;
  return NIC_OK;
}

int nic_layer_times(nic_ctx* c, double* ms_sum, int64_t* launches) {
  if (!c) return fail(NIC_EINVAL, "nic_layer_times: NULL ctx");
  DeviceGuard guard(c->device);
  for (int i = 0; i < L_COUNT; ++i) {
    int rc = collect_layer(c, i);
    if (rc) return rc;
    if (ms_sum) ms_sum[i] = c->ms_sum[i];
    if (launches) launches[i] = c->launches[i];
  }
  return NIC_OK;
}

}  // extern "C"
