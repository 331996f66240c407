// Internal kernel interface (not part of the public C-ABI; see include/nic.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nic {

int set_error(int code, const char* msg);  // nic_last_error() text of this thread (nic_capi.hip)

// Activation formats in HBM: fp32 NHWC (exact-fp32 mode) or "split" NHWC: per pixel
// [hi: C f16][lo: C f16] with x = hi + lo, hi = f16(x), lo = f16(x - hi) (f16x3 mode; the
// same 4 B per element, split once by the producer's epilogue).
// IN_U8_CODES: the u8 latent as exact f16 codes (0..255); the 1/255 of the dequantiser is
// folded into the epilogue scale, so the activation needs no lo half (2 MFMAs per MAC)
enum InMode { IN_F32 = 0, IN_U8_LATENT = 1, IN_SPLIT = 2, IN_SPLIT_DMA = 3, IN_U8_CODES = 4 };
enum OutMode { OUT_F32 = 0, OUT_U8_LATENT = 1, OUT_SPLIT = 2 };

enum LayerId {
  L_CONV1 = 0, L_CONV2, L_CONV3, L_CONV4, L_CONV8,
  L_DCONV1, L_DCONV5, L_DCONV6, L_DCONV7, L_DCONV8,
  L_COUNT
};

// f16 range guard of the split format: a split-f16 producer whose fp32 value reaches the
// f16 limit (|v| >= 65504, or non-finite) stores `epoch` into *flag (one word per ctx); the
// exact-fp32 re-run of the pass is gated on *gate == epoch (fp32 kernels exit otherwise).
constexpr float kF16Limit = 65504.0f;
struct RangeGuard {
  int* flag = nullptr;        // f16x3 producers: set to epoch on overflow
  const int* gate = nullptr;  // fp32 kernels: run only when *gate == epoch
  int* trips = nullptr;       // head kernel of a gated re-run: +1 when it runs
  int epoch = 0;
};

struct ConvArgs {
  RangeGuard rg;
  const float* in;        // [P][H][W][Cin] fp32 (IN_F32)
  const uint8_t* in_u8;   // [N][H][W][96] latent (IN_U8_LATENT)
  float* out;             // [P][OH][OW][Cout] fp32 (OUT_F32)
  const float* res;       // residual, same layout as out
  const uint16_t* in_s;   // [P][H][W][2][Cin] split f16 (IN_SPLIT)
  uint16_t* out_s;        // [P][OH][OW][2][Cout] split f16 (OUT_SPLIT)
  const uint16_t* res_s;  // residual in split format
  const char* zero16;     // >= 16 zero bytes in global memory (DMA source for padding)
  uint8_t* out_u8;        // [N][OH][OW][96] latent (OUT_U8_LATENT)
  float* out_f32_latent;  // optional clipped fp32 latent, same layout as out_u8
  const float* w;         // fp32 path: repacked weights [2 models][taps][Cin/8][2][Cout][4]
  const uint16_t* wx;     // f16x3 path: [2 models][taps][Cin/16][hi,lo][2][Cout][8] fp16 of w*2^k
  float wscale[2];        // f16x3 path: 2^-k per model (exact), undoes the weight pre-scale
  const float* bias;      // [2][Cout]
  int P, nimg;            // planes (= 3 * nimg), images
  int H, W;               // input spatial dims
  int OH, OW;             // output spatial dims
  int pad_y, pad_x;       // forward conv TF-SAME pad_lo
  int tiles_x;            // set by the launcher
  int tiles_y, ntiles;    // pipelined kernels: tile grid (set by the launcher)
  int ws_taps;            // weight-stationary kernels: taps per model in wx
  int ws_ngrp;            // weight-stationary kernels: block groups (tap set x model)
  int ws_blk[9];          // weight-stationary kernels: first block of each group, then the grid
  int ws_xcd;             // weight-stationary kernels: logical block = XCD-contiguous remap of blockIdx
  // conv8 (f16x3, OUT_U8_LATENT) with the latent histogram folded in (nic_encode_entropy):
  // the counts [3 nimg][256], zero on entry, added to with device-scope atomics
  uint32_t* hist_part;
  // fused k3 residual pair (conv3 -> conv4 -> + x, dconv5 -> dconv6 -> + x): the second
  // layer's weights (wx / wscale / bias are the first layer's), rows per block segment
  const uint16_t* wx2;
  float wscale2[2];
  const float* bias2;
  int seg_rows;
  // conv1 fused into conv2 (f16x3): the colour plane is computed from the RGB input and
  // conv1's split output is written straight into conv2's LDS halo (no HBM round trip)
  const uint8_t* rgb;     // [N][H0][W0][3]
  const uint16_t* wx1;    // conv1 MFMA A fragments [2 models][2 co tiles][hi,lo][64 lanes][8] of w*2^k
  float wscale1[2];       // 2^-k per model for wx1
  const float* bias1;     // [2][32]
  int H0, W0;             // image size (conv1 input)
  int p1y, p1x;           // conv1 TF-SAME pad_lo
  uint16_t* cplane;       // padded split colour planes [hi, lo][P][cp_h][cp_w] f16 (c12_plane_geom)
  int cp_h, cp_w;
  // dconv8 projection fused into dconv7 (f16x3): per dconv7 output pixel the 25 phase-tap
  // dot products with dconv8's kernel, tile-major [P][4 phases][tiles_y][tiles_x][25][64 px]
  float* proj;
  const uint16_t* proj_w;  // MFMA B fragments [2 models][2 tap blocks][Cin/32][hi,lo][64 lanes][8] of w8*2^k
  float proj_scale[2];     // 2^-k per model
};

struct Conv1Args {
  RangeGuard rg;
  const uint8_t* rgb;  // [N][H][W][3]
  float* out;          // [P][OH][OW][32] fp32 (exact mode)
  uint16_t* out_s;     // [P][OH][OW][2][32] split f16 (f16x3 mode), used when non-null
  const float* w;      // [2][26][32]
  const float* bias;   // [2][32]
  int P, nimg, H, W, OH, OW, pad_y, pad_x, tiles_x, tiles_y;
};

struct Dconv8Args {
  RangeGuard rg;
  const float* in;      // [P][H][W][64] fp32 (exact mode)
  const uint16_t* in_s; // [P][H][W][2][64] split f16 (f16x3 mode)
  const char* zero16;   // DMA padding source
  uint8_t* out_u8;      // [N][2H][2W][3]
  float* out_f32;       // optional clipped fp32 RGB, same layout
  const float* w;       // fp32 path: [2][25 phase-taps][64]
  const uint16_t* wx;   // f16x3 path: [2][9 nbr][2 chunk][hi,lo][64 lanes][8] MFMA A fragments
  float wscale[2];      // f16x3 path: 2^-k per model
  const float* bias;    // [2]
  int nimg, H, W, tiles_x, tiles_y;
  const float* proj;           // gather kernel: dconv7's projections (ConvArgs::proj layout)
  int tiles_y7, tiles_x7;      // gather kernel: dconv7's 8x8 tile grid over its coarse input
};

// The gated exact-fp32 re-run of a split-f16 pass as one launch (stages run in
// order with grid barriers; every block exits at once unless gate.gate == gate.epoch).
constexpr int kChainMax = 6;
constexpr int kChainQWords = 2 * kChainMax + 1;  // Fp32Chain::q
struct Fp32Chain {
  RangeGuard gate;  // gate + trips of the re-run (the stages' own rg fields are unused)
  int* q;           // kChainQWords zeroed device words: per stage next tile, tiles done; blocks out
  int nstage;
  int diag_late;    // NIC_DIAG_CHAIN (launch_fp32_chain fills it): block 0 starts ~1 ms late
  int total[kChainMax];     // tiles of each stage
  int kind[kChainMax];      // LayerId; L_CONV1 -> c1, L_DCONV8 -> d8, other layers -> c[s]
  ConvArgs c[kChainMax];
  Conv1Args c1;
  Dconv8Args d8;
};
hipError_t chain_add_layer(Fp32Chain& ch, LayerId id, ConvArgs a);
hipError_t chain_add_conv1(Fp32Chain& ch, Conv1Args a);
hipError_t chain_add_dconv8(Fp32Chain& ch, Dconv8Args a);
hipError_t launch_fp32_chain(const Fp32Chain& ch, hipStream_t st);
void fp32_chain_launch_info(int* blocks_per_cu, int* grid, int* cooperative);  // current device

hipError_t upload_constants(const float* u8_to_unit, const float* ycbcr, const float* ycbcr_inv, const float* off);
hipError_t launch_layer(LayerId id, const ConvArgs& a, hipStream_t st);      // exact fp32 MFMA
hipError_t launch_layer_x3(LayerId id, const ConvArgs& a, hipStream_t st);   // split-f16 (3-pass) MFMA
// the residual pair x -> leaky(conv_b(leaky(conv_a(x)))) + x of two k3 s1 64-channel layers as
// one launch (split-f16), for planes up to K3P_MAX_W columns; false: use two launches
bool k3pair_supported(int H, int W);
hipError_t launch_k3pair_x3(const ConvArgs& a, hipStream_t st);
hipError_t launch_conv12_x3(const ConvArgs& a, hipStream_t st);  // conv1 fused into conv2 (f16x3)
// the fused conv1's padded colour planes: origin offsets and plane size in f16 elements
// (a.cplane must hold 2 * P * hp * wp of them)
void c12_plane_geom(int OH, int OW, int pad_y, int pad_x, int p1y, int p1x, int* oy, int* ox, int* hp, int* wp);
hipError_t launch_conv1(Conv1Args a, hipStream_t st);
hipError_t launch_dconv8(Dconv8Args a, hipStream_t st);      // exact fp32 VALU
// f16x3 decoder tail with dconv8 split across two kernels: dconv7 writes the 25 projections
// of every output pixel instead of its 64 channels, the gather sums them per output pixel
hipError_t launch_dconv7_proj_x3(const ConvArgs& a, hipStream_t st);
hipError_t launch_dconv8_gather(Dconv8Args a, hipStream_t st);
// histogram entropy: per-block partial counts into `part` (hist_scratch_bytes), then one
// reduce kernel writes counts (optional) and bits/symbol (optional)
size_t hist_scratch_bytes(int nimg, int plane_px);
hipError_t launch_hist(const uint8_t* z, int nimg, int plane_px, uint32_t* part, uint32_t* counts, float* bits,
                       hipStream_t st);
// the histogram folded into conv8 (nic_encode_entropy): whether the split-f16 conv8 launch can
// count for this shape (each block's strided walk visits >= 2 tiles of every plane it touches:
// blocks of a model group <= conv8 tiles per plane / 2), the [3 nimg][256] count accumulator
// conv8's blocks add into with device-scope atomics (LDS histograms alternated by plane parity,
// flushed one tile after the plane changes), and the reduce that reads + clears it (counts /
// bits; a tripped range guard -- the latent rewritten by the exact-fp32 re-run -- recounts from z)
bool hist_fold_supported(int nimg, int h8, int w8);
size_t hist_fold_scratch_bytes(int nimg, int h8, int w8);
hipError_t launch_hist_fold(uint32_t* part, const uint8_t* z, int nimg, int h8, int w8, RangeGuard trip,
                            uint32_t* counts, float* bits, hipStream_t st);
hipError_t launch_pack(const uint8_t* src, uint8_t* dst, int nimg, int h8, int w8, bool unpack, hipStream_t st);

// --- quality metrics (nic_quality.hip) ---------------------------------------------------
constexpr int kSsimScales = 5;  // tf.image.ssim_multiscale power_factors

struct SsimScaleArgs {
  const uint8_t* a8;  // scale 0: u8 NHWC (N,H,W,3)
  const uint8_t* b8;
  const float* af;    // scales 1..4: planar fp32 (P,H,W)
  const float* bf;
  double2* part;      // [P][tiles] (sum ssim, sum cs) per output tile
  int P, H, W, tiles_x, tiles;
};

struct SsimCombineArgs {
  const double2* part;
  size_t offset[kSsimScales];  // in double2 units
  int tiles[kSsimScales];
  int64_t valid[kSsimScales];  // valid filter outputs per plane
  float* out;                  // (N,)
  float* per_scale;            // optional (N,3,5,2): mean ssim, mean cs
};

// Scratch layout of one MS-SSIM evaluation: pooled images of scales 1..4, then the tile sums.
struct SsimPlan {
  int h[kSsimScales], w[kSsimScales], tiles_x[kSsimScales], tiles[kSsimScales];
  int64_t valid[kSsimScales];
  size_t img_off[kSsimScales];  // bytes
  size_t part_off[kSsimScales]; // double2 units after img_bytes
  size_t img_bytes, bytes;
};
hipError_t upload_ssim_constants();  // per device, from nic_create
void ssim_plan(int nimg, int H, int W, SsimPlan* plan);
hipError_t launch_ms_ssim(const uint8_t* a, const uint8_t* b, int nimg, int H, int W, void* scratch, float* out,
                          float* per_scale, hipStream_t st);
hipError_t launch_sq_err(const uint8_t* a, const uint8_t* b, int nimg, int64_t bytes, unsigned long long* sse,
                         hipStream_t st);

// --- training side path (nic_train.hip) ------------------------------------------------------
size_t train_scale_work_floats();
size_t train_wgrad_work_floats(int n, int uh, int uw, int kh, int kw, int ca, int cb);
size_t train_gather_work_bytes(int kh, int kw, int cin, int cout);
hipError_t launch_absmax_scale(const float* x, long long n, float* scale, float* work, hipStream_t st);
hipError_t launch_conv_gather(const float* x, int n, int h, int w, int cin, const float* wt, int kh, int kw, int layout,
                              int stride, int pad_y, int pad_x, int transposed, const float* bias, const float* x_scale,
                              const float* w_scale, float* y, int oh, int ow, int cout, int act, void* work, hipStream_t st);
size_t train_abg_work_floats(long long rows, int cols);
hipError_t launch_act_bias_grad(const float* y, const float* dy, long long rows, int cols, int act, float* dz, float* db,
                                float* dz_scale, float* work, hipStream_t st);
hipError_t launch_conv_wgrad(const float* gat, int n, int gh, int gw, int ca, const float* dir, int uh, int uw, int cb,
                             int kh, int kw, int stride, int pad_y, int pad_x, const float* gat_scale,
                             const float* dir_scale, float* dw, float* work, hipStream_t st);
// tf.keras Adam over `count` tensors (table: {var, m, v, grad, n} int64 records on the device)
hipError_t launch_adam_keras(const long long* table, int count, long long max_n, float alpha, float beta1,
                             float beta2, float eps, hipStream_t st);
size_t train_ssim_work_floats(int n, long long hw);
hipError_t launch_ssim_map(const float* mx, const float* my, const float* sxy, const float* sxx, int n, long long hw,
                           float c1, float c2, float* out, float* work, hipStream_t st);
hipError_t launch_ssim_map_grad(const float* mx, const float* my, const float* sxy, const float* sxx, const float* g,
                                int n, long long hw, float c1, float c2, float* gmx, float* gmy, float* gsxy,
                                float* gsxx, hipStream_t st);
hipError_t launch_gauss1d(const float* in, int n, int hi, int wi, const float* taps, int nt, int vertical, int adjoint,
                          float* out, int ho, int wo, hipStream_t st);

}  // namespace nic
