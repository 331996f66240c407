/*
 * nic.h -- C-ABI of the MI355X-native learned-image-codec hot path.
 *
 * Drop-in boundary for the reference's TF2 codec surface
 * (AlexFuster/Neural_network_image_compression, tf2_0/src):
 *
 *   reference                                   replaced by
 *   ------------------------------------------  -----------------------------------------
 *   Encoder()/Decoder() + ProClass.load(path)   nic_create + nic_set_weights
 *     encoder.py:34-36, decoder.py:35-37,
 *     utils.py:15-17, 26-28
 *   Encoder.__call__(x) encoder.py:38-47        nic_encode (device) / nic_encode_host (NumPy)
 *   Decoder.__call__(z) decoder.py:39-48        nic_decode (device) / nic_decode_host (NumPy)
 *   ProClass._feed_batch pack/unpack            nic_pack_latent / nic_unpack_latent
 *     utils.py:35-36, 39-40
 *   disc_entropy tf1_13/src/training.py:66-71   nic_entropy_hist (nic_encode_entropy: fused
 *                                                 into the encoder's conv8)
 *   tf.image.ssim_multiscale(x1, x2, 255)       nic_ms_ssim
 *     tf2_0/tests/calc_ssim.py:13
 *   PSNR (the benchmark's quality figure)       nic_sq_err
 *   Training step convolutions, forward and     nic_conv_gather / nic_conv_wgrad /
 *     backward (tf2_0/src/training.py:74-151,     nic_absmax_scale / nic_gauss_1d
 *     Keras Conv2D / Conv2DTranspose SAME, SSIM)  (training side path)
 *   Training step optimiser (training.py:147-149, nic_adam_keras
 *     tf.keras Adam)
 *
 * Conventions
 *  - Every buffer argument is a DEVICE pointer owned by the caller (e.g. a torch-ROCm
 *    tensor's data_ptr()); inputs are never written.  The library owns only the weights
 *    and a scratch workspace inside the nic_ctx, grown on demand (call nic_reserve to
 *    size it ahead so no allocation happens in a timed or graph-captured call).
 *  - Work is enqueued asynchronously on the caller's hipStream_t (NULL = default
 *    stream).  One nic_ctx must not be used by two threads at once; distinct contexts
 *    are independent.  There is no global mutable state besides the per-thread error.
 *  - Layouts are NHWC uint8: images (N, H, W, 3); latents (N, ceil(H/8), ceil(W/8), 96)
 *    with channels Y0..31, Cb0..31, Cr0..31 (encoder.py:45).  Sizes need not be multiples
 *    of 8: like the reference, decode returns (N, 8h, 8w, 3).
 *  - Return 0 on success or a negative NIC_E* code; nic_last_error() describes the most
 *    recent failure on the calling thread.
 */
#ifndef NIC_H_
#define NIC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nic_ctx nic_ctx;

enum {
  NIC_OK = 0,
  NIC_EINVAL = -1,      /* null pointer, bad enum, bad layer name          */
  NIC_ESHAPE = -2,      /* tensor shape does not match the architecture    */
  NIC_ENOWEIGHTS = -3,  /* encode/decode before every tensor was set       */
  NIC_EHIP = -4,        /* HIP runtime error                               */
  NIC_ENOMEM = -5,      /* device allocation failed                        */
  NIC_ERANGE = -6       /* NIC_RANGE_ERROR: a split-f16 activation left the f16 range */
};

/* model_id values for nic_set_weights (checkpoint names encoder{Y,CbCr}, decoder{Y,CbCr},
 * training.py:167-172) */
enum {
  NIC_MODEL_ENCODER_Y = 0,
  NIC_MODEL_ENCODER_CBCR = 1,
  NIC_MODEL_DECODER_Y = 2,
  NIC_MODEL_DECODER_CBCR = 3
};

/* Arithmetic of the convolutions:
 *   NIC_PRECISION_FP32  -- exact-fp32 MFMA (v_mfma_f32_32x32x2_f32) for conv2..conv8 and
 *     dconv1..dconv7: an fp32 FMA chain; conv1 and dconv8 as fp32 VALU FMA.
 *   NIC_PRECISION_F16X3 -- split-f16 MFMA (default) for every convolution, conv1 (fused
 *     into conv2's kernel) and dconv8 included: each fp32 operand x = hi + lo with hi, lo
 *     f16 and weights pre-scaled by 2^k; a*w ~ a_hi*w_hi + a_hi*w_lo + a_lo*w_hi on
 *     v_mfma_f32_16x16x32_f16 / v_mfma_f32_32x32x16_f16 with fp32 accumulation.  Error
 *     ~2^-22 relative per product, i.e. at the level of fp32 accumulation-order
 *     differences.  The split format holds |x| < 65504 (the f16 range): see the range guard.
 *     Its kernels use 32-bit offsets inside one plane: images whose 64-channel level
 *     (ceil(h/4) x ceil(w/4), resp. 2*h8 x 2*w8 for decode) exceeds 2^22 pixels (~67 MP per
 *     image) run the NIC_PRECISION_FP32 kernels instead (same results class, no error).
 * Bias, activations, residuals, colour transforms and quantisers are fp32 in both modes. */
enum { NIC_PRECISION_FP32 = 0, NIC_PRECISION_F16X3 = 1 };

/* f16 range guard of NIC_PRECISION_F16X3 (the reference, encoder.py:19-32 / decoder.py:19-32,
 * has no activation bound; trained weights may drive an activation past the f16 range).
 * Every kernel that stores a split activation tracks max |x| and, at |x| >= 65504 or a
 * non-finite x, marks the ctx's range word with the pass's epoch.  Then:
 *   NIC_RANGE_FALLBACK (default) -- every split-f16 encode/decode pass is followed on the
 *     same stream by the exact-fp32 pass (NIC_PRECISION_FP32 kernels) gated on that mark:
 *     its kernels exit at once unless the split pass tripped, in which case they recompute
 *     and overwrite every output.  No host synchronisation; results always fp32-class.
 *   NIC_RANGE_ERROR -- the call synchronises its stream after the split pass and returns
 *     NIC_ERANGE if it tripped (outputs undefined).
 * nic_range_trips (synchronising) counts the passes that tripped since nic_create.
 * A FALLBACK re-run runs as one chained launch whose stages hand their tiles out through
 * device-side queues (no grid barrier): it completes whatever share of the grid is resident,
 * so a tripped FALLBACK call always returns the exact-fp32 outputs. */
enum { NIC_RANGE_FALLBACK = 0, NIC_RANGE_ERROR = 1 };
int nic_set_range_policy(nic_ctx* ctx, int policy);
int nic_range_trips(nic_ctx* ctx, int64_t* passes);
/* How the chained exact-fp32 re-run launches on ctx's device: its resident blocks per CU
 * (occupancy; informational -- the queued stages need no co-residency), the grid (one block
 * per CU) and whether it uses a cooperative launch (always 0: a plain launch). */
int nic_rerun_launch_info(nic_ctx* ctx, int* blocks_per_cu, int* grid, int* cooperative);

/* ABI version: major * 10000 + minor * 100 + patch */
int nic_version(void);

/* Host copies of the fp32 colour constants the device uses: fp32(ycbcr_kernel) (utils.py:7),
 * fp32(inv(ycbcr_kernel)) computed in float64 (utils.py:8), fp32(ycbcr_off) (utils.py:9).
 * Row-major 3x3; any pointer may be NULL. */
int nic_constants(float* ycbcr9, float* ycbcr_inv9, float* off3);

/* Human-readable description of the last error on this thread ("" if none). */
const char* nic_last_error(void);

/* Create a context on HIP device `device`. */
int nic_create(int device, nic_ctx** out);
int nic_destroy(nic_ctx* ctx);

/* Upload one tensor in its Keras layout from HOST memory (fp32, C order).
 *   layer: "conv1".."conv8" (Conv2D kernel (kh,kw,Cin,Cout), encoder.py:10-17) or
 *          "dconv1".."dconv8" (Conv2DTranspose kernel (kh,kw,Cout,Cin), decoder.py:10-17),
 *          followed by "/kernel" or "/bias" (bias shape (Cout,)).
 * The kernel is repacked to the device-native fragment layout.  Synchronous. */
int nic_set_weights(nic_ctx* ctx, int model_id, const char* layer, const float* host, const int64_t* shape,
                    int ndim);

int nic_set_precision(nic_ctx* ctx, int mode);
int nic_get_precision(nic_ctx* ctx, int* mode);

/* 1 when every tensor of the encoder pair (resp. decoder pair) has been set. */
int nic_weights_ready(nic_ctx* ctx, int* encoder_ready, int* decoder_ready);

/* Grow the workspace so encode of (n, h, w) images and decode of their latents allocate
 * nothing.  Synchronous. */
int nic_reserve(nic_ctx* ctx, int n, int h, int w);

/* Latent spatial size for an h x w image: ceil(h/8), ceil(w/8) (TF SAME, three s2 convs). */
int nic_latent_shape(int h, int w, int* h8, int* w8);

/* Encoder.__call__: rgb (n,h,w,3) u8 -> latent (n,h8,w8,96) u8.
 * prequant (nullable): (n,h8,w8,96) fp32, the clipped encoder output before round(x*255). */
int nic_encode(nic_ctx* ctx, const uint8_t* rgb, int n, int h, int w, uint8_t* latent, float* prequant,
               void* stream);

/* Decoder.__call__: latent (n,h8,w8,96) u8 -> rgb (n,8*h8,8*w8,3) u8.
 * rgb_f32 (nullable): the clipped fp32 RGB before round(x*255). */
int nic_decode(nic_ctx* ctx, const uint8_t* latent, int n, int h8, int w8, uint8_t* rgb, float* rgb_f32,
               void* stream);

/* Host-array surface: Encoder.__call__ / Decoder.__call__ on NumPy batches (encoder.py:38-47,
 * decoder.py:39-48 hand host arrays in and out around every call).  rgb / latent are HOST
 * pointers; the call is ordered after the work queued on `stream` and returns with the
 * outputs written (synchronous).  The batch runs as `chunks` (1..16) chunks on the ctx's own
 * streams, chunk k+1's H2D and chunk k-1's D2H overlapping chunk k's device pass; page-locked
 * buffers are DMA'd directly, pageable ones staged through the ctx's pinned buffers. */
int nic_encode_host(nic_ctx* ctx, const uint8_t* rgb, int n, int h, int w, uint8_t* latent, int chunks,
                    void* stream);
int nic_decode_host(nic_ctx* ctx, const uint8_t* latent, int n, int h8, int w8, uint8_t* rgb, int chunks,
                    void* stream);

/* Histogram entropy of each latent plane (tf1_13/src/training.py:66-71).
 * Plane order is the reference's concat along the batch: row p = plane p/n (Y,Cb,Cr) of
 * image p%n.  counts (nullable): (3n, 256) uint32.  bits (nullable): (3n,) fp32
 * bits/symbol.  Needs a ctx only for its scratch. */
int nic_entropy_hist(nic_ctx* ctx, const uint8_t* latent, int n, int h8, int w8, uint32_t* counts, float* bits,
                     void* stream);

/* Encode + histogram entropy of the new latent in one pass (BASELINE config 5: the encoder
 * followed by disc_entropy, tf1_13/src/training.py:66-71): same outputs as nic_encode then
 * nic_entropy_hist -- latent, counts (nullable), bits (nullable) -- with the codes counted in
 * conv8's epilogue as it quantises them (no re-read of the latent).  Shapes where the fold does
 * not apply (exact-fp32 precision, latents too small for one plane per block range) run the
 * two calls. */
int nic_encode_entropy(nic_ctx* ctx, const uint8_t* rgb, int n, int h, int w, uint8_t* latent, uint32_t* counts,
                       float* bits, void* stream);
/* 1 in *folds when nic_encode_entropy on (n, h, w) images (counts or bits requested) takes the
 * folded form on ctx's device and precision, 0 when it runs the two calls.  Shapes the call
 * refuses (NIC_ESHAPE: bad sizes, n > 21845, latent planes over 2^31 / 6 codes) and n = 0 are
 * refused the same way. */
int nic_encode_entropy_fold(nic_ctx* ctx, int n, int h, int w, int* folds);

/* MS-SSIM of tf.image.ssim_multiscale(a, b, max_val=255) (tf2_0/tests/calc_ssim.py:13)
 * per image: a, b u8 (n,h,w,3) -> ms_ssim (n,) fp32.  TF defaults: 11-tap Gaussian
 * (sigma 1.5), k1 0.01, k2 0.03, power factors (0.0448, 0.2856, 0.3001, 0.2363, 0.1333),
 * SYMMETRIC-padded 2x2 average pooling between scales; every scale >= 11 px: h, w >= 161.
 * per_scale (nullable): (n,3,5,2) fp32 mean SSIM and mean cs per channel and scale.
 * fp32 filtering, fp64 reductions.  Needs a ctx only for its scratch. */
int nic_ms_ssim(nic_ctx* ctx, const uint8_t* a, const uint8_t* b, int n, int h, int w, float* ms_ssim,
                float* per_scale, void* stream);

/* Exact per-image sum of squared differences of two u8 tensors of n images of
 * bytes_per_image bytes: sse (n,) uint64.  PSNR = 10 log10(255^2 * bytes / sse). */
int nic_sq_err(const uint8_t* a, const uint8_t* b, int n, int64_t bytes_per_image, uint64_t* sse, void* stream);

/* PNG files of m u8 images (h, w, channels = 1 or 3) in HOST memory, on `threads` host
 * threads (no GPU, no ctx; w * channels <= 16384), in one of two encoders' settings:
 *   NIC_PNG_PILLOW  Pillow with optimize=True, the reference's bitstream writer save_img
 *                   (utils.py:85-87): adaptive per-row filter (least sum of |signed bytes|,
 *                   first on ties), zlib level 9 / window 15 / memLevel 9 / Z_FILTERED,
 *                   65,536-B IDATs -- byte for byte Pillow's file (tests/test_png_encode.py;
 *                   Pillow and this library link the same zlib 1.2.11 here).
 *   NIC_PNG_TF      tf.image.encode_png(compression=-1), what get_bpp sizes
 *                   (training.py:12-21): libpng 1.6 defaults -- the same filter heuristic,
 *                   zlib default level (6) / memLevel 9 (png_io sets MAX_MEM_LEVEL) /
 *                   Z_FILTERED, libpng's window reduction and CMF rewrite for small images and
 *                   its filter pruning for 1-row / 1-column images, 8,192-B IDATs.  TensorFlow is
 *                   not importable here: parity with its own output is UNPINNED.
 * nic_png_encode writes file i at out + i * out_stride (out_stride >= nic_png_bound; out may
 * be NULL for sizes only) and its byte count to sizes[i].  nic_png_sizes = the Pillow sizes
 * (the val_bpp of training.py:157-163 and the RD harness). */
#define NIC_PNG_PILLOW 0
#define NIC_PNG_TF 1
int nic_png_bound(int h, int w, int channels, int mode, int64_t* bytes);
int nic_png_encode(const uint8_t* images, int m, int h, int w, int channels, int mode, uint8_t* out,
                   int64_t out_stride, int64_t* sizes, int threads);
int nic_png_sizes(const uint8_t* images, int m, int h, int w, int channels, int64_t* sizes, int threads);

/* Bitstream image layout of ProClass._feed_batch: (n,h8,w8,96) <-> (n,4*h8,8*w8,3), each
 * plane a raw C-order reshape (utils.py:35-36, 39-40). */
int nic_pack_latent(const uint8_t* latent, int n, int h8, int w8, uint8_t* packed, void* stream);
int nic_unpack_latent(const uint8_t* packed, int n, int h8, int w8, uint8_t* latent, void* stream);

/* ---- Training side path (tf2_0/src/training.py:74-151): the step's convolutions ------------
 * NHWC fp32 device tensors, split-f16x3 MFMA (fp32-class), kernels of Keras layouts, no ctx.
 * Every forward and backward convolution of the step is one of two GEMMs:
 *
 * nic_conv_gather: y[b][oy][ox][co] = bias[co] + sum over taps (ky,kx), ci of
 *     x[b][src_y][src_x][ci] * W(ky,kx,ci,co), with
 *       transposed = 0: src = stride * o + k - pad   (Conv2D forward; input grad of Conv2DTranspose)
 *       transposed = 1: src = (o + pad - k) / stride, taps where it divides (Conv2DTranspose
 *                       forward; input grad of Conv2D)
 *     W(ky,kx,ci,co) = wt[((ky*kw+kx)*cin + ci)*cout + co]  (wt_layout 0, Conv2D HWIO)
 *                    = wt[((ky*kw+kx)*cout + co)*cin + ci]  (wt_layout 1, Conv2DTranspose HWOI)
 *     bias nullable; x_scale / w_scale nullable device floats (power-of-two operand scales from
 *     nic_absmax_scale, undone exactly in the epilogue).  work: 16-B aligned device scratch of
 *     nic_conv_gather_work() bytes (the split weights).  cin, cout <= 64.
 * nic_conv_gather_act: the same with act = 1 applying the layers' activation in the epilogue,
 *     y = leaky_relu(bias + sum, 0.2) (Keras Conv2D(..., activation=tf.nn.leaky_relu),
 *     encoder.py:10-17 / decoder.py:10-17); act = 0 is nic_conv_gather.
 * nic_act_bias_grad: the backward of that epilogue over a (rows, cols) NHWC tensor (rows = n h w):
 *     dz = dy * (act && !(y > 0) ? 0.2 : 1) (tf.nn.leaky_relu's gradient, from the layer's output
 *     y), db[c] = sum over rows of dz[row][c] (BiasAddGrad) and dz_scale[0] = nic_absmax_scale
 *     of dz, from one pass; any output may be NULL (not all; act = 0 and dz NULL: dz is dy).
 *     Deterministic (per-block column sums in `work`, added in block order); work must hold
 *     nic_act_bias_grad_work() floats.  cols <= 64.
 * nic_conv_wgrad: dw[ky][kx][a][b'] = sum over b, u of
 *     gat[b][stride*uy+ky-pad_y][stride*ux+kx-pad_x][a] * dir[b][uy][ux][b']
 *     (Conv2D: gat = x, dir = dy, dw HWIO; Conv2DTranspose: gat = dy, dir = x, dw HWOI);
 *     deterministic (per-slice partials in `work`, summed in order); work must hold
 *     nic_conv_wgrad_work() floats.  ca, cb <= 64.
 * nic_absmax_scale: scale[0] = 2^(13 - floor(log2 max|x|)) (1 for 0 / non-finite), so the
 *     split-f16 operands keep every bit of tiny gradients; work >= 512 floats.
 * nic_gauss_1d: one-channel planes (n,h,w): VALID correlation with ntaps taps along x
 *     (vertical 0) or y, or its adjoint (the input gradient); the SSIM loss's separable
 *     Gaussian (tf.image.ssim, training.py:119-121).
 * nic_ssim_map: the SSIM loss's map from its Gaussian-filtered terms (tf.image.ssim,
 *     training.py:119-121): per pixel of n planes of hw pixels, from mx = G*x, my = G*y,
 *     sxy = G*(x y), sxx = G*(x^2 + y^2): num0 = (mx my) 2, den0 = mx mx + my my,
 *     lum = (num0 + c1)/(den0 + c1), cs = ((2 sxy - num0) + c2)/((sxx - den0) + c2); ssim_mean[i] =
 *     mean of lum cs over plane i (deterministic; work >= nic_ssim_map_work() floats).
 * nic_ssim_map_grad: the gradients of sum_i g[i] ssim_mean[i] with respect to mx, my, sxy, sxx.
 * nic_adam_keras: the step's optimiser update (training.py:147-149, tf.keras Adam = TF's
 *     ResourceApplyAdam) over `count` tensors in one launch; table = device int64 records
 *     {var, m, v, grad, n} (pointers to fp32 device buffers, n elements), max_n their largest n:
 *       m += (g - m)*(1 - beta1);  v += (g*g - v)*(1 - beta2);  var -= (m*alpha)/(sqrt(v) + epsilon)
 *     each op an fp32 rounding; alpha = lr*sqrt(1 - beta2^t)/(1 - beta1^t) from the caller. */
int nic_conv_gather_work(int kh, int kw, int cin, int cout, int64_t* bytes);
int nic_conv_gather(const float* x, int n, int h, int w, int cin, const float* wt, int kh, int kw, int wt_layout,
                    int stride, int pad_y, int pad_x, int transposed, const float* bias, const float* x_scale,
                    const float* w_scale, float* y, int oh, int ow, int cout, void* work, int64_t work_bytes,
                    void* stream);
int nic_conv_gather_act(const float* x, int n, int h, int w, int cin, const float* wt, int kh, int kw, int wt_layout,
                        int stride, int pad_y, int pad_x, int transposed, const float* bias, const float* x_scale,
                        const float* w_scale, float* y, int oh, int ow, int cout, int act, void* work,
                        int64_t work_bytes, void* stream);
int nic_act_bias_grad_work(int64_t rows, int cols, int64_t* floats);
int nic_act_bias_grad(const float* y, const float* dy, int64_t rows, int cols, int act, float* dz, float* db,
                      float* dz_scale, float* work, int64_t work_floats, void* stream);
int nic_conv_wgrad_work(int n, int uh, int uw, int kh, int kw, int ca, int cb, int64_t* floats);
int nic_conv_wgrad(const float* gat, int n, int gh, int gw, int ca, const float* dir, int uh, int uw, int cb, int kh,
                   int kw, int stride, int pad_y, int pad_x, const float* gat_scale, const float* dir_scale, float* dw,
                   float* work, int64_t work_floats, void* stream);
int nic_absmax_scale(const float* x, int64_t count, float* scale, float* work, void* stream);
int nic_gauss_1d(const float* in, int n, int h_in, int w_in, const float* taps, int ntaps, int vertical, int adjoint,
                 float* out, int h_out, int w_out, void* stream);
int nic_ssim_map_work(int n, int64_t hw, int64_t* floats);
int nic_ssim_map(const float* mx, const float* my, const float* sxy, const float* sxx, int n, int64_t hw, float c1,
                 float c2, float* ssim_mean, float* work, int64_t work_floats, void* stream);
int nic_ssim_map_grad(const float* mx, const float* my, const float* sxy, const float* sxx, const float* g, int n,
                      int64_t hw, float c1, float c2, float* gmx, float* gmy, float* gsxy, float* gsxx, void* stream);
int nic_adam_keras(const int64_t* table, int count, int64_t max_n, float alpha, float beta1, float beta2,
                   float epsilon, void* stream);

/* Per-layer device timing.  With timing on, every kernel launch of encode/decode is
 * bracketed by a hipEvent pair on the caller's stream (the stream the kernel runs on);
 * nic_layer_times returns, per layer in the order conv1, conv2, conv3, conv4, conv8,
 * dconv1, dconv5, dconv6, dconv7, dconv8 (NIC_LAYER_COUNT entries), the summed
 * milliseconds and launch counts since timing was (re)enabled.  Both synchronise on
 * the recorded events. */
#define NIC_LAYER_COUNT 10
int nic_set_timing(nic_ctx* ctx, int enable);
int nic_layer_times(nic_ctx* ctx, double* ms_sum, int64_t* launches);

#ifdef __cplusplus
}
#endif

#endif /* NIC_H_ */
