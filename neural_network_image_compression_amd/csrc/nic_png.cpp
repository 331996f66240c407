// PNG files of u8 images on host threads, in one of two encoders' exact settings.
//
// Reference: the bitstream writer save_img (tf2_0/src/utils.py:85-87) is Pillow with
// optimize=True; the training target get_bpp (tf2_0/src/training.py:12-21) sizes
// tf.image.encode_png (compression=-1) output of every latent plane reshaped to (4h, 8w).
//
// NIC_PNG_PILLOW -- Pillow 12 / libImaging ZipEncode for an 8-bit L or RGB image with
// optimize=True, as established against Pillow's own files (tests/test_png_sizes.py,
// tests/test_png_encode.py: byte for byte):
//   * every row is filtered with the PNG filter (None, Sub, Up, Average, Paeth; neighbours a
//     pixel = 1 or 3 bytes back) whose output bytes, read as signed, have the least sum of
//     absolute values (first on ties);
//   * the filtered rows (filter byte + row) go through zlib deflate level 9, window 15,
//     memLevel 9, Z_FILTERED, in one stream;
//   * the stream is cut into IDAT chunks of 65,536 bytes (the encoder's buffer size for
//     rows up to 16,384 bytes), framed by the signature, IHDR and IEND:
//     size = 8 + 25 + sum(12 + idat_i) + 12.
// NIC_PNG_TF -- tf.image.encode_png(compression=-1): TensorFlow's png_io WriteImageToBuffer
// on libpng 1.6 defaults: the same adaptive filter choice (libpng's minimum-sum-of-absolute-
// differences heuristic over all five filters, first on ties, zero row above the first),
// deflate at zlib's default level (Z_DEFAULT_COMPRESSION = 6), memLevel 9 (png_io's
// png_set_compression_mem_level(MAX_MEM_LEVEL) after the level), Z_FILTERED, the
// window reduced for images under 16 KiB of filtered data (png_deflate_claim; the stream is
// the same, only the zlib header's window field differs, which optimize_cmf rewrites as
// libpng does), IDAT chunks of libpng's 8,192-byte zbuffer, no ancillary chunks.  TensorFlow
// is not importable here, so this mode is a restatement of those libraries' published
// behaviour: parity with TF's own output is unpinned.  libpng's png_write_start_row prunes the
// candidate filters of degenerate images: one row drops Up, Average and Paeth, one pixel
// column drops Sub, Average and Paeth (restated here in TF mode; Pillow tries all five).
// Byte equality with Pillow also assumes the deflate Pillow links is the same algorithm as the
// system zlib this library links (-lz): true for the image's Pillow (tests/test_png_encode.py
// compares the files); a Pillow built on zlib-ng or libdeflate would choose other matches.
// One image per task, a fixed pool of std::threads, no Python.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/nic.h"

namespace nic {
int set_error(int code, const char* msg);  // nic_capi.hip
}

namespace {

struct PngMode {
  int level, mem_level, idat;  // deflate level, memLevel, IDAT chunk size
  bool libpng;                 // window reduction + CMF rewrite of libpng (NIC_PNG_TF)
};
constexpr PngMode kModes[2] = {{9, 9, 65536, false}, {Z_DEFAULT_COMPRESSION, 9, 8192, true}};

inline int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// filtered rows of one image of h rows of w bytes (bpp bytes per pixel) into out
// ((w + 1) * h bytes); cand: 5 * w scratch; zeros: w zero bytes; allowed: bit f set = filter f
// is a candidate (libpng's pruning in TF mode)
void filter_rows(const uint8_t* img, int h, int w, int bpp, uint8_t* out, uint8_t* cand, const uint8_t* zeros,
                 unsigned allowed) {
  const uint8_t* prev = zeros;  // the row above the first is zero
  for (int r = 0; r < h; ++r) {
    const uint8_t* x = img + (size_t)r * w;
    long best_sum = -1;
    int best = 0;
    for (int f = 0; f < 5; ++f) {
      if (!((allowed >> f) & 1u)) continue;
      uint8_t* o = cand + (size_t)f * w;
      long sum = 0;
      for (int i = 0; i < w; ++i) {
        const int a = i >= bpp ? x[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
        int pred = 0;
        switch (f) {
          case 0: pred = 0; break;
          case 1: pred = a; break;
          case 2: pred = b; break;
          case 3: pred = (a + b) >> 1; break;
          default: pred = paeth(a, b, c); break;
        }
        const uint8_t v = (uint8_t)(x[i] - pred);
        o[i] = v;
        sum += std::abs((int)(int8_t)v);
      }
      if (best_sum < 0 || sum < best_sum) {
        best_sum = sum;
        best = f;
      }
    }
    uint8_t* dst = out + (size_t)r * (w + 1);
    dst[0] = (uint8_t)best;
    std::memcpy(dst + 1, cand + (size_t)best * w, (size_t)w);
    prev = x;
  }
}

// libpng 1.6 png_deflate_claim: the window shrinks while data + 262 fits in half of it
int libpng_window_bits(size_t data) {
  int wb = 15;
  if (data <= 16384) {
    unsigned half = 1u << (wb - 1);
    while (data + 262 <= half) {
      half >>= 1;
      --wb;
    }
  }
  return std::max(wb, 9);  // zlib >= 1.2.9 deflates an 8-bit window as 9 (optimize_cmf fixes the header)
}

// libpng 1.6 optimize_cmf: the zlib header's CINFO lowered to the smallest window covering
// the uncompressed data, FCHECK recomputed
void libpng_optimize_cmf(uint8_t* z, size_t data) {
  if (data > 16384) return;
  unsigned cmf = z[0];
  if ((cmf & 0x0f) != 8 || (cmf & 0xf0) > 0x70) return;
  unsigned cinfo = cmf >> 4, half = 1u << (cinfo + 7);
  if (data > half) return;
  do {
    half >>= 1;
    --cinfo;
  } while (cinfo > 0 && data <= half);
  cmf = (cmf & 0x0f) | (cinfo << 4);
  z[0] = (uint8_t)cmf;
  unsigned t = z[1] & 0xe0;
  t += 0x1f - ((cmf << 8) + t) % 0x1f;
  z[1] = (uint8_t)t;
}

// the deflated stream of the filtered rows into buf; its length or -1
long deflate_rows(const uint8_t* data, size_t n, const PngMode& md, std::vector<uint8_t>& buf) {
  z_stream s;
  std::memset(&s, 0, sizeof(s));
  const int wb = md.libpng ? libpng_window_bits(n) : 15;
  if (deflateInit2(&s, md.level, Z_DEFLATED, wb, md.mem_level, Z_FILTERED) != Z_OK) return -1;
  buf.resize(deflateBound(&s, (uLong)n) + 64);
  s.next_in = const_cast<Bytef*>(data);
  s.avail_in = (uInt)n;
  s.next_out = buf.data();
  s.avail_out = (uInt)buf.size();
  const int rc = deflate(&s, Z_FINISH);
  const long len = rc == Z_STREAM_END ? (long)s.total_out : -1;
  deflateEnd(&s);
  if (len >= 2 && md.libpng) libpng_optimize_cmf(buf.data(), n);
  return len;
}

long png_file_size(long zlen, int idat) {
  const long chunks = std::max(1L, (zlen + idat - 1) / idat);
  return 8 + 25 + 12 * chunks + zlen + 12;
}

inline uint8_t* put32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
  return p + 4;
}

// one chunk (length, type, data, CRC over type + data) at p; returns the end
uint8_t* put_chunk(uint8_t* p, const char* type, const uint8_t* data, uint32_t len) {
  p = put32(p, len);
  std::memcpy(p, type, 4);
  if (len) std::memcpy(p + 4, data, len);
  const uint32_t crc = (uint32_t)crc32(0L, p, len + 4);
  return put32(p + 4 + len, crc);
}

void write_png(uint8_t* out, int h, int w_px, int channels, const uint8_t* z, long zlen, int idat) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  std::memcpy(out, sig, 8);
  uint8_t ihdr[13];
  put32(ihdr, (uint32_t)w_px);
  put32(ihdr + 4, (uint32_t)h);
  ihdr[8] = 8;                          // bit depth
  ihdr[9] = channels == 3 ? 2 : 0;      // colour type: RGB / greyscale
  ihdr[10] = ihdr[11] = ihdr[12] = 0;   // deflate, adaptive filtering, no interlace
  uint8_t* p = put_chunk(out + 8, "IHDR", ihdr, 13);
  long off = 0;
  do {
    const long n = std::min<long>(idat, zlen - off);
    p = put_chunk(p, "IDAT", z + off, (uint32_t)n);
    off += n;
  } while (off < zlen);
  put_chunk(p, "IEND", nullptr, 0);
}

int check_shape(const char* fn, int m, int h, int w, int channels, int mode) {
  if (m < 0 || h <= 0 || w <= 0) return -1;
  if (channels != 1 && channels != 3) return -2;
  if (mode != NIC_PNG_PILLOW && mode != NIC_PNG_TF) return -3;
  (void)fn;
  // one 65,536-B Pillow encoder buffer per row (the IDAT rule above); images under 1 GB
  if ((long long)w * channels + 1 > 16385 || (long long)h * (w * channels + 1) > (1LL << 30)) return -4;
  return 0;
}

int shape_error(const char* fn, int e) {
  static thread_local char msg[160];
  const char* what = e == -1 ? "bad image shape" : e == -2 ? "channels must be 1 or 3" : e == -3 ? "unknown mode"
                                                                                                   : "rows wider than 16384 bytes or images above 1 GB";
  std::snprintf(msg, sizeof(msg), "%s: %s", fn, what);
  return nic::set_error(e == -2 || e == -3 ? NIC_EINVAL : NIC_ESHAPE, msg);
}

// upper bound of one file: zlib's conservative deflateBound (any level / memLevel / window)
// + zlib framing + chunk overhead
long long bound_bytes(int h, int w, int channels, int mode) {
  const long long raw = (long long)h * ((long long)w * channels + 1);
  const long long z = raw + ((raw + 7) >> 3) + ((raw + 63) >> 6) + 5 + 6 + 64;
  return png_file_size((long)z, kModes[mode].idat);
}

}  // namespace

extern "C" int nic_png_bound(int h, int w, int channels, int mode, int64_t* bytes) {
  if (!bytes) return nic::set_error(NIC_EINVAL, "nic_png_bound: NULL argument");
  const int e = check_shape("nic_png_bound", 0, h, w, channels, mode);
  if (e) return shape_error("nic_png_bound", e);
  *bytes = bound_bytes(h, w, channels, mode);
  return NIC_OK;
}

extern "C" int nic_png_encode(const uint8_t* images, int m, int h, int w, int channels, int mode, uint8_t* out,
                              int64_t out_stride, int64_t* sizes, int threads) {
  const int e = check_shape("nic_png_encode", m, h, w, channels, mode);
  if (e) return shape_error("nic_png_encode", e);
  if (m == 0) return NIC_OK;
  if (!images || !sizes) return nic::set_error(NIC_EINVAL, "nic_png_encode: NULL argument");
  if (out && out_stride < bound_bytes(h, w, channels, mode))
    return nic::set_error(NIC_ESHAPE, "nic_png_encode: out_stride below nic_png_bound");
  const PngMode& md = kModes[mode];
  const int bpp = channels, wb = w * channels;  // bytes per pixel / per row
  // libpng png_write_start_row (TF mode): None 0, Sub 1, Up 2, Average 3, Paeth 4
  unsigned allowed = 0x1fu;
  if (md.libpng && h == 1) allowed &= ~((1u << 2) | (1u << 3) | (1u << 4));
  if (md.libpng && w == 1) allowed &= ~((1u << 1) | (1u << 3) | (1u << 4));
  const int nt = std::max(1, std::min(threads > 0 ? threads : 1, m));
  std::atomic<int> next{0}, failed{0};
  auto work = [&]() {
    std::vector<uint8_t> filt((size_t)h * (wb + 1)), cand((size_t)5 * wb), zeros((size_t)wb, 0), z;
    for (int i = next.fetch_add(1); i < m; i = next.fetch_add(1)) {
      filter_rows(images + (size_t)i * h * wb, h, wb, bpp, filt.data(), cand.data(), zeros.data(), allowed);
      const long len = deflate_rows(filt.data(), filt.size(), md, z);
      if (len < 0) {
        failed.store(1);
        sizes[i] = -1;
        continue;
      }
      sizes[i] = png_file_size(len, md.idat);
      if (out) write_png(out + (size_t)i * (size_t)out_stride, h, w, channels, z.data(), len, md.idat);
    }
  };
  if (nt == 1) {
    work();
  } else {
    std::vector<std::thread> pool;
    pool.reserve(nt);
    for (int t = 0; t < nt; ++t) pool.emplace_back(work);
    for (auto& t : pool) t.join();
  }
  return failed.load() ? nic::set_error(NIC_EINVAL, "nic_png_encode: zlib deflate failed") : NIC_OK;
}

extern "C" int nic_png_sizes(const uint8_t* images, int m, int h, int w, int channels, int64_t* sizes, int threads) {
  const int e = check_shape("nic_png_sizes", m, h, w, channels, NIC_PNG_PILLOW);
  if (e) return shape_error("nic_png_sizes", e);
  return nic_png_encode(images, m, h, w, channels, NIC_PNG_PILLOW, nullptr, 0, sizes, threads);
}
