// PNG byte counts of u8 latent planes, bit-exact to Pillow's encoder, on host threads.
//
// Reference: get_bpp (tf2_0/src/training.py:12-21) sizes 8 * len(PNG) of every latent plane
// reshaped to (4h, 8w); the reference's own writer save_img (utils.py:85-87) is Pillow with
// optimize=True, which this build's training target follows (training.py png_bpp_planes).
// Pillow 12 / libImaging ZipEncode for an 8-bit L or RGB image with optimize=True, as
// established against Pillow's own output (tests/test_png_sizes.py):
//   * every row is filtered with the PNG filter (None, Sub, Up, Average, Paeth; neighbours a
//     pixel = 1 or 3 bytes back) whose output bytes, read as signed, have the least sum of
//     absolute values (first on ties);
//   * the filtered rows (filter byte + row) go through zlib deflate level 9, window 15,
//     memLevel 9, Z_FILTERED, in one stream;
//   * the stream is cut into IDAT chunks of 65,536 bytes (the encoder's buffer size for
//     rows up to 16,384 bytes), framed by the signature, IHDR and IEND:
//     size = 8 + 25 + sum(12 + idat_i) + 12.
// Only the size is needed, so no chunk or CRC is formed.  One image per task, a fixed pool
// of std::threads, no Python (the Pillow path spends much of its time in the interpreter).
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/nic.h"

namespace nic {
int set_error(int code, const char* msg);  // nic_capi.hip
}

namespace {

inline int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// filtered rows of one image of h rows of w bytes (bpp bytes per pixel) into out
// ((w + 1) * h bytes); cand: 5 * w scratch; zeros: w zero bytes
void filter_rows(const uint8_t* img, int h, int w, int bpp, uint8_t* out, uint8_t* cand, const uint8_t* zeros) {
  const uint8_t* prev = zeros;  // the row above the first is zero
  for (int r = 0; r < h; ++r) {
    const uint8_t* x = img + (size_t)r * w;
    long best_sum = -1;
    int best = 0;
    for (int f = 0; f < 5; ++f) {
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

// deflated length of the filtered stream (level 9, window 15, memLevel 9, Z_FILTERED)
long deflated_len(const uint8_t* data, size_t n, std::vector<uint8_t>& buf) {
  z_stream s;
  std::memset(&s, 0, sizeof(s));
  if (deflateInit2(&s, 9, Z_DEFLATED, 15, 9, Z_FILTERED) != Z_OK) return -1;
  buf.resize(deflateBound(&s, (uLong)n) + 64);
  s.next_in = const_cast<Bytef*>(data);
  s.avail_in = (uInt)n;
  s.next_out = buf.data();
  s.avail_out = (uInt)buf.size();
  const int rc = deflate(&s, Z_FINISH);
  const long len = rc == Z_STREAM_END ? (long)s.total_out : -1;
  deflateEnd(&s);
  return len;
}

}  // namespace

extern "C" int nic_png_sizes(const uint8_t* images, int m, int h, int w, int channels, int64_t* sizes, int threads) {
  if (m < 0 || h <= 0 || w <= 0) return nic::set_error(NIC_ESHAPE, "nic_png_sizes: bad image shape");
  if (channels != 1 && channels != 3) return nic::set_error(NIC_EINVAL, "nic_png_sizes: channels must be 1 or 3");
  const uint8_t* planes = images;
  const int bpp = channels;
  w *= channels;  // bytes per row
  if (m == 0) return NIC_OK;
  if (!planes || !sizes) return nic::set_error(NIC_EINVAL, "nic_png_sizes: NULL argument");
  if ((long long)w + 1 > 16385 || (long long)h * (w + 1) > (1LL << 30))  // one 65,536-B encoder buffer per row
    return nic::set_error(NIC_ESHAPE, "nic_png_sizes: rows wider than 16384 bytes or images above 1 GB");
  const int nt = std::max(1, std::min(threads > 0 ? threads : 1, m));
  std::atomic<int> next{0}, failed{0};
  auto work = [&]() {
    std::vector<uint8_t> filt((size_t)h * (w + 1)), cand((size_t)5 * w), zeros((size_t)w, 0), out;
    for (int i = next.fetch_add(1); i < m; i = next.fetch_add(1)) {
      filter_rows(planes + (size_t)i * h * w, h, w, bpp, filt.data(), cand.data(), zeros.data());
      const long len = deflated_len(filt.data(), filt.size(), out);
      if (len < 0) {
        failed.store(1);
        sizes[i] = -1;
        continue;
      }
      const long chunks = std::max(1L, (len + 65535) / 65536);
      sizes[i] = 8 + 25 + 12 * chunks + len + 12;
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
  return failed.load() ? nic::set_error(NIC_EINVAL, "nic_png_sizes: zlib deflate failed") : NIC_OK;
}
