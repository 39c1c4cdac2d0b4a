// Keypoint-dataset item loader, host side: the per-item file decode of
// perseus/detector/data.py:73-102 (PIL PNG -> RGB f32 / 255, tifffile depth page 0, PIL
// segmentation PNG -> 0/1 mask) as native PNG / TIFF decoders and one batch call over a
// pool of host threads (the reference runs __getitem__ in 8 DataLoader worker processes,
// validate.py:99-105).  The decoded batch is exactly what data.py returns; the HDF5 index
// (file names, pixel coordinates) is read by the caller.
//
// PNG: chunk walk, one zlib inflate over the concatenated IDATs, the five row filters,
// then PIL's mode semantics (convert("RGB") or the raw samples).  TIFF: page 0, strips,
// none / LZW / Deflate, horizontal and floating-point predictors, either byte order.
// Anything else is refused with a message (include/perseus_amd_loader.h lists the cases).
#include <fcntl.h>
#include <sched.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "perseus_amd.h"
#include "perseus_amd_loader.h"

namespace pa {
void set_error(const char* fmt, ...);
}

#define LD_CHECK(cond, ...)          \
  do {                               \
    if (!(cond)) {                   \
      ::pa::set_error(__VA_ARGS__);  \
      return PA_EINVAL;              \
    }                                \
  } while (0)

namespace {

// ------------------------------------------------------------------------- PNG
inline uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | (uint32_t)p[3];
}

struct Png {
  int w = 0, h = 0, depth = 0, ctype = 0, interlace = 0, nplte = 0;
  uint8_t plte[256][3] = {};
  std::vector<uint8_t> idat;
};

int png_channels(int ctype) { return ctype == 2 ? 3 : ctype == 4 ? 2 : ctype == 6 ? 4 : 1; }

int png_parse(const uint8_t* b, size_t n, Png& p, bool data) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  LD_CHECK(b && n >= 8 && !memcmp(b, sig, 8), "png: not a PNG file");
  size_t o = 8;
  bool ihdr = false;
  while (o + 12 <= n) {
    const uint32_t len = be32(b + o);
    LD_CHECK(len <= n - o - 12, "png: truncated chunk at byte %zu", o);
    const uint8_t* t = b + o + 4;
    const uint8_t* d = b + o + 8;
    if (!memcmp(t, "IHDR", 4)) {
      LD_CHECK(len == 13, "png: IHDR length %u", len);
      p.w = (int)be32(d);
      p.h = (int)be32(d + 4);
      p.depth = d[8];
      p.ctype = d[9];
      p.interlace = d[12];
      LD_CHECK(d[10] == 0 && d[11] == 0, "png: compression / filter method %d / %d", d[10], d[11]);
      ihdr = true;
      if (!data) break;
    } else if (!memcmp(t, "PLTE", 4)) {
      LD_CHECK(len % 3 == 0 && len <= 768, "png: PLTE length %u", len);
      p.nplte = (int)(len / 3);
      memcpy(p.plte, d, len);
    } else if (!memcmp(t, "IDAT", 4)) {
      p.idat.insert(p.idat.end(), d, d + len);
    } else if (!memcmp(t, "IEND", 4)) {
      break;
    }
    o += 12 + (size_t)len;
  }
  LD_CHECK(ihdr, "png: no IHDR");
  LD_CHECK(p.w > 0 && p.h > 0 && p.w <= 65536 && p.h <= 65536, "png: size %d x %d", p.w, p.h);
  LD_CHECK(p.interlace == 0, "png: interlaced files are not supported");
  const bool ok = (p.depth == 8 && (p.ctype == 0 || p.ctype == 2 || p.ctype == 3 || p.ctype == 4 || p.ctype == 6)) ||
                  (p.ctype == 3 && (p.depth == 1 || p.depth == 2 || p.depth == 4));
  LD_CHECK(ok, "png: colour type %d at bit depth %d is not supported", p.ctype, p.depth);
  return PA_OK;
}

inline uint8_t paeth(int a, int b, int c) {
  const int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  return (uint8_t)(pa <= pb && pa <= pc ? a : (pb <= pc ? b : c));
}

// samples: the unfiltered image, `stride` bytes per row
int png_unpack(const uint8_t* b, size_t n, Png& p, std::vector<uint8_t>& img, size_t& stride) {
  const int r = png_parse(b, n, p, true);
  if (r) return r;
  const int bits = p.depth * png_channels(p.ctype);
  const int bpp = bits >= 8 ? bits / 8 : 1;
  stride = ((size_t)p.w * bits + 7) / 8;
  std::vector<uint8_t> raw((stride + 1) * p.h);
  z_stream z;
  memset(&z, 0, sizeof z);
  LD_CHECK(inflateInit(&z) == Z_OK, "png: zlib init");
  z.next_in = p.idat.data();
  z.avail_in = (uInt)p.idat.size();
  z.next_out = raw.data();
  z.avail_out = (uInt)raw.size();
  const int zr = inflate(&z, Z_FINISH);
  const size_t got = z.total_out;
  inflateEnd(&z);
  LD_CHECK(zr == Z_STREAM_END && got == raw.size(), "png: image data inflates to %zu of %zu bytes (zlib %d)", got,
           raw.size(), zr);
  img.assign(stride * p.h, 0);
  std::vector<uint8_t> zero(stride, 0);
  for (int y = 0; y < p.h; ++y) {
    const uint8_t f = raw[y * (stride + 1)];
    const uint8_t* s = raw.data() + y * (stride + 1) + 1;
    uint8_t* dst = img.data() + y * stride;
    const uint8_t* up = y ? img.data() + (y - 1) * stride : zero.data();
    const size_t k = (size_t)bpp < stride ? (size_t)bpp : stride;  // the first pixel has no left neighbour
    switch (f) {
      case 0: memcpy(dst, s, stride); break;
      case 1:
        memcpy(dst, s, k);
        for (size_t i = k; i < stride; ++i) dst[i] = (uint8_t)(s[i] + dst[i - bpp]);
        break;
      case 2:
        for (size_t i = 0; i < stride; ++i) dst[i] = (uint8_t)(s[i] + up[i]);
        break;
      case 3:
        for (size_t i = 0; i < k; ++i) dst[i] = (uint8_t)(s[i] + (up[i] >> 1));
        for (size_t i = k; i < stride; ++i) dst[i] = (uint8_t)(s[i] + ((dst[i - bpp] + up[i]) >> 1));
        break;
      case 4:
        for (size_t i = 0; i < k; ++i) dst[i] = (uint8_t)(s[i] + up[i]);  // paeth(0, b, 0) = b
        for (size_t i = k; i < stride; ++i) dst[i] = (uint8_t)(s[i] + paeth(dst[i - bpp], up[i], up[i - bpp]));
        break;
      default: LD_CHECK(false, "png: row %d has filter type %d", y, f);
    }
  }
  return PA_OK;
}

int png_decode(const uint8_t* b, size_t n, int rgb, uint8_t* out, size_t cap) {
  Png p;
  std::vector<uint8_t> img;
  size_t stride = 0;
  const int r = png_unpack(b, n, p, img, stride);
  if (r) return r;
  const int ch = png_channels(p.ctype);
  const size_t np = (size_t)p.w * p.h;
  LD_CHECK(out && cap >= np * (rgb ? 3 : ch), "png: output buffer %zu bytes < %zu", cap, np * (rgb ? 3 : ch));
  if (p.ctype == 3 && p.depth == 8) {  // palette indices, one per byte
    for (int y = 0; y < p.h; ++y) {
      const uint8_t* s = img.data() + y * stride;
      uint8_t* o = out + (size_t)y * p.w * (rgb ? 3 : 1);
      if (!rgb) {
        memcpy(o, s, p.w);
        continue;
      }
      for (int x = 0; x < p.w; ++x, o += 3) {
        const int idx = s[x];
        for (int c = 0; c < 3; ++c) o[c] = idx < p.nplte ? p.plte[idx][c] : 0;
      }
    }
    return PA_OK;
  }
  if (p.ctype == 3) {  // palette: packed indices, MSB first
    const int per = 8 / p.depth, mask = (1 << p.depth) - 1;
    for (int y = 0; y < p.h; ++y)
      for (int x = 0; x < p.w; ++x) {
        const uint8_t byte = img[y * stride + x / per];
        const int idx = (byte >> (8 - p.depth * (x % per + 1))) & mask;
        uint8_t* o = out + ((size_t)y * p.w + x) * (rgb ? 3 : 1);
        if (rgb) {
          for (int c = 0; c < 3; ++c) o[c] = idx < p.nplte ? p.plte[idx][c] : 0;
        } else {
          o[0] = (uint8_t)idx;
        }
      }
    return PA_OK;
  }
  if (!rgb) {
    for (int y = 0; y < p.h; ++y) memcpy(out + (size_t)y * p.w * ch, img.data() + y * stride, (size_t)p.w * ch);
    return PA_OK;
  }
  for (int y = 0; y < p.h; ++y) {  // convert("RGB"): gray replicated, alpha dropped
    const uint8_t* s = img.data() + y * stride;
    uint8_t* o = out + (size_t)y * p.w * 3;
    if (ch == 3) {
      memcpy(o, s, (size_t)p.w * 3);
    } else if (ch == 4) {
      for (int x = 0; x < p.w; ++x, s += 4, o += 3) {
        o[0] = s[0];
        o[1] = s[1];
        o[2] = s[2];
      }
    } else {
      for (int x = 0; x < p.w; ++x, s += ch, o += 3) o[0] = o[1] = o[2] = s[0];
    }
  }
  return PA_OK;
}

// ------------------------------------------------------------------------ TIFF
struct Tif {
  bool le = true;
  int w = 0, h = 0, bps = 0, spp = 1, comp = 1, pred = 1, fmt = 1, planar = 1;
  uint32_t rps = 0xffffffffu;
  std::vector<uint32_t> off, cnt;
};

struct TifReader {
  const uint8_t* b;
  size_t n;
  bool le;
  uint16_t u16(size_t o) const { return le ? (uint16_t)(b[o] | b[o + 1] << 8) : (uint16_t)(b[o] << 8 | b[o + 1]); }
  uint32_t u32(size_t o) const {
    return le ? (uint32_t)b[o] | (uint32_t)b[o + 1] << 8 | (uint32_t)b[o + 2] << 16 | (uint32_t)b[o + 3] << 24
              : be32(b + o);
  }
};

// values of one IFD entry (SHORT or LONG), read from the entry or its offset
int tif_values(const TifReader& rd, size_t e, std::vector<uint32_t>& v) {
  const uint16_t type = rd.u16(e + 2);
  const uint32_t count = rd.u32(e + 4);
  const size_t sz = type == 3 ? 2 : type == 4 ? 4 : 0;
  LD_CHECK(sz && count >= 1 && count <= (1u << 24), "tiff: tag %u has type %u / count %u", rd.u16(e), type, count);
  size_t at = e + 8;
  if (sz * count > 4) {
    at = rd.u32(e + 8);
    LD_CHECK(at + sz * count <= rd.n, "tiff: tag %u values outside the file", rd.u16(e));
  }
  v.resize(count);
  for (uint32_t i = 0; i < count; ++i) v[i] = sz == 2 ? rd.u16(at + 2 * i) : rd.u32(at + 4 * i);
  return PA_OK;
}

int tif_parse(const uint8_t* b, size_t n, Tif& t) {
  LD_CHECK(b && n >= 8 && ((b[0] == 'I' && b[1] == 'I') || (b[0] == 'M' && b[1] == 'M')), "tiff: not a TIFF file");
  const TifReader rd{b, n, b[0] == 'I'};
  t.le = rd.le;
  LD_CHECK(rd.u16(2) == 42, "tiff: version %u (BigTIFF is not supported)", rd.u16(2));
  const size_t ifd = rd.u32(4);
  LD_CHECK(ifd + 2 <= n, "tiff: IFD offset");
  const int ne = rd.u16(ifd);
  LD_CHECK(ifd + 2 + 12 * (size_t)ne <= n, "tiff: IFD entries");
  std::vector<uint32_t> v;
  for (int i = 0; i < ne; ++i) {
    const size_t e = ifd + 2 + 12 * (size_t)i;
    const uint16_t tag = rd.u16(e);
    if (tag == 322 || tag == 323 || tag == 324 || tag == 325) LD_CHECK(false, "tiff: tiled images are not supported");
    if (tag != 256 && tag != 257 && tag != 258 && tag != 259 && tag != 273 && tag != 277 && tag != 278 &&
        tag != 279 && tag != 284 && tag != 317 && tag != 339)
      continue;
    const int r = tif_values(rd, e, v);
    if (r) return r;
    switch (tag) {
      case 256: t.w = (int)v[0]; break;
      case 257: t.h = (int)v[0]; break;
      case 258:
        t.bps = (int)v[0];
        for (uint32_t x : v) LD_CHECK((int)x == t.bps, "tiff: mixed bits per sample");
        break;
      case 259: t.comp = (int)v[0]; break;
      case 273: t.off = v; break;
      case 277: t.spp = (int)v[0]; break;
      case 278: t.rps = v[0]; break;
      case 279: t.cnt = v; break;
      case 284: t.planar = (int)v[0]; break;
      case 317: t.pred = (int)v[0]; break;
      case 339: t.fmt = (int)v[0]; break;
    }
  }
  LD_CHECK(t.w > 0 && t.h > 0 && t.w <= 65536 && t.h <= 65536, "tiff: size %d x %d", t.w, t.h);
  LD_CHECK(t.spp == 1, "tiff: %d samples per pixel (one supported)", t.spp);
  LD_CHECK((t.fmt == 3 && t.bps == 32) || (t.fmt == 1 && (t.bps == 8 || t.bps == 16)),
           "tiff: sample format %d at %d bits is not supported", t.fmt, t.bps);
  LD_CHECK(t.comp == 1 || t.comp == 5 || t.comp == 8 || t.comp == 32946, "tiff: compression %d is not supported",
           t.comp);
  LD_CHECK(t.pred == 1 || t.pred == 2 || t.pred == 3, "tiff: predictor %d", t.pred);
  LD_CHECK(t.pred != 3 || t.fmt == 3, "tiff: floating-point predictor on integer samples");
  if (t.rps == 0 || t.rps > (uint32_t)t.h) t.rps = (uint32_t)t.h;
  const size_t strips = (t.h + t.rps - 1) / t.rps;
  LD_CHECK(t.off.size() == strips && t.cnt.size() == strips, "tiff: %zu strip offsets / %zu counts for %zu strips",
           t.off.size(), t.cnt.size(), strips);
  for (size_t s = 0; s < strips; ++s)
    LD_CHECK((size_t)t.off[s] + t.cnt[s] <= n, "tiff: strip %zu outside the file", s);
  return PA_OK;
}

// TIFF LZW (MSB-first codes, 9-12 bits, code width raised one code early as libtiff does)
int lzw_decode(const uint8_t* in, size_t n, uint8_t* out, size_t want) {
  struct Ent {
    int prefix, len;
    uint8_t first, last;
  };
  std::vector<Ent> tab(4096);
  for (int i = 0; i < 256; ++i) tab[i] = Ent{-1, 1, (uint8_t)i, (uint8_t)i};
  int next = 258, width = 9, prev = -1;
  size_t bitpos = 0, o = 0;
  const size_t nbits = n * 8;
  auto emit = [&](int code) {  // write the string of `code` at out[o ..]
    const int len = tab[code].len;
    if (o + len > want) return false;
    for (int c = code, i = len - 1; i >= 0; --i, c = tab[c].prefix) out[o + i] = tab[c].last;
    o += len;
    return true;
  };
  while (bitpos + width <= nbits) {
    int code = 0;
    for (int i = 0; i < width; ++i, ++bitpos) code = code << 1 | ((in[bitpos >> 3] >> (7 - (bitpos & 7))) & 1);
    if (code == 257) break;
    if (code == 256) {
      next = 258;
      width = 9;
      prev = -1;
      continue;
    }
    if (prev < 0) {
      LD_CHECK(code < 256, "tiff lzw: first code %d after a clear", code);
      LD_CHECK(emit(code), "tiff lzw: output overflow");
      prev = code;
      continue;
    }
    LD_CHECK(code <= next && next < 4096, "tiff lzw: code %d beyond table %d", code, next);
    const uint8_t first = code < next ? tab[code].first : tab[prev].first;
    tab[next] = Ent{prev, tab[prev].len + 1, tab[prev].first, first};
    ++next;
    LD_CHECK(emit(code), "tiff lzw: output overflow");
    if (next + 1 >= (1 << width) && width < 12) ++width;
    prev = code;
  }
  LD_CHECK(o == want, "tiff lzw: strip decodes to %zu of %zu bytes", o, want);
  return PA_OK;
}

int tif_decode(const uint8_t* b, size_t n, float* out, size_t cap) {
  Tif t;
  int r = tif_parse(b, n, t);
  if (r) return r;
  const size_t bytes = t.bps / 8, row = (size_t)t.w * bytes;
  LD_CHECK(out && cap >= (size_t)t.w * t.h, "tiff: output buffer %zu floats < %zu", cap, (size_t)t.w * t.h);
  std::vector<uint8_t> buf(row * t.h);
  for (size_t s = 0, y0 = 0; y0 < (size_t)t.h; ++s, y0 += t.rps) {
    const size_t rows = (size_t)t.h - y0 < t.rps ? (size_t)t.h - y0 : t.rps;
    const size_t want = rows * row;
    uint8_t* dst = buf.data() + y0 * row;
    const uint8_t* src = b + t.off[s];
    if (t.comp == 1) {
      LD_CHECK(t.cnt[s] >= want, "tiff: strip %zu has %u of %zu bytes", s, t.cnt[s], want);
      memcpy(dst, src, want);
    } else if (t.comp == 5) {
      r = lzw_decode(src, t.cnt[s], dst, want);
      if (r) return r;
    } else {
      uLongf got = (uLongf)want;
      const int zr = uncompress(dst, &got, src, t.cnt[s]);
      LD_CHECK(zr == Z_OK && got == want, "tiff: strip %zu inflates to %lu of %zu bytes (zlib %d)", s,
               (unsigned long)got, want, zr);
    }
  }
  const bool swap = t.le != (__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__);
  std::vector<uint8_t> tmp(row);
  for (int y = 0; y < t.h; ++y) {
    uint8_t* p = buf.data() + y * row;
    if (t.pred == 3) {  // floating point: byte-wise accumulate, then byte planes (MSB first) -> values
      for (size_t i = 1; i < row; ++i) p[i] = (uint8_t)(p[i] + p[i - 1]);
      memcpy(tmp.data(), p, row);
      for (int x = 0; x < t.w; ++x)
        for (size_t k = 0; k < bytes; ++k) p[x * bytes + k] = tmp[(bytes - 1 - k) * t.w + x];  // native little-endian
    } else if (swap && bytes > 1) {
      for (int x = 0; x < t.w; ++x)
        for (size_t k = 0; k < bytes / 2; ++k) std::swap(p[x * bytes + k], p[x * bytes + bytes - 1 - k]);
    }
    if (t.pred == 2) {  // horizontal differencing on the (native-order) samples
      if (bytes == 1) {
        for (int x = 1; x < t.w; ++x) p[x] = (uint8_t)(p[x] + p[x - 1]);
      } else if (bytes == 2) {
        uint16_t* q = reinterpret_cast<uint16_t*>(p);
        for (int x = 1; x < t.w; ++x) q[x] = (uint16_t)(q[x] + q[x - 1]);
      } else {
        uint32_t* q = reinterpret_cast<uint32_t*>(p);
        for (int x = 1; x < t.w; ++x) q[x] = q[x] + q[x - 1];
      }
    }
    float* o = out + (size_t)y * t.w;
    if (t.fmt == 3) {
      memcpy(o, p, row);
    } else if (bytes == 2) {
      const uint16_t* q = reinterpret_cast<const uint16_t*>(p);
      for (int x = 0; x < t.w; ++x) o[x] = (float)q[x];
    } else {
      for (int x = 0; x < t.w; ++x) o[x] = (float)p[x];
    }
  }
  return PA_OK;
}

// ----------------------------------------------------------------------- batch
int read_file(const char* path, std::vector<uint8_t>& data) {
  const int fd = open(path, O_RDONLY);
  LD_CHECK(fd >= 0, "cannot open %s", path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    LD_CHECK(false, "cannot stat %s", path);
  }
  data.resize((size_t)st.st_size);
  size_t got = 0;
  while (got < data.size()) {
    const ssize_t r = read(fd, data.data() + got, data.size() - got);
    if (r <= 0) break;
    got += (size_t)r;
  }
  close(fd);
  LD_CHECK(got == data.size(), "short read of %s", path);
  return PA_OK;
}

int load_item(const char* img_path, const char* depth_path, const char* seg_path, int32_t asset, int h, int w,
              float* image, float* depth, uint8_t* seg, std::vector<uint8_t>& file, std::vector<uint8_t>& px) {
  const size_t np = (size_t)h * w;
  int r, ph, pw, pc;
  if (img_path) {
    if ((r = read_file(img_path, file))) return r;
    if ((r = pa_png_info(file.data(), file.size(), &ph, &pw, &pc))) return r;
    LD_CHECK(ph == h && pw == w, "%s: %d x %d, expected %d x %d", img_path, ph, pw, h, w);
    px.resize(np * 3);
    if ((r = png_decode(file.data(), file.size(), 1, px.data(), px.size()))) return r;
    for (int c = 0; c < 3; ++c)  // data.py:88: np.float32 samples .transpose(2, 0, 1) / 255.0 (f32 division)
      for (size_t i = 0; i < np; ++i) image[c * np + i] = (float)px[i * 3 + c] / 255.0f;
  }
  if (depth_path) {
    if ((r = read_file(depth_path, file))) return r;
    if ((r = pa_tiff_info(file.data(), file.size(), &ph, &pw))) return r;
    LD_CHECK(ph == h && pw == w, "%s: %d x %d, expected %d x %d", depth_path, ph, pw, h, w);
    if ((r = tif_decode(file.data(), file.size(), depth, np))) return r;
  }
  if (seg_path) {
    if ((r = read_file(seg_path, file))) return r;
    if ((r = pa_png_info(file.data(), file.size(), &ph, &pw, &pc))) return r;
    LD_CHECK(ph == h && pw == w && pc == 1, "%s: %d x %d x %d, expected %d x %d x 1", seg_path, ph, pw, pc, h, w);
    px.resize(np);
    if ((r = png_decode(file.data(), file.size(), 0, px.data(), px.size()))) return r;
    for (size_t i = 0; i < np; ++i) seg[i] = (int)px[i] == asset + 1 ? 1 : 0;  // data.py:93-95
  }
  return PA_OK;
}

// Every extern "C" entry point runs its body through `guarded`: a C++ exception
// (bad_alloc from a header-sized buffer, system_error from thread creation) must not
// cross the C ABI / ctypes boundary, where it would std::terminate the caller.
template <class F>
int guarded(const char* where, F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    ::pa::set_error("%s: out of host memory", where);
    return PA_ENOMEM;
  } catch (const std::exception& e) {
    ::pa::set_error("%s: %s", where, e.what());
    return PA_EINVAL;
  } catch (...) {
    ::pa::set_error("%s: unknown C++ exception", where);
    return PA_EINVAL;
  }
}

}  // namespace

extern "C" {

int pa_png_info(const uint8_t* buf, size_t n, int* h, int* w, int* channels) {
  return guarded("pa_png_info", [&]() {
    Png p;
    const int r = png_parse(buf, n, p, false);
    if (r) return r;
    if (h) *h = p.h;
    if (w) *w = p.w;
    if (channels) *channels = png_channels(p.ctype);
    return (int)PA_OK;
  });
}

int pa_png_decode(const uint8_t* buf, size_t n, int rgb, uint8_t* out, size_t cap) {
  return guarded("pa_png_decode", [&]() { return png_decode(buf, n, rgb, out, cap); });
}

int pa_tiff_info(const uint8_t* buf, size_t n, int* h, int* w) {
  return guarded("pa_tiff_info", [&]() {
    Tif t;
    const int r = tif_parse(buf, n, t);
    if (r) return r;
    if (h) *h = t.h;
    if (w) *w = t.w;
    return (int)PA_OK;
  });
}

int pa_tiff_decode_f32(const uint8_t* buf, size_t n, float* out, size_t cap) {
  return guarded("pa_tiff_decode_f32", [&]() { return tif_decode(buf, n, out, cap); });
}

int pa_load_keypoint_items(const char* const* image_paths, const char* const* depth_paths,
                           const char* const* seg_paths, const int32_t* asset_ids, int B, int h, int w,
                           int n_threads, float* image, float* depth, uint8_t* seg) {
  LD_CHECK(B >= 0 && h > 0 && w > 0, "loader: B=%d h=%d w=%d", B, h, w);
  LD_CHECK(!image_paths || image, "loader: image paths without an image buffer");
  LD_CHECK(!depth_paths || depth, "loader: depth paths without a depth buffer");
  LD_CHECK(!seg_paths || (seg && asset_ids), "loader: segmentation paths need seg and asset_ids");
  if (B == 0) return PA_OK;
  if (n_threads <= 0) {
    cpu_set_t cs;
    n_threads = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) : 1;
  }
  if (n_threads > B) n_threads = B;
  const size_t np = (size_t)h * w;
  std::atomic<int> next{0};
  std::atomic<int> failed{0};
  std::mutex mu;
  std::string msg;
  int first_rc = PA_OK;
  auto work = [&]() {
    std::vector<uint8_t> file, px;
    for (int i; !failed.load(std::memory_order_relaxed) && (i = next.fetch_add(1)) < B;) {
      // pa_last_error is thread-local: the item's message is taken on the thread that failed
      const int r = guarded("pa_load_keypoint_items", [&]() {
        return load_item(image_paths ? image_paths[i] : nullptr, depth_paths ? depth_paths[i] : nullptr,
                         seg_paths ? seg_paths[i] : nullptr, asset_ids ? asset_ids[i] : 0, h, w,
                         image ? image + (size_t)i * 3 * np : nullptr, depth ? depth + (size_t)i * np : nullptr,
                         seg ? seg + (size_t)i * np : nullptr, file, px);
      });
      if (r) {
        std::lock_guard<std::mutex> g(mu);
        if (!failed.exchange(1)) {
          msg = std::string("item ") + std::to_string(i) + ": " + pa_last_error();
          first_rc = r;
        }
      }
    }
  };
  return guarded("pa_load_keypoint_items", [&]() {
    std::vector<std::thread> pool;
    // reserved before any thread starts: emplace_back then never reallocates, so the only
    // throw inside the loop is the thread's own construction (a bad_alloc here leaves no
    // joinable thread behind)
    pool.reserve(n_threads > 1 ? n_threads - 1 : 0);
    for (int t = 1; t < n_threads; ++t) {
      try {
        pool.emplace_back(work);
      } catch (...) {
        break;  // fewer threads: the calling thread and those already started finish the batch
      }
    }
    work();
    for (auto& t : pool) t.join();
    if (failed.load()) {
      ::pa::set_error("%s", msg.c_str());
      return first_rc;
    }
    return (int)PA_OK;
  });
}

}  // extern "C"
