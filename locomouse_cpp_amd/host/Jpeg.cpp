// Jpeg.cpp — sequential Huffman JPEG decoding to BGR channel 0 (see Jpeg.hpp).
//
// The stream is decoded component plane by component plane (every block's
// coefficients straight through the ISLOW IDCT into its plane; a plane not
// needed for channel 0 — Cr of a YCbCr image — is entropy-decoded only), then
// channel 0 is formed row by row from the planes.  The arithmetic follows
// ITU-T T.81 (Huffman decoding F.2.2, restart markers B.2.1) and libjpeg's
// decompression defaults (jidctint.c, jdsample.c, jdcolor.c), the decoder
// the reference's OpenCV build links for still images.
#include "Jpeg.hpp"

#include <algorithm>
#include <cstring>

namespace locomouse {
namespace {

// Zig-zag scan position -> natural (row-major) coefficient index, padded so a
// corrupt run length past 63 lands on a harmless slot.
constexpr uint8_t kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// ITU-T T.81 Annex K.3 tables (what MJPEG "AVI1" frames leave out).
constexpr uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
constexpr uint8_t kDcChromBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
constexpr uint8_t kDcVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
constexpr uint8_t kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
constexpr uint8_t kAcLumVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
constexpr uint8_t kAcChromBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
constexpr uint8_t kAcChromVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

constexpr int kLook = 9;  // Huffman lookahead bits

// Canonical Huffman table (T.81 C.2 / F.2.2.3) with a 9-bit lookahead.
struct Huff {
  bool defined = false;
  uint16_t look[1 << kLook];  // (length << 8) | symbol; 0 = longer code
  int32_t maxcode[18];        // largest code of each length, -1 if none
  int32_t valoff[17];         // symbol index = code + valoff[length]
  uint8_t vals[256];
};

bool build_huff(Huff& h, const uint8_t bits[16], const uint8_t* vals, int nvals) {
  int total = 0;
  for (int l = 0; l < 16; ++l) total += bits[l];
  if (total > 256 || total > nvals) return false;
  std::memset(h.look, 0, sizeof(h.look));
  std::memcpy(h.vals, vals, (size_t)total);
  int code = 0, k = 0;
  for (int l = 1; l <= 16; ++l) {
    h.valoff[l] = k - code;
    for (int i = 0; i < bits[l - 1]; ++i, ++k, ++code)
      if (l <= kLook) {
        const int sh = kLook - l;
        for (int j = 0; j < (1 << sh); ++j) h.look[(code << sh) | j] = (uint16_t)((l << 8) | vals[k]);
      }
    h.maxcode[l] = bits[l - 1] ? code - 1 : -1;
    if (bits[l - 1] && code >= (1 << l)) return false;  // over-subscribed (or an all-ones code)
    code <<= 1;
  }
  h.maxcode[17] = 0x7FFFFFFF;
  h.defined = true;
  return true;
}

// Entropy-coded segment reader: byte stuffing (FF 00) removed, fill bytes
// (FF FF ..) skipped, stops at a marker and feeds zeros past it (libjpeg's
// behaviour on premature markers).
struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t buf = 0;
  int cnt = 0;
  bool marker = false;

  void refill() {
    while (cnt <= 56) {
      unsigned b = 0;
      if (!marker && p < end) {
        b = *p++;
        if (b == 0xFF) {
          const uint8_t* q = p;
          while (q < end && *q == 0xFF) ++q;
          if (q < end && *q == 0) {
            p = q + 1;
          } else {  // a marker: leave p on its FF
            marker = true;
            p = q - 1;
            b = 0;
          }
        }
      }
      buf |= (uint64_t)b << (56 - cnt);
      cnt += 8;
    }
  }
  unsigned get(int n) {  // n in 1..16, cnt >= n
    const unsigned v = (unsigned)(buf >> (64 - n));
    buf <<= n;
    cnt -= n;
    return v;
  }
  int decode(const Huff& h) {
    const unsigned e = h.look[buf >> (64 - kLook)];
    if (e >> 8) {
      buf <<= (e >> 8);
      cnt -= (int)(e >> 8);
      return (int)(e & 255);
    }
    int l = kLook + 1;
    int32_t code = (int32_t)(buf >> (64 - l));
    while (code > h.maxcode[l]) {
      ++l;
      code = (int32_t)(buf >> (64 - l));
    }
    if (l > 16) {  // not a code (corrupt data): libjpeg returns symbol 0
      buf <<= 16;
      cnt -= 16;
      return 0;
    }
    buf <<= l;
    cnt -= l;
    return h.vals[(code + h.valoff[l]) & 255];
  }
  // Restart: drop the remaining bits, step over the RSTn marker.
  void restart() {
    buf = 0;
    cnt = 0;
    if (!marker) {  // find the marker
      while (p < end) {
        if (*p == 0xFF && p + 1 < end && p[1] != 0 && p[1] != 0xFF) break;
        ++p;
      }
    }
    if (p + 1 < end && p[1] >= 0xD0 && p[1] <= 0xD7) p += 2;
    marker = false;
  }
};

inline int extend(unsigned v, int s) { return (int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v; }

// libjpeg's post-IDCT range limit: x + 128 clamped to 0..255 for |x| < 512,
// wrapping by 1024 beyond (prepare_range_limit_table's layout).
struct RangeLimit {
  uint8_t t[1024];
  RangeLimit() {
    for (int i = 0; i < 1024; ++i) {
      if (i < 128) t[i] = (uint8_t)(i + 128);
      else if (i < 512) t[i] = 255;
      else if (i < 896) t[i] = 0;
      else t[i] = (uint8_t)(i - 896);
    }
  }
};
const RangeLimit kRange;

// ISLOW inverse DCT (libjpeg jidctint.c: Loeffler-Ligtenberg-Moschytz with
// 13-bit constants, 2 extra bits between the column and row passes), with
// dequantisation folded into the column pass.
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                  F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
constexpr int kConstBits = 13, kPass1 = 2;

// JLONG arithmetic (64-bit on LP64, as jidctint.c): with 16-bit quantisation
// tables (SOF1) the products exceed 32 bits.  The column pass's workspace is
// int, as libjpeg's.
inline int64_t descale(int64_t x, int n) { return (x + ((int64_t)1 << (n - 1))) >> n; }
inline int64_t left_shift(int64_t a, int b) { return (int64_t)((uint64_t)a << b); }  // LEFT_SHIFT (jdct.h)

void idct_islow(const int16_t* coef, const uint16_t* q, uint8_t* out, int pitch) {
  int32_t ws[64];
  for (int c = 0; c < 8; ++c) {
    const int16_t* in = coef + c;
    const uint16_t* qq = q + c;
    int32_t* w = ws + c;
    if (!(in[8] | in[16] | in[24] | in[32] | in[40] | in[48] | in[56])) {
      const int32_t dc = (int32_t)left_shift((int32_t)in[0] * (int32_t)qq[0], kPass1);  // int dcval (wraps like libjpeg)
      for (int r = 0; r < 8; ++r) w[8 * r] = dc;
      continue;
    }
    int64_t z2 = (int32_t)in[16] * (int32_t)qq[16], z3 = (int32_t)in[48] * (int32_t)qq[48];
    int64_t z1 = (z2 + z3) * F0541;
    int64_t tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
    z2 = (int32_t)in[0] * (int32_t)qq[0];
    z3 = (int32_t)in[32] * (int32_t)qq[32];
    int64_t tmp0 = left_shift(z2 + z3, kConstBits), tmp1 = left_shift(z2 - z3, kConstBits);
    const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = (int32_t)in[56] * (int32_t)qq[56];
    tmp1 = (int32_t)in[40] * (int32_t)qq[40];
    tmp2 = (int32_t)in[24] * (int32_t)qq[24];
    tmp3 = (int32_t)in[8] * (int32_t)qq[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * F1175;
    tmp0 *= F0298;
    tmp1 *= F2053;
    tmp2 *= F3072;
    tmp3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 = z3 * -F1961 + z5;
    z4 = z4 * -F0390 + z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    constexpr int s = kConstBits - kPass1;
    w[0] = (int32_t)descale(t10 + tmp3, s);
    w[56] = (int32_t)descale(t10 - tmp3, s);
    w[8] = (int32_t)descale(t11 + tmp2, s);
    w[48] = (int32_t)descale(t11 - tmp2, s);
    w[16] = (int32_t)descale(t12 + tmp1, s);
    w[40] = (int32_t)descale(t12 - tmp1, s);
    w[24] = (int32_t)descale(t13 + tmp0, s);
    w[32] = (int32_t)descale(t13 - tmp0, s);
  }
  constexpr int s2 = kConstBits + kPass1 + 3;
  for (int r = 0; r < 8; ++r) {
    const int32_t* w = ws + 8 * r;
    uint8_t* o = out + (size_t)r * pitch;
    if (!(w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7])) {
      const uint8_t v = kRange.t[(int)descale(w[0], kPass1 + 3) & 1023];
      std::memset(o, v, 8);
      continue;
    }
    int64_t z2 = w[2], z3 = w[6];
    int64_t z1 = (z2 + z3) * F0541;
    int64_t tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
    int64_t tmp0 = left_shift((int64_t)w[0] + w[4], kConstBits), tmp1 = left_shift((int64_t)w[0] - w[4], kConstBits);
    const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = w[7];
    tmp1 = w[5];
    tmp2 = w[3];
    tmp3 = w[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * F1175;
    tmp0 *= F0298;
    tmp1 *= F2053;
    tmp2 *= F3072;
    tmp3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 = z3 * -F1961 + z5;
    z4 = z4 * -F0390 + z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    o[0] = kRange.t[(int)descale(t10 + tmp3, s2) & 1023];
    o[7] = kRange.t[(int)descale(t10 - tmp3, s2) & 1023];
    o[1] = kRange.t[(int)descale(t11 + tmp2, s2) & 1023];
    o[6] = kRange.t[(int)descale(t11 - tmp2, s2) & 1023];
    o[2] = kRange.t[(int)descale(t12 + tmp1, s2) & 1023];
    o[5] = kRange.t[(int)descale(t12 - tmp1, s2) & 1023];
    o[3] = kRange.t[(int)descale(t13 + tmp0, s2) & 1023];
    o[4] = kRange.t[(int)descale(t13 - tmp0, s2) & 1023];
  }
}

// jdcolor.c's Cb -> B term: round(1.772 * 2^16 * (cb - 128)) >> 16.
struct CbToB {
  int16_t t[256];
  CbToB() {
    const int32_t fix = (int32_t)(1.772 * 65536.0 + 0.5);
    for (int i = 0; i < 256; ++i) t[i] = (int16_t)((fix * (i - 128) + (1 << 15)) >> 16);
  }
};
const CbToB kCbB;

struct Component {
  int id = 0, h = 1, v = 1, tq = 0;
  int td = 0, ta = 0;      // scan tables
  int dw = 0, dh = 0;      // downsampled size (jdinput.c: ceil(W * h / Hmax))
  int pitch = 0, prows = 0;
  int pred = 0;
  bool need = false;       // plane feeds channel 0
  std::vector<uint8_t> plane;
};

struct Decoder {
  uint16_t qt[4][64];
  bool qdef[4] = {false, false, false, false};
  Huff dc[4], ac[4];
  int W = 0, H = 0, nc = 0, hmax = 1, vmax = 1, restart = 0;
  bool sof = false, jfif = false, adobe = false;
  int adobe_transform = -1;
  Component comp[3];
  std::string why;

  bool fail(const char* m) {
    why = m;
    return false;
  }

  static int u16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

  bool parse_dqt(const uint8_t* p, int n) {
    while (n > 0) {
      const int pq = p[0] >> 4, tq = p[0] & 15;
      const int sz = 1 + 64 * (pq ? 2 : 1);
      if (tq > 3 || pq > 1 || n < sz) return fail("bad DQT segment");
      for (int k = 0; k < 64; ++k) qt[tq][kNatural[k]] = (uint16_t)(pq ? u16(p + 1 + 2 * k) : p[1 + k]);
      qdef[tq] = true;
      p += sz;
      n -= sz;
    }
    return true;
  }

  bool parse_dht(const uint8_t* p, int n) {
    while (n > 0) {
      if (n < 17) return fail("bad DHT segment");
      const int tc = p[0] >> 4, th = p[0] & 15;
      int total = 0;
      for (int l = 0; l < 16; ++l) total += p[1 + l];
      if (tc > 1 || th > 3 || total > 256 || n < 17 + total) return fail("bad DHT segment");
      if (!build_huff(tc ? ac[th] : dc[th], p + 1, p + 17, total)) return fail("bad Huffman table");
      p += 17 + total;
      n -= 17 + total;
    }
    return true;
  }

  bool parse_sof(const uint8_t* p, int n) {
    if (sof) return fail("more than one frame header");
    if (n < 6) return fail("bad SOF segment");
    if (p[0] != 8) return fail("only 8-bit JPEG samples are supported");
    H = u16(p + 1);
    W = u16(p + 3);
    nc = p[5];
    if (W <= 0 || H <= 0) return fail("JPEG image of zero size (DNL not supported)");
    if (nc != 1 && nc != 3) return fail("only 1- or 3-component JPEG images are supported");
    if (n < 6 + 3 * nc) return fail("bad SOF segment");
    hmax = vmax = 1;
    for (int c = 0; c < nc; ++c) {
      Component& C = comp[c];
      C.id = p[6 + 3 * c];
      C.h = p[7 + 3 * c] >> 4;
      C.v = p[7 + 3 * c] & 15;
      C.tq = p[8 + 3 * c];
      if (C.h < 1 || C.h > 4 || C.v < 1 || C.v > 4 || C.tq > 3) return fail("bad JPEG component parameters");
      hmax = std::max(hmax, C.h);
      vmax = std::max(vmax, C.v);
    }
    const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
    for (int c = 0; c < nc; ++c) {
      Component& C = comp[c];
      C.dw = (W * C.h + hmax - 1) / hmax;
      C.dh = (H * C.v + vmax - 1) / vmax;
      C.pitch = mcux * C.h * 8;
      C.prows = mcuy * C.v * 8;
    }
    sof = true;
    return true;
  }

  // Colour space as libjpeg's default_decompress_parms picks it.
  bool is_rgb() const {
    if (nc != 3) return false;
    if (jfif) return false;
    if (adobe) return adobe_transform == 0;
    return comp[0].id == 'R' && comp[1].id == 'G' && comp[2].id == 'B';
  }

  void fill_default_tables() {
    if (!dc[0].defined) build_huff(dc[0], kDcLumBits, kDcVals, 12);
    if (!dc[1].defined) build_huff(dc[1], kDcChromBits, kDcVals, 12);
    if (!ac[0].defined) build_huff(ac[0], kAcLumBits, kAcLumVals, 162);
    if (!ac[1].defined) build_huff(ac[1], kAcChromBits, kAcChromVals, 162);
  }

  void decode_block(Bits& b, Component& C, int16_t* blk) {
    std::memset(blk, 0, 64 * sizeof(int16_t));
    if (b.cnt < 32) b.refill();
    const int s = b.decode(dc[C.td]);
    if (s) {
      if (b.cnt < 16) b.refill();
      C.pred += extend(b.get(s > 16 ? 16 : s), s > 16 ? 16 : s);
    }
    blk[0] = (int16_t)C.pred;
    const Huff& A = ac[C.ta];
    for (int k = 1; k < 64;) {
      if (b.cnt < 32) b.refill();
      const int rs = b.decode(A);
      const int r = rs >> 4, sz = rs & 15;
      if (sz) {
        k += r;
        blk[kNatural[k]] = (int16_t)extend(b.get(sz), sz);
        ++k;
      } else {
        if (r != 15) break;
        k += 16;
      }
    }
  }

  // One scan (interleaved when ns > 1), starting at `data`; returns the
  // position after the entropy-coded segment (at its terminating marker).
  const uint8_t* decode_scan(const uint8_t* data, const uint8_t* end, int ns, const int* idx) {
    Bits b{data, end};
    for (int i = 0; i < ns; ++i) comp[idx[i]].pred = 0;
    int16_t blk[64];
    const bool single = ns == 1;
    const int mcux = single ? (comp[idx[0]].dw + 7) / 8 : (W + 8 * hmax - 1) / (8 * hmax);
    const int mcuy = single ? (comp[idx[0]].dh + 7) / 8 : (H + 8 * vmax - 1) / (8 * vmax);
    int todo = restart;
    for (int my = 0; my < mcuy; ++my)
      for (int mx = 0; mx < mcux; ++mx) {
        if (restart && todo == 0) {
          b.restart();
          for (int i = 0; i < ns; ++i) comp[idx[i]].pred = 0;
          todo = restart;
        }
        for (int i = 0; i < ns; ++i) {
          Component& C = comp[idx[i]];
          const int bh = single ? 1 : C.h, bv = single ? 1 : C.v;
          for (int v = 0; v < bv; ++v)
            for (int h = 0; h < bh; ++h) {
              decode_block(b, C, blk);
              if (!C.need) continue;
              const int bx = mx * bh + h, by = my * bv + v;
              idct_islow(blk, qt[C.tq], C.plane.data() + (size_t)by * 8 * C.pitch + bx * 8, C.pitch);
            }
        }
        --todo;
      }
    // Leave the reader on the next marker.
    const uint8_t* p = b.p;
    if (!b.marker)
      while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0 && p[1] != 0xFF)) ++p;
    return p;
  }

  bool run(const uint8_t* d, size_t n) {
    const uint8_t* end = d + n;
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return fail("not a JPEG image (no SOI)");
    const uint8_t* p = d + 2;
    bool scanned = false;
    for (;;) {
      while (p < end && *p != 0xFF) ++p;  // garbage between segments
      while (p < end && *p == 0xFF) ++p;
      if (p >= end) break;
      const int m = *p++;
      if (m == 0xD9) break;                         // EOI
      if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;  // TEM / stray RSTn
      if (m == 0xD8) return fail("nested SOI");
      if (end - p < 2) return fail("truncated JPEG segment");
      const int len = u16(p);
      if (len < 2 || end - p < len) return fail("truncated JPEG segment");
      const uint8_t* s = p + 2;
      const int sn = len - 2;
      p += len;
      switch (m) {
        case 0xC0:
        case 0xC1:
          if (!parse_sof(s, sn)) return false;
          break;
        case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7:
        case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
          return fail("only sequential Huffman JPEG is supported (progressive/lossless/arithmetic found)");
        case 0xC4:
          if (!parse_dht(s, sn)) return false;
          break;
        case 0xDB:
          if (!parse_dqt(s, sn)) return false;
          break;
        case 0xDD:
          if (sn < 2) return fail("bad DRI segment");
          restart = u16(s);
          break;
        case 0xE0:
          if (sn >= 5 && std::memcmp(s, "JFIF\0", 5) == 0) jfif = true;
          break;
        case 0xEE:
          if (sn >= 12 && std::memcmp(s, "Adobe", 5) == 0) {
            adobe = true;
            adobe_transform = s[11];
          }
          break;
        case 0xDA: {
          if (!sof) return fail("scan before frame header");
          if (sn < 1) return fail("bad SOS segment");
          const int ns = s[0];
          if (ns < 1 || ns > nc || sn < 1 + 2 * ns + 3) return fail("bad SOS segment");
          int idx[3];
          for (int i = 0; i < ns; ++i) {
            const int cid = s[1 + 2 * i];
            int c = 0;
            while (c < nc && comp[c].id != cid) ++c;
            if (c == nc) return fail("scan names an unknown component");
            idx[i] = c;
            comp[c].td = s[2 + 2 * i] >> 4;
            comp[c].ta = s[2 + 2 * i] & 15;
            if (comp[c].td > 3 || comp[c].ta > 3) return fail("bad SOS table selector");
          }
          if (!scanned) {  // first scan: decide which planes channel 0 needs
            const bool rgb = is_rgb();
            for (int c = 0; c < nc; ++c) {
              comp[c].need = nc == 1 || (rgb ? c == 2 : c <= 1);
              if (comp[c].need) comp[c].plane.assign((size_t)comp[c].pitch * comp[c].prows, 0);
            }
          }
          fill_default_tables();
          for (int i = 0; i < ns; ++i) {
            const Component& C = comp[idx[i]];
            if (!dc[C.td].defined || !ac[C.ta].defined) return fail("scan uses an undefined Huffman table");
            if (C.need && !qdef[C.tq]) return fail("component uses an undefined quantisation table");
          }
          p = decode_scan(p, end, ns, idx);
          scanned = true;
          break;
        }
        default:
          break;  // APPn, COM, DNL, ...
      }
    }
    if (!scanned) return fail("JPEG image has no scan");
    return true;
  }

  // Plane row y of component C at full resolution (upsampled by libjpeg's
  // fancy filters for 2x horizontal and/or 2x vertical, by replication for
  // other ratios) into `o` (W samples).
  void upsample_row(const Component& C, int y, uint8_t* o, std::vector<int>& tmp) const {
    const int hx = hmax / C.h, vx = vmax / C.v;
    const bool hfit = hmax % C.h == 0, vfit = vmax % C.v == 0;
    const uint8_t* P = C.plane.data();
    if (hx == 1 && vx == 1 && hfit && vfit) {
      std::memcpy(o, P + (size_t)y * C.pitch, (size_t)W);
      return;
    }
    if ((hx == 2 || hx == 1) && (vx == 2 || vx == 1) && hfit && vfit) {
      const int dw = C.dw;
      if (vx == 2) {  // vertical triangle: 3/4 nearer row + 1/4 the next one (edge rows replicate)
        const int r = y >> 1;
        const int r2 = (y & 1) ? std::min(r + 1, C.dh - 1) : std::max(r - 1, 0);
        const uint8_t* a = P + (size_t)r * C.pitch;
        const uint8_t* b = P + (size_t)r2 * C.pitch;
        tmp.resize((size_t)dw);
        for (int x = 0; x < dw; ++x) tmp[x] = 3 * a[x] + b[x];
        if (hx == 1) {  // h1v2_fancy_upsample
          const int bias = (y & 1) ? 2 : 1;
          for (int x = 0; x < W; ++x) o[x] = (uint8_t)((tmp[x] + bias) >> 2);
          return;
        }
        // h2v2_fancy_upsample
        auto put = [&](int ox, int v) {
          if (ox < W) o[ox] = (uint8_t)v;
        };
        if (dw == 1) {
          put(0, (tmp[0] * 4 + 8) >> 4);
          put(1, (tmp[0] * 4 + 7) >> 4);
          return;
        }
        put(0, (tmp[0] * 4 + 8) >> 4);
        put(1, (tmp[0] * 3 + tmp[1] + 7) >> 4);
        for (int x = 1; x < dw - 1; ++x) {
          put(2 * x, (tmp[x] * 3 + tmp[x - 1] + 8) >> 4);
          put(2 * x + 1, (tmp[x] * 3 + tmp[x + 1] + 7) >> 4);
        }
        put(2 * dw - 2, (tmp[dw - 1] * 3 + tmp[dw - 2] + 8) >> 4);
        put(2 * dw - 1, (tmp[dw - 1] * 4 + 7) >> 4);
        return;
      }
      // h2v1_fancy_upsample
      const uint8_t* a = P + (size_t)y * C.pitch;
      auto put = [&](int ox, int v) {
        if (ox < W) o[ox] = (uint8_t)v;
      };
      if (dw == 1) {
        put(0, a[0]);
        put(1, a[0]);
        return;
      }
      put(0, a[0]);
      put(1, (a[0] * 3 + a[1] + 2) >> 2);
      for (int x = 1; x < dw - 1; ++x) {
        put(2 * x, (a[x] * 3 + a[x - 1] + 1) >> 2);
        put(2 * x + 1, (a[x] * 3 + a[x + 1] + 2) >> 2);
      }
      put(2 * dw - 2, (a[dw - 1] * 3 + a[dw - 2] + 1) >> 2);
      put(2 * dw - 1, a[dw - 1]);
      return;
    }
    // Integral (or non-integral) ratios: sample replication.
    const int r = std::min(y * C.v / vmax, C.prows - 1);
    const uint8_t* a = P + (size_t)r * C.pitch;
    for (int x = 0; x < W; ++x) o[x] = a[std::min(x * C.h / hmax, C.pitch - 1)];
  }

  void channel0(uint8_t* out) const {
    std::vector<int> tmp;
    if (nc == 1) {
      for (int y = 0; y < H; ++y) upsample_row(comp[0], y, out + (size_t)y * W, tmp);
      return;
    }
    if (is_rgb()) {  // channel 0 = B = third component
      for (int y = 0; y < H; ++y) upsample_row(comp[2], y, out + (size_t)y * W, tmp);
      return;
    }
    std::vector<uint8_t> cb((size_t)W);
    for (int y = 0; y < H; ++y) {
      uint8_t* o = out + (size_t)y * W;
      upsample_row(comp[0], y, o, tmp);
      upsample_row(comp[1], y, cb.data(), tmp);
      for (int x = 0; x < W; ++x) {
        const int b = o[x] + kCbB.t[cb[x]];
        o[x] = (uint8_t)(b < 0 ? 0 : b > 255 ? 255 : b);
      }
    }
  }
};

}  // namespace

bool decode_jpeg_channel0(const uint8_t* data, size_t size, int& rows, int& cols, std::vector<uint8_t>& out,
                          std::string* err) {
  Decoder D;
  if (!D.run(data, size)) {
    if (err) *err = D.why;
    return false;
  }
  rows = D.H;
  cols = D.W;
  out.resize((size_t)rows * cols);
  D.channel0(out.data());
  return true;
}

bool decode_jpeg_channel0_into(const uint8_t* data, size_t size, int rows, int cols, uint8_t* out, std::string* err) {
  Decoder D;
  if (!D.run(data, size)) {
    if (err) *err = D.why;
    return false;
  }
  if (D.H != rows || D.W != cols) {
    if (err)
      *err = "JPEG frame is " + std::to_string(D.W) + "x" + std::to_string(D.H) + ", the video header says " +
             std::to_string(cols) + "x" + std::to_string(rows);
    return false;
  }
  D.channel0(out);
  return true;
}

}  // namespace locomouse
