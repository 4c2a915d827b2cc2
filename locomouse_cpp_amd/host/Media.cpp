// Media.cpp — see Media.hpp.
#include "Media.hpp"

#include "Jpeg.hpp"

#include <zlib.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>

#include <unistd.h>

namespace locomouse {

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint32_t le32(const uint8_t* p) { return (uint32_t)p[3] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[1] << 8 | p[0]; }
uint16_t le16(const uint8_t* p) { return (uint16_t)(p[1] << 8 | p[0]); }

int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

}  // namespace

bool read_png_gray(const std::string& path, int& rows, int& cols, std::vector<uint8_t>& pixels) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (d.size() < 8 || std::memcmp(d.data(), sig, 8) != 0) return false;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> z;
  for (size_t p = 8; p + 12 <= d.size();) {
    const uint32_t len = be32(&d[p]);
    if (p + 12 + (size_t)len > d.size()) return false;
    const char* type = (const char*)&d[p + 4];
    const uint8_t* body = &d[p + 8];
    if (!std::memcmp(type, "IHDR", 4) && len >= 13) {
      w = be32(body);
      h = be32(body + 4);
      depth = body[8];
      ctype = body[9];
      interlace = body[12];
    } else if (!std::memcmp(type, "IDAT", 4)) {
      z.insert(z.end(), body, body + len);
    } else if (!std::memcmp(type, "IEND", 4)) {
      break;
    }
    p += 12 + len;
  }
  int ch = ctype == 0 ? 1 : ctype == 4 ? 2 : ctype == 2 ? 3 : ctype == 6 ? 4 : 0;
  if (!w || !h || depth != 8 || !ch || interlace) return false;
  const size_t stride = (size_t)w * ch;
  std::vector<uint8_t> raw((stride + 1) * h);
  uLongf out_len = (uLongf)raw.size();
  if (uncompress(raw.data(), &out_len, z.data(), (uLong)z.size()) != Z_OK || out_len != raw.size()) return false;
  std::vector<uint8_t> img(stride * h), zero(stride, 0);
  for (uint32_t y = 0; y < h; ++y) {  // unfilter (PNG spec §9)
    const uint8_t ft = raw[y * (stride + 1)];
    const uint8_t* src = &raw[y * (stride + 1) + 1];
    uint8_t* cur = &img[y * stride];
    const uint8_t* up = y ? &img[(y - 1) * stride] : zero.data();
    for (size_t x = 0; x < stride; ++x) {
      const int a = x >= (size_t)ch ? cur[x - ch] : 0, b = up[x], c = x >= (size_t)ch ? up[x - ch] : 0;
      int v = src[x];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: return false;
      }
      cur[x] = (uint8_t)v;
    }
  }
  rows = (int)h;
  cols = (int)w;
  pixels.resize((size_t)w * h);
  // png_set_rgb_to_gray_fixed(29900, 58700): 15-bit weights 9797, 19234, 3737
  const uint32_t rc = 9797, gc = 19234, bc = 32768 - 9797 - 19234;
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    const uint8_t* px = &img[i * ch];
    if (ch <= 2) {
      pixels[i] = px[0];  // alpha dropped
    } else {
      const uint32_t r = px[0], g = px[1], b = px[2];
      pixels[i] = (r == g && r == b) ? (uint8_t)r : (uint8_t)((rc * r + gc * g + bc * b) >> 15);
    }
  }
  return true;
}

AviReader::~AviReader() {
  if (f_) std::fclose(f_);
}

bool AviReader::open(const std::string& path) {
  if (f_) std::fclose(f_);
  f_ = std::fopen(path.c_str(), "rb");
  if (!f_) return false;
  frames_.clear();
  next_ = 0;
  uint8_t hdr[12];
  if (std::fread(hdr, 1, 12, f_) != 12 || std::memcmp(hdr, "RIFF", 4) || std::memcmp(hdr + 8, "AVI ", 4)) return false;
  std::fseek(f_, 0, SEEK_END);
  const long file_end = std::ftell(f_);
  bool have_format = false;
  int video_stream = -1, stream_index = -1;
  uint32_t compression = 0;
  // Walk the chunk tree: hdrl/strl for the format, movi for the frames.
  struct Span {
    long pos, end;
    bool movi;
  };
  std::vector<Span> stack{{12, std::min<long>(file_end, 8 + (long)le32(hdr + 4)), false}};
  while (!stack.empty()) {
    Span& s = stack.back();
    if (s.pos + 8 > s.end) {
      stack.pop_back();
      continue;
    }
    uint8_t ck[12];
    std::fseek(f_, s.pos, SEEK_SET);
    if (std::fread(ck, 1, 8, f_) != 8) return false;
    const uint32_t size = le32(ck + 4);
    const long body = s.pos + 8, next = body + (long)size + (size & 1);
    const bool in_movi = s.movi;
    s.pos = next;
    if (!std::memcmp(ck, "LIST", 4)) {
      if (std::fread(ck + 8, 1, 4, f_) != 4) return false;
      stack.push_back({body + 4, std::min(next, file_end), in_movi || !std::memcmp(ck + 8, "movi", 4)});
      continue;
    }
    if (in_movi) {
      // ##db / ##dc of the video stream (stream number in the first two characters)
      if ((ck[2] == 'd' && (ck[3] == 'b' || ck[3] == 'c')) && ck[0] >= '0' && ck[0] <= '9' && ck[1] >= '0' &&
          ck[1] <= '9' && (ck[0] - '0') * 10 + (ck[1] - '0') == video_stream)
        frames_.emplace_back(body, size);
      continue;
    }
    std::vector<uint8_t> b(std::min<uint32_t>(size, 4096));
    if (!b.empty() && std::fread(b.data(), 1, b.size(), f_) != b.size()) return false;
    if (!std::memcmp(ck, "strh", 4) && b.size() >= 8) {
      ++stream_index;
      if (!std::memcmp(b.data(), "vids", 4) && video_stream < 0) video_stream = stream_index;
    } else if (!std::memcmp(ck, "strf", 4) && stream_index == video_stream && video_stream >= 0 && !have_format &&
               b.size() >= 40) {
      width_ = (int)le32(&b[4]);
      const int32_t hh = (int32_t)le32(&b[8]);
      bottom_up_ = hh > 0;
      height_ = hh > 0 ? hh : -hh;
      bits_ = le16(&b[14]);
      compression = le32(&b[16]);
      uint32_t n_pal = le32(&b[32]);
      if (bits_ == 8 && compression == 0) {
        if (!n_pal) n_pal = 256;
        palette_blue_.assign(256, 0);
        for (uint32_t k = 0; k < n_pal && 40 + 4 * k < b.size(); ++k) palette_blue_[k] = b[40 + 4 * k];
      }
      have_format = true;
    }
  }
  const bool grey = compression == 0x30303859u /* 'Y800' */ || compression == 0x59455247u /* 'GREY' */;
  mjpeg_ = compression == 0x47504A4Du /* 'MJPG' */ || compression == 0x67706A6Du /* 'mjpg' */ ||
           compression == 0x4745504Au /* 'JPEG' */ || compression == 0x6765706Au /* 'jpeg' */ ||
           compression == 0x31495641u /* 'AVI1' */;
  const bool ok = have_format && width_ > 0 && height_ > 0 &&
                  ((compression == 0 && (bits_ == 24 || bits_ == 8)) || (grey && bits_ == 8) || mjpeg_);
  if (!ok) {
    std::fclose(f_);
    f_ = nullptr;
    return false;
  }
  if (grey || mjpeg_) palette_blue_.clear(), bottom_up_ = false;
  return true;
}

bool AviReader::read(uint8_t* channel0) {
  if (!f_ || next_ >= frames_.size()) return false;
  return read_at(next_++, channel0);
}

bool AviReader::read_at(size_t index, uint8_t* channel0) const {
  if (!f_ || index >= frames_.size()) return false;
  const auto fr = frames_[index];
  if (mjpeg_) {  // one JPEG image per chunk, decoded to channel 0 of its BGR rendering (Jpeg.hpp)
    thread_local std::vector<uint8_t> jpg;
    jpg.resize(fr.second);
    for (size_t got = 0; got < fr.second;) {
      const ssize_t r = pread(fileno(f_), jpg.data() + got, fr.second - got, (off_t)(fr.first + (long)got));
      if (r <= 0) return false;
      got += (size_t)r;
    }
    return decode_jpeg_channel0_into(jpg.data(), jpg.size(), height_, width_, channel0);
  }
  const size_t bpp = (size_t)bits_ / 8, stride = ((size_t)width_ * bpp + 3) & ~(size_t)3;
  const size_t tight = (size_t)width_ * bpp;
  const bool padded = fr.second >= stride * (size_t)height_;
  const size_t row_bytes = padded ? stride : tight;
  if (fr.second < row_bytes * (size_t)height_) return false;
  const bool direct = bpp == 1 && palette_blue_.empty() && !bottom_up_ && row_bytes == (size_t)width_;
  thread_local std::vector<uint8_t> buf;
  uint8_t* data = channel0;
  if (!direct) {
    buf.resize(row_bytes * (size_t)height_);
    data = buf.data();
  }
  const size_t want = row_bytes * (size_t)height_;
  for (size_t got = 0; got < want;) {
    const ssize_t r = pread(fileno(f_), data + got, want - got, (off_t)(fr.first + (long)got));
    if (r <= 0) return false;
    got += (size_t)r;
  }
  if (direct) return true;
  bool identity = !palette_blue_.empty();
  for (int k = 0; identity && k < 256; ++k) identity = palette_blue_[k] == k;
  for (int y = 0; y < height_; ++y) {
    const uint8_t* src = data + (size_t)(bottom_up_ ? height_ - 1 - y : y) * row_bytes;
    uint8_t* dst = channel0 + (size_t)y * width_;
    if (bpp == 3) {
      for (int x = 0; x < width_; ++x) dst[x] = src[3 * x];  // B of BGR
    } else if (!palette_blue_.empty() && !identity) {
      const uint8_t* lut = palette_blue_.data();
      for (int x = 0; x < width_; ++x) dst[x] = lut[src[x]];
    } else {
      std::memcpy(dst, src, (size_t)width_);  // grey, or a palette whose blue is the index
    }
  }
  return true;
}

}  // namespace locomouse
