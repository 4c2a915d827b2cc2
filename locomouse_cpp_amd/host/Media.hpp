// Media.hpp — the image and video readers behind the reference's CLI
// (SURVEY.md §8(f) row 2), native because OpenCV is absent:
//
//   read_png_gray  cv::imread(BKG_FILE, CV_LOAD_IMAGE_GRAYSCALE)  (LocoMouse_class.cpp:405-419)
//   AviReader      cv::VideoCapture(VIDEO_FILE); V >> F; extractChannel(F, F, 0)
//                  (:376-403, :1273-1293) for uncompressed AVI (BI_RGB 24-bit
//                  BGR or 8-bit palettised, and 8-bit 'Y800'/'GREY') and MJPEG
//                  AVI ('MJPG'/'JPEG'/'AVI1': sequential Huffman JPEG per
//                  frame, Jpeg.hpp); channel 0 of the decoded BGR frame is
//                  blue.  Other codecs (H.264 …) are not decoded: opening
//                  such a file fails like a VideoCapture that cannot open it.
#ifndef LOCOMOUSE_HOST_MEDIA_HPP
#define LOCOMOUSE_HOST_MEDIA_HPP

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace locomouse {

// 8-bit PNG (grey, grey+alpha, RGB, RGBA; no interlace, no palette) as one
// grey channel.  Colour is reduced with libpng's png_set_rgb_to_gray(1,
// 0.299, 0.587) fixed-point weights (what OpenCV's PNG decoder requests for
// IMREAD_GRAYSCALE; exact byte parity with a given libpng build is unpinned).
// Returns false when the file cannot be read or decoded (!BKG.data).
bool read_png_gray(const std::string& path, int& rows, int& cols, std::vector<uint8_t>& pixels);

class AviReader {
 public:
  AviReader() = default;
  ~AviReader();
  AviReader(const AviReader&) = delete;
  AviReader& operator=(const AviReader&) = delete;

  bool open(const std::string& path);  // V.isOpened()
  int rows() const { return height_; }
  int cols() const { return width_; }
  uint32_t frame_count() const { return (uint32_t)frames_.size(); }  // CAP_PROP_FRAME_COUNT
  bool read(uint8_t* channel0);        // V >> F + extractChannel(F, F, 0); false at the end
  void rewind() { next_ = 0; }         // V.set(CV_CAP_PROP_POS_FRAMES, 0)
  // Frame `index` (0-based) without moving the read position; safe to call
  // from several threads at once (pread on the file descriptor).
  bool read_at(size_t index, uint8_t* channel0) const;

 private:
  std::FILE* f_ = nullptr;
  int width_ = 0, height_ = 0, bits_ = 0;
  bool bottom_up_ = true;
  bool mjpeg_ = false;
  std::vector<uint8_t> palette_blue_;  // 8-bit palettised: blue of each entry
  std::vector<std::pair<long, uint32_t>> frames_;  // (file offset, size) of each frame chunk
  size_t next_ = 0;
};

}  // namespace locomouse

#endif
