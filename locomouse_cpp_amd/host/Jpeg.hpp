// Jpeg.hpp — baseline JPEG decoding for MJPEG AVI frames (SURVEY.md §8(f)
// row 2): the reference opens its video with cv::VideoCapture (LocoMouse_class.cpp
// :367-400) and reads BGR frames (:1282) of which it keeps channel 0 (:1293);
// MJPEG is the compressed format LocoMouse recordings use.  OpenCV is absent,
// so the decoding is native:
//
//   * sequential Huffman JPEG (SOF0 baseline, SOF1 extended, 8-bit samples),
//     1 component (grey) or 3 (YCbCr, or RGB with an Adobe transform of 0),
//     any sampling factors, interleaved and non-interleaved scans, restart
//     intervals; frames without DHT (the "AVI1" MJPEG convention) use the
//     standard tables of ITU-T T.81 Annex K.3;
//   * the arithmetic restates libjpeg's defaults bit for bit: the ISLOW
//     integer IDCT (jidctint.c), "fancy" triangle upsampling of subsampled
//     chroma with edge replication (jdsample.c h2v1 / h2v2 / h1v2), and the
//     fixed-point YCbCr->RGB tables (jdcolor.c) — channel 0 is B = Y +
//     1.772 (Cb - 128), range-limited; a grey JPEG's channel 0 is Y.
//
// Parity: pinned against libjpeg-turbo through Pillow's decoder
// (tests/test_mjpeg.py).  OpenCV's FFmpeg backend decodes MJPEG with FFmpeg's
// own IDCT and swscale colour conversion, whose rounding differs by a grey
// level here and there; that path cannot be pinned here (no OpenCV/FFmpeg).
#ifndef LOCOMOUSE_HOST_JPEG_HPP
#define LOCOMOUSE_HOST_JPEG_HPP

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace locomouse {

// Decodes one JPEG image to channel 0 of its BGR rendering (rows x cols u8,
// row-major, into `out`).  Returns false (with a reason in *err) for data it
// cannot decode: progressive/lossless/arithmetic coding, 12-bit samples,
// 2 or 4 components, truncated headers.
bool decode_jpeg_channel0(const uint8_t* data, size_t size, int& rows, int& cols, std::vector<uint8_t>& out,
                          std::string* err = nullptr);

// Same, into a caller buffer of exactly rows x cols bytes (the size must
// match the image); no allocation for the output.
bool decode_jpeg_channel0_into(const uint8_t* data, size_t size, int rows, int cols, uint8_t* out,
                               std::string* err = nullptr);

}  // namespace locomouse

#endif
