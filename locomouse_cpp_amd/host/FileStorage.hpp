// FileStorage.hpp — reader for the OpenCV FileStorage YAML files the
// reference's CLI consumes (config.yml, the model file, the calibration file;
// SURVEY.md §8(f) row 2).  OpenCV is not available, so the subset those files
// use is read natively: a top-level mapping of scalars (int / real / string),
// flow sequences and maps, block maps and sequences, and `!!opencv-matrix`
// nodes (rows, cols, dt, data).
//
// Lookup semantics follow OpenCV 3.x's operator>> (persistence.hpp): a missing
// key reads as 0 / 0.0 / "" / an empty matrix; a real read into an int is
// cvRound-ed (half to even); a string read into a number gives INT_MAX / 1e300.
#ifndef LOCOMOUSE_HOST_FILESTORAGE_HPP
#define LOCOMOUSE_HOST_FILESTORAGE_HPP

#include <string>
#include <utility>
#include <vector>

namespace locomouse {

// cv::Mat read from an !!opencv-matrix node; values widened to double.
struct FsMat {
  int rows = 0, cols = 0;
  char dt = 'd';  // u c w s i f d (CV_8U .. CV_64F)
  std::vector<double> v;
  bool empty() const { return v.empty(); }
  double at(int r, int c) const { return v[(size_t)r * cols + c]; }
};

class FsNode {
 public:
  enum Kind { NONE, INT, REAL, STR, SEQ, MAP, MAT };
  Kind kind = NONE;
  long long i = 0;
  double f = 0;
  std::string s;
  std::vector<FsNode> seq;
  std::vector<std::pair<std::string, FsNode>> map;
  FsMat mat;

  const FsNode& operator[](const std::string& key) const;  // NONE when absent
  bool empty() const { return kind == NONE; }
  int to_int() const;
  double to_double() const;
  std::string to_string() const;
  FsMat to_mat() const;  // empty unless an !!opencv-matrix
};

// Parses `path`; returns false when the file cannot be opened (isOpened()).
// Malformed content throws std::runtime_error (cv::Exception in OpenCV).
bool read_file_storage(const std::string& path, FsNode& root);
FsNode parse_file_storage(const std::string& text);

}  // namespace locomouse

#endif
