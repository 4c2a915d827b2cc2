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

// cv::FileStorage(path, WRITE) for YAML, with the reference's stream protocol:
//   fs << "name" << value;   fs << "name" << "{" ... "}";   fs << "name" << "[" ... "]";
//   "[:" / "{:" open flow collections; inside a sequence values take no name.
// The text follows OpenCV's YAML emitter: "%YAML:1.0" / "---" header, block
// collections indented by 3, flow collections opened on the key's line and
// wrapped past column 71, ints as %d, reals as "%d." when integral else
// "%.16e", !!opencv-matrix maps for matrices (rows, cols, dt, data).
class FsWriter {
 public:
  explicit FsWriter(const std::string& path);
  ~FsWriter();
  FsWriter(const FsWriter&) = delete;
  FsWriter& operator=(const FsWriter&) = delete;
  bool isOpened() const;
  void release();  // closes open collections and the file

  FsWriter& operator<<(const char* s);  // a name, a bracket, or a string value
  FsWriter& operator<<(const std::string& s) { return *this << s.c_str(); }
  FsWriter& operator<<(int v);
  FsWriter& operator<<(double v);
  // An int32 matrix (rows x cols, row-major) as !!opencv-matrix with dt: i.
  void write_mat_i(const int* data, int rows, int cols);

 private:
  struct Level {
    int indent;
    bool map, flow, empty;
  };
  void scalar(const char* key, const std::string* data);
  void start(const char* key, bool map, bool flow, const char* type);
  void end();
  void flush();
  void value(const std::string& text);
  struct Impl;
  Impl* f_;
  std::vector<Level> stack_;
  std::string line_;
  int space_ = 0;
  bool name_expected_ = true;
  std::string elname_;
};

std::string fs_real(double v);  // OpenCV's YAML text of a double

}  // namespace locomouse

#endif
