// FileStorage.cpp — see FileStorage.hpp.
#include "FileStorage.hpp"

#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace locomouse {

namespace {

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r"), b = s.find_last_not_of(" \t\r");
  return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

FsNode scalar(const std::string& raw) {
  FsNode n;
  std::string t = trim(raw);
  if (t.size() >= 2 && (t[0] == '"' || t[0] == '\'') && t.back() == t[0]) {
    n.kind = FsNode::STR;
    n.s = t.substr(1, t.size() - 2);
    return n;
  }
  if (t.empty()) {
    n.kind = FsNode::STR;
    return n;
  }
  char* end = nullptr;
  errno = 0;
  long long v = std::strtoll(t.c_str(), &end, 0);
  if (end && *end == 0 && errno == 0) {
    n.kind = FsNode::INT;
    n.i = v;
    return n;
  }
  std::string l;
  for (char c : t) l += (char)std::tolower((unsigned char)c);
  if (l == ".inf" || l == "+.inf") return n.kind = FsNode::REAL, n.f = INFINITY, n;
  if (l == "-.inf") return n.kind = FsNode::REAL, n.f = -INFINITY, n;
  if (l == ".nan") return n.kind = FsNode::REAL, n.f = NAN, n;
  double d = std::strtod(t.c_str(), &end);
  if (end && *end == 0) {
    n.kind = FsNode::REAL;
    n.f = d;
    return n;
  }
  n.kind = FsNode::STR;
  n.s = t;
  return n;
}

// Flow collections: [a, b, [c]] and {k: v, ...}.
struct Flow {
  const std::string& t;
  size_t p = 0;
  void ws() {
    while (p < t.size() && (t[p] == ' ' || t[p] == '\t' || t[p] == '\n' || t[p] == '\r')) ++p;
  }
  FsNode value() {
    ws();
    if (p >= t.size()) throw std::runtime_error("FileStorage: unexpected end of a flow collection.");
    if (t[p] == '[') {
      FsNode n;
      n.kind = FsNode::SEQ;
      ++p;
      ws();
      if (p < t.size() && t[p] == ']') return ++p, n;
      for (;;) {
        n.seq.push_back(value());
        ws();
        if (p < t.size() && t[p] == ',') {
          ++p;
          continue;
        }
        if (p < t.size() && t[p] == ']') return ++p, n;
        throw std::runtime_error("FileStorage: malformed flow sequence.");
      }
    }
    if (t[p] == '{') {
      FsNode n;
      n.kind = FsNode::MAP;
      ++p;
      ws();
      if (p < t.size() && t[p] == '}') return ++p, n;
      for (;;) {
        ws();
        size_t c = t.find(':', p);
        if (c == std::string::npos) throw std::runtime_error("FileStorage: malformed flow map.");
        std::string key = trim(t.substr(p, c - p));
        p = c + 1;
        n.map.emplace_back(key, value());
        ws();
        if (p < t.size() && t[p] == ',') {
          ++p;
          continue;
        }
        if (p < t.size() && t[p] == '}') return ++p, n;
        throw std::runtime_error("FileStorage: malformed flow map.");
      }
    }
    size_t a = p;
    if (t[p] == '"' || t[p] == '\'') {
      const char q = t[p];
      size_t e = t.find(q, p + 1);
      if (e == std::string::npos) throw std::runtime_error("FileStorage: unterminated string.");
      p = e + 1;
    } else {
      while (p < t.size() && t[p] != ',' && t[p] != ']' && t[p] != '}') ++p;
    }
    return scalar(t.substr(a, p - a));
  }
};

struct Line {
  int indent;
  std::string text;  // without indentation and comment
};

std::string strip_comment(const std::string& s) {
  char q = 0;
  for (size_t k = 0; k < s.size(); ++k) {
    if (q) {
      if (s[k] == q) q = 0;
    } else if (s[k] == '"' || s[k] == '\'') {
      q = s[k];
    } else if (s[k] == '#') {
      return s.substr(0, k);
    }
  }
  return s;
}

int bracket_balance(const std::string& s) {
  int b = 0;
  char q = 0;
  for (char c : s) {
    if (q) {
      if (c == q) q = 0;
    } else if (c == '"' || c == '\'') {
      q = c;
    } else if (c == '[' || c == '{') {
      ++b;
    } else if (c == ']' || c == '}') {
      --b;
    }
  }
  return b;
}

FsNode to_matrix(const FsNode& m) {
  FsNode n;
  n.kind = FsNode::MAT;
  const FsNode& rows = m["rows"];
  const FsNode& cols = m["cols"];
  const FsNode& dt = m["dt"];
  const FsNode& data = m["data"];
  if (rows.kind != FsNode::INT || cols.kind != FsNode::INT || dt.kind != FsNode::STR)
    throw std::runtime_error("FileStorage: !!opencv-matrix needs rows, cols and dt.");
  n.mat.rows = (int)rows.i;
  n.mat.cols = (int)cols.i;
  const std::string d = dt.s;
  if (d.size() != 1 || std::string("ucwsifd").find(d[0]) == std::string::npos)
    throw std::runtime_error("FileStorage: unsupported matrix dt '" + d + "' (single-channel u c w s i f d).");
  n.mat.dt = d[0];
  for (const FsNode& e : data.seq) {
    if (e.kind == FsNode::INT)
      n.mat.v.push_back((double)e.i);
    else if (e.kind == FsNode::REAL)
      n.mat.v.push_back(e.f);
    else
      throw std::runtime_error("FileStorage: non-numeric matrix data.");
  }
  if ((long long)n.mat.v.size() != (long long)n.mat.rows * n.mat.cols)
    throw std::runtime_error("FileStorage: matrix data size does not match rows x cols.");
  return n;
}

class BlockParser {
 public:
  explicit BlockParser(std::vector<Line> lines) : L(std::move(lines)) {}
  FsNode document() {
    if (L.empty()) return FsNode{};
    FsNode root = block(L[0].indent);
    if (k != L.size()) throw std::runtime_error("FileStorage: unexpected indentation at '" + L[k].text + "'.");
    return root;
  }

 private:
  std::vector<Line> L;
  size_t k = 0;

  // Everything from `first` on, plus continuation lines until brackets close.
  std::string gather(std::string first) {
    int balance = bracket_balance(first);  // incremental: matrices span thousands of lines
    while (balance > 0 && k < L.size()) {
      balance += bracket_balance(L[k].text);
      first += " ";
      first += L[k++].text;
    }
    if (balance != 0) throw std::runtime_error("FileStorage: unbalanced brackets.");
    return first;
  }

  FsNode value_after(std::string rest, int indent) {
    rest = trim(rest);
    bool matrix = false;
    if (rest.rfind("!!opencv-matrix", 0) == 0) {
      matrix = true;
      rest = trim(rest.substr(15));
    } else if (!rest.empty() && rest[0] == '!') {  // other tags: ignore the tag
      size_t sp = rest.find(' ');
      rest = sp == std::string::npos ? std::string() : trim(rest.substr(sp));
    }
    FsNode n;
    if (rest.empty()) {
      if (k < L.size() && L[k].indent > indent && (L[k].text[0] == '[' || L[k].text[0] == '{')) {
        const std::string t = gather(L[k++].text);  // "-" then an indented flow value ("[]" of an empty entry)
        Flow fl{t};
        n = fl.value();
      } else if (k < L.size() && L[k].indent > indent) n = block(L[k].indent);
      else if (k < L.size() && L[k].indent == indent && L[k].text.rfind("- ", 0) == 0) n = block(indent);
    } else if (rest[0] == '[' || rest[0] == '{') {
      std::string t = gather(rest);
      Flow fl{t};
      n = fl.value();
    } else {
      n = scalar(rest);
    }
    return matrix ? to_matrix(n) : n;
  }

  FsNode block(int indent) {
    FsNode n;
    const bool is_seq = L[k].text.rfind("- ", 0) == 0 || L[k].text == "-";
    n.kind = is_seq ? FsNode::SEQ : FsNode::MAP;
    while (k < L.size() && L[k].indent == indent) {
      const std::string t = L[k].text;
      if (is_seq) {
        if (t.rfind("-", 0) != 0) break;
        ++k;
        n.seq.push_back(value_after(t.substr(1), indent));
      } else {
        size_t c = t.find(':');
        if (c == std::string::npos) throw std::runtime_error("FileStorage: expected 'key: value' at '" + t + "'.");
        ++k;
        std::string key = trim(t.substr(0, c));
        if (key.size() >= 2 && (key[0] == '"' || key[0] == '\'')) key = key.substr(1, key.size() - 2);
        n.map.emplace_back(key, value_after(t.substr(c + 1), indent));
      }
    }
    return n;
  }
};

const FsNode& none_node() {
  static const FsNode n;
  return n;
}

}  // namespace

const FsNode& FsNode::operator[](const std::string& key) const {
  for (const auto& kv : map)
    if (kv.first == key) return kv.second;
  return none_node();
}

int FsNode::to_int() const {
  if (kind == INT) return (int)i;
  if (kind == REAL) return (int)std::nearbyint(f);  // cvRound: half to even
  if (kind == NONE) return 0;
  return INT_MAX;
}

double FsNode::to_double() const {
  if (kind == INT) return (double)i;
  if (kind == REAL) return f;
  if (kind == NONE) return 0;
  return 1e300;
}

std::string FsNode::to_string() const { return kind == STR ? s : std::string(); }

FsMat FsNode::to_mat() const { return kind == MAT ? mat : FsMat{}; }

FsNode parse_file_storage(const std::string& text) {
  std::vector<Line> lines;
  std::istringstream in(text);
  std::string raw;
  bool first = true;
  while (std::getline(in, raw)) {
    std::string s = strip_comment(raw);
    if (trim(s).empty()) continue;
    if (first && s.rfind("%YAML", 0) == 0) {
      first = false;
      continue;
    }
    first = false;
    if (trim(s) == "---" || trim(s) == "...") continue;
    int ind = 0;
    while (ind < (int)s.size() && s[ind] == ' ') ++ind;
    lines.push_back({ind, trim(s)});
  }
  return BlockParser(std::move(lines)).document();
}

bool read_file_storage(const std::string& path, FsNode& root) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  root = parse_file_storage(ss.str());
  return true;
}

// ------------------------------------------------------------------ writer
// OpenCV's YAML emitter (persistence_yml.cpp: writeScalar, startWriteStruct,
// endWriteStruct; FileStorage::Impl::flush and operator<< (const String&)).

struct FsWriter::Impl {
  std::ofstream out;
};

static constexpr int kYmlIndent = 3, kWrapMargin = 71;

std::string fs_real(double v) {
  char buf[64];
  if (std::isnan(v)) return ".Nan";
  if (std::isinf(v)) return v < 0 ? "-.Inf" : ".Inf";
  const double r = std::nearbyint(v);  // cvRound
  if (r == v && std::fabs(r) <= (double)INT_MAX) {
    std::snprintf(buf, sizeof buf, "%d.", (int)r);
  } else {
    std::snprintf(buf, sizeof buf, "%.16e", v);
  }
  return buf;
}

FsWriter::FsWriter(const std::string& path) : f_(new Impl) {
  f_->out.open(path, std::ios::binary);
  if (f_->out) f_->out << "%YAML:1.0\n---\n";
  stack_.push_back({0, true, false, true});
}

FsWriter::~FsWriter() {
  release();
  delete f_;
}

bool FsWriter::isOpened() const { return (bool)f_->out && f_->out.is_open(); }

void FsWriter::release() {
  if (!f_->out.is_open()) return;
  while (stack_.size() > 1) end();
  flush();
  f_->out.close();
}

void FsWriter::flush() {
  if ((int)line_.size() > space_) f_->out << line_ << '\n';
  const int ind = stack_.back().indent;
  line_.assign((size_t)ind, ' ');
  space_ = ind;
}

void FsWriter::scalar(const char* key, const std::string* data) {
  Level& cur = stack_.back();
  if (key && !*key) key = nullptr;
  if (cur.map != (key != nullptr))
    throw std::runtime_error("FsWriter: an element without a name in a map, or with a name in a sequence.");
  const int keylen = key ? (int)std::strlen(key) : 0, datalen = data ? (int)data->size() : 0;
  if (cur.flow) {
    if (!cur.empty) line_ += ',';
    const int new_offset = (int)line_.size() + keylen + datalen;
    if (new_offset > kWrapMargin && new_offset - cur.indent > 10) flush();
    else line_ += ' ';
  } else {
    flush();
    if (!cur.map) {
      line_ += '-';
      if (data) line_ += ' ';
    }
  }
  if (key) {
    line_ += key;
    line_ += ':';
    if (!cur.flow && data) line_ += ' ';
  }
  if (data) line_ += *data;
  cur.empty = false;
}

void FsWriter::start(const char* key, bool map, bool flow, const char* type) {
  std::string data;
  bool has = false;
  if (type && !*type) type = nullptr;
  if (flow) {
    data = type ? std::string("!!") + type + " " + (map ? '{' : '[') : std::string(1, map ? '{' : '[');
    has = true;
  } else if (type) {
    data = std::string("!!") + type;
    has = true;
  }
  const Level parent = stack_.back();
  scalar(key, has ? &data : nullptr);
  stack_.push_back({parent.indent + (parent.flow ? 0 : kYmlIndent + (flow ? 1 : 0)), map, flow, true});
  if (!flow) flush();
}

void FsWriter::end() {
  if (stack_.size() < 2) throw std::runtime_error("FsWriter: extra closing bracket.");
  const Level cur = stack_.back();
  if (cur.flow) {
    if ((int)line_.size() > cur.indent && !cur.empty) line_ += ' ';
    line_ += cur.map ? '}' : ']';
  } else if (cur.empty) {
    flush();
    line_ += cur.map ? "{}" : "[]";
  }
  stack_.pop_back();
  stack_.back().empty = false;
}

void FsWriter::value(const std::string& text) {
  const bool in_map = stack_.back().map;
  if (in_map && name_expected_) throw std::runtime_error("FsWriter: no element name has been given.");
  scalar(in_map ? elname_.c_str() : nullptr, &text);
  elname_.clear();
  name_expected_ = stack_.back().map;
}

FsWriter& FsWriter::operator<<(const char* s) {
  if (!isOpened() || !s) return *this;
  const char c = *s;
  const bool in_map = stack_.back().map;
  if (c == '}' || c == ']') {
    if ((c == '}') != in_map) throw std::runtime_error("FsWriter: closing bracket does not match.");
    end();
    name_expected_ = stack_.back().map;
    elname_.clear();
  } else if (in_map && name_expected_) {
    elname_ = s;
    name_expected_ = false;
  } else if (c == '{' || c == '[') {
    bool flow = false;
    const char* t = s + 1;
    if (*t == ':') {
      ++t;
      if (!*t) flow = true;
    }
    start(in_map ? elname_.c_str() : nullptr, c == '{', flow, t);
    elname_.clear();
    name_expected_ = c == '{';
  } else {
    value(s);
  }
  return *this;
}

FsWriter& FsWriter::operator<<(int v) {
  if (isOpened()) value(std::to_string(v));
  return *this;
}

FsWriter& FsWriter::operator<<(double v) {
  if (isOpened()) value(fs_real(v));
  return *this;
}

void FsWriter::write_mat_i(const int* data, int rows, int cols) {
  if (!isOpened()) return;
  start(stack_.back().map ? elname_.c_str() : nullptr, true, false, "opencv-matrix");
  elname_.clear();
  name_expected_ = true;
  *this << "rows" << rows << "cols" << cols << "dt" << "i" << "data" << "[:";
  for (long long k = 0; k < (long long)rows * cols; ++k) *this << data[k];
  *this << "]";
  end();
  name_expected_ = stack_.back().map;
}

}  // namespace locomouse
