// MyMat.hpp — the cost-matrix containers handed to the match2nd tracker.
//
// Same names and element semantics as the reference's MyMat / MATSPARSE
// (MyMat/MyMat.hpp:20-95, MyMat.cpp): MyMat is a column-major double matrix
// (values[j*nrows + i], MyMat.cpp:64-70); MATSPARSE is MATLAB's CSC layout
// (Ir row indices, Jc column starts with Jc[0] = 0 and ncols+1 entries, Pr
// values; MyMat.cpp:141-178).  Storage is std::vector here, so copies are
// deep and nothing leaks (the reference's copy-assign leaks, MyMat.cpp:230-255).
#ifndef LOCOMOUSE_HOST_MYMAT_HPP
#define LOCOMOUSE_HOST_MYMAT_HPP

#include <ostream>
#include <vector>

namespace locomouse {

class MyMat {
  std::vector<double> values;
  int nrows = 0, ncols = 0, numel = 0;

 public:
  MyMat() = default;
  MyMat(unsigned n, unsigned m) : values((size_t)n * m, 0.0), nrows((int)n), ncols((int)m), numel((int)(n * m)) {}

  void put(unsigned i, unsigned j, double val);
  double get(unsigned i, unsigned j) const;
  inline int Nrows() const { return nrows; }
  inline int Ncols() const { return ncols; }
  inline int Numel() const { return numel; }
  inline double* getValues() { return values.data(); }
  inline const double* getValues() const { return values.data(); }
};

class MATSPARSE {
  std::vector<int> Ir, Jc;
  std::vector<double> Pr;
  int nzel = 0, n_rows = 0, n_cols = 0;

 public:
  MATSPARSE() = default;
  explicit MATSPARSE(const MyMat* M);  // dense -> CSC, column by column, zeros dropped
  // CSC arrays as recorded by the device path (jc: ncols+1 entries).
  MATSPARSE(int rows, int cols, const int* jc, const int* ir, const double* pr);

  // The reference's get() returns 0 before its lookup (MyMat.cpp:371-374);
  // kept for drop-in behaviour.  at() is the lookup it intended.
  double get(int irow, int icol) const;
  double at(int irow, int icol) const;
  inline int* getIr() const { return const_cast<int*>(Ir.data()); }
  inline int* getJc() const { return const_cast<int*>(Jc.data()); }
  inline double* getPr() const { return const_cast<double*>(Pr.data()); }
  inline int nz() const { return nzel; }
  inline int Nrows() const { return n_rows; }
  inline int Ncols() const { return n_cols; }

  bool operator==(const MATSPARSE& o) const;
};

std::ostream& operator<<(std::ostream& out, const MyMat& M);

}  // namespace locomouse

#ifndef LOCOMOUSE_NO_GLOBAL_NAMES
using locomouse::MATSPARSE;
using locomouse::MyMat;
#endif

#endif
