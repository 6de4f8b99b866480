// combblas_amd/CombBLAS.h -- C++ mirror of the reference's SpGEMM operator
// surface over libcbg's C ABI (include/cbg.h).  Header-only.
//
//   reference (include/CombBLAS/...)              this header (namespace combblas_amd)
//   SpDCCols<IT,NT>            SpDCCols.h         SpDCCols<IT,NT>   (device DCSC tile)
//   CommGrid(MPI_Comm,r,c)     CommGrid.h         CommGrid(MPI_Comm,r,c) -> RCCL grid
//   SpParMat<IT,NT,DER>        SpParMat.h         SpParMat<IT,NT,DER>
//   PlusTimesSRing/MinPlusSRing Semirings.h:212   PlusTimesSRing/MinPlusSRing
//   LocalHybridSpGEMM          mtSpGEMM.h:212     LocalHybridSpGEMM  (returns SpTuples*, device entries)
//   SpTuples<IT,NT>            SpTuples.h:65      SpTuples (col-major entries in HBM, host accessors)
//   SpDCCols Create/GetArrays/ SpDCCols.cpp:733,   same names; GetArrays lists DEVICE addresses
//     Transpose/Merge/ColSplit 825,853,1194,936
//   LocalSpGEMM (heap)         mtSpGEMM.h:73      LocalSpGEMM (same kernel; summation order differs only)
//   Mult_AnXBn_DoubleBuff      ParFriends.h:798   Mult_AnXBn_DoubleBuff
//   Mult_AnXBn_Synch           ParFriends.h:1004  Mult_AnXBn_Synch
//   PSpGEMM                    SpParMat.h:454     PSpGEMM
//   MemEfficientSpGEMM         ParFriends.h:449   MemEfficientSpGEMM (phases; no MCL pruning)
//   SpParMat::Transpose        SpParMat.cpp:3528  Transpose (square grids, RCCL send/recv)
//   SpParMat::DimApply         SpParMat.cpp:801   DimApply (dense vector given as its global values)
//   SpParMat::ReadDistribute   SpParMat.cpp:4211  ReadDistribute (text / HKDT binary triples)
//   FullyDistVec::ReadDistribute FullyDistVec.cpp:495 ReadDistributeVector (global values)
//   SpParMat::operator+=       SpParMat.cpp:741   operator+= (device merge)
//   SpDCCols/SpParMat ==       SpDCCols.h:74, SpParMat.cpp:2878  operator== (ErrorTolerantEqual)
//
// Same template parameters and call shapes, so MultTiming/MultTest-style
// drivers (tools/multtiming.cpp) compile against it.  Misuse that the
// reference MPI_Aborts on (DIMMISMATCH 3002, MATRIXALIAS 3005, NOTSQUARE 3003)
// aborts here with the same code.  Define CBG_NO_MPI to use a single-process grid.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "../../../include/cbg.h"

#ifndef CBG_NO_MPI
#include <mpi.h>
#endif

namespace combblas_amd {

inline void cbg_abort_on(int rc, const char* what) {
  if (rc == CBG_OK) return;
  std::fprintf(stderr, "%s: libcbg error %d: %s\n", what, rc, cbg_last_error());
#ifndef CBG_NO_MPI
  int init = 0;
  MPI_Initialized(&init);
  if (init) MPI_Abort(MPI_COMM_WORLD, rc);
#endif
  std::exit(rc);
}

// ---------------------------------------------------------------- semirings
enum Dim { Column = 0, Row = 1 };  // SpDefs.h
// functors usable with DimApply (std::multiplies<double> etc. of the reference)
template <class T> struct multiplies { static const int code = CBG_OP_MULTIPLIES; T operator()(T a, T b) const { return a * b; } };
template <class T> struct plus { static const int code = CBG_OP_PLUS; T operator()(T a, T b) const { return a + b; } };

// Operations.h maximum<T> (the BinOp MultTest passes to ParallelReadMM)
template <class T>
struct maximum {
  T operator()(const T& a, const T& b) const { return a < b ? b : a; }
};

template <class T1, class T2>
struct PlusTimesSRing {
  typedef T1 T_promote;
  static constexpr int code = CBG_PLUS_TIMES;
  static T1 id() { return 0; }
  static bool returnedSAID() { return false; }
  static T1 add(const T1& a, const T1& b) { return a + b; }
  static T1 multiply(const T1& a, const T2& b) { return a * b; }
};
template <class T1, class T2>
struct MinPlusSRing {
  typedef T1 T_promote;
  static constexpr int code = CBG_MIN_PLUS;
  static T1 id() { return std::numeric_limits<T1>::max(); }
  static bool returnedSAID() { return false; }
  static T1 add(const T1& a, const T1& b) { return b < a ? b : a; }
  static T1 multiply(const T1& a, const T2& b) {
    const T1 inf = std::numeric_limits<T1>::max();
    return (a == inf || b == inf) ? inf : a + b;
  }
};

// ---------------------------------------------------------------- tiles
// LocArr / Arr (LocArr.h:36-58): the arrays GetArrays() lists.  Here `addr` is a
// DEVICE pointer (a broadcast buffer for RCCL, not for MPI) and, because the
// tile's arrays have different widths (cp int64, jc/ir int32, numx f64),
// every entry also carries its element size.
template <class V, class C>
struct LocArr {
  LocArr() : addr(nullptr), count(0), elem_bytes(0) {}
  LocArr(V* a, C c, size_t eb) : addr(a), count(c), elem_bytes(eb) {}
  V* addr;
  C count;
  size_t elem_bytes;
};
template <class IT, class NT>
struct Arr {
  Arr(IT indsize, IT numsize) {
    indarrs.resize(indsize);
    numarrs.resize(numsize);
  }
  std::vector<LocArr<void, IT>> indarrs;  // cp (int64), jc (int32), ir (int32)
  std::vector<LocArr<NT, IT>> numarrs;    // numx
  IT totalsize() { return (IT)(indarrs.size() + numarrs.size()); }
};

template <class IT, class NT>
class SpTuples;

// SpDCCols<IT,NT>: a DCSC tile resident in HBM (int32 local indices, f64 values).
template <class IT, class NT>
class SpDCCols {
 public:
  typedef IT LocalIT;
  typedef NT LocalNT;
  static const IT esscount = 4;  // SpDCCols.cpp:45-46

  SpDCCols() { t_ = cbg_tile{}; }
  explicit SpDCCols(const cbg_tile& dev) : t_(dev) {}
  // SpDCCols(const SpTuples&, bool transpose) (SpDCCols.cpp:108-190): the tuples
  // (column-major, rows ascending) become this tile; a transposed view is built
  // with Transpose() (SpTuples::SortRowBased + the transpose constructor)
  SpDCCols(const SpTuples<IT, NT>& T, bool transpose);
  // from column-sorted host tuples (row, col, value), as SpDCCols(nRow,nCol,nTuples,tuples,false)
  SpDCCols(IT nRow, IT nCol, IT nTuples, const std::tuple<IT, IT, NT>* tuples, bool transpose = false) {
    if (transpose) throw std::invalid_argument("row-sorted input is not supported");
    std::vector<int64_t> cp(1, 0);
    std::vector<int32_t> jc, ir(nTuples);
    std::vector<double> val(nTuples);
    for (IT i = 0; i < nTuples; ++i) {
      const IT c = std::get<1>(tuples[i]);
      if (jc.empty() || jc.back() != (int32_t)c) {
        if (!jc.empty()) cp.push_back(i);
        jc.push_back((int32_t)c);
      }
      ir[i] = (int32_t)std::get<0>(tuples[i]);
      val[i] = (double)std::get<2>(tuples[i]);
    }
    cp.push_back(nTuples);
    if (jc.empty()) cp.assign(1, 0);
    cbg_tile h{nRow, nCol, (int64_t)nTuples, (int64_t)jc.size(), cp.data(), jc.data(), ir.data(), val.data(), 0, 0};
    cbg_abort_on(cbg_tile_upload(&h, &t_), "SpDCCols upload");
  }
  ~SpDCCols() { cbg_tile_free(&t_); }
  SpDCCols(const SpDCCols&) = delete;
  SpDCCols& operator=(const SpDCCols&) = delete;

  IT getnrow() const { return (IT)t_.m; }
  IT getncol() const { return (IT)t_.n; }
  int64_t getnnz() const { return t_.nnz; }
  int64_t getnzc() const { return t_.nzc; }
  bool isZero() const { return t_.nnz == 0; }
  // SpDCCols::operator== (SpDCCols.h:74-81): exact structure, values within EPSILON (SpDefs.h:64)
  bool operator==(const SpDCCols& rhs) const {
    int eq = 0;
    cbg_abort_on(cbg_tile_equal(&t_, &rhs.t_, 0.01, &eq), "SpDCCols::operator==");
    return eq != 0;
  }
  std::vector<IT> GetEssentials() const { return {(IT)t_.nnz, (IT)t_.m, (IT)t_.n, (IT)t_.nzc}; }
  // SpDCCols::Create(essentials) / CreateImpl (SpDCCols.cpp:733-745): an
  // uninitialised device tile {nnz, m, n, nzc} -- the receiving side of BCastMatrix
  void Create(const std::vector<IT>& ess) {
    if ((IT)ess.size() != esscount) cbg_abort_on(CBG_ERR_INVALIDPARAMS, "Create: esscount");
    cbg_tile t{};
    cbg_abort_on(cbg_tile_alloc((int64_t)ess[1], (int64_t)ess[2], (int64_t)ess[0], (int64_t)ess[3], &t), "Create");
    reset(t);
  }
  // SpDCCols::GetArrays (SpDCCols.cpp:825-851): indarrs {cp[nzc+1], jc[nzc], ir[nnz]},
  // numarrs {numx[nnz]}, device addresses (NULL / 0 for an empty tile)
  Arr<IT, NT> GetArrays() const {
    Arr<IT, NT> a(3, 1);
    if (t_.nnz > 0) {
      a.indarrs[0] = LocArr<void, IT>(t_.cp, (IT)(t_.nzc + 1), sizeof(int64_t));
      a.indarrs[1] = LocArr<void, IT>(t_.jc, (IT)t_.nzc, sizeof(int32_t));
      a.indarrs[2] = LocArr<void, IT>(t_.ir, (IT)t_.nnz, sizeof(int32_t));
      a.numarrs[0] = LocArr<NT, IT>(reinterpret_cast<NT*>(t_.val), (IT)t_.nnz, sizeof(double));
    } else {
      a.indarrs[0] = LocArr<void, IT>(nullptr, 0, sizeof(int64_t));
      a.indarrs[1] = LocArr<void, IT>(nullptr, 0, sizeof(int32_t));
      a.indarrs[2] = LocArr<void, IT>(nullptr, 0, sizeof(int32_t));
      a.numarrs[0] = LocArr<NT, IT>(nullptr, 0, sizeof(double));
    }
    return a;
  }
  // SpDCCols::Transpose (SpDCCols.cpp:853-873): in place
  void Transpose() {
    cbg_tile t{};
    cbg_abort_on(cbg_tile_transpose(&t_, &t), "Transpose");
    reset(t);
  }
  // SpDCCols::Merge (SpDCCols.cpp:1194-1223): *this = [partA | partB]; both are emptied
  void Merge(SpDCCols& partA, SpDCCols& partB) {
    cbg_tile parts[2] = {partA.t_, partB.t_}, t{};
    cbg_abort_on(cbg_tile_concat_cols(parts, 2, &t), "Merge");
    partA.reset(cbg_tile{});
    partB.reset(cbg_tile{});
    reset(t);
  }
  // SpDCCols::ColSplit (SpDCCols.cpp:936-970): `parts` pieces cut at
  // (i+1)*(n/parts), the last taking the rest; destroys *this
  void ColSplit(int parts, std::vector<SpDCCols>& matrices) {
    const int64_t w = t_.n / parts;
    matrices.clear();
    matrices.reserve(parts);
    cbg_tile rest = t_;
    bool own_rest = false;
    for (int i = 0; i + 1 < parts; ++i) {
      cbg_tile l{}, r{};
      cbg_abort_on(cbg_tile_split_cols(&rest, w, &l, &r), "ColSplit");
      if (own_rest) cbg_tile_free(&rest);
      matrices.emplace_back(l);
      rest = r;
      own_rest = true;
    }
    if (!own_rest) {  // one part: a copy
      cbg_tile l{}, r{};
      cbg_abort_on(cbg_tile_split_cols(&rest, t_.n, &l, &r), "ColSplit");
      cbg_tile_free(&r);
      rest = l;
    }
    matrices.emplace_back(rest);
    reset(cbg_tile{});
  }
  // SpDCCols::ColConcatenate (ParFriends.h:724-725): the pieces side by side
  void ColConcatenate(std::vector<SpDCCols>& matrices) {
    std::vector<cbg_tile> v;
    for (auto& m : matrices) v.push_back(m.t_);
    cbg_tile t{};
    cbg_abort_on(cbg_tile_concat_cols(v.data(), (int)v.size(), &t), "ColConcatenate");
    for (auto& m : matrices) m.reset(cbg_tile{});
    reset(t);
  }
  SpDCCols(SpDCCols&& o) noexcept : t_(o.t_) { o.t_ = cbg_tile{}; }
  SpDCCols& operator=(SpDCCols&& o) noexcept {
    if (this != &o) {
      cbg_tile_free(&t_);
      t_ = o.t_;
      o.t_ = cbg_tile{};
    }
    return *this;
  }
  const cbg_tile* tile() const { return &t_; }
  cbg_tile* tile() { return &t_; }
  cbg_tile release() {
    cbg_tile t = t_;
    t_ = cbg_tile{};
    return t;
  }

  // SpDCCols::Split (SpDCCols.cpp:905-930): columns [0,n/2) and [n/2,n)
  void Split(SpDCCols& a, SpDCCols& b) {
    cbg_tile l{}, r{};
    cbg_abort_on(cbg_tile_split_cols(&t_, t_.n / 2, &l, &r), "Split");
    a.reset(l);
    b.reset(r);
  }
  void reset(const cbg_tile& t) {
    cbg_tile_free(&t_);
    t_ = t;
  }
  // host copy as (cp, jc, ir, val)
  void download(std::vector<int64_t>& cp, std::vector<int32_t>& jc, std::vector<int32_t>& ir,
                std::vector<double>& val) const {
    cp.resize(t_.nzc + 1);
    jc.resize(t_.nzc);
    ir.resize(t_.nnz);
    val.resize(t_.nnz);
    cbg_tile h{0, 0, 0, 0, cp.data(), jc.data(), ir.data(), val.data(), 0, 0};
    cbg_abort_on(cbg_tile_download(&t_, &h), "download");
  }

 private:
  cbg_tile t_;
};

// SpTuples<IT,NT> (SpTuples.h:65-297): the local multiply's output container.
// The reference's is an AoS array of (row, col, value) tuples, column-major with
// rows ascending; here the same entries stay on the device in that order, held
// as the DCSC arrays the kernels emit (one device allocation, no AoS copy).
// getnnz/getnrow/getncol, rowindex/colindex/numvalue(i) (host accessors, the
// entries are fetched from HBM on first use), and SpDCCols(SpTuples, false)
// mirror the reference's use in LocalHybridSpGEMM callers (ParFriends.h:888-896).
template <class IT, class NT>
class SpTuples {
 public:
  explicit SpTuples(const cbg_tile& t) : t_(t) {}
  ~SpTuples() { cbg_tile_free(&t_); }
  SpTuples(const SpTuples&) = delete;
  SpTuples& operator=(const SpTuples&) = delete;
  int64_t getnnz() const { return t_.nnz; }
  IT getnrow() const { return (IT)t_.m; }
  IT getncol() const { return (IT)t_.n; }
  IT rowindex(int64_t i) const { return (IT)host().ir[i]; }
  IT colindex(int64_t i) const { return (IT)host().col[i]; }
  NT numvalue(int64_t i) const { return (NT)host().val[i]; }
  const cbg_tile* tile() const { return &t_; }
  cbg_tile release() {
    cbg_tile t = t_;
    t_ = cbg_tile{};
    return t;
  }

 private:
  struct Host {
    std::vector<int32_t> ir, col;
    std::vector<double> val;
  };
  const Host& host() const {
    if (!h_) {
      h_.reset(new Host());
      std::vector<int64_t> cp(t_.nzc + 1);
      std::vector<int32_t> jc(t_.nzc);
      h_->ir.resize(t_.nnz);
      h_->val.resize(t_.nnz);
      cbg_tile h{0, 0, 0, 0, cp.data(), jc.data(), h_->ir.data(), h_->val.data(), 0, 0};
      cbg_abort_on(cbg_tile_download(&t_, &h), "SpTuples");
      h_->col.resize(t_.nnz);
      for (int64_t i = 0; i < t_.nzc; ++i)
        for (int64_t p = cp[i]; p < cp[i + 1]; ++p) h_->col[p] = jc[i];
    }
    return *h_;
  }
  cbg_tile t_;
  mutable std::unique_ptr<Host> h_;
};

template <class IT, class NT>
SpDCCols<IT, NT>::SpDCCols(const SpTuples<IT, NT>& T, bool transpose) {
  cbg_tile c{}, r{};
  // a device copy of the tuples' arrays (the reference copies the tuples too)
  cbg_abort_on(cbg_tile_split_cols(T.tile(), T.tile()->n, &c, &r), "SpDCCols(SpTuples)");
  cbg_tile_free(&r);
  t_ = c;
  if (transpose) Transpose();
}

// ---------------------------------------------------------------- grid
class CommGrid {
 public:
#ifndef CBG_NO_MPI
  // CommGrid(MPI_COMM_WORLD, 0, 0): square grid or NOTSQUARE (src/CommGrid.cpp:37-75).
  // One rank per GPU; the RCCL unique id travels by MPI_Bcast.
  CommGrid(MPI_Comm world, int nrowproc, int ncolproc) {
    MPI_Comm_rank(world, &rank_);
    MPI_Comm_size(world, &size_);
    char id[CBG_UNIQUE_ID_BYTES] = {0};
    if (rank_ == 0) cbg_abort_on(cbg_get_unique_id(id), "ncclGetUniqueId");
    MPI_Bcast(id, CBG_UNIQUE_ID_BYTES, MPI_BYTE, 0, world);
    int ndev = 1;
    cbg_device_count(&ndev);
    cbg_set_device(rank_ % (ndev > 0 ? ndev : 1));
    cbg_abort_on(cbg_grid_create(rank_, size_, nrowproc, ncolproc, id, &g_), "CommGrid");
    int dummy;
    cbg_grid_info(g_, &dummy, &dummy, &rows_, &cols_, &prow_, &pcol_);
  }
#endif
  // single-process 1x1 grid
  CommGrid() {
    static cbg_host_comm self = {[](void*, int, void*, size_t, int) { return 0; },
                                 [](void*, int, const void* in, void* out, size_t b) {
                                   std::memcpy(out, in, b);
                                   return 0;
                                 },
                                 nullptr};
    cbg_abort_on(cbg_grid_create_host(0, 1, 1, 1, &self, &g_), "CommGrid");
  }
  ~CommGrid() { cbg_grid_destroy(g_); }
  CommGrid(const CommGrid&) = delete;
  CommGrid& operator=(const CommGrid&) = delete;

  int GetRank() const { return rank_; }
  int GetSize() const { return size_; }
  int GetGridRows() const { return rows_; }
  int GetGridCols() const { return cols_; }
  int GetRankInProcRow() const { return pcol_; }
  int GetRankInProcCol() const { return prow_; }
  cbg_grid* handle() const { return g_; }
  bool operator==(const CommGrid& o) const { return rows_ == o.rows_ && cols_ == o.cols_ && size_ == o.size_; }

 private:
  cbg_grid* g_ = nullptr;
  int rank_ = 0, size_ = 1, rows_ = 1, cols_ = 1, prow_ = 0, pcol_ = 0;
};

// ---------------------------------------------------------------- distributed matrix
template <class IT, class NT, class DER>
class SpParMat {
 public:
  SpParMat() = default;
  explicit SpParMat(std::shared_ptr<CommGrid> grid) : commGrid(grid) {}
  SpParMat(DER* seq, std::shared_ptr<CommGrid> grid, IT gm, IT gn) : spSeq(seq), commGrid(grid), m_(gm), n_(gn) {}
  SpParMat(SpParMat&& o) noexcept : spSeq(o.spSeq), commGrid(o.commGrid), m_(o.m_), n_(o.n_) { o.spSeq = nullptr; }
  SpParMat& operator=(SpParMat&& o) noexcept {
    if (this != &o) {
      delete spSeq;
      spSeq = o.spSeq;
      o.spSeq = nullptr;
      commGrid = o.commGrid;
      m_ = o.m_;
      n_ = o.n_;
    }
    return *this;
  }
  ~SpParMat() { delete spSeq; }
  SpParMat(const SpParMat&) = delete;

  // Graph500 R-MAT tile of this rank (GenWriteMatrix.cpp:101-114 semantics)
  static SpParMat rmat(std::shared_ptr<CommGrid> g, int scale, int ef, uint64_t seed = 0xDECAFBADULL) {
    cbg_tile t{};
    cbg_abort_on(cbg_rmat_tile(scale, ef, seed, g->GetGridRows(), g->GetGridCols(), g->GetRankInProcCol(),
                               g->GetRankInProcRow(), &t),
                 "rmat");
    const IT nv = (IT)1 << scale;
    return SpParMat(new DER(t), g, nv, nv);
  }

  // SpParMat::ParallelReadMM (SpParMat.cpp:3980-4117): Matrix Market coordinate
  // real / integer / pattern (value 1), symmetric or hermitian entries mirrored
  // (SpHelper::push_to_vectors, SpHelper.h:75-91), duplicates combined with BinOp
  // in column-major order (SpTuples::RemoveDuplicates).  Every rank parses the
  // file and keeps its block (the reference splits the bytes across ranks and
  // redistributes; the tiles are the same).
  template <typename BinOp>
  void ParallelReadMM(const std::string& filename, bool onebased, BinOp binop) {
    FILE* f = std::fopen(filename.c_str(), "r");
    if (!f) cbg_abort_on(3004, ("Matrix-market file " + filename + " can not be found").c_str());  // NOFILE
    char line[1024], mm[64], obj[64], fmt[64], field[64], sym[64];
    if (!std::fgets(line, sizeof line, f) || std::sscanf(line, "%63s %63s %63s %63s %63s", mm, obj, fmt, field, sym) != 5 ||
        std::strcmp(fmt, "coordinate") != 0)
      cbg_abort_on(CBG_ERR_INVALIDPARAMS, "Could not process Matrix Market banner");
    const bool pattern = std::strcmp(field, "pattern") == 0;
    const bool symmetric = std::strcmp(sym, "symmetric") == 0 || std::strcmp(sym, "hermitian") == 0;
    long long m = 0, n = 0, nz = 0;
    while (std::fgets(line, sizeof line, f))
      if (line[0] != '%' && std::sscanf(line, "%lld %lld %lld", &m, &n, &nz) == 3) break;
    const int pr = commGrid->GetGridRows(), pc = commGrid->GetGridCols();
    const int r = commGrid->GetRankInProcCol(), c = commGrid->GetRankInProcRow();
    const long long mper = m / pr, nper = n / pc;  // SpParMat::Owner (SpParMat.cpp:5068-5097)
    const long long r0 = r * mper, r1 = (r == pr - 1) ? m : r0 + mper;
    const long long c0 = c * nper, c1 = (c == pc - 1) ? n : c0 + nper;
    std::vector<std::tuple<IT, IT, NT>> t;
    auto keep = [&](long long i, long long j, double v) {
      if (i >= r0 && i < r1 && j >= c0 && j < c1) t.emplace_back((IT)(i - r0), (IT)(j - c0), (NT)v);
    };
    while (std::fgets(line, sizeof line, f)) {
      long long i, j;
      double v = 1.0;
      const int got = pattern ? std::sscanf(line, "%lld %lld", &i, &j) : std::sscanf(line, "%lld %lld %lg", &i, &j, &v);
      if (got < 2) continue;
      if (onebased) { --i; --j; }
      keep(i, j, v);
      if (symmetric && i != j) keep(j, i, v);
    }
    std::fclose(f);
    std::stable_sort(t.begin(), t.end(), [](const std::tuple<IT, IT, NT>& a, const std::tuple<IT, IT, NT>& b) {
      return std::get<1>(a) != std::get<1>(b) ? std::get<1>(a) < std::get<1>(b) : std::get<0>(a) < std::get<0>(b);
    });
    std::vector<std::tuple<IT, IT, NT>> u;
    for (auto& x : t) {
      if (!u.empty() && std::get<0>(u.back()) == std::get<0>(x) && std::get<1>(u.back()) == std::get<1>(x))
        std::get<2>(u.back()) = binop(std::get<2>(u.back()), std::get<2>(x));
      else
        u.push_back(x);
    }
    delete spSeq;
    spSeq = new DER((IT)(r1 - r0), (IT)(c1 - c0), (IT)u.size(), u.data(), false);
    m_ = (IT)m;
    n_ = (IT)n;
  }

  // SpParMat::ReadDistribute (SpParMat.cpp:4211-4540), the GalerkinNew input:
  // text = '%' comment lines, "m n nnz", then nnz lines "i j [v]" (1-based, a
  // missing value reads 1); binary = "HKDT" + uint64 {version, objsize, format, m,
  // n, nnz} + nnz {int64 row, int64 col, double val} records (0-based).  Tuples
  // sorted column-major, duplicates kept (SpDCCols::Create).  Every rank reads
  // the file and keeps its block; the master argument is accepted for the
  // reference's signature.
  void ReadDistribute(const std::string& filename, int master = 0) {
    (void)master;
    FILE* f = std::fopen(filename.c_str(), "rb");
    if (!f) cbg_abort_on(3004, ("ReadDistribute: file " + filename + " can not be found").c_str());  // NOFILE
    long long m = 0, n = 0, nz = 0;
    std::vector<long long> ri, ci;
    std::vector<double> vv;
    char magic[4] = {0};
    if (std::fread(magic, 1, 4, f) == 4 && std::memcmp(magic, "HKDT", 4) == 0) {
      uint64_t h[6];
      if (std::fread(h, sizeof h, 1, f) != 1 || h[2] != 0)
        cbg_abort_on(CBG_ERR_INVALIDPARAMS, "ReadDistribute: bad binary header");
      m = (long long)h[3];
      n = (long long)h[4];
      nz = (long long)h[5];
      struct Rec { int64_t r, c; double v; } rec;
      for (long long k = 0; k < nz && std::fread(&rec, sizeof rec, 1, f) == 1; ++k) {
        ri.push_back(rec.r);
        ci.push_back(rec.c);
        vv.push_back(rec.v);
      }
    } else {
      std::rewind(f);
      char line[1024];
      while (std::fgets(line, sizeof line, f))
        if (line[0] != '%' && std::sscanf(line, "%lld %lld %lld", &m, &n, &nz) == 3) break;
      for (long long k = 0; k < nz && std::fgets(line, sizeof line, f); ++k) {
        long long i, j;
        double v = 1.0;
        if (std::sscanf(line, "%lld %lld %lg", &i, &j, &v) < 2) { --k; continue; }
        ri.push_back(i - 1);
        ci.push_back(j - 1);
        vv.push_back(v);
      }
    }
    std::fclose(f);
    const int pr = commGrid->GetGridRows(), pc = commGrid->GetGridCols();
    const int r = commGrid->GetRankInProcCol(), c = commGrid->GetRankInProcRow();
    const long long mper = m / pr, nper = n / pc;  // SpParMat::Owner (SpParMat.cpp:5068-5097)
    const long long r0 = r * mper, r1 = (r == pr - 1) ? m : r0 + mper;
    const long long c0 = c * nper, c1 = (c == pc - 1) ? n : c0 + nper;
    std::vector<std::tuple<IT, IT, NT>> t;
    for (size_t k = 0; k < ri.size(); ++k)
      if (ri[k] >= r0 && ri[k] < r1 && ci[k] >= c0 && ci[k] < c1)
        t.emplace_back((IT)(ri[k] - r0), (IT)(ci[k] - c0), (NT)vv[k]);
    std::stable_sort(t.begin(), t.end(), [](const std::tuple<IT, IT, NT>& a, const std::tuple<IT, IT, NT>& b) {
      return std::get<1>(a) != std::get<1>(b) ? std::get<1>(a) < std::get<1>(b) : std::get<0>(a) < std::get<0>(b);
    });
    delete spSeq;
    spSeq = new DER((IT)(r1 - r0), (IT)(c1 - c0), (IT)t.size(), t.data(), false);
    m_ = (IT)m;
    n_ = (IT)n;
  }

  IT getnrow() const { return m_; }
  IT getncol() const { return n_; }
  int64_t getnnz() const {  // SpParMat::getnnz (Allreduce, SpParMat.cpp:772-778)
    int64_t v = spSeq ? spSeq->getnnz() : 0;
    cbg_abort_on(cbg_grid_allreduce_sum_i64(commGrid->handle(), &v), "getnnz");
    return v;
  }
  DER& seq() const { return *spSeq; }
  std::shared_ptr<CommGrid> getcommgrid() const { return commGrid; }
  // SpParMat::Transpose (SpParMat.cpp:3528-3590): in place, square grids
  void Transpose() {
    cbg_tile t{};
    cbg_abort_on(cbg_grid_transpose(commGrid->handle(), spSeq->tile(), &t), "Transpose");
    spSeq->reset(t);
    std::swap(m_, n_);
  }
  // SpParMat::DimApply (SpParMat.cpp:801) with the distributed vector's global
  // values (FullyDistVec is not on this path); op: a functor class below
  template <typename Op>
  void DimApply(Dim dim, const std::vector<double>& global, Op) {
    const int parts = dim == Column ? commGrid->GetGridCols() : commGrid->GetGridRows();
    const int idx = dim == Column ? commGrid->GetRankInProcRow() : commGrid->GetRankInProcCol();
    const int64_t total = dim == Column ? (int64_t)n_ : (int64_t)m_;
    const int64_t per = total / parts, lo = idx * per;
    cbg_abort_on(cbg_tile_dim_apply(spSeq->tile(), dim == Column ? CBG_DIM_COLUMN : CBG_DIM_ROW, global.data() + lo,
                                    Op::code),
                 "DimApply");
  }
  // SpParMat::operator+= (SpParMat.cpp:741): union with duplicates added
  SpParMat& operator+=(const SpParMat& rhs) {
    cbg_tile parts[2] = {*spSeq->tile(), *rhs.spSeq->tile()}, c{};
    cbg_abort_on(cbg_merge(parts, 2, CBG_PLUS_TIMES, &c, nullptr), "operator+=");
    spSeq->reset(c);
    return *this;
  }
  // restriction operator (mfiles/genrestrict.m role): n x n/order
  static SpParMat restriction(std::shared_ptr<CommGrid> g, int scale, int order, uint64_t seed = 0x5EED) {
    cbg_tile t{};
    cbg_abort_on(cbg_restriction_tile(scale, order, seed, g->GetGridRows(), g->GetGridCols(), g->GetRankInProcCol(),
                                      g->GetRankInProcRow(), &t),
                 "restriction");
    const IT n = (IT)1 << scale;
    return SpParMat(new DER(t), g, n, n / order);
  }

  // rows (dim 0) or columns (dim 1) [lo, hi) as a distributed matrix of their own
  SpParMat BlockExtract(int dim, IT lo, IT hi) const {
    cbg_tile t{};
    cbg_abort_on(cbg_grid_block_extract(commGrid->handle(), spSeq->tile(), m_, n_, dim, lo, hi, &t), "BlockSplit");
    return SpParMat(new DER(t), commGrid, dim == 0 ? hi - lo : m_, dim == 1 ? hi - lo : n_);
  }
  // block starts of BlockSplit / BlockSpGEMM::getBlockOffsets: n / nb per
  // block, the first n % nb blocks one longer, n at the end
  static std::vector<IT> BlockOffsets(IT n, int nb) {
    std::vector<IT> o(nb + 1);
    const IT bs = n / nb, r = n % nb;
    for (int b = 0; b < nb; ++b) o[b] = std::min((IT)b, r) * (bs + 1) + ((IT)b < r ? 0 : (IT)b - r) * bs;
    o[nb] = n;
    return o;
  }
  // SpParMat::BlockSplit (SpParMat.cpp:2974-3058): br x bc blocks, each a
  // distributed matrix on this grid in the standard layout
  std::vector<std::vector<SpParMat>> BlockSplit(int br, int bc) const {
    std::vector<std::vector<SpParMat>> out(br);
    if ((br == 1 && bc == 1) || (IT)br > m_ || (IT)bc > n_) {
      out.resize(1);
      out[0].push_back(BlockExtract(0, 0, m_));  // a copy of *this
      return out;
    }
    const std::vector<IT> ro = BlockOffsets(m_, br), co = BlockOffsets(n_, bc);
    for (int i = 0; i < br; ++i) {
      SpParMat R = BlockExtract(0, ro[i], ro[i + 1]);
      for (int j = 0; j < bc; ++j) out[i].push_back(bc == 1 ? std::move(R) : R.BlockExtract(1, co[j], co[j + 1]));
    }
    return out;
  }

  // SpParMat::operator== (SpParMat.cpp:2878-2884): local equality, AND over the grid
  bool operator==(const SpParMat& rhs) const {
    int64_t bad = (*spSeq == *rhs.spSeq) ? 0 : 1;
    cbg_abort_on(cbg_grid_allreduce_sum_i64(commGrid->handle(), &bad), "SpParMat::operator==");
    return bad == 0;
  }

  DER* spSeq = nullptr;
  std::shared_ptr<CommGrid> commGrid;

 private:
  IT m_ = 0, n_ = 0;
};

// ---------------------------------------------------------------- products
// LocalHybridSpGEMM (mtSpGEMM.h:213-217): the caller owns the returned
// SpTuples* (delete it, or build an SpDCCols from it as ParFriends.h:888-896
// does); clearA/clearB delete the inputs (mtSpGEMM.h:443-446)
template <class SR, class NTO, class IT, class NT1, class NT2>
SpTuples<IT, NTO>* LocalHybridSpGEMM(const SpDCCols<IT, NT1>& A, const SpDCCols<IT, NT2>& B, bool clearA, bool clearB,
                                     IT* aux = nullptr) {
  (void)aux;
  cbg_tile c{};
  cbg_abort_on(cbg_local_spgemm(A.tile(), B.tile(), SR::code, &c, nullptr), "LocalHybridSpGEMM");
  if (clearA) delete const_cast<SpDCCols<IT, NT1>*>(&A);
  if (clearB) delete const_cast<SpDCCols<IT, NT2>*>(&B);
  return new SpTuples<IT, NTO>(c);
}
// LocalSpGEMM (heap kernel, mtSpGEMM.h:73-202): same C structure; the heap's
// summation order only changes fp rounding, so it runs the same device kernel
template <class SR, class NTO, class IT, class NT1, class NT2>
SpTuples<IT, NTO>* LocalSpGEMM(const SpDCCols<IT, NT1>& A, const SpDCCols<IT, NT2>& B, bool clearA, bool clearB) {
  return LocalHybridSpGEMM<SR, NTO>(A, B, clearA, clearB);
}

namespace detail {
template <class SR, class NUO, class UDERO, class IU, class NU1, class NU2, class UDERA, class UDERB>
SpParMat<IU, NUO, UDERO> summa(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B, int algo, bool clearA,
                               bool clearB, int exec) {
  if ((void*)&A == (void*)&B) cbg_abort_on(CBG_ERR_MATRIXALIAS, "Can not multiply, inputs alias");
  if (A.getncol() != B.getnrow()) cbg_abort_on(CBG_ERR_DIMMISMATCH, "Can not multiply, dimensions does not match");
  if (!(*A.commGrid == *B.commGrid)) cbg_abort_on(CBG_ERR_GRIDMISMATCH, "Grids don't confirm for multiplication");
  cbg_tile c{};
  cbg_abort_on(cbg_summa_spgemm(A.commGrid->handle(), A.spSeq->tile(), B.spSeq->tile(), A.getncol(), B.getnrow(),
                                SR::code, algo, exec, &c),
               algo == CBG_DOUBLEBUFF ? "Mult_AnXBn_DoubleBuff" : "Mult_AnXBn_Synch");
  SpParMat<IU, NUO, UDERO> C(new UDERO(c), A.commGrid, A.getnrow(), B.getncol());
  if (clearA) { delete A.spSeq; A.spSeq = nullptr; }
  if (clearB) { delete B.spSeq; B.spSeq = nullptr; }
  return C;
}
}  // namespace detail

// ParFriends.h:798-800 signature
template <typename SR, typename NUO, typename UDERO, typename IU, typename NU1, typename NU2, typename UDERA,
          typename UDERB>
SpParMat<IU, NUO, UDERO> Mult_AnXBn_DoubleBuff(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B,
                                                bool clearA = false, bool clearB = false, int exec = CBG_EXEC_PANEL) {
  return detail::summa<SR, NUO, UDERO>(A, B, CBG_DOUBLEBUFF, clearA, clearB, exec);
}
// ParFriends.h:1004-1006 signature
template <typename SR, typename NUO, typename UDERO, typename IU, typename NU1, typename NU2, typename UDERA,
          typename UDERB>
SpParMat<IU, NUO, UDERO> Mult_AnXBn_Synch(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B,
                                           bool clearA = false, bool clearB = false, int exec = CBG_EXEC_PANEL) {
  return detail::summa<SR, NUO, UDERO>(A, B, CBG_SYNCH, clearA, clearB, exec);
}
// ParFriends.h:449-451 signature.  Phases cut B's local tile by columns and C is
// column-concatenated; the Markov-clustering pruning arguments must keep their
// no-pruning values (hardThreshold, selectNum, recoverNum, recoverPct <= 0);
// perProcessMemory > 0 (GB) picks the phase count from memory like the
// reference (ParFriends.h:482-535; see cbg_summa_spgemm_memeff), phases < 1 is
// reset to 1 (:469-473); kselectVersion/computationKernel select CPU kernels of
// the reference and are unused here.
template <typename SR, typename NUO, typename UDERO, typename IU, typename NU1, typename NU2, typename UDERA,
          typename UDERB>
SpParMat<IU, NUO, UDERO> MemEfficientSpGEMM(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B, int phases,
                                             NUO hardThreshold, IU selectNum, IU recoverNum, NUO recoverPct,
                                             int kselectVersion, int computationKernel, int64_t perProcessMemory) {
  (void)kselectVersion;
  (void)computationKernel;
  if (hardThreshold > 0 || selectNum > 0 || recoverNum > 0 || recoverPct > 0)
    cbg_abort_on(CBG_ERR_INVALIDPARAMS, "MemEfficientSpGEMM: pruning is not supported");
  if (A.getncol() != B.getnrow()) cbg_abort_on(CBG_ERR_DIMMISMATCH, "Can not multiply, dimensions does not match");
  if (phases < 1) phases = 1;
  cbg_tile c{};
  cbg_abort_on(cbg_summa_spgemm_memeff(A.commGrid->handle(), A.spSeq->tile(), B.spSeq->tile(), A.getncol(),
                                       B.getnrow(), SR::code, CBG_DOUBLEBUFF, CBG_EXEC_PANEL, phases,
                                       perProcessMemory > 0 ? perProcessMemory : 0, nullptr, nullptr, &c),
               "MemEfficientSpGEMM");
  return SpParMat<IU, NUO, UDERO>(new UDERO(c), A.commGrid, A.getnrow(), B.getncol());
}

// BlockSpGEMM (BlockSpGEMM.h:14-131): C = A*B block by block, A split into br
// row blocks and B into bc column blocks (bi = 1), each block product a
// Mult_AnXBn_DoubleBuff
template <typename IT, typename NTA, typename DERA, typename NTB, typename DERB>
struct BlockSpGEMM {
  BlockSpGEMM(SpParMat<IT, NTA, DERA>& A, SpParMat<IT, NTB, DERB>& B, int br, int bc, int bi = 1)
      : br_(br), bc_(bc), bi_(bi), cur_block_(0) {
    if (bi_ != 1) cbg_abort_on(CBG_ERR_NOTSUPPORTED, "BlockSpGEMM: bi must be 1");
    A_blocks_ = A.BlockSplit(br_, bi_);
    B_blocks_ = B.BlockSplit(bi_, bc_);
    nr_ = A.getnrow();
    nc_ = B.getncol();
  }
  template <typename SR, typename NTC, typename DERC>
  SpParMat<IT, NTC, DERC> getNextBlock(IT& roffset, IT& coffset) {
    const int rbid = cur_block_ / bc_, cbid = cur_block_ % bc_;
    ++cur_block_;
    return getBlockId<SR, NTC, DERC>(rbid, cbid, roffset, coffset);
  }
  bool hasNext() { return cur_block_ < br_ * bc_; }
  template <typename SR, typename NTC, typename DERC>
  SpParMat<IT, NTC, DERC> getBlockId(int rbid, int cbid, IT& roffset, IT& coffset) {
    roffset = getBlockOffsets(true)[rbid];
    coffset = getBlockOffsets(false)[cbid];
    return Mult_AnXBn_DoubleBuff<SR, NTC, DERC>(A_blocks_[rbid][0], B_blocks_[0][cbid], false, false);
  }
  std::vector<IT> getBlockOffsets(bool is_row) {
    return SpParMat<IT, NTA, DERA>::BlockOffsets(is_row ? nr_ : nc_, is_row ? br_ : bc_);
  }

 private:
  std::vector<std::vector<SpParMat<IT, NTA, DERA>>> A_blocks_;
  std::vector<std::vector<SpParMat<IT, NTB, DERB>>> B_blocks_;
  int br_, bc_, bi_, cur_block_;
  IT nr_ = 0, nc_ = 0;
};

// SpParMat.h:454-467
template <typename SR, typename IU, typename NU1, typename NU2, typename UDERA, typename UDERB>
SpParMat<IU, typename SR::T_promote, UDERA> PSpGEMM(SpParMat<IU, NU1, UDERA>& A, SpParMat<IU, NU2, UDERB>& B) {
  return Mult_AnXBn_Synch<SR, typename SR::T_promote, UDERA>(A, B);
}

// FullyDistVec<IT,double>::ReadDistribute (FullyDistVec.cpp:495 ->
// FullyDistSpVec.cpp:1397-1437) as the global values DimApply takes: header
// "m n nnz", then "i j v" lines (1-based); the index is the row of a column
// vector (n == 1), else the column; absent entries are 0.
inline std::vector<double> ReadDistributeVector(const std::string& filename) {
  FILE* f = std::fopen(filename.c_str(), "r");
  if (!f) cbg_abort_on(3004, ("ReadDistribute: file " + filename + " can not be found").c_str());  // NOFILE
  char line[1024];
  long long m = 0, n = 0, nz = 0;
  if (!std::fgets(line, sizeof line, f) || std::sscanf(line, "%lld %lld %lld", &m, &n, &nz) != 3)
    cbg_abort_on(CBG_ERR_INVALIDPARAMS, "ReadDistribute: bad vector header");
  std::vector<double> out((size_t)(n == 1 ? m : n), 0.0);
  for (long long k = 0; k < nz && std::fgets(line, sizeof line, f); ++k) {
    long long i, j;
    double v = 1.0;
    if (std::sscanf(line, "%lld %lld %lg", &i, &j, &v) < 2) continue;
    const long long x = (n == 1 ? i : j) - 1;
    if (x >= 0 && x < (long long)out.size()) out[(size_t)x] = v;
  }
  std::fclose(f);
  return out;
}

}  // namespace combblas_amd
