// plugin_surface.cpp -- the tile type's plugin surface on the C++ mirror
// (SpMat.h:54-174 requirements: Create(essentials), GetEssentials, GetArrays,
// Split/Merge, ColSplit/ColConcatenate, Transpose; LocalHybridSpGEMM returning
// SpTuples*, SpDCCols(SpTuples, false) as ParFriends.h:888-896 uses them).
// Checks on one GPU; prints "PLUGIN OK".
#include "combblas_amd/CombBLAS.h"

using namespace combblas_amd;
typedef SpDCCols<int, double> DCCols;
typedef SpParMat<int, double, DCCols> PMat;
typedef PlusTimesSRing<double, double> PT;

#define CHECK(c)                                           \
  do {                                                     \
    if (!(c)) {                                            \
      std::printf("FAILED: %s (line %d)\n", #c, __LINE__); \
      return 1;                                            \
    }                                                      \
  } while (0)

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rc = 0;
  {
    auto grid = std::make_shared<CommGrid>();  // single-process 1x1 grid
    const int scale = argc > 1 ? std::atoi(argv[1]) : 10;
    PMat A = PMat::rmat(grid, scale, 16), B = PMat::rmat(grid, scale, 16);
    // LocalHybridSpGEMM -> SpTuples* -> SpDCCols(tuples, false), as ParFriends.h:888-896
    SpTuples<int, double>* t = LocalHybridSpGEMM<PT, double>(A.seq(), B.seq(), false, false);
    DCCols C(*t, false);
    PMat Cs = Mult_AnXBn_Synch<PT, double, DCCols>(A, B);
    CHECK(C == Cs.seq());
    CHECK(t->getnnz() == C.getnnz() && t->getnrow() == A.getnrow() && t->getncol() == B.getncol());
    // the first column's rows ascend (col-major order, rows ascending)
    CHECK(t->colindex(0) <= t->colindex(1) && (t->colindex(0) != t->colindex(1) || t->rowindex(0) < t->rowindex(1)));
    delete t;
    // GetEssentials / Create / GetArrays
    std::vector<int> ess = C.GetEssentials();
    DCCols R;
    R.Create(ess);
    CHECK(R.GetEssentials() == ess);
    Arr<int, double> arr = C.GetArrays();
    CHECK(arr.totalsize() == 4 && arr.indarrs[0].count == ess[3] + 1 && arr.indarrs[2].count == ess[0] &&
          arr.numarrs[0].count == ess[0] && arr.indarrs[0].elem_bytes == 8 && arr.indarrs[1].elem_bytes == 4);
    // Split / Merge restore the tile
    DCCols L0, R0;
    C.Split(L0, R0);
    DCCols M;
    M.Merge(L0, R0);
    CHECK(M == Cs.seq());
    // ColSplit / ColConcatenate restore the tile
    std::vector<DCCols> pieces;
    M.ColSplit(3, pieces);
    CHECK(pieces.size() == 3 && M.getnnz() == 0);
    DCCols K;
    K.ColConcatenate(pieces);
    CHECK(K == Cs.seq());
    // Transpose twice is the identity; once it swaps the dimensions
    K.Transpose();
    CHECK(K.getnrow() == Cs.seq().getncol() && K.getnnz() == Cs.seq().getnnz());
    K.Transpose();
    CHECK(K == Cs.seq());
    std::printf("PLUGIN OK nnz %lld\n", (long long)C.getnnz());
  }
  MPI_Finalize();
  return rc;
}
