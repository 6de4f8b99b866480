// adapter_check.cpp -- compile/link check of integration/ParFriends_cbg.h against
// the reference's headers (TEST INFRASTRUCTURE: built only where /root/reference
// exists, by oracle/Makefile).  Run as `adapter_check A.mtx` on a GPU box it
// multiplies A*A with the reference's own CPU Mult_AnXBn_Synch and with the
// adapter (the drop-in specializations and the *_cbg functions), plus-times and
// min-plus, and compares them with the reference's SpParMat::operator==.
#include "ParFriends_cbg.h"

#include <cstdio>

using namespace combblas;
typedef SpDCCols<int64_t, double> DCCols;
typedef SpParMat<int64_t, double, DCCols> PMat;

// semiring types the adapter does not specialize: the reference's own template
// (its CPU LocalHybridSpGEMM + MultiwayMerge) computes the control products
struct RefPlusTimes : PlusTimesSRing<double, double> {};
struct RefMinPlus : MinPlusSRing<double, double> {};

int main(int argc, char* argv[]) {
  MPI_Init(&argc, &argv);
  int ok = 1;
  if (argc > 1) {
    auto grid = std::make_shared<CommGrid>(MPI_COMM_WORLD, 0, 0);
    PMat A(grid), B(grid);
    A.ParallelReadMM(argv[1], true, maximum<double>());
    B.ParallelReadMM(argv[1], true, maximum<double>());
    PMat Cref = Mult_AnXBn_Synch<RefPlusTimes, double, DCCols>(A, B);
    PMat Cdrop = Mult_AnXBn_DoubleBuff<PlusTimesSRing<double, double>, double, DCCols>(A, B);  // drop-in
    PMat Csyn = Mult_AnXBn_Synch<PlusTimesSRing<double, double>, double, DCCols>(A, B);        // drop-in
    PMat Cps = PSpGEMM<PlusTimesSRing<double, double>>(A, B);                                  // via Synch
    PMat Cdb = Mult_AnXBn_DoubleBuff_cbg(A, B);
    PMat Csy = Mult_AnXBn_Synch_cbg(A, B);
    PMat Mref = Mult_AnXBn_Synch<RefMinPlus, double, DCCols>(A, B);
    PMat Mdrop = Mult_AnXBn_DoubleBuff<MinPlusSRing<double, double>, double, DCCols>(A, B);
    ok = (Cref == Cdrop) && (Cref == Csyn) && (Cref == Cps) && (Cref == Cdb) && (Cref == Csy) && (Mref == Mdrop);
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    if (rank == 0) std::printf("%s nnz %lld\n", ok ? "ADAPTER OK" : "ADAPTER MISMATCH", (long long)Cdrop.getnnz());
  }
  MPI_Finalize();
  return ok ? 0 : 1;
}
