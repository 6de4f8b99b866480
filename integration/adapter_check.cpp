// adapter_check.cpp -- compile/link check of integration/ParFriends_cbg.h against
// the reference's headers (TEST INFRASTRUCTURE: built only where /root/reference
// exists, by tests/test_capi.py).  Run as `adapter_check A.mtx` on a GPU box it
// multiplies A*A with the reference's Mult_AnXBn_Synch and with the adapter and
// compares them with the reference's SpParMat::operator==.
#include <mpi.h>
#include <cstdio>
#include "CombBLAS/CombBLAS.h"
#include "ParFriends_cbg.h"

using namespace combblas;
typedef SpDCCols<int64_t, double> DCCols;
typedef SpParMat<int64_t, double, DCCols> PMat;

int main(int argc, char* argv[]) {
  MPI_Init(&argc, &argv);
  int ok = 1;
  if (argc > 1) {
    auto grid = std::make_shared<CommGrid>(MPI_COMM_WORLD, 0, 0);
    PMat A(grid), B(grid);
    A.ParallelReadMM(argv[1], true, maximum<double>());
    B.ParallelReadMM(argv[1], true, maximum<double>());
    PMat Cref = Mult_AnXBn_Synch<PlusTimesSRing<double, double>, double, DCCols>(A, B);
    PMat Cdb = Mult_AnXBn_DoubleBuff_cbg(A, B);
    PMat Csy = Mult_AnXBn_Synch_cbg(A, B);
    ok = (Cref == Cdb) && (Cref == Csy);
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    if (rank == 0) std::printf("%s nnz %lld\n", ok ? "ADAPTER OK" : "ADAPTER MISMATCH", (long long)Cdb.getnnz());
  }
  MPI_Finalize();
  return ok ? 0 : 1;
}
