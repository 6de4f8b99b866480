// multtest.cpp -- the SpGEMM part of MultTest (reference ReleaseTests/MultTest.cpp:95-180)
// on the MI355X path, written against the C++ mirror header combblas_amd/CombBLAS.h.
//
//   mpirun -n P ./multtest <MatrixA.mtx> <MatrixB.mtx> <MatrixC.mtx>
//
// Reads A, B and the control product with ParallelReadMM (onebased, maximum<double>),
// multiplies with Mult_AnXBn_Synch and Mult_AnXBn_DoubleBuff (and MemEfficientSpGEMM
// with 2 phases) and compares with operator==, printing the reference's messages.
// The SpMV / SpMSpV checks of MultTest are not on the SpGEMM path.
#include <mpi.h>

#include <cstdio>
#include <string>

#include "combblas_amd/CombBLAS.h"

using namespace combblas_amd;
typedef SpDCCols<int, double> DCCols;
typedef SpParMat<int, double, DCCols> PMat;
typedef PlusTimesSRing<double, double> PTDOUBLEDOUBLE;

int main(int argc, char* argv[]) {
  MPI_Init(&argc, &argv);
  int myrank;
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  if (argc < 4) {
    if (myrank == 0) std::printf("Usage: ./multtest <MatrixA> <MatrixB> <MatrixC>\n");
    MPI_Finalize();
    return -1;
  }
  int failures = 0;
  {
    auto fullWorld = std::make_shared<CommGrid>(MPI_COMM_WORLD, 0, 0);
    PMat A(fullWorld), B(fullWorld), CControl(fullWorld);
    A.ParallelReadMM(argv[1], true, maximum<double>());
    B.ParallelReadMM(argv[2], true, maximum<double>());
    CControl.ParallelReadMM(argv[3], true, maximum<double>());
    auto report = [&](bool ok, const char* good, const char* bad) {
      if (myrank == 0) std::printf("%s\n", ok ? good : bad);
      failures += ok ? 0 : 1;
    };
    {
      PMat C = Mult_AnXBn_Synch<PTDOUBLEDOUBLE, double, DCCols>(A, B);
      report(CControl == C, "Synchronous Multiplication working correctly",
             "ERROR in Synchronous Multiplication, go fix it!");
    }
    {
      PMat C = Mult_AnXBn_DoubleBuff<PTDOUBLEDOUBLE, double, DCCols>(A, B);
      report(CControl == C, "Double buffered multiplication working correctly",
             "ERROR in double buffered multiplication, go fix it!");
    }
    {
      PMat C = MemEfficientSpGEMM<PTDOUBLEDOUBLE, double, DCCols>(A, B, 2, 0.0, 0, 0, 0.0, 1, 1, 0);
      report(CControl == C, "Phased (MemEfficientSpGEMM) multiplication working correctly",
             "ERROR in phased multiplication, go fix it!");
    }
  }
  MPI_Finalize();
  return failures;
}
