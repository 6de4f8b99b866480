// galerkin.cpp -- GalerkinNew (reference ReleaseTests/GalerkinNew.cpp:96-153) on the
// MI355X path, written against the C++ mirror header.  Synthetic operands: A = R-MAT
// (off-diagonal, loops removed) plus a seeded diagonal, T = restriction operator.
//   mpirun -n P ./galerkin <scale> [order]        (P a perfect square)
// or the reference's file arguments (triples files read by ReadDistribute):
//   mpirun -n P ./galerkin <Matrix> <OffDiagonal> <Diagonal> <T>
#include <mpi.h>

#include <cstdio>
#include <random>

#include "combblas_amd/CombBLAS.h"

using namespace combblas_amd;
typedef SpDCCols<int, double> DCCols;
typedef SpParMat<int, double, DCCols> PMat;
typedef PlusTimesSRing<double, double> PTDD;

int main(int argc, char* argv[]) {
  MPI_Init(&argc, &argv);
  int myrank;
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  const bool files = argc >= 5;
  const int scale = !files && argc > 1 ? std::atoi(argv[1]) : 16, order = !files && argc > 2 ? std::atoi(argv[2]) : 2;
  int rc = 0;
  {
    auto fullWorld = std::make_shared<CommGrid>(MPI_COMM_WORLD, 0, 0);
    PMat A(fullWorld), L(fullWorld), T(fullWorld), S(fullWorld), SD(fullWorld);
    std::vector<double> dvec;
    if (files) {  // GalerkinNew.cpp:92-101
      A.ReadDistribute(argv[1], 0);
      L.ReadDistribute(argv[2], 0);
      T.ReadDistribute(argv[4], 0);
      S.ReadDistribute(argv[4], 0);
      SD.ReadDistribute(argv[4], 0);
      dvec = ReadDistributeVector(argv[3]);
      if (myrank == 0) std::printf("Data read\n");
    } else {
      const int n = 1 << scale;
      dvec.resize(n);
      std::mt19937_64 rng(7);
      std::uniform_real_distribution<double> u(0.5, 1.5);
      for (auto& x : dvec) x = u(rng);
      L = PMat::rmat(fullWorld, scale, 16);
      A = PMat::rmat(fullWorld, scale, 16);
      // A = L + D: D has this rank's diagonal entries
      const int pr = fullWorld->GetGridRows(), pc = fullWorld->GetGridCols();
      const int r = fullWorld->GetRankInProcCol(), c = fullWorld->GetRankInProcRow();
      const int mper = n / pr, nper = n / pc;
      const int r0 = r * mper, r1 = r == pr - 1 ? n : r0 + mper, c0 = c * nper, c1 = c == pc - 1 ? n : c0 + nper;
      std::vector<std::tuple<int, int, double>> t;
      for (int i = std::max(r0, c0); i < std::min(r1, c1); ++i) t.emplace_back(i - r0, i - c0, dvec[i]);
      PMat D(new DCCols(r1 - r0, c1 - c0, (int)t.size(), t.data(), false), fullWorld, n, n);
      A += D;
      T = PMat::restriction(fullWorld, scale, order);
      S = PMat::restriction(fullWorld, scale, order);
      SD = PMat::restriction(fullWorld, scale, order);
    }
    S.Transpose();
    PMat AT = PSpGEMM<PTDD>(A, T);
    PMat SAT = PSpGEMM<PTDD>(S, AT);
    PMat LT = PSpGEMM<PTDD>(L, T);
    PMat SLT = PSpGEMM<PTDD>(S, LT);
    SD.Transpose();
    SD.DimApply(Column, dvec, multiplies<double>());
    PMat SDT = PSpGEMM<PTDD>(SD, T);
    SLT += SDT;
    if (SLT == SAT) {
      if (myrank == 0) std::printf("Splitting approach is correct\n");
    } else {
      if (myrank == 0) std::printf("Error in splitting, go fix it\n");
      rc = 1;
    }
    MPI_Barrier(MPI_COMM_WORLD);
    double t1 = MPI_Wtime();
    {
      PMat X = PSpGEMM<PTDD>(A, T);
      PMat Y = PSpGEMM<PTDD>(S, X);
      cbg_synchronize();
    }
    MPI_Barrier(MPI_COMM_WORLD);
    double t2 = MPI_Wtime();
    if (myrank == 0) {
      std::printf("Full restriction (without splitting) finished\n");
      std::printf("%.6lf seconds elapsed per iteration\n", t2 - t1);
    }
  }
  MPI_Finalize();
  return rc;
}
