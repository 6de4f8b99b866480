// multtiming.cpp -- MultTiming (reference ReleaseTests/MultTiming.cpp) on the
// MI355X path, written against the C++ mirror header combblas_amd/CombBLAS.h.
//
//   mpirun -n P ./multtiming A.triples B.triples      (triples file: "m n nnz" then 1-based i j v)
//   mpirun -n P ./multtiming --rmat <scale> [ef]      (Graph500 R-MAT A, B = copy of A)
//
// One MPI rank per GPU; P must be a perfect square (CommGrid(world,0,0)).
// Prints the same lines as the reference driver.
#include <mpi.h>

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

#include "combblas_amd/CombBLAS.h"

using namespace combblas_amd;
typedef SpDCCols<int, double> DCCols;
typedef SpParMat<int, double, DCCols> PMat;
typedef PlusTimesSRing<double, double> PTDOUBLEDOUBLE;
#define ITERATIONS 1

// rank-local block of a triples file (block distribution of SpParMat::Owner)
static PMat read_triples(const std::string& path, std::shared_ptr<CommGrid> g) {
  std::ifstream in(path);
  if (!in) {
    std::fprintf(stderr, "cannot open %s\n", path.c_str());
    MPI_Abort(MPI_COMM_WORLD, 3004);  // NOFILE
  }
  std::string line;
  long long m = 0, n = 0, nnz = 0;
  while (std::getline(in, line)) {
    if (line.empty() || line[0] == '%') continue;
    std::istringstream ss(line);
    ss >> m >> n >> nnz;
    break;
  }
  const int pr = g->GetGridRows(), pc = g->GetGridCols(), r = g->GetRankInProcCol(), c = g->GetRankInProcRow();
  const long long mper = m / pr, nper = n / pc;
  const long long r0 = r * mper, r1 = (r == pr - 1) ? m : r0 + mper;
  const long long c0 = c * nper, c1 = (c == pc - 1) ? n : c0 + nper;
  std::vector<std::tuple<int, int, double>> t;
  long long i, j;
  double v;
  while (in >> i >> j >> v) {
    --i;
    --j;
    if (i >= r0 && i < r1 && j >= c0 && j < c1) t.emplace_back((int)(i - r0), (int)(j - c0), v);
  }
  std::sort(t.begin(), t.end(), [](const std::tuple<int, int, double>& a, const std::tuple<int, int, double>& b) {
    return std::get<1>(a) != std::get<1>(b) ? std::get<1>(a) < std::get<1>(b) : std::get<0>(a) < std::get<0>(b);
  });
  return PMat(new DCCols((int)(r1 - r0), (int)(c1 - c0), (int)t.size(), t.data(), false), g, (int)m, (int)n);
}

int main(int argc, char* argv[]) {
  MPI_Init(&argc, &argv);
  int myrank;
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  if (argc < 3) {
    if (myrank == 0) std::printf("Usage: ./multtiming <MatrixA> <MatrixB> | --rmat <scale> [ef]\n");
    MPI_Finalize();
    return -1;
  }
  {
    auto grid = std::make_shared<CommGrid>(MPI_COMM_WORLD, 0, 0);
    std::string a1 = argv[1];
    PMat A, B;
    if (a1 == "--rmat") {
      const int scale = std::atoi(argv[2]), ef = argc > 3 ? std::atoi(argv[3]) : 16;
      A = PMat::rmat(grid, scale, ef);
      B = PMat::rmat(grid, scale, ef);
    } else {
      A = read_triples(argv[1], grid);
      B = read_triples(argv[2], grid);
    }
    {
      PMat C = Mult_AnXBn_DoubleBuff<PTDOUBLEDOUBLE, double, DCCols>(A, B);
      const int64_t cnnz = C.getnnz();
      if (myrank == 0) std::printf("C has a total of %lld nonzeros\nWarmed up for DoubleBuff\n", (long long)cnnz);
    }
    MPI_Barrier(MPI_COMM_WORLD);
    double t1 = MPI_Wtime();
    for (int i = 0; i < ITERATIONS; i++) {
      PMat C = Mult_AnXBn_DoubleBuff<PTDOUBLEDOUBLE, double, DCCols>(A, B);
      cbg_synchronize();
    }
    MPI_Barrier(MPI_COMM_WORLD);
    double t2 = MPI_Wtime();
    if (myrank == 0) {
      std::printf("Double buffered multiplications finished\n");
      std::printf("%.6lf seconds elapsed per iteration\n", (t2 - t1) / (double)ITERATIONS);
    }
    {
      PMat C = Mult_AnXBn_Synch<PTDOUBLEDOUBLE, double, DCCols>(A, B);
    }
    MPI_Barrier(MPI_COMM_WORLD);
    t1 = MPI_Wtime();
    for (int i = 0; i < ITERATIONS; i++) {
      PMat C = Mult_AnXBn_Synch<PTDOUBLEDOUBLE, double, DCCols>(A, B);
      cbg_synchronize();
    }
    MPI_Barrier(MPI_COMM_WORLD);
    t2 = MPI_Wtime();
    if (myrank == 0) {
      std::printf("Synchronous multiplications finished\n");
      std::printf("%.6lf seconds elapsed per iteration\n", (t2 - t1) / (double)ITERATIONS);
    }
    {
      // MemEfficientSpGEMM with 4 phases (ParFriends.h:449) must equal the
      // unphased product (SpParMat::operator==, SpParMat.cpp:2878)
      PMat C = Mult_AnXBn_Synch<PTDOUBLEDOUBLE, double, DCCols>(A, B);
      PMat Cp = MemEfficientSpGEMM<PTDOUBLEDOUBLE, double, DCCols>(A, B, 4, 0.0, 0, 0, 0.0, 1, 1, 0);
      const bool same = (C == Cp);
      if (myrank == 0) std::printf("MemEfficientSpGEMM (4 phases) %s the unphased product\n", same ? "equals" : "DIFFERS from");
    }
  }
  MPI_Finalize();
  return 0;
}
