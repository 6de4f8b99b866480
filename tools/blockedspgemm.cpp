// blockedspgemm.cpp -- ReleaseTests/BlockedSpGEMM.cpp (BlockSpGEMM over ParallelReadMM
// inputs) on the MI355X path, written against the C++ mirror header combblas_amd/CombBLAS.h.
//
//   mpirun -n P ./blockedspgemm <MatrixA.mtx> <MatrixB.mtx> <br> <bc>
//
// Prints the reference's lines ("A m n nnz", "B m n nnz", then per block "block size
// m n nnz offsets r c"), and, beyond the reference, checks that the block nonzeros add
// up to nnz(Mult_AnXBn_Synch(A, B)) ("BlockSpGEMM blocks cover A*B").
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#include "combblas_amd/CombBLAS.h"

using namespace combblas_amd;
typedef int64_t IT;
typedef double NT;
typedef SpDCCols<IT, NT> DER;
typedef SpParMat<IT, NT, DER> PMat;
typedef PlusTimesSRing<NT, NT> SR_PT;

int main(int argc, char* argv[]) {
  MPI_Init(&argc, &argv);
  int myrank;
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  if (argc < 5) {
    if (myrank == 0) std::printf("Usage: ./BlockedSpGEMM <MatrixA> <MatrixB> <br> <bc>\n");
    MPI_Finalize();
    return -1;
  }
  int rc = 0;
  {
    const int br = std::atoi(argv[3]), bc = std::atoi(argv[4]);
    auto fullWorld = std::make_shared<CommGrid>(MPI_COMM_WORLD, 0, 0);
    PMat A(fullWorld), B(fullWorld);
    A.ParallelReadMM(argv[1], true, maximum<NT>());
    long long nnz = A.getnnz();
    if (myrank == 0) std::printf("A %lld %lld %lld\n", (long long)A.getnrow(), (long long)A.getncol(), nnz);
    B.ParallelReadMM(argv[2], true, maximum<NT>());
    nnz = B.getnnz();
    if (myrank == 0) std::printf("B %lld %lld %lld\n", (long long)B.getnrow(), (long long)B.getncol(), nnz);
    BlockSpGEMM<IT, NT, DER, NT, DER> bspgemm(A, B, br, bc);
    IT roffset, coffset;
    long long total = 0;
    while (bspgemm.hasNext()) {
      auto C = bspgemm.getNextBlock<SR_PT, NT, DER>(roffset, coffset);
      nnz = C.getnnz();
      total += nnz;
      if (myrank == 0)
        std::printf("block size %lld %lld %lld offsets %lld %lld\n", (long long)C.getnrow(), (long long)C.getncol(),
                    nnz, (long long)roffset, (long long)coffset);
    }
    PMat Cfull = Mult_AnXBn_Synch<SR_PT, NT, DER>(A, B);
    const long long want = Cfull.getnnz();
    rc = total == want ? 0 : 1;
    if (myrank == 0)
      std::printf(rc == 0 ? "BlockSpGEMM blocks cover A*B (%lld nonzeros)\n" : "ERROR: blocks hold %lld nonzeros\n",
                  total);
  }
  MPI_Finalize();
  return rc;
}
