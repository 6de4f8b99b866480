// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY (golden-vector generator).
//
// Our own driver program that links the *reference* CombBLAS sources found
// under /root/reference (built by oracle/Makefile target `ref`, output in
// oracle/_ref/, never shipped, never on the product path).  It exercises the
// reference's own code for the hot path so that tests/golden/ fixtures are
// produced by the reference itself:
//
//   gen   <scale> <ef> <out.cbgt>            DistEdgeList::GenGraph500Data
//                                            (DistEdgeList.cpp:223-280) ->
//                                            SpParMat(DEL,false) (SpParMat.cpp:3140)
//                                            -> RemoveLoops (SpParMat.cpp:3257),
//                                            exactly as GenWriteMatrix.cpp:101-114.
//   readmm <file.mtx> <out.cbgt>             ParallelReadMM (SpParMat.cpp:3980)
//   readtriples <file> <out.cbgt>            ReadDistribute (SpParMat.cpp:4211)
//   mult <algo> <sr> <A.cbgt> <B.cbgt> <out>  algo in {local, heap, doublebuff, synch}
//                                            sr in {plus, minplus}; out=".cbgt" file
//                                            or "-" for digest only
//   multphased <algo> <sr> <A> <B> <phases> [first count]  B column pieces (SpDCCols::ColSplit), one
//                                            Mult_AnXBn_<algo> per piece, C digested and freed
//   symbolic <A.cbgt> <B.cbgt>               estimateFLOP + estimateNNZ_Hash totals
//                                            (mtSpGEMM.h:1056,805)
//   digest <file.cbgt>
//
// Under mpirun -n P (P square) the tile of every rank is written to
// <out>.r<rank> (grid position in the header) and the digest is reduced.
//
// The .cbgt tile format (ours): "CBGT0001", int64 m,n,nnz,nzc,
// grid_rows, grid_cols, grid_r, grid_c, row_off, col_off, then
// int64 cp[nzc+1], int32 jc[nzc], int32 ir[nnz], double val[nnz].

#include <mpi.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <string>
#include <vector>
#include <iostream>
#include "CombBLAS/CombBLAS.h"

using namespace combblas;

typedef int64_t LIT;
typedef SpDCCols<LIT, double> DCCols;
typedef SpParMat<int64_t, double, DCCols> PMat;
typedef PlusTimesSRing<double, double> PT;
typedef MinPlusSRing<double, double> MP;

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

struct Digest {
  // nnz, nzc, structural hash (sum of mix64(col<<32|row), order-free),
  // value-weighted hash (sum of mix64(..)*bits(val)), value sum, order flag
  uint64_t nnz = 0, nzc = 0, hs = 0, hv = 0;
  double vsum = 0.0;
  uint64_t unsorted = 0;
};

// digest of one tile in GLOBAL coordinates
static Digest tile_digest(const DCCols& T, int64_t roff, int64_t coff) {
  Digest d;
  if (T.getnnz() == 0) return d;
  Dcsc<LIT, double>* dc = T.GetDCSC();
  d.nnz = dc->nz;
  d.nzc = dc->nzc;
  for (LIT i = 0; i < dc->nzc; ++i) {
    uint64_t col = (uint64_t)(dc->jc[i] + coff);
    for (LIT p = dc->cp[i]; p < dc->cp[i + 1]; ++p) {
      uint64_t row = (uint64_t)(dc->ir[p] + roff);
      uint64_t h = mix64((col << 32) | row);
      d.hs += h;
      uint64_t vb;
      double v = dc->numx[p];
      std::memcpy(&vb, &v, 8);
      d.hv += h * mix64(vb);
      d.vsum += v;
      if (p > dc->cp[i] && dc->ir[p] <= dc->ir[p - 1]) d.unsorted++;
    }
    if (i > 0 && dc->jc[i] <= dc->jc[i - 1]) d.unsorted++;
  }
  return d;
}

static void print_digest(const char* tag, const Digest& d) {
  printf("{\"tag\": \"%s\", \"nnz\": %llu, \"nzc\": %llu, \"hs\": \"%016llx\", \"hv\": \"%016llx\", \"vsum\": %.17g, \"unsorted\": %llu}\n",
         tag, (unsigned long long)d.nnz, (unsigned long long)d.nzc, (unsigned long long)d.hs,
         (unsigned long long)d.hv, d.vsum, (unsigned long long)d.unsorted);
  fflush(stdout);
}

static Digest reduce_digest(const Digest& d, MPI_Comm comm) {
  Digest r;
  uint64_t in[5] = {d.nnz, d.nzc, d.hs, d.hv, d.unsorted}, out[5];
  MPI_Allreduce(in, out, 5, MPI_UINT64_T, MPI_SUM, comm);  // wraps mod 2^64
  r.nnz = out[0]; r.nzc = out[1]; r.hs = out[2]; r.hv = out[3]; r.unsorted = out[4];
  MPI_Allreduce(&d.vsum, &r.vsum, 1, MPI_DOUBLE, MPI_SUM, comm);
  return r;
}

static void place(const PMat& M, int64_t& roff, int64_t& coff) {
  // same arithmetic as the (private) SpParMat::GetPlaceInGlobalGrid, SpParMat.cpp:5103-5116
  auto g = M.getcommgrid();
  roff = g->GetRankInProcCol() * (M.getnrow() / g->GetGridRows());
  coff = g->GetRankInProcRow() * (M.getncol() / g->GetGridCols());
}

static void write_tile(const std::string& path, const PMat& M) {
  const DCCols& T = M.seq();
  auto grid = M.getcommgrid();
  int64_t roff, coff;
  place(M, roff, coff);
  int64_t hdr[10] = {(int64_t)T.getnrow(), (int64_t)T.getncol(), (int64_t)T.getnnz(), (int64_t)T.getnzc(),
                     grid->GetGridRows(), grid->GetGridCols(), grid->GetRankInProcCol(), grid->GetRankInProcRow(),
                     roff, coff};
  std::string p = path;
  if (grid->GetSize() > 1) p += ".r" + std::to_string(grid->GetRank());
  FILE* f = fopen(p.c_str(), "wb");
  if (!f) { perror(p.c_str()); MPI_Abort(MPI_COMM_WORLD, 1); }
  fwrite("CBGT0001", 1, 8, f);
  fwrite(hdr, 8, 10, f);
  int64_t nzc = hdr[3], nnz = hdr[2];
  std::vector<int64_t> cp(nzc + 1, 0);
  std::vector<int32_t> jc(nzc), ir(nnz);
  std::vector<double> val(nnz);
  if (nnz > 0) {
    Dcsc<LIT, double>* dc = T.GetDCSC();
    for (int64_t i = 0; i <= nzc; ++i) cp[i] = dc->cp[i];
    for (int64_t i = 0; i < nzc; ++i) jc[i] = (int32_t)dc->jc[i];
    for (int64_t i = 0; i < nnz; ++i) { ir[i] = (int32_t)dc->ir[i]; val[i] = dc->numx[i]; }
  }
  fwrite(cp.data(), 8, nzc + 1, f);
  fwrite(jc.data(), 4, nzc, f);
  fwrite(ir.data(), 4, nnz, f);
  fwrite(val.data(), 8, nnz, f);
  fclose(f);
}

// Read a GLOBAL matrix stored as a single .cbgt (1x1 tile) and distribute its
// tuples to the current grid via the block distribution of SpParMat::Owner.
static PMat* read_global_tile(const std::string& path, std::shared_ptr<CommGrid> grid) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) { perror(path.c_str()); MPI_Abort(MPI_COMM_WORLD, 1); }
  char magic[8];
  int64_t hdr[10];
  if (fread(magic, 1, 8, f) != 8 || fread(hdr, 8, 10, f) != 10) MPI_Abort(MPI_COMM_WORLD, 2);
  int64_t m = hdr[0], n = hdr[1], nnz = hdr[2], nzc = hdr[3];
  std::vector<int64_t> cp(nzc + 1);
  std::vector<int32_t> jc(nzc), ir(nnz);
  std::vector<double> val(nnz);
  size_t ok = fread(cp.data(), 8, nzc + 1, f);
  ok += fread(jc.data(), 4, nzc, f);
  ok += fread(ir.data(), 4, nnz, f);
  ok += fread(val.data(), 8, nnz, f);
  (void)ok;
  fclose(f);
  int pr = grid->GetGridRows(), pc = grid->GetGridCols();
  int myr = grid->GetRankInProcCol(), myc = grid->GetRankInProcRow();
  int64_t mper = m / pr, nper = n / pc;
  int64_t lm = (myr == pr - 1) ? m - myr * mper : mper;
  int64_t ln = (myc == pc - 1) ? n - myc * nper : nper;
  std::vector<std::tuple<LIT, LIT, double>> tup;
  for (int64_t i = 0; i < nzc; ++i) {
    int64_t col = jc[i];
    int oc = (nper != 0) ? std::min((int)(col / nper), pc - 1) : pc - 1;
    if (oc != myc) continue;
    for (int64_t p = cp[i]; p < cp[i + 1]; ++p) {
      int64_t row = ir[p];
      int orow = (mper != 0) ? std::min((int)(row / mper), pr - 1) : pr - 1;
      if (orow != myr) continue;
      tup.emplace_back(row - orow * mper, col - oc * nper, val[p]);
    }
  }
  // already column-sorted, rows ascending
  DCCols* T = new DCCols((LIT)lm, (LIT)ln, (LIT)tup.size(), tup.data(), false);
  return new PMat(T, grid);
}

template <class SR>
static PMat run_mult(const std::string& algo, PMat& A, PMat& B) {
  if (algo == "doublebuff") return Mult_AnXBn_DoubleBuff<SR, double, DCCols>(A, B);
  if (algo == "synch") return Mult_AnXBn_Synch<SR, double, DCCols>(A, B);
  // local kernels: 1x1 grid only
  const DCCols& Aseq = A.seq();
  const DCCols& Bseq = B.seq();
  SpTuples<LIT, double>* t;
  if (algo == "heap")
    t = LocalSpGEMM<SR, double>(Aseq, Bseq, false, false);
  else
    t = LocalHybridSpGEMM<SR, double>(Aseq, Bseq, false, false);
  DCCols* C = new DCCols(*t, false);
  delete t;
  return PMat(C, A.getcommgrid());
}

int main(int argc, char* argv[]) {
  MPI_Init(&argc, &argv);
  int rank, nprocs;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
  if (argc < 2) {
    if (rank == 0) fprintf(stderr, "usage: see header of ref_driver.cpp\n");
    MPI_Finalize();
    return 1;
  }
  {  // scope: every CombBLAS object dies before MPI_Finalize
  std::string cmd = argv[1];
  auto grid = std::make_shared<CommGrid>(MPI_COMM_WORLD, 0, 0);
  if (cmd == "gen") {
    unsigned scale = atoi(argv[2]), ef = atoi(argv[3]);
    double initiator[4] = {.57, .19, .19, .05};
    DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>();
    DEL->GenGraph500Data(initiator, scale, ef, true, true);
    PMat G(*DEL, false);
    delete DEL;
    int64_t removed = G.RemoveLoops();
    if (rank == 0) printf("{\"tag\": \"gen_loops_removed\", \"value\": %lld}\n", (long long)removed);
    write_tile(argv[4], G);
    int64_t ro, co;
    place(G, ro, co);
    Digest d = reduce_digest(tile_digest(G.seq(), ro, co), MPI_COMM_WORLD);
    if (rank == 0) print_digest("A", d);
  } else if (cmd == "readmm" || cmd == "readtriples") {
    PMat A(grid);
    if (cmd == "readmm")
      A.ParallelReadMM(argv[2], true, maximum<double>());
    else
      A.ReadDistribute(argv[2], 0);
    write_tile(argv[3], A);
    int64_t ro, co;
    place(A, ro, co);
    Digest d = reduce_digest(tile_digest(A.seq(), ro, co), MPI_COMM_WORLD);
    if (rank == 0) print_digest("A", d);
  } else if (cmd == "mult") {
    std::string algo = argv[2], sr = argv[3];
    PMat* A = read_global_tile(argv[4], grid);
    PMat* B = read_global_tile(argv[5], grid);
    double t0 = MPI_Wtime();
    PMat C = (sr == "minplus") ? run_mult<MP>(algo, *A, *B) : run_mult<PT>(algo, *A, *B);
    double t1 = MPI_Wtime();
    int64_t ro, co;
    place(C, ro, co);
    Digest d = reduce_digest(tile_digest(C.seq(), ro, co), MPI_COMM_WORLD);
    if (rank == 0) {
      print_digest(("C_" + algo + "_" + sr).c_str(), d);
      printf("{\"tag\": \"time_%s\", \"seconds\": %.6f, \"nprocs\": %d}\n", algo.c_str(), t1 - t0, nprocs);
    }
    if (std::string(argv[6]) != "-") write_tile(argv[6], C);
  } else if (cmd == "multphased") {
    // multphased <algo> <sr> <A.cbgt> <B.cbgt> <phases>  (1x1 grid): B cut into column
    // pieces by the reference's SpDCCols::ColSplit, as MemEfficientSpGEMM does
    // (ParFriends.h:552-553), each piece multiplied with Mult_AnXBn_<algo> and its C
    // digested and freed before the next (C larger than host memory).  Prints the
    // summed digest and the summed multiply time (the CPU baseline at scale 22).
    // optional [first count]: only phases first .. first+count-1 (one process per
    // phase keeps the host's memory bounded: the reference's heap grows across calls)
    std::string algo = argv[2], sr = argv[3];
    const int phases = atoi(argv[6]);
    const int first = argc > 7 ? atoi(argv[7]) : 0;
    const int count = argc > 8 ? atoi(argv[8]) : phases;
    if (nprocs != 1) { fprintf(stderr, "multphased: 1x1 only\n"); MPI_Abort(MPI_COMM_WORLD, 1); }
    PMat* A = read_global_tile(argv[4], grid);
    PMat* B = read_global_tile(argv[5], grid);
    const int64_t n = B->getncol();
    DCCols copyB = B->seq();
    delete B;
    std::vector<DCCols> pieces;
    copyB.ColSplit(phases, pieces);
    Digest tot;
    double secs = 0;
    for (int p = 0; p < (int)pieces.size(); ++p) {
      if (p < first || p >= first + count) {
        pieces[p] = DCCols();
        continue;
      }
      PMat Bp(new DCCols(pieces[p]), grid);
      pieces[p] = DCCols();
      double t0 = MPI_Wtime();
      PMat C = (sr == "minplus") ? run_mult<MP>(algo, *A, Bp) : run_mult<PT>(algo, *A, Bp);
      secs += MPI_Wtime() - t0;
      Digest d = tile_digest(C.seq(), 0, (int64_t)p * (n / phases));
      tot.nnz += d.nnz; tot.nzc += d.nzc; tot.hs += d.hs; tot.hv += d.hv; tot.vsum += d.vsum;
      tot.unsorted += d.unsorted;
      printf("{\"tag\": \"phase\", \"phase\": %d, \"nnz\": %llu, \"seconds\": %.3f}\n", p,
             (unsigned long long)d.nnz, secs);
      fflush(stdout);
    }
    print_digest(("C_" + algo + "_" + sr).c_str(), tot);
    printf("{\"tag\": \"time_%s\", \"seconds\": %.6f, \"nprocs\": %d, \"phases\": %d}\n", algo.c_str(), secs,
           nprocs, phases);
  } else if (cmd == "symbolic") {
    PMat* A = read_global_tile(argv[2], grid);
    PMat* B = read_global_tile(argv[3], grid);
    const DCCols& Aseq = A->seq();
    const DCCols& Bseq = B->seq();
    double t0 = MPI_Wtime();
    LIT* flop = estimateFLOP(Aseq, Bseq);
    LIT* cnt = estimateNNZ_Hash(Aseq, Bseq, flop);
    double t1 = MPI_Wtime();
    int64_t F = 0, N = 0, mx = 0;
    for (LIT i = 0; i < Bseq.getnzc(); ++i) { F += flop[i]; N += cnt[i]; mx = std::max<int64_t>(mx, cnt[i]); }
    printf("{\"tag\": \"symbolic\", \"flops\": %lld, \"nnzC\": %lld, \"maxcol\": %lld, \"seconds\": %.3f}\n",
           (long long)F, (long long)N, (long long)mx, t1 - t0);
    delete[] flop;
    delete[] cnt;
  } else {
    if (rank == 0) fprintf(stderr, "unknown command %s\n", cmd.c_str());
  }
  }
  MPI_Finalize();
  return 0;
}
