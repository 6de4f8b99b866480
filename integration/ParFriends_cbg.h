// ParFriends_cbg.h -- the adapter a CombBLAS maintainer adds next to
// Mult_AnXBn_DoubleBuff (include/CombBLAS/ParFriends.h:798) so that the
// reference's own drivers (MultTest, MultTiming, GalerkinNew) multiply on
// MI355X through libcbg's C ABI (include/cbg.h).  It includes
// "CombBLAS/CombBLAS.h" itself, so a driver picks up the GPU path with this one
// extra include (or `-include ParFriends_cbg.h` on its compile line) and no
// other change: the explicit specializations at the end replace the
// reference's Mult_AnXBn_DoubleBuff / Mult_AnXBn_Synch templates for the
// concrete types the ReleaseTests instantiate (PlusTimesSRing<double,double>
// and MinPlusSRing<double,double> on SpDCCols<int|int64_t, double>), and
// PSpGEMM (SpParMat.h:454-467), which calls Mult_AnXBn_Synch, follows.
// INTEGRATION.md section 2; compiled against the reference headers by
// oracle/Makefile (adapter_check.cpp, and ReleaseTests/MultTiming.cpp unmodified).
#pragma once
#include <mpi.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <map>
#include <vector>

#include "CombBLAS/CombBLAS.h"
#include "cbg.h"

namespace combblas {

// Dcsc arrays (SpDCCols::GetArrays, SpDCCols.cpp:825-851) -> device tile
template <class IT>
static cbg_tile cbg_upload(const SpDCCols<IT, double>& T) {
  std::vector<int64_t> cp;
  std::vector<int32_t> jc, ir;
  cbg_tile h{(int64_t)T.getnrow(), (int64_t)T.getncol(), (int64_t)T.getnnz(), 0,
             nullptr, nullptr, nullptr, nullptr, 0, 0};
  if (T.getnnz()) {
    Dcsc<IT, double>* d = T.GetDCSC();
    h.nzc = d->nzc;
    cp.assign(d->cp, d->cp + d->nzc + 1);
    jc.assign(d->jc, d->jc + d->nzc);
    ir.assign(d->ir, d->ir + d->nz);
    h.cp = cp.data();
    h.jc = jc.data();
    h.ir = ir.data();
    h.val = d->numx;
  } else {
    cp.assign(1, 0);
    h.cp = cp.data();
  }
  cbg_tile dev{};
  if (int rc = cbg_tile_upload(&h, &dev)) MPI_Abort(MPI_COMM_WORLD, rc);
  return dev;
}

// largest value IT may hold here: numeric_limits<IT>::max(), or the test hook
// CBG_ADAPTER_IT_MAX when that is smaller (tests force the overflow path)
template <class IT>
static int64_t cbg_index_limit() {
  int64_t lim = (int64_t)std::numeric_limits<IT>::max();
  if (const char* e = std::getenv("CBG_ADAPTER_IT_MAX")) lim = std::min<int64_t>(lim, std::atoll(e));
  return lim;
}

// device tile -> SpDCCols with no host tuples: SpDCCols(size, nRow, nCol, nzc)
// (SpDCCols.cpp:55-62) allocates the Dcsc of exactly nnz entries and nzc
// columns (Dcsc(nnz, nzcol), dcsc.cpp:44-52: cp/jc/ir/numx, dcsc.h:124-131),
// and the download writes C's arrays into it: the values straight into numx,
// the indices straight where their width is IT's (int32 ir/jc for IT = int,
// int64 cp for IT = int64_t), through one staging copy otherwise.  A C whose
// nnz or dimensions IT cannot represent aborts with a message (the tuples
// constructor's (IT)t.size() wrapped silently).
template <class IT>
static SpDCCols<IT, double>* cbg_download(const cbg_tile& C) {
  const int64_t lim = cbg_index_limit<IT>();
  if (C.nnz > lim || C.m > lim || C.n > lim) {
    std::fprintf(stderr,
                 "[cbg adapter] C of %lld x %lld with %lld nonzeros exceeds the index type's range (%lld): "
                 "use SpDCCols<int64_t, double>\n",
                 (long long)C.m, (long long)C.n, (long long)C.nnz, (long long)lim);
    MPI_Abort(MPI_COMM_WORLD, CBG_ERR_NOTSUPPORTED);
  }
  if (C.nnz == 0) return new SpDCCols<IT, double>(0, (IT)C.m, (IT)C.n, 0);
  SpDCCols<IT, double>* T = new SpDCCols<IT, double>((IT)C.nnz, (IT)C.m, (IT)C.n, (IT)C.nzc);
  Dcsc<IT, double>* d = T->GetDCSC();
  constexpr bool narrow = sizeof(IT) == sizeof(int32_t);
  std::vector<int64_t> cp64(narrow ? C.nzc + 1 : 0);
  std::vector<int32_t> jc32(narrow ? 0 : C.nzc), ir32(narrow ? 0 : C.nnz);
  cbg_tile h{0, 0, 0, 0,
             narrow ? cp64.data() : reinterpret_cast<int64_t*>(d->cp),
             narrow ? reinterpret_cast<int32_t*>(d->jc) : jc32.data(),
             narrow ? reinterpret_cast<int32_t*>(d->ir) : ir32.data(),
             d->numx, 0, 0};
  if (int rc = cbg_tile_download(&C, &h)) MPI_Abort(MPI_COMM_WORLD, rc);
  if (narrow) {
    for (int64_t i = 0; i <= C.nzc; ++i) d->cp[i] = (IT)cp64[i];
  } else {
    for (int64_t i = 0; i < C.nzc; ++i) d->jc[i] = (IT)jc32[i];
    for (int64_t p = 0; p < C.nnz; ++p) d->ir[p] = (IT)ir32[p];
  }
  return T;
}

// one RCCL grid per CommGrid, created collectively from its world communicator
static cbg_grid* cbg_grid_of(CommGrid& g) {
  static std::map<MPI_Comm, cbg_grid*> cache;
  MPI_Comm w = g.GetWorld();
  if (cache.count(w)) return cache[w];
  char id[CBG_UNIQUE_ID_BYTES] = {0};
  if (g.GetRank() == 0) cbg_get_unique_id(id);
  MPI_Bcast(id, CBG_UNIQUE_ID_BYTES, MPI_BYTE, 0, w);
  int ndev = 1;
  cbg_device_count(&ndev);
  cbg_set_device(g.GetRank() % (ndev > 0 ? ndev : 1));
  cbg_grid* h = nullptr;
  if (int rc = cbg_grid_create(g.GetRank(), g.GetSize(), g.GetGridRows(), g.GetGridCols(), id, &h))
    MPI_Abort(MPI_COMM_WORLD, rc);
  return cache[w] = h;
}

// Mult_AnXBn_DoubleBuff / _Synch on MI355X: same compliance checks and abort
// codes (ParFriends.h:160-183, SpDefs.h:69-76), the local tiles copied to HBM
// and back (a driver that keeps tiles resident uses the mirror header instead)
template <class IT>
SpParMat<IT, double, SpDCCols<IT, double>> Mult_AnXBn_cbg(SpParMat<IT, double, SpDCCols<IT, double>>& A,
                                                           SpParMat<IT, double, SpDCCols<IT, double>>& B,
                                                           int algo = CBG_DOUBLEBUFF,
                                                           int semiring = CBG_PLUS_TIMES) {
  typedef SpParMat<IT, double, SpDCCols<IT, double>> PM;
  if (!CheckSpGEMMCompliance(A, B)) return PM(A.getcommgrid());
  cbg_tile a = cbg_upload(*A.seqptr()), b = cbg_upload(*B.seqptr()), c{};
  int rc = cbg_summa_spgemm(cbg_grid_of(*A.getcommgrid()), &a, &b, A.getncol(), B.getnrow(), semiring, algo,
                            CBG_EXEC_PANEL, &c);
  if (rc) MPI_Abort(MPI_COMM_WORLD, rc);  // every rank returns the same code (cbg_grid_agree)
  SpDCCols<IT, double>* C = cbg_download<IT>(c);
  cbg_tile_free(&a);
  cbg_tile_free(&b);
  cbg_tile_free(&c);
  return PM(C, A.getcommgrid());
}

template <class IT>
SpParMat<IT, double, SpDCCols<IT, double>> Mult_AnXBn_DoubleBuff_cbg(SpParMat<IT, double, SpDCCols<IT, double>>& A,
                                                                      SpParMat<IT, double, SpDCCols<IT, double>>& B) {
  return Mult_AnXBn_cbg(A, B, CBG_DOUBLEBUFF);
}
template <class IT>
SpParMat<IT, double, SpDCCols<IT, double>> Mult_AnXBn_Synch_cbg(SpParMat<IT, double, SpDCCols<IT, double>>& A,
                                                                 SpParMat<IT, double, SpDCCols<IT, double>>& B) {
  return Mult_AnXBn_cbg(A, B, CBG_SYNCH);
}

// ---------------------------------------------------------------------------
// Drop-in: explicit specializations of the reference templates
//   template<SR, NUO, UDERO, IU, NU1, NU2, UDERA, UDERB>
//   SpParMat<IU,NUO,UDERO> Mult_AnXBn_DoubleBuff(SpParMat<IU,NU1,UDERA>&, SpParMat<IU,NU2,UDERB>&,
//                                               bool clearA, bool clearB)   ParFriends.h:798-800
//   ... Mult_AnXBn_Synch                                                    ParFriends.h:1004-1006
// for the types MultTiming.cpp:58,71,83,92 / MultTest.cpp:162,173 /
// GalerkinNew.cpp:105-152 (through PSpGEMM) instantiate.  clearA / clearB free
// the inputs' local tiles after the multiply, like the reference (:966-993).
// CBG_ADAPTER_VERBOSE=1 prints one line per call on rank 0 (tests).
// ---------------------------------------------------------------------------
template <class IT>
static SpParMat<IT, double, SpDCCols<IT, double>> cbg_dropin(SpParMat<IT, double, SpDCCols<IT, double>>& A,
                                                             SpParMat<IT, double, SpDCCols<IT, double>>& B,
                                                             bool clearA, bool clearB, int algo, int semiring,
                                                             const char* name) {
  if (std::getenv("CBG_ADAPTER_VERBOSE") && A.getcommgrid()->GetRank() == 0)
    std::fprintf(stderr, "[cbg adapter] %s on MI355X (libcbg), semiring %d\n", name, semiring);
  SpParMat<IT, double, SpDCCols<IT, double>> C = Mult_AnXBn_cbg(A, B, algo, semiring);
  if (clearA) A.FreeMemory();
  if (clearB) B.FreeMemory();
  return C;
}

#define CBG_DROPIN(FN, ALGO, SRT, SRCODE, IT)                                                                     \
  template <>                                                                                                   \
  inline SpParMat<IT, double, SpDCCols<IT, double>>                                                             \
  FN<SRT, double, SpDCCols<IT, double>, IT, double, double, SpDCCols<IT, double>, SpDCCols<IT, double>>(          \
      SpParMat<IT, double, SpDCCols<IT, double>> & A, SpParMat<IT, double, SpDCCols<IT, double>> & B, bool clearA, \
      bool clearB) {                                                                                            \
    return cbg_dropin<IT>(A, B, clearA, clearB, ALGO, SRCODE, #FN);                                            \
  }
#define CBG_DROPIN_ALL(IT)                                                                          \
  CBG_DROPIN(Mult_AnXBn_DoubleBuff, CBG_DOUBLEBUFF, PlusTimesSRing<double CBG_COMMA double>, CBG_PLUS_TIMES, IT) \
  CBG_DROPIN(Mult_AnXBn_Synch, CBG_SYNCH, PlusTimesSRing<double CBG_COMMA double>, CBG_PLUS_TIMES, IT)           \
  CBG_DROPIN(Mult_AnXBn_DoubleBuff, CBG_DOUBLEBUFF, MinPlusSRing<double CBG_COMMA double>, CBG_MIN_PLUS, IT)     \
  CBG_DROPIN(Mult_AnXBn_Synch, CBG_SYNCH, MinPlusSRing<double CBG_COMMA double>, CBG_MIN_PLUS, IT)
#define CBG_COMMA ,
CBG_DROPIN_ALL(int)
CBG_DROPIN_ALL(int64_t)
#undef CBG_DROPIN_ALL
#undef CBG_DROPIN
#undef CBG_COMMA

}  // namespace combblas
