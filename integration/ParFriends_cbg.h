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

#include <cstdio>
#include <cstdlib>
#include <map>
#include <tuple>
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

// device tile -> SpDCCols (the tuples constructor, SpDCCols.cpp:197)
template <class IT>
static SpDCCols<IT, double>* cbg_download(const cbg_tile& C) {
  std::vector<int64_t> cp(C.nzc + 1);
  std::vector<int32_t> jc(C.nzc), ir(C.nnz);
  std::vector<double> v(C.nnz);
  cbg_tile h{0, 0, 0, 0, cp.data(), jc.data(), ir.data(), v.data(), 0, 0};
  if (int rc = cbg_tile_download(&C, &h)) MPI_Abort(MPI_COMM_WORLD, rc);
  std::vector<std::tuple<IT, IT, double>> t;
  t.reserve(C.nnz);
  for (int64_t i = 0; i < C.nzc; ++i)
    for (int64_t p = cp[i]; p < cp[i + 1]; ++p) t.emplace_back((IT)ir[p], (IT)jc[i], v[p]);
  return new SpDCCols<IT, double>((IT)C.m, (IT)C.n, (IT)t.size(), t.data(), false);
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
