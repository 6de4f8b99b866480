// ParFriends_cbg.h -- the adapter a CombBLAS maintainer adds next to
// Mult_AnXBn_DoubleBuff (include/CombBLAS/ParFriends.h:798) so that the
// reference's own drivers (MultTest, MultTiming, GalerkinNew) multiply on
// MI355X through libcbg's C ABI (include/cbg.h).  Include it after
// "CombBLAS/CombBLAS.h"; IT = int64_t or int.  INTEGRATION.md section 2;
// compiled and linked against the reference headers by
// tests/test_capi.py::test_reference_adapter_compiles (integration/adapter_check.cpp).
#pragma once
#include <map>
#include <tuple>
#include <vector>

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

}  // namespace combblas
