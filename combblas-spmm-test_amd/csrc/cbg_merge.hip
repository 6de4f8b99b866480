// cbg_merge.hip -- on-device multiway merge of column-sorted partial products.
//
// Replaces MergeAll (serial heap merge, reference Friends.h:657-741) used by
// Mult_AnXBn_DoubleBuff and MultiwayMerge (MultiwayMerge.h:409-526) used by
// Mult_AnXBn_Synch.  Both sum entries with equal (row, col) with SR::add and
// keep the (col, row) order.
//
// MI355X formulation: merging P partial tiles P_1..P_P (all m x n) is the
// product  [P_1 | P_2 | ... | P_P] * [I; I; ...; I]  with the stacked identity
// carrying the semiring's multiplicative unit (1.0 for plus-times, 0.0 for
// min-plus, both exact).  The merge therefore runs on the same LDS-hash /
// dense-slab kernels as the local multiply (cbg_local.hip): per output column
// the P sorted runs are accumulated in LDS and emitted row-sorted, instead of
// a heap that pops one tuple at a time.
#include "cbg_device.h"
#include "cbg_internal.h"

namespace cbg {

__global__ void k_identity_stack(int64_t n, int P, double unit, int64_t* __restrict__ cp, int32_t* __restrict__ jc,
                                 int32_t* __restrict__ ir, double* __restrict__ val) {
  int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j > n) return;
  cp[j] = j * P;
  if (j == n) return;
  jc[j] = (int32_t)j;
  for (int k = 0; k < P; ++k) {
    ir[j * P + k] = (int32_t)(k * n + j);
    val[j * P + k] = unit;
  }
}

void merge_tiles(const std::vector<cbg_tile>& parts, int64_t m, int64_t n, int semiring, cbg_tile& C, hipStream_t s) {
  std::vector<cbg_tile> live;
  for (auto& p : parts)
    if (p.nnz > 0) live.push_back(p);
  if (live.empty()) {
    tile_alloc_device(C, m, n, 0, 0);
    return;
  }
  const int P = (int)live.size();
  int64_t tot = 0;
  for (auto& p : live) tot += p.nnz;
  if (tot >= (int64_t)INT32_MAX || (int64_t)P * n >= (int64_t)INT32_MAX)
    throw HipError("merge: partial products exceed 2^31 entries; use CBG_EXEC_PANEL", CBG_ERR_NOTSUPPORTED);
  std::vector<int64_t> off(P);
  for (int k = 0; k < P; ++k) off[k] = (int64_t)k * n;
  cbg_tile Acat{}, Id{};
  tile_concat_cols(live, off, m, (int64_t)P * n, Acat, s);
  tile_alloc_device(Id, (int64_t)P * n, n, (int64_t)P * n, n);
  hipLaunchKernelGGL(k_identity_stack, dim3((unsigned)((n + 256) / 256)), dim3(256), 0, s, n, P,
                     semiring == CBG_MIN_PLUS ? 0.0 : 1.0, Id.cp, Id.jc, Id.ir, Id.val);
  try {
    local_spgemm(Acat, Id, semiring, C, s, nullptr);
  } catch (...) {
    tile_free_device(Acat);
    tile_free_device(Id);
    throw;
  }
  tile_free_device(Acat);
  tile_free_device(Id);
}

}  // namespace cbg
