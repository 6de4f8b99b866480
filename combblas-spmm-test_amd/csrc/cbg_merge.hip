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

MergeStats& merge_stats() {
  static thread_local MergeStats m;
  return m;
}

// entries a merge product may stack (A operand of the local multiply: int32
// offsets in its column maps); CBG_MERGE_CHUNK lowers it (tests of the
// chunked path at small sizes)
static int64_t merge_chunk_entries() {
  static const char* e = getenv("CBG_MERGE_CHUNK");
  const int64_t v = e ? atoll(e) : (int64_t)1 << 30;
  return std::max<int64_t>(v, 1);
}

// one product [P_1 | ... | P_k] * [I; ...; I] over the columns of the parts
static void merge_product(const std::vector<cbg_tile>& live, int64_t m, int64_t n, int semiring, cbg_tile& C,
                          hipStream_t s, OutSink* sink) {
  const int P = (int)live.size();
  std::vector<int64_t> off(P);
  for (int k = 0; k < P; ++k) off[k] = (int64_t)k * n;
  TileGuard Acat, Id;
  tile_concat_cols(live, off, m, (int64_t)P * n, Acat.t, s);
  tile_alloc_device(Id.t, (int64_t)P * n, n, (int64_t)P * n, n);
  hipLaunchKernelGGL(k_identity_stack, dim3((unsigned)((n + 256) / 256)), dim3(256), 0, s, n, P,
                     semiring == CBG_MIN_PLUS ? 0.0 : 1.0, Id.t.cp, Id.t.jc, Id.t.ir, Id.t.val);
  // a merge is not SpGEMM work: keep it out of the multiply statistics
  const LocalStats saved = thread_stats();
  LocalStats mine;
  try {
    local_spgemm(Acat.t, Id.t, semiring, C, s, &mine, sink);
  } catch (...) {
    thread_stats() = saved;
    throw;
  }
  thread_stats() = saved;
  MergeStats& ms = merge_stats();
  ms.entries_in += Acat.t.nnz;
  ms.entries_out += mine.nnz;
  ms.ms += mine.ms_symbolic + mine.ms_numeric;
}

void merge_tiles(const std::vector<cbg_tile>& parts, int64_t m, int64_t n, int semiring, cbg_tile& C, hipStream_t s) {
  std::vector<cbg_tile> live;
  for (auto& p : parts)
    if (p.nnz > 0) live.push_back(p);
  if (live.empty()) {
    tile_alloc_device(C, m, n, 0, 0);
    return;
  }
  const int64_t P = (int64_t)live.size();
  int64_t tot = 0;
  for (auto& p : live) tot += p.nnz;
  const int64_t lim = merge_chunk_entries();
  const int64_t lim_cols = ((int64_t)1 << 30) / P;  // stacked identity: P * cols rows < 2^31
  if (tot <= lim && n <= lim_cols) {
    merge_product(live, m, n, semiring, C, s, nullptr);
    return;
  }
  // column chunks with at most `lim` stacked entries each (a chunk still over
  // the limit is halved again), merged one after another into one arena:
  // the merged tile is their column concatenation without a copy
  int64_t K = std::max<int64_t>((tot + lim - 1) / lim, (n + lim_cols - 1) / lim_cols);
  K = std::min<int64_t>(K, n);
  std::vector<std::pair<int64_t, int64_t>> todo;  // column ranges, processed from the back
  for (int64_t k = K - 1; k >= 0; --k) todo.emplace_back(k * n / K, (k + 1) * n / K);
  EntryArena arena;
  std::vector<TileGuard> out;
  std::vector<cbg_tile> outv;
  std::vector<int64_t> offs;
  while (!todo.empty()) {
    const auto r = todo.back();
    todo.pop_back();
    if (r.second <= r.first) continue;
    std::vector<TileGuard> sl;
    std::vector<cbg_tile> slv;
    int64_t sub = 0;
    for (auto& p : live) {
      TileGuard g;
      tile_slice_cols(p, r.first, r.second, g.t, s);
      sub += g.t.nnz;
      if (g.t.nnz > 0) {
        slv.push_back(g.t);
        sl.push_back(std::move(g));
      }
    }
    if (sub > lim && r.second - r.first > 1) {
      const int64_t mid = r.first + (r.second - r.first) / 2;
      todo.emplace_back(mid, r.second);
      todo.emplace_back(r.first, mid);
      continue;
    }
    if (sub >= (int64_t)INT32_MAX)
      throw HipError("merge: one output column holds 2^31 or more partial entries", CBG_ERR_NOTSUPPORTED);
    TileGuard Cc;
    if (slv.empty()) {
      tile_alloc_device(Cc.t, m, r.second - r.first, 0, 0);
    } else {
      merge_product(slv, m, r.second - r.first, semiring, Cc.t, s, &arena);
    }
    outv.push_back(Cc.t);
    offs.push_back(r.first);
    out.push_back(std::move(Cc));
  }
  // chunks with no entries own their (empty) arrays; the others point into the arena
  tile_assemble_cols(outv, offs, m, n, arena, C, s);
}

}  // namespace cbg
