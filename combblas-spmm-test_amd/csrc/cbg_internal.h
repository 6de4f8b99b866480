// cbg_internal.h -- host-side internals of the MI355X SpGEMM library (libcbg).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/cbg.h"

namespace cbg {

struct HipError : std::runtime_error {
  int code;
  HipError(const std::string& s, int c) : std::runtime_error(s), code(c) {}
};

#define CBG_HIP(x)                                                                                  \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess)                                                                           \
      throw ::cbg::HipError(std::string(#x) + ": " + hipGetErrorString(e_) + " @" + __FILE__ + ":" + \
                                std::to_string(__LINE__),                                           \
                            CBG_ERR_HIP);                                                           \
  } while (0)

// Caching device allocator: blocks are rounded up (>= 2 MiB granules for big
// requests) and recycled by size so that repeated multiplies never touch
// hipMalloc/hipFree in steady state (cdna_hip_programming.md Guideline 9).
//
// Growable arrays (reserve_growable/grow) are a reserved virtual range whose
// physical pages are mapped on demand (hipMemAddressReserve + hipMemCreate +
// hipMemMap): a C tile assembled from several multiplies (pipeline pieces,
// merge chunks) is written in place, with no concatenation copy, and holds
// only the memory it uses.  A freed growable block stays mapped in the cache
// (like the hipMalloc blocks) and is handed out again, so steady-state calls
// map nothing; trim() (also run before an allocation is retried on OOM)
// unmaps and releases them.
class DevicePool {
 public:
  void* alloc(size_t bytes);
  void free(void* p);
  void trim();  // release every cached block
  bool release_largest_cached();  // hipFree the largest cached (non-growable) block; false if none
  void* reserve_growable(size_t max_bytes);
  void grow(void* base, size_t bytes);  // map [base, base + bytes)
  size_t bytes_in_use() const { return in_use_; }
  // allocation serial of the live block that contains p (a block handed out
  // again gets a new one); 0 if p is not in a live pool block
  uint64_t serial_of(const void* p);
  size_t bytes_cached() const { return cached_; }
  // Debug mode (CBG_POOL_QUARANTINE=1, read once): a freed block is poisoned at
  // once on a stream of its own (0xff bytes: row ids -1, values NaN), racing any
  // kernel that may still use it, and is not handed out again before
  // quarantine_release() (a device synchronization; every local multiply's end),
  // so a buffer released while a kernel can still read it shows up as a wrong
  // result, not as a rare race with the block's next owner.
  bool quarantine() const { return quarantine_; }
  void quarantine_release();
  DevicePool();
  ~DevicePool() { trim(); }

 private:
  struct Growable {
    size_t reserved = 0, mapped = 0;
    std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> chunks;
  };
  void release_growable(void* base, Growable& g);
  std::mutex mu_;
  std::multimap<size_t, void*> free_;
  std::map<void*, size_t> live_;
  std::map<void*, Growable> grow_;        // growable blocks in use
  std::map<void*, Growable> grow_cache_;  // freed growable blocks, still mapped, reused first
  std::map<void*, uint64_t> serial_;      // live blocks (regular and growable) -> allocation serial
  uint64_t next_serial_ = 0;
  size_t in_use_ = 0, cached_ = 0;
  bool quarantine_ = false;
  std::vector<std::pair<void*, size_t>> quar_;  // freed, poisoned, not yet reusable
  hipStream_t poison_ = nullptr;
};
DevicePool& pool();

// cbg_tile.reserved bit: ir/val point into memory the tile does not own (an
// EntryArena's ranges); tile_free_device then frees only cp and jc
constexpr int32_t TILE_BORROWED_ENTRIES = 1;

// where a local multiply puts C's row ids and values (default: fresh pool blocks)
struct OutSink {
  virtual void place(int64_t nnz, int32_t** ir, double** val) = 0;
  virtual ~OutSink() = default;
};
// C entries of consecutive multiplies laid end to end in two growable arrays
struct EntryArena : OutSink {
  int32_t* ir = nullptr;
  double* val = nullptr;
  int64_t used = 0;
  EntryArena();
  ~EntryArena() override;
  void place(int64_t nnz, int32_t** pir, double** pval) override;
  void detach() { ir = nullptr; val = nullptr; used = 0; }
  EntryArena(const EntryArena&) = delete;
  EntryArena& operator=(const EntryArena&) = delete;
};

// RAII device buffer from the pool
template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  DBuf() = default;
  explicit DBuf(size_t count) { reset(count); }
  void reset(size_t count) {
    release();
    n = count;
    if (count) p = static_cast<T*>(pool().alloc(count * sizeof(T)));
  }
  void release() {
    if (p) pool().free(p);
    p = nullptr;
    n = 0;
  }
  T* detach() {
    T* q = p;
    p = nullptr;
    n = 0;
    return q;
  }
  ~DBuf() { release(); }
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
};

// pool blocks whose release waits until the owner's streams are joined and
// synchronized (buffers of kernels running on a side stream)
struct DeferredFree {
  std::vector<void*> ptrs;
  bool synced = false;  // set by the owner after its streams are synchronized
  template <class T>
  void take(DBuf<T>& b) {
    if (b.p) ptrs.push_back(b.detach());
  }
  ~DeferredFree() {
    // an error path leaves without the owner's final sync: kernels may still
    // use the buffers, so wait before they can be handed out again
    if (!synced && !ptrs.empty()) (void)hipDeviceSynchronize();
    for (void* q : ptrs) pool().free(q);
    if (pool().quarantine()) pool().quarantine_release();
  }
};

// local SpGEMM (cbg_local.hip)
struct LocalStats {
  int64_t flops = 0;
  int64_t nnz = 0;
  int64_t n_big = 0, n_slabs = 0;
  double ms_symbolic = 0, ms_numeric = 0;
  int64_t work[CBG_WORK_N] = {};  // cbg_last_work_stats
};
// Every call accumulates into the calling thread's stats (reset by the C ABI
// at the start of each public entry point); `st` optionally receives this call's.
// sink: where C's entries go (C.reserved gets TILE_BORROWED_ENTRIES).
void local_spgemm(const cbg_tile& A, const cbg_tile& B, int semiring, cbg_tile& C, hipStream_t s,
                  LocalStats* st = nullptr, OutSink* sink = nullptr);
LocalStats& thread_stats();
// CUs the persistent slab kernels leave free for communication (cbg_local.hip)
int& comm_reserve_cus();
struct CommReserve {  // scope of a local multiply that runs while a broadcast is in flight
  int prev;
  explicit CommReserve(int cus) : prev(comm_reserve_cus()) { comm_reserve_cus() = cus; }
  ~CommReserve() { comm_reserve_cus() = prev; }
};
// merges run as products (cbg_merge.hip) but are not SpGEMM work: their
// multiplies are kept out of thread_stats() and summed here instead
struct MergeStats {
  int64_t entries_in = 0, entries_out = 0;
  double ms = 0;
};
MergeStats& merge_stats();
// the last PANEL SUMMA's pipelining: pieces multiplied, measured broadcast
// time of the first piece, and the transfer of the rest it estimated
struct SummaInfo {
  int pieces = 0;
  double bcast_ms_piece0 = 0, est_hidden_ms = 0, piece_cost_ms = 0;
  int oom_splits = 0;  // phases computed as column halves after an out-of-memory
  // 0: one piece, no decision; 1: pipelined (RCCL, > 1 remote B tile);
  // 2: adaptive, kept two pieces; 3: adaptive, rejoined into one
  int rule = 0;
  int64_t bytes_recv = 0;      // A and B tile bytes this rank received
  double exposed_comm_ms = 0;  // compute-stream waits for the broadcasts (events)
};
// the last MemEfficientSpGEMM call's phase plan: phases run, and when they
// were chosen from memory, this rank's product flops, estimated nnz(C) and
// the C bytes a phase may take
struct PhasePlan {
  int phases = 0, automatic = 0;
  int64_t flops = 0, nnz_est = 0;
  double c_budget_bytes = 0;
  double ms = 0;  // host time of the planning (collectives and sample included)
};
PhasePlan& phase_plan();
SummaInfo& summa_info();
// A-side preparation (column maps of A) kept across the local multiplies of
// one MemEfficientSpGEMM call, whose phases all multiply the same A: between
// aprep_begin() and aprep_end() on a thread, a local multiply whose A has the
// same arrays, the same pool allocations of them (DevicePool::serial_of: a
// freed and re-allocated block at the same address is a different A) and the
// same sizes as the previous one reuses its maps.
void aprep_begin();
void aprep_end();
struct APrepScope {
  APrepScope() { aprep_begin(); }
  ~APrepScope() { aprep_end(); }
};

// device exclusive scan of n int64 values -> out[0..n], returns nothing (total at out[n]).
// df: the scan's temporaries are released with df (no host synchronization);
// without it the scan synchronizes the stream before returning them.
struct DeferredFree;
void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s, DeferredFree* df = nullptr);
void exclusive_scan_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, hipStream_t s, DeferredFree* df = nullptr);

// thin big columns of the local multiply (cbg_thin.hip): the n columns perm[]
// (fthin products in all) expanded, sorted and reduced into tir/tval[base ...];
// cnt[col] = their nnz, tslot[col] = their first temporary position
// (E = their B entries); thin_copy moves them to C after the column scan
// (ainl: optional inline records of A's columns, see k_inline_cols)
void thin_columns(const int32_t* perm, int n, int64_t E, int64_t fthin, const cbg_tile& A, const cbg_tile& B,
                  const int2* cmap, const int4* ainl, int semiring, int32_t* cnt, int64_t* tslot, int32_t* tir,
                  double* tval, int64_t base, hipStream_t s, DeferredFree& df);
void thin_copy(const int32_t* perm, int n, const int64_t* tslot, const int32_t* cnt, const int64_t* colptr,
               const int32_t* tir, const double* tval, int32_t* out_ir, double* out_val, hipStream_t s);

// radix sort of (key, value) pairs (cbg_sort.hip): LSD over the 8-bit digits
// that `varying` marks as possibly nonzero, stable, 64-bit counts; the sorted
// pairs end in `keys` / `vals` (the DBufs may be swapped with temporaries).
// With df the temporaries are handed to it (no host synchronization: the
// caller's stream sync releases them), else the call synchronizes the stream.
template <typename K>
void radix_sort_pairs(DBuf<K>& keys, DBuf<double>& vals, int64_t n, unsigned long long varying, hipStream_t s,
                      DeferredFree* df = nullptr);
// equal consecutive keys combined with the semiring's add (in order); returns the
// runs (one readback: a host synchronization; temporaries to df when given)
template <typename K>
int64_t reduce_by_key(const K* keys, const double* vals, int64_t n, int semiring, K* ukeys, double* uvals,
                      hipStream_t s, DeferredFree* df = nullptr);

// multiway merge of column-sorted partial tiles (cbg_merge.hip)
// int64 entry counts: column chunks of < 2^30 stacked entries (CBG_MERGE_CHUNK
// overrides) each run as one product into an EntryArena
void merge_tiles(const std::vector<cbg_tile>& parts, int64_t m, int64_t n, int semiring, cbg_tile& C,
                 hipStream_t s);

// tile helpers (cbg_tile.hip)
void tile_free_device(cbg_tile& t);
void tile_alloc_device(cbg_tile& t, int64_t m, int64_t n, int64_t nnz, int64_t nzc);
// owner of a device tile inside host loops: freed on scope exit (exceptions included)
struct TileGuard {
  cbg_tile t{};
  TileGuard() = default;
  explicit TileGuard(const cbg_tile& x) : t(x) {}
  ~TileGuard();
  cbg_tile release() {
    cbg_tile r = t;
    t = cbg_tile{};
    return r;
  }
  TileGuard(TileGuard&& o) noexcept : t(o.release()) {}
  TileGuard& operator=(TileGuard&& o) noexcept;
  TileGuard(const TileGuard&) = delete;
  TileGuard& operator=(const TileGuard&) = delete;
};
void tile_split_cols(const cbg_tile& T, int64_t cut, cbg_tile& L, cbg_tile& R, hipStream_t s);
// columns [a, b) / rows [a, b) of T as a new tile (re-based), one copy
void tile_slice_cols(const cbg_tile& T, int64_t a, int64_t b, cbg_tile& out, hipStream_t s);
void tile_slice_rows(const cbg_tile& T, int64_t a, int64_t b, cbg_tile& out, hipStream_t s);
// column concatenation of tiles whose entries already lie end to end in
// `arena` (parts[k].ir == arena.ir + sum of the earlier parts' nnz): only cp
// and jc are built; `out` takes over the arena's arrays
void tile_assemble_cols(const std::vector<cbg_tile>& parts, const std::vector<int64_t>& col_off, int64_t m,
                        int64_t n, EntryArena& arena, cbg_tile& out, hipStream_t s);
void tile_split_rows(const cbg_tile& T, int64_t cut, cbg_tile& Top, cbg_tile& Bot, hipStream_t s);
void tile_concat_cols(const std::vector<cbg_tile>& parts, const std::vector<int64_t>& col_off, int64_t m,
                      int64_t n, cbg_tile& out, hipStream_t s);
void tile_concat_rows(const std::vector<cbg_tile>& parts, const std::vector<int64_t>& row_off, int64_t m,
                      int64_t n, cbg_tile& out, hipStream_t s);
bool tile_equal(const cbg_tile& a, const cbg_tile& b, double eps, hipStream_t s);
// phase planning: dim 0 = nonzeros per column (length n), 1 = per row (length m),
// into the device array d zero-padded to `padded` entries (stream synchronized)
void tile_counts_device(const cbg_tile& t, int dim, int32_t* d, int64_t padded, hipStream_t s);
// sum over B's entries (k, j) of a[k] (device array of B.m values): A*B's flops for A's column counts
int64_t entry_sum_device(const cbg_tile& B, const int32_t* a, hipStream_t s);
// sum_k a[k] * b[k] over k < K with a, b stored as blocks (see cbg_tile.hip)
int64_t blocked_dot_device(const int32_t* a, int64_t astride, const std::vector<int64_t>& aoff, const int32_t* b,
                           int64_t bstride, const std::vector<int64_t>& boff, int64_t K, hipStream_t s);
// the columns of T whose id is a multiple of stride (same shape and ids), and
// the rows whose id is (renumbered row / stride: ceil(m / stride) rows)
void tile_sample_cols(const cbg_tile& T, int stride, cbg_tile& out, hipStream_t s);
void tile_sample_rows(const cbg_tile& T, int stride, cbg_tile& out, hipStream_t s);
// estimateFLOP + estimateNNZ_Hash totals of A*B without the numeric phase
void local_symbolic(const cbg_tile& A, const cbg_tile& B, hipStream_t s, int64_t* flops, int64_t* nnz);

// Galerkin path operations (cbg_ops.hip)
void tile_transpose(const cbg_tile& T, cbg_tile& out, hipStream_t s);
void tile_dim_apply(cbg_tile& t, int dim, const double* vec_host, int op, hipStream_t s);
void restriction_tile(int scale, int order, uint64_t seed, int pr, int pc, int prow, int pcol, cbg_tile& out,
                      hipStream_t s);
// values U[-1, 1) from a hash of (seed, global column, global row) (test inputs)
void tile_random_values(cbg_tile& t, uint64_t seed, int64_t roff, int64_t coff, hipStream_t s);

// measured HBM bandwidth: 16-B-per-lane device copy (cbg_ops.hip)
double hbm_copy_gbps(int64_t bytes, int reps);
void store_probe(int64_t bytes, int width);

}  // namespace cbg
