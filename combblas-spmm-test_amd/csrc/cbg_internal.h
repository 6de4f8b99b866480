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
class DevicePool {
 public:
  void* alloc(size_t bytes);
  void free(void* p);
  void trim();  // release every cached block
  size_t bytes_in_use() const { return in_use_; }
  size_t bytes_cached() const { return cached_; }
  ~DevicePool() { trim(); }

 private:
  std::mutex mu_;
  std::multimap<size_t, void*> free_;
  std::map<void*, size_t> live_;
  size_t in_use_ = 0, cached_ = 0;
};
DevicePool& pool();

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
  template <class T>
  void take(DBuf<T>& b) {
    if (b.p) ptrs.push_back(b.detach());
  }
  ~DeferredFree() {
    for (void* q : ptrs) pool().free(q);
  }
};

// local SpGEMM (cbg_local.hip)
struct LocalStats {
  int64_t flops = 0;
  int64_t nnz = 0;
  int64_t n_big = 0, n_slabs = 0;
  double ms_symbolic = 0, ms_numeric = 0;
};
// Every call accumulates into the calling thread's stats (reset by the C ABI
// at the start of each public entry point); `st` optionally receives this call's.
void local_spgemm(const cbg_tile& A, const cbg_tile& B, int semiring, cbg_tile& C, hipStream_t s,
                  LocalStats* st = nullptr);
LocalStats& thread_stats();
// A-side preparation (column maps of A) kept across the local multiplies of
// one MemEfficientSpGEMM call, whose phases all multiply the same A: between
// aprep_begin() and aprep_end() on a thread, a local multiply whose A has the
// same arrays and sizes as the previous one reuses its maps.
void aprep_begin();
void aprep_end();
struct APrepScope {
  APrepScope() { aprep_begin(); }
  ~APrepScope() { aprep_end(); }
};

// device exclusive scan of n int64 values -> out[0..n], returns nothing (total at out[n])
void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s);
void exclusive_scan_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, hipStream_t s);

// multiway merge of column-sorted partial tiles (cbg_merge.hip)
void merge_tiles(const std::vector<cbg_tile>& parts, int64_t m, int64_t n, int semiring, cbg_tile& C,
                 hipStream_t s);

// tile helpers (cbg_tile.hip)
void tile_free_device(cbg_tile& t);
void tile_alloc_device(cbg_tile& t, int64_t m, int64_t n, int64_t nnz, int64_t nzc);
void tile_split_cols(const cbg_tile& T, int64_t cut, cbg_tile& L, cbg_tile& R, hipStream_t s);
void tile_split_rows(const cbg_tile& T, int64_t cut, cbg_tile& Top, cbg_tile& Bot, hipStream_t s);
void tile_concat_cols(const std::vector<cbg_tile>& parts, const std::vector<int64_t>& col_off, int64_t m,
                      int64_t n, cbg_tile& out, hipStream_t s);
void tile_concat_rows(const std::vector<cbg_tile>& parts, const std::vector<int64_t>& row_off, int64_t m,
                      int64_t n, cbg_tile& out, hipStream_t s);
bool tile_equal(const cbg_tile& a, const cbg_tile& b, double eps, hipStream_t s);

// Galerkin path operations (cbg_ops.hip)
void tile_transpose(const cbg_tile& T, cbg_tile& out, hipStream_t s);
void tile_dim_apply(cbg_tile& t, int dim, const double* vec_host, int op, hipStream_t s);
void restriction_tile(int scale, int order, uint64_t seed, int pr, int pc, int prow, int pcol, cbg_tile& out,
                      hipStream_t s);

// measured HBM bandwidth: 16-B-per-lane device copy (cbg_ops.hip)
double hbm_copy_gbps(int64_t bytes, int reps);

}  // namespace cbg
