// cbg_capi.cpp -- extern "C" boundary of libcbg (declared in include/cbg.h).
// Every entry point catches exceptions and returns the reference's abort code
// (SpDefs.h:69-76) or a >= 3100 runtime code; cbg_last_error() has the text.
#include <cstring>

#include "cbg_internal.h"

struct cbg_grid;
namespace cbg {
void rmat_tile(int scale, int ef, uint64_t userseed, int pr, int pc, int prow, int pcol, cbg_tile& out, hipStream_t s);
void tile_digest(const cbg_tile& t, int64_t roff, int64_t coff, uint64_t* hs, uint64_t* hv, double* vsum,
                 uint64_t* unsorted, hipStream_t s);
bool tile_equal(const cbg_tile& a, const cbg_tile& b, double eps, hipStream_t s);
int grid_shape(int nranks, int& rows, int& cols);
cbg_grid* grid_create_rccl(int rank, int nranks, int rows, int cols, const void* uid);
cbg_grid* grid_create_host(int rank, int nranks, int rows, int cols, const cbg_host_comm* hc);
void grid_destroy(cbg_grid* g);
void allreduce_f64(cbg_grid* g, double* v, bool max);
void allreduce_sum_i64(cbg_grid* g, int64_t* v);
void barrier(cbg_grid* g);
int summa_spgemm(cbg_grid* g, const cbg_tile& A, const cbg_tile& B, int64_t A_gncol, int64_t B_gnrow, int sr, int algo,
                 int exec, cbg_tile& C);
int summa_spgemm_phased(cbg_grid* g, const cbg_tile& A, const cbg_tile& B, int64_t A_gncol, int64_t B_gnrow, int sr,
                        int algo, int exec, int phases, int64_t mem_gb, cbg_phase_fn fn, void* user, cbg_tile* C);
int grid_transpose(cbg_grid* g, const cbg_tile& T, cbg_tile& out);
int agree(cbg_grid* g, int rc);
std::string& step_error();
int grid_block_extract(cbg_grid* g, const cbg_tile& T, int64_t gm, int64_t gn, int dim, int64_t lo, int64_t hi,
                       cbg_tile& out);
}  // namespace cbg

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

template <class F>
int guard(F&& f) {
  try {
    g_err.clear();
    return f();
  } catch (const cbg::HipError& e) {
    return fail(e.code, e.what());
  } catch (const std::exception& e) {
    return fail(CBG_ERR_HIP, e.what());
  } catch (...) {
    return fail(CBG_ERR_HIP, "unknown error");
  }
}

hipStream_t default_stream() {
  static thread_local hipStream_t s = nullptr;
  if (!s) CBG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  return s;
}
hipStream_t as_stream(void* p) { return p ? static_cast<hipStream_t>(p) : default_stream(); }

int check_tile(const cbg_tile* t, bool need_device, const char* name) {
  if (!t) return fail(CBG_ERR_INVALIDPARAMS, std::string(name) + " is NULL");
  if (need_device && !t->on_device) return fail(CBG_ERR_INVALIDPARAMS, std::string(name) + " is not a device tile");
  if (t->m < 0 || t->n < 0 || t->nnz < 0 || t->nzc < 0 || t->nzc > t->n)
    return fail(CBG_ERR_INVALIDPARAMS, std::string(name) + " has inconsistent sizes");
  if (t->m >= INT32_MAX || t->n >= INT32_MAX)
    return fail(CBG_ERR_INVALIDPARAMS, std::string(name) + ": local dimensions must fit int32");
  return CBG_OK;
}
}  // namespace

extern "C" {

const char* cbg_version(void) { return "libcbg 0.1 (gfx950)"; }
const char* cbg_last_error(void) { return g_err.c_str(); }

int cbg_set_device(int device) {
  return guard([&] {
    CBG_HIP(hipSetDevice(device));
    return CBG_OK;
  });
}
int cbg_device_count(int* count) {
  return guard([&] {
    CBG_HIP(hipGetDeviceCount(count));
    return CBG_OK;
  });
}
int cbg_pool_stats(size_t* in_use, size_t* cached) {
  if (in_use) *in_use = cbg::pool().bytes_in_use();
  if (cached) *cached = cbg::pool().bytes_cached();
  return CBG_OK;
}
int cbg_pool_trim(void) {
  return guard([&] {
    cbg::pool().trim();
    return CBG_OK;
  });
}
int cbg_hbm_copy_bandwidth(int64_t bytes, int reps, double* gbps) {
  if (!gbps || bytes <= 0 || reps <= 0) return fail(CBG_ERR_INVALIDPARAMS, "cbg_hbm_copy_bandwidth: bad arguments");
  return guard([&] {
    *gbps = cbg::hbm_copy_gbps(bytes, reps);
    return CBG_OK;
  });
}

int cbg_store_probe(int64_t bytes, int width) {
  if (bytes <= 0 || bytes % 256 || (width != 4 && width != 8))
    return fail(CBG_ERR_INVALIDPARAMS, "cbg_store_probe: bytes a positive multiple of 256, width 4 or 8");
  return guard([&] {
    cbg::store_probe(bytes, width);
    return CBG_OK;
  });
}

int cbg_synchronize(void) {
  return guard([&] {
    CBG_HIP(hipDeviceSynchronize());
    return CBG_OK;
  });
}

int cbg_tile_upload(const cbg_tile* h, cbg_tile* d) {
  if (int rc = check_tile(h, false, "host tile")) return rc;
  if (!d) return fail(CBG_ERR_INVALIDPARAMS, "dst is NULL");
  return guard([&] {
    cbg_tile t{};
    cbg::tile_alloc_device(t, h->m, h->n, h->nnz, h->nzc);
    hipStream_t s = default_stream();
    CBG_HIP(hipMemcpyAsync(t.cp, h->cp, sizeof(int64_t) * (h->nzc + 1), hipMemcpyHostToDevice, s));
    if (h->nzc) CBG_HIP(hipMemcpyAsync(t.jc, h->jc, sizeof(int32_t) * h->nzc, hipMemcpyHostToDevice, s));
    if (h->nnz) {
      CBG_HIP(hipMemcpyAsync(t.ir, h->ir, sizeof(int32_t) * h->nnz, hipMemcpyHostToDevice, s));
      CBG_HIP(hipMemcpyAsync(t.val, h->val, sizeof(double) * h->nnz, hipMemcpyHostToDevice, s));
    }
    CBG_HIP(hipStreamSynchronize(s));
    *d = t;
    return CBG_OK;
  });
}

int cbg_tile_download(const cbg_tile* d, cbg_tile* h) {
  if (int rc = check_tile(d, true, "device tile")) return rc;
  if (!h || !h->cp || (d->nzc && !h->jc) || (d->nnz && (!h->ir || !h->val)))
    return fail(CBG_ERR_INVALIDPARAMS, "host arrays missing");
  return guard([&] {
    hipStream_t s = default_stream();
    CBG_HIP(hipMemcpyAsync(h->cp, d->cp, sizeof(int64_t) * (d->nzc + 1), hipMemcpyDeviceToHost, s));
    if (d->nzc) CBG_HIP(hipMemcpyAsync(h->jc, d->jc, sizeof(int32_t) * d->nzc, hipMemcpyDeviceToHost, s));
    if (d->nnz) {
      CBG_HIP(hipMemcpyAsync(h->ir, d->ir, sizeof(int32_t) * d->nnz, hipMemcpyDeviceToHost, s));
      CBG_HIP(hipMemcpyAsync(h->val, d->val, sizeof(double) * d->nnz, hipMemcpyDeviceToHost, s));
    }
    CBG_HIP(hipStreamSynchronize(s));
    h->m = d->m;
    h->n = d->n;
    h->nnz = d->nnz;
    h->nzc = d->nzc;
    h->on_device = 0;
    return CBG_OK;
  });
}

int cbg_tile_free(cbg_tile* t) {
  if (!t) return CBG_OK;
  return guard([&] {
    if (t->on_device) cbg::tile_free_device(*t);
    return CBG_OK;
  });
}

int cbg_tile_alloc(int64_t m, int64_t n, int64_t nnz, int64_t nzc, cbg_tile* out) {
  if (!out || m < 0 || n < 0 || nnz < 0 || nzc < 0 || nzc > n || (nzc == 0) != (nnz == 0))
    return fail(CBG_ERR_INVALIDPARAMS, "bad tile sizes");
  return guard([&] {
    cbg_tile t{};
    cbg::tile_alloc_device(t, m, n, nnz, nzc);
    if (nzc > 0) CBG_HIP(hipMemset(t.cp, 0, sizeof(int64_t)));
    *out = t;
    return CBG_OK;
  });
}

int cbg_tile_concat_cols(const cbg_tile* parts, int nparts, cbg_tile* out) {
  if (!parts || nparts <= 0 || !out) return fail(CBG_ERR_INVALIDPARAMS, "no parts");
  int64_t n = 0;
  std::vector<int64_t> off;
  for (int i = 0; i < nparts; ++i) {
    if (int rc = check_tile(&parts[i], true, "part")) return rc;
    if (parts[i].m != parts[0].m) return fail(CBG_ERR_DIMMISMATCH, "parts differ in row count");
    off.push_back(n);
    n += parts[i].n;
  }
  if (n >= INT32_MAX) return fail(CBG_ERR_INVALIDPARAMS, "local dimensions must fit int32");
  return guard([&] {
    std::vector<cbg_tile> v(parts, parts + nparts);
    cbg::tile_concat_cols(v, off, parts[0].m, n, *out, default_stream());
    return CBG_OK;
  });
}

int cbg_device_memory(size_t* free_bytes, size_t* total_bytes) {
  return guard([&] {
    size_t f = 0, t = 0;
    CBG_HIP(hipMemGetInfo(&f, &t));
    if (free_bytes) *free_bytes = f;
    if (total_bytes) *total_bytes = t;
    return CBG_OK;
  });
}

int cbg_tile_split_cols(const cbg_tile* t, int64_t cut, cbg_tile* l, cbg_tile* r) {
  if (int rc = check_tile(t, true, "tile")) return rc;
  if (cut < 0 || cut > t->n) return fail(CBG_ERR_INVALIDPARAMS, "cut out of range");
  return guard([&] {
    cbg::tile_split_cols(*t, cut, *l, *r, default_stream());
    return CBG_OK;
  });
}

int cbg_tile_split_rows(const cbg_tile* t, int64_t cut, cbg_tile* top, cbg_tile* bot) {
  if (int rc = check_tile(t, true, "tile")) return rc;
  if (cut < 0 || cut > t->m) return fail(CBG_ERR_INVALIDPARAMS, "cut out of range");
  return guard([&] {
    cbg::tile_split_rows(*t, cut, *top, *bot, default_stream());
    return CBG_OK;
  });
}

int cbg_tile_digest(const cbg_tile* t, int64_t roff, int64_t coff, uint64_t* hs, uint64_t* hv, double* vsum,
                    uint64_t* unsorted) {
  if (int rc = check_tile(t, true, "tile")) return rc;
  if (!hs || !hv || !vsum) return fail(CBG_ERR_INVALIDPARAMS, "digest outputs missing");
  return guard([&] {
    cbg::tile_digest(*t, roff, coff, hs, hv, vsum, unsorted, default_stream());
    return CBG_OK;
  });
}

int cbg_tile_equal(const cbg_tile* a, const cbg_tile* b, double epsilon, int* equal) {
  if (int rc = check_tile(a, true, "a")) return rc;
  if (int rc = check_tile(b, true, "b")) return rc;
  if (!equal || !(epsilon >= 0)) return fail(CBG_ERR_INVALIDPARAMS, "bad equality parameters");
  return guard([&] {
    *equal = cbg::tile_equal(*a, *b, epsilon, default_stream()) ? 1 : 0;
    return CBG_OK;
  });
}

int cbg_tile_transpose(const cbg_tile* t, cbg_tile* out) {
  if (int rc = check_tile(t, true, "tile")) return rc;
  if (!out) return fail(CBG_ERR_INVALIDPARAMS, "out is NULL");
  return guard([&] {
    cbg::tile_transpose(*t, *out, default_stream());
    return CBG_OK;
  });
}

int cbg_tile_dim_apply(cbg_tile* t, int dim, const double* vec, int op) {
  if (int rc = check_tile(t, true, "tile")) return rc;
  if ((dim != CBG_DIM_COLUMN && dim != CBG_DIM_ROW) || op < CBG_OP_MULTIPLIES || op > CBG_OP_MAX ||
      (!vec && (dim == CBG_DIM_COLUMN ? t->n : t->m) > 0))
    return fail(CBG_ERR_INVALIDPARAMS, "bad DimApply parameters");
  return guard([&] {
    cbg::tile_dim_apply(*t, dim, vec, op, default_stream());
    return CBG_OK;
  });
}

int cbg_restriction_tile(int scale, int order, uint64_t seed, int pr, int pc, int prow, int pcol, cbg_tile* out) {
  if (scale < 1 || scale > 30 || order < 1 || ((int64_t)1 << scale) / order < 1 || pr < 1 || pc < 1 || prow < 0 ||
      prow >= pr || pcol < 0 || pcol >= pc || !out)
    return fail(CBG_ERR_INVALIDPARAMS, "bad restriction parameters");
  return guard([&] {
    cbg::restriction_tile(scale, order, seed, pr, pc, prow, pcol, *out, default_stream());
    return CBG_OK;
  });
}

int cbg_tile_random_values(cbg_tile* t, uint64_t seed, int64_t row_off, int64_t col_off) {
  if (int rc = check_tile(t, true, "tile")) return rc;
  if (row_off < 0 || col_off < 0) return fail(CBG_ERR_INVALIDPARAMS, "negative offsets");
  return guard([&] {
    cbg::tile_random_values(*t, seed, row_off, col_off, default_stream());
    return CBG_OK;
  });
}

static const char* summa_msg(int rc);

int cbg_grid_transpose(cbg_grid* g, const cbg_tile* local, cbg_tile* out) {
  if (!g) return fail(CBG_ERR_INVALIDPARAMS, "grid is NULL");
  if (int rc = check_tile(local, true, "tile")) return rc;
  if (!out) return fail(CBG_ERR_INVALIDPARAMS, "out is NULL");
  return guard([&]() -> int {
    CBG_HIP(hipDeviceSynchronize());
    cbg::step_error().clear();
    int rc = cbg::grid_transpose(g, *local, *out);
    if (rc == CBG_ERR_NOTSQUARE) return fail(rc, "SpParMat::Transpose needs a square grid");
    if (rc) return fail(rc, cbg::step_error().empty() ? summa_msg(rc) : "this rank: " + cbg::step_error());
    return CBG_OK;
  });
}

int cbg_grid_block_extract(cbg_grid* g, const cbg_tile* local, int64_t gm, int64_t gn, int dim, int64_t lo,
                           int64_t hi, cbg_tile* out) {
  if (!g) return fail(CBG_ERR_INVALIDPARAMS, "grid is NULL");
  if (int rc = check_tile(local, true, "tile")) return rc;
  if (!out) return fail(CBG_ERR_INVALIDPARAMS, "out is NULL");
  return guard([&]() -> int {
    CBG_HIP(hipDeviceSynchronize());
    cbg::step_error().clear();
    int rc = cbg::grid_block_extract(g, *local, gm, gn, dim, lo, hi, *out);
    if (rc == CBG_ERR_INVALIDPARAMS && cbg::step_error().empty())
      return fail(rc, "block range outside the matrix or bad dim");
    if (rc) return fail(rc, cbg::step_error().empty() ? summa_msg(rc) : "this rank: " + cbg::step_error());
    return CBG_OK;
  });
}

int cbg_rmat_tile(int scale, int ef, uint64_t seed, int pr, int pc, int prow, int pcol, cbg_tile* out) {
  if (scale < 1 || scale > 30 || ef < 1 || pr < 1 || pc < 1 || prow < 0 || prow >= pr || pcol < 0 || pcol >= pc || !out)
    return fail(CBG_ERR_INVALIDPARAMS, "bad R-MAT parameters");
  if (((int64_t)1 << scale) * ef >= ((int64_t)1 << 31))
    return fail(CBG_ERR_NOTSUPPORTED, "edge count must stay below 2^31");
  return guard([&] {
    cbg::rmat_tile(scale, ef, seed, pr, pc, prow, pcol, *out, default_stream());
    return CBG_OK;
  });
}

int cbg_local_spgemm(const cbg_tile* A, const cbg_tile* B, int sr, cbg_tile* C, void* stream) {
  if (int rc = check_tile(A, true, "A")) return rc;
  if (int rc = check_tile(B, true, "B")) return rc;
  if (!C) return fail(CBG_ERR_INVALIDPARAMS, "C is NULL");
  if (sr != CBG_PLUS_TIMES && sr != CBG_MIN_PLUS) return fail(CBG_ERR_INVALIDPARAMS, "unknown semiring");
  if (A->n != B->m) return fail(CBG_ERR_DIMMISMATCH, "A.ncol != B.nrow");
  if (A->nnz >= INT32_MAX || B->nnz >= INT32_MAX) return fail(CBG_ERR_NOTSUPPORTED, "A/B tiles need nnz < 2^31");
  return guard([&] {
    cbg::thread_stats() = cbg::LocalStats{};
    cbg::local_spgemm(*A, *B, sr, *C, as_stream(stream));
    return CBG_OK;
  });
}

int cbg_local_symbolic(const cbg_tile* A, const cbg_tile* B, int64_t* flops, int64_t* nnz, void* stream) {
  if (int rc = check_tile(A, true, "A")) return rc;
  if (int rc = check_tile(B, true, "B")) return rc;
  if (A->n != B->m) return fail(CBG_ERR_DIMMISMATCH, "A.ncol != B.nrow");
  if (A->nnz >= INT32_MAX || B->nnz >= INT32_MAX) return fail(CBG_ERR_NOTSUPPORTED, "A/B tiles need nnz < 2^31");
  // the multiply's flops and symbolic kernels only: no C is formed
  return guard([&] {
    cbg::local_symbolic(*A, *B, as_stream(stream), flops, nnz);
    return CBG_OK;
  });
}

int cbg_merge(const cbg_tile* parts, int nparts, int sr, cbg_tile* C, void* stream) {
  if (nparts <= 0 || !parts || !C) return fail(CBG_ERR_INVALIDPARAMS, "no parts");
  for (int i = 0; i < nparts; ++i) {
    if (int rc = check_tile(&parts[i], true, "part")) return rc;
    if (parts[i].m != parts[0].m || parts[i].n != parts[0].n)
      return fail(CBG_ERR_DIMMISMATCH, "Dimensions do not match on MergeAll()");  // Friends.h:672-678
  }
  return guard([&] {
    cbg::thread_stats() = cbg::LocalStats{};
    cbg::merge_stats() = cbg::MergeStats{};
    std::vector<cbg_tile> v(parts, parts + nparts);
    cbg::merge_tiles(v, parts[0].m, parts[0].n, sr, *C, as_stream(stream));
    return CBG_OK;
  });
}

int cbg_last_stats(int64_t* flops, int64_t* nnz, double* ms_sym, double* ms_num, int64_t* n_big, int64_t* n_slabs) {
  const cbg::LocalStats& g_stats = cbg::thread_stats();
  if (flops) *flops = g_stats.flops;
  if (nnz) *nnz = g_stats.nnz;
  if (ms_sym) *ms_sym = g_stats.ms_symbolic;
  if (ms_num) *ms_num = g_stats.ms_numeric;
  if (n_big) *n_big = g_stats.n_big;
  if (n_slabs) *n_slabs = g_stats.n_slabs;
  return CBG_OK;
}

int cbg_last_work_stats(int64_t* counts, int n) {
  const cbg::LocalStats& g_stats = cbg::thread_stats();
  for (int i = 0; counts && i < n && i < CBG_WORK_N; ++i) counts[i] = g_stats.work[i];
  return CBG_WORK_N;
}

// ---------------- grid ----------------
int cbg_get_unique_id(void* id);  // cbg_summa_id.cpp

int cbg_grid_create(int rank, int nranks, int rows, int cols, const void* uid, cbg_grid** out) {
  if (!out || !uid || rank < 0 || rank >= nranks) return fail(CBG_ERR_INVALIDPARAMS, "bad grid parameters");
  if (int rc = cbg::grid_shape(nranks, rows, cols))
    return fail(rc, rc == CBG_ERR_NOTSQUARE ? "This version only works on a square logical processor grid"
                                            : "grid rows*cols != nranks");
  return guard([&] {
    *out = cbg::grid_create_rccl(rank, nranks, rows, cols, uid);
    return CBG_OK;
  });
}

int cbg_grid_create_host(int rank, int nranks, int rows, int cols, const cbg_host_comm* hc, cbg_grid** out) {
  if (!out || !hc || !hc->bcast || !hc->allgather || rank < 0 || rank >= nranks)
    return fail(CBG_ERR_INVALIDPARAMS, "bad grid parameters");
  if (int rc = cbg::grid_shape(nranks, rows, cols)) return fail(rc, "grid shape");
  return guard([&] {
    *out = cbg::grid_create_host(rank, nranks, rows, cols, hc);
    return CBG_OK;
  });
}

int cbg_grid_destroy(cbg_grid* g) {
  return guard([&] {
    cbg::grid_destroy(g);
    return CBG_OK;
  });
}

int cbg_grid_barrier(cbg_grid* g) {
  if (!g) return fail(CBG_ERR_INVALIDPARAMS, "grid is NULL");
  return guard([&] {
    cbg::barrier(g);
    return CBG_OK;
  });
}
int cbg_grid_allreduce_max(cbg_grid* g, double* v) {
  if (!g || !v) return fail(CBG_ERR_INVALIDPARAMS, "grid is NULL");
  return guard([&] {
    cbg::allreduce_f64(g, v, true);
    return CBG_OK;
  });
}
int cbg_grid_allreduce_sum_i64(cbg_grid* g, int64_t* v) {
  if (!g || !v) return fail(CBG_ERR_INVALIDPARAMS, "grid is NULL");
  return guard([&] {
    cbg::allreduce_sum_i64(g, v);
    return CBG_OK;
  });
}

// Collective entry points: a check that fails on some ranks only is agreed on
// over the grid before returning, so every rank returns the code (the
// reference MPI_Aborts every rank, SpDefs.h:69-76).
static const char* summa_msg(int rc) {
  return rc == CBG_ERR_DIMMISMATCH   ? "Can not multiply, dimensions does not match"
         : rc == CBG_ERR_MATRIXALIAS ? "Can not multiply, inputs alias"
         : rc == CBG_ERR_NOTSQUARE   ? "needs a square grid"
         : rc == CBG_ERR_INVALIDPARAMS
             ? "bad parameters (a B tile with fewer columns than phases, or a phase callback failed)"
         : rc == CBG_ERR_OOM ? "device memory exhausted on a rank of the grid"
         : rc == CBG_ERR_RCCL ? "communication failure on the grid"
                              : "failed on a rank of the grid";
}

static int summa_args(const cbg_tile* A, const cbg_tile* B, int sr, int algo, int exec) {
  if (int rc = check_tile(A, true, "A")) return rc;
  if (int rc = check_tile(B, true, "B")) return rc;
  if ((sr != CBG_PLUS_TIMES && sr != CBG_MIN_PLUS) || (algo != CBG_DOUBLEBUFF && algo != CBG_SYNCH) ||
      (exec != CBG_EXEC_PANEL && exec != CBG_EXEC_STAGED))
    return fail(CBG_ERR_INVALIDPARAMS, "bad summa parameters");
  if (A->nnz >= INT32_MAX || B->nnz >= INT32_MAX) return fail(CBG_ERR_NOTSUPPORTED, "A/B tiles need nnz < 2^31");
  return CBG_OK;
}

int cbg_summa_spgemm(cbg_grid* g, const cbg_tile* A, const cbg_tile* B, int64_t A_gncol, int64_t B_gnrow, int sr,
                     int algo, int exec, cbg_tile* C) {
  if (!g) return fail(CBG_ERR_INVALIDPARAMS, "grid is NULL");
  int arg = summa_args(A, B, sr, algo, exec);
  if (!arg && !C) arg = fail(CBG_ERR_INVALIDPARAMS, "C is NULL");
  if (!arg && A == B) arg = fail(CBG_ERR_MATRIXALIAS, "inputs alias (make a temporary copy of one of them first)");
  const std::string why = g_err;
  return guard([&]() -> int {
    cbg::thread_stats() = cbg::LocalStats{};
    cbg::merge_stats() = cbg::MergeStats{};
    if (arg) return fail(cbg::agree(g, arg), why);  // before any device call: peers must not block
    CBG_HIP(hipDeviceSynchronize());
    cbg::step_error().clear();
    int rc = cbg::summa_spgemm(g, *A, *B, A_gncol, B_gnrow, sr, algo, exec, *C);
    if (rc) return fail(rc, cbg::step_error().empty() ? summa_msg(rc) : "this rank: " + cbg::step_error());
    return CBG_OK;
  });
}

int cbg_summa_spgemm_memeff(cbg_grid* g, const cbg_tile* A, const cbg_tile* B, int64_t A_gncol, int64_t B_gnrow,
                            int sr, int algo, int exec, int phases, int64_t per_process_memory_gb, cbg_phase_fn fn,
                            void* user, cbg_tile* C) {
  if (!g) return fail(CBG_ERR_INVALIDPARAMS, "grid is NULL");
  // A and B may alias: B is copied (ParFriends.h:547-549)
  int arg = summa_args(A, B, sr, algo, exec);
  if (!arg && !C && !fn) arg = fail(CBG_ERR_INVALIDPARAMS, "neither C nor a phase callback");
  const std::string why = g_err;
  return guard([&]() -> int {
    cbg::thread_stats() = cbg::LocalStats{};
    cbg::merge_stats() = cbg::MergeStats{};
    if (arg) return fail(cbg::agree(g, arg), why);  // before any device call: peers must not block
    CBG_HIP(hipDeviceSynchronize());
    cbg::step_error().clear();
    int rc = cbg::summa_spgemm_phased(g, *A, *B, A_gncol, B_gnrow, sr, algo, exec, phases, per_process_memory_gb, fn,
                                      user, C);
    if (rc) return fail(rc, cbg::step_error().empty() ? summa_msg(rc) : "this rank: " + cbg::step_error());
    return CBG_OK;
  });
}

int cbg_summa_spgemm_phased(cbg_grid* g, const cbg_tile* A, const cbg_tile* B, int64_t A_gncol, int64_t B_gnrow,
                            int sr, int algo, int exec, int phases, cbg_phase_fn fn, void* user, cbg_tile* C) {
  return cbg_summa_spgemm_memeff(g, A, B, A_gncol, B_gnrow, sr, algo, exec, phases, 0, fn, user, C);
}

int cbg_last_phase_plan(int* phases, int* automatic, int64_t* flops, int64_t* nnz_est, double* c_budget_bytes,
                        int* oom_splits, double* plan_ms) {
  const cbg::PhasePlan& p = cbg::phase_plan();
  if (phases) *phases = p.phases;
  if (automatic) *automatic = p.automatic;
  if (flops) *flops = p.flops;
  if (nnz_est) *nnz_est = p.nnz_est;
  if (c_budget_bytes) *c_budget_bytes = p.c_budget_bytes;
  if (oom_splits) *oom_splits = cbg::summa_info().oom_splits;
  if (plan_ms) *plan_ms = p.ms;
  return CBG_OK;
}

int cbg_grid_agree(cbg_grid* g, int local_rc, int* agreed) {
  if (!g || !agreed) return fail(CBG_ERR_INVALIDPARAMS, "grid or output is NULL");
  return guard([&] {
    *agreed = cbg::agree(g, local_rc);
    return CBG_OK;
  });
}

int cbg_last_summa_info(int* pieces, double* bcast_ms_piece0, double* est_hidden_ms, double* piece_cost_ms) {
  const cbg::SummaInfo& i = cbg::summa_info();
  if (pieces) *pieces = i.pieces;
  if (bcast_ms_piece0) *bcast_ms_piece0 = i.bcast_ms_piece0;
  if (est_hidden_ms) *est_hidden_ms = i.est_hidden_ms;
  if (piece_cost_ms) *piece_cost_ms = i.piece_cost_ms;
  return CBG_OK;
}

int cbg_last_summa_comm(int* rule, int64_t* bytes_recv, double* exposed_comm_ms) {
  const cbg::SummaInfo& i = cbg::summa_info();
  if (rule) *rule = i.rule;
  if (bytes_recv) *bytes_recv = i.bytes_recv;
  if (exposed_comm_ms) *exposed_comm_ms = i.exposed_comm_ms;
  return CBG_OK;
}

int cbg_merge_stats(int64_t* entries_in, int64_t* entries_out, double* ms) {
  const cbg::MergeStats& m = cbg::merge_stats();
  if (entries_in) *entries_in = m.entries_in;
  if (entries_out) *entries_out = m.entries_out;
  if (ms) *ms = m.ms;
  return CBG_OK;
}

int cbg_grid_info(const cbg_grid* g, int* rank, int* nranks, int* rows, int* cols, int* prow, int* pcol);

}  // extern "C"
