// cbg_summa.cpp -- 2D Sparse SUMMA over RCCL (xGMI), one process per GPU.
//
// Replaces, for the SpGEMM path:
//   CommGrid (reference src/CommGrid.cpp:37-75; rank -> (rank / cols, rank % cols),
//             row/col communicators by MPI_Comm_split)       -> ncclCommInitRank + ncclCommSplit
//   ProductGrid (CommGrid.cpp:164-180)                        -> grid reuse (no per-call dup)
//   SpParHelper::GetSetSizes (SpParHelper.cpp:797-809)        -> one allgather of {m,n,nnz,nzc}
//   SpParHelper::BCastMatrix (SpParHelper.cpp:582-600)        -> 4 x ncclBroadcast in a group
//   Mult_AnXBn_DoubleBuff / Mult_AnXBn_Synch (ParFriends.h:798-1108)
//
// Two execution modes with identical results (up to fp summation order):
//   PANEL  : every rank gathers its A block row and B block column (the same
//            broadcasts as the SUMMA stages, issued back to back on the comm
//            stream), concatenates them in HBM and runs ONE local multiply.
//            No partial products, no merge (the reference's dominant cost,
//            69 % of DoubleBuff at 1x1).  Works on any pr x pc grid because
//            the inner coordinates are global.
//            The B block column arrives in column pieces: the broadcast of
//            piece p+1 runs on the comm stream while piece p multiplies on
//            the compute stream (double buffering), and the pieces' C entries
//            are written end to end into one growable arena (no copy).
//   STAGED : the reference's stage structure (sqrt(P) stages for Synch,
//            2 sqrt(P) half-tile stages for DoubleBuff on square grids),
//            generalized to pr x pc grids by cutting the inner dimension at
//            the union of A's column-block and B's row-block boundaries; the
//            broadcast of stage s+1 runs on the comm stream while stage s
//            multiplies on the compute stream; partial products are merged
//            on device (cbg_merge.hip, 64-bit entry counts).
//
// Failure semantics.  The reference MPI_Aborts the whole job on a failed
// check (ParFriends.h:160-183, SpDefs.h:69-76).  Here every collective entry
// point agrees on a return code: after each local step the ranks take the
// maximum of their codes over the world (agree()), so a rank-local failure
// (an OOM inside the local multiply, a receive buffer that cannot be
// allocated, a HIP error) makes every rank leave the call with that code,
// after the collectives already posted have drained, instead of the others
// blocking in the next broadcast.  Communicator failures (an RCCL async
// error, or no progress for CBG_COMM_TIMEOUT_S seconds, default 600) abort
// the grid's communicators (ncclCommAbort); the grid is then unusable and
// every later call returns CBG_ERR_RCCL.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <thread>

#include "cbg_internal.h"

namespace cbg {

struct RcclError : std::runtime_error {
  explicit RcclError(const std::string& s) : std::runtime_error(s) {}
};
#define CBG_NCCL(x)                                                                                   \
  do {                                                                                                \
    ncclResult_t r_ = (x);                                                                            \
    if (r_ != ncclSuccess)                                                                            \
      throw ::cbg::HipError(std::string(#x) + ": " + ncclGetErrorString(r_), CBG_ERR_RCCL);           \
  } while (0)

}  // namespace cbg

struct cbg_grid {
  int rank = 0, nranks = 1, pr = 1, pc = 1, prow = 0, pcol = 0;
  bool host_mode = false;
  cbg_host_comm hc{};
  ncclComm_t world = nullptr, row = nullptr, col = nullptr;
  hipStream_t compute = nullptr, comm = nullptr;
  hipEvent_t ev_comm = nullptr;
  hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;  // timing of the first piece's broadcast
  bool broken = false;  // communicators aborted: every later collective fails
  int64_t calls = 0;    // SUMMA calls made on this grid (fault-injection index)
  int64_t redist_calls = 0;  // Transpose / BlockSplit calls (CBG_FAULT_INJECT_REDIST index)
  bool fault_armed = false;
};

namespace cbg {

enum { COMM_WORLD = 0, COMM_ROW = 1, COMM_COL = 2 };

static ncclComm_t pick(cbg_grid* g, int which) {
  return which == COMM_ROW ? g->row : which == COMM_COL ? g->col : g->world;
}
static int comm_size(cbg_grid* g, int which) { return which == COMM_ROW ? g->pc : which == COMM_COL ? g->pr : g->nranks; }
static int comm_rank(cbg_grid* g, int which) { return which == COMM_ROW ? g->pcol : which == COMM_COL ? g->prow : g->rank; }

void grid_setup_streams(cbg_grid* g) {
  CBG_HIP(hipStreamCreateWithFlags(&g->compute, hipStreamNonBlocking));
  CBG_HIP(hipStreamCreateWithFlags(&g->comm, hipStreamNonBlocking));
  CBG_HIP(hipEventCreateWithFlags(&g->ev_comm, hipEventDisableTiming));
  CBG_HIP(hipEventCreate(&g->ev_t0));
  CBG_HIP(hipEventCreate(&g->ev_t1));
}

int grid_shape(int nranks, int& rows, int& cols) {
  if (rows == 0 && cols == 0) {  // CommGrid.cpp:44-53: square or NOTSQUARE
    int r = 1;
    while ((r + 1) * (r + 1) <= nranks) ++r;
    if (r * r != nranks) return CBG_ERR_NOTSQUARE;
    rows = cols = r;
  }
  if (rows <= 0 || cols <= 0 || rows * cols != nranks) return CBG_ERR_INVALIDPARAMS;
  return CBG_OK;
}

cbg_grid* grid_create_rccl(int rank, int nranks, int rows, int cols, const void* uid) {
  std::unique_ptr<cbg_grid> g(new cbg_grid());
  g->rank = rank;
  g->nranks = nranks;
  g->pr = rows;
  g->pc = cols;
  g->prow = rank / cols;
  g->pcol = rank % cols;
  grid_setup_streams(g.get());
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  CBG_NCCL(ncclCommInitRank(&g->world, nranks, id, rank));
  CBG_NCCL(ncclCommSplit(g->world, g->prow, g->pcol, &g->row, nullptr));  // row comm: rank = pcol
  CBG_NCCL(ncclCommSplit(g->world, g->pcol, g->prow, &g->col, nullptr));  // col comm: rank = prow
  return g.release();
}

cbg_grid* grid_create_host(int rank, int nranks, int rows, int cols, const cbg_host_comm* hc) {
  std::unique_ptr<cbg_grid> g(new cbg_grid());
  g->rank = rank;
  g->nranks = nranks;
  g->pr = rows;
  g->pc = cols;
  g->prow = rank / cols;
  g->pcol = rank % cols;
  g->host_mode = true;
  g->hc = *hc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
    grid_setup_streams(g.get());
  } else {
    (void)hipGetLastError();  // no device: only the host collectives (agree, barrier) are usable
  }
  return g.release();
}

void grid_destroy(cbg_grid* g) {
  if (!g) return;
  if (g->row) ncclCommDestroy(g->row);
  if (g->col) ncclCommDestroy(g->col);
  if (g->world) ncclCommDestroy(g->world);
  if (g->compute) (void)hipStreamDestroy(g->compute);
  if (g->comm) (void)hipStreamDestroy(g->comm);
  if (g->ev_comm) (void)hipEventDestroy(g->ev_comm);
  if (g->ev_t0) (void)hipEventDestroy(g->ev_t0);
  if (g->ev_t1) (void)hipEventDestroy(g->ev_t1);
  delete g;
}

// ---------------------------------------------------------------------------
// collectives
// ---------------------------------------------------------------------------
static void host_check(cbg_grid* g, int rc, const char* what) {
  if (rc != 0) {
    g->broken = true;  // a peer is gone or the transport failed: no later call can agree
    throw HipError(std::string("host transport ") + what + " failed", CBG_ERR_RCCL);
  }
}

static double comm_timeout_s() {
  static const char* e = getenv("CBG_COMM_TIMEOUT_S");
  const double t = e ? atof(e) : 600.0;
  return t > 0 ? t : 600.0;
}

// ncclCommAbort on every communicator of the grid (pending operations are
// cancelled); the grid is unusable afterwards
static void abort_comms(cbg_grid* g) {
  for (ncclComm_t* c : {&g->row, &g->col, &g->world})
    if (*c) {
      (void)ncclCommAbort(*c);
      *c = nullptr;
    }
  g->broken = true;
}

static void check_usable(cbg_grid* g) {
  if (g->broken) throw HipError("grid communicators were aborted after an earlier failure", CBG_ERR_RCCL);
}

// Wait for the comm stream (the caller's collectives) with a watchdog:
// an RCCL async error on any communicator, or no completion within
// CBG_COMM_TIMEOUT_S, aborts the communicators instead of hanging.
static void wait_comm(cbg_grid* g) {
  if (g->host_mode) {
    CBG_HIP(hipStreamSynchronize(g->comm));
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const double limit = comm_timeout_s();
  int spins = 0;
  for (;;) {
    hipError_t q = hipStreamQuery(g->comm);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) {
      (void)hipGetLastError();
      abort_comms(g);
      throw HipError(std::string("comm stream: ") + hipGetErrorString(q), CBG_ERR_HIP);
    }
    for (ncclComm_t c : {g->world, g->row, g->col}) {
      ncclResult_t ae = ncclSuccess;
      if (c && ncclCommGetAsyncError(c, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
        abort_comms(g);
        throw HipError(std::string("RCCL async error: ") + ncclGetErrorString(ae), CBG_ERR_RCCL);
      }
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > limit) {
      abort_comms(g);
      throw HipError("collective made no progress for " + std::to_string((int)limit) +
                         " s (CBG_COMM_TIMEOUT_S); communicators aborted",
                     CBG_ERR_RCCL);
    }
    if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(spins > 4096 ? 200 : 20));
  }
}

// allgather of n int64 per rank (host buffers)
void allgather_i64(cbg_grid* g, int which, const int64_t* in, int64_t* out, int n) {
  check_usable(g);
  const int P = comm_size(g, which);
  if (g->host_mode) {
    if (P == 1) {
      std::memcpy(out, in, sizeof(int64_t) * n);
      return;
    }
    host_check(g, g->hc.allgather(g->hc.user, which, in, out, sizeof(int64_t) * n), "allgather");
    return;
  }
  // RCCL: executed for one-rank communicators too (a 1x1 RCCL grid runs the same calls)
  DBuf<int64_t> d(P * n + n);
  CBG_HIP(hipMemcpyAsync(d.p + P * n, in, sizeof(int64_t) * n, hipMemcpyHostToDevice, g->comm));
  CBG_NCCL(ncclAllGather(d.p + P * n, d.p, n, ncclInt64, pick(g, which), g->comm));
  CBG_HIP(hipMemcpyAsync(out, d.p, sizeof(int64_t) * P * n, hipMemcpyDeviceToHost, g->comm));
  wait_comm(g);
}

// allgather of `bytes` bytes per rank (host buffers)
static void allgather_bytes(cbg_grid* g, int which, const void* in, void* out, size_t bytes) {
  check_usable(g);
  const int P = comm_size(g, which);
  if (bytes == 0) return;
  if (g->host_mode) {
    if (P == 1) {
      std::memcpy(out, in, bytes);
      return;
    }
    host_check(g, g->hc.allgather(g->hc.user, which, in, out, bytes), "allgather");
    return;
  }
  DBuf<char> d((size_t)(P + 1) * bytes);
  CBG_HIP(hipMemcpyAsync(d.p + P * bytes, in, bytes, hipMemcpyHostToDevice, g->comm));
  CBG_NCCL(ncclAllGather(d.p + P * bytes, d.p, bytes, ncclInt8, pick(g, which), g->comm));
  CBG_HIP(hipMemcpyAsync(out, d.p, (size_t)P * bytes, hipMemcpyDeviceToHost, g->comm));
  wait_comm(g);
}

// allgather of `bytes` bytes per rank of DEVICE buffers (stream-ordered on the
// comm stream and waited for); the host transport stages through host memory
static void allgather_device(cbg_grid* g, int which, const void* in, void* out, size_t bytes) {
  check_usable(g);
  if (bytes == 0) return;
  const int P = comm_size(g, which);
  if (P == 1) {
    CBG_HIP(hipMemcpy(out, in, bytes, hipMemcpyDeviceToDevice));
    return;
  }
  if (g->host_mode) {
    std::vector<char> h(bytes), all((size_t)P * bytes);
    CBG_HIP(hipMemcpy(h.data(), in, bytes, hipMemcpyDeviceToHost));
    allgather_bytes(g, which, h.data(), all.data(), bytes);
    CBG_HIP(hipMemcpy(out, all.data(), all.size(), hipMemcpyHostToDevice));
    return;
  }
  CBG_NCCL(ncclAllGather(in, out, bytes, ncclInt8, pick(g, which), g->comm));
  wait_comm(g);
}

void allreduce_f64(cbg_grid* g, double* v, bool max) {
  check_usable(g);
  if (g->host_mode) {
    if (g->nranks == 1) return;
    std::vector<double> all(g->nranks);
    host_check(g, g->hc.allgather(g->hc.user, COMM_WORLD, v, all.data(), sizeof(double)), "allgather");
    double r = all[0];
    for (double x : all) r = max ? std::max(r, x) : r + x;
    *v = r;
    return;
  }
  DBuf<double> d(1);
  CBG_HIP(hipMemcpyAsync(d.p, v, sizeof(double), hipMemcpyHostToDevice, g->comm));
  CBG_NCCL(ncclAllReduce(d.p, d.p, 1, ncclFloat64, max ? ncclMax : ncclSum, g->world, g->comm));
  CBG_HIP(hipMemcpyAsync(v, d.p, sizeof(double), hipMemcpyDeviceToHost, g->comm));
  wait_comm(g);
}

void allreduce_sum_i64(cbg_grid* g, int64_t* v) {
  std::vector<int64_t> all(g->nranks);
  allgather_i64(g, COMM_WORLD, v, all.data(), 1);
  int64_t s = 0;
  for (auto x : all) s += x;
  *v = s;
}

void barrier(cbg_grid* g) {
  double z = 0;
  allreduce_f64(g, &z, true);
}

// The agreed code of a collective step: max over the world of the ranks'
// local codes (0 = success).  Every rank calls it at the same points, so a
// failed rank never leaves its peers blocked in a broadcast it skipped.
int agree(cbg_grid* g, int rc) {
  int64_t v = rc, w = 0;
  std::vector<int64_t> all(g->nranks);
  allgather_i64(g, COMM_WORLD, &v, all.data(), 1);
  for (auto x : all) w = std::max(w, x);
  return (int)w;
}
// agree() that also reduces one value over the world: *vmin / *vmax receive
// its minimum / maximum (one allgather, the same point of the protocol)
static int agree_val(cbg_grid* g, int rc, int64_t val, int64_t* vmin, int64_t* vmax) {
  int64_t v[2] = {rc, val};
  std::vector<int64_t> all((size_t)2 * g->nranks);
  allgather_i64(g, COMM_WORLD, v, all.data(), 2);
  int64_t w = 0, lo = val, hi = val;
  for (int r = 0; r < g->nranks; ++r) {
    w = std::max(w, all[2 * r]);
    lo = std::min(lo, all[2 * r + 1]);
    hi = std::max(hi, all[2 * r + 1]);
  }
  if (vmin) *vmin = lo;
  if (vmax) *vmax = hi;
  return (int)w;
}

// Test hook (CBG_FAULT_INJECT="rank:k1,k2,..."): in the listed SUMMA calls
// that rank `rank` makes on a grid (counted from 0 over the grid's life), the
// first local multiply fails as an out-of-memory would.
static void arm_fault(cbg_grid* g) {
  static const char* e = getenv("CBG_FAULT_INJECT");
  const int64_t k = g->calls++;
  g->fault_armed = false;
  if (!e) return;
  const char* c = strchr(e, ':');
  if (!c || atoi(e) != g->rank) return;
  for (const char* q = c + 1; *q;) {
    char* end = nullptr;
    const long long at = strtoll(q, &end, 10);
    if (end == q) break;
    if (at == k) g->fault_armed = true;
    q = *end == ',' ? end + 1 : end;
  }
}
static void maybe_inject_fault(cbg_grid* g) {
  if (!g->fault_armed) return;
  g->fault_armed = false;
  throw HipError("injected fault (CBG_FAULT_INJECT) in SUMMA call " + std::to_string(g->calls - 1), CBG_ERR_OOM);
}
// the same for the redistributions (Transpose, BlockSplit):
// CBG_FAULT_INJECT_REDIST="rank:k1,k2,..." counts their calls on a grid, and
// the listed calls of that rank fail their receive-buffer allocation as an
// out-of-memory would
static bool redist_fault(cbg_grid* g) {
  static const char* e = getenv("CBG_FAULT_INJECT_REDIST");
  const int64_t k = g->redist_calls++;
  if (!e) return false;
  const char* c = strchr(e, ':');
  if (!c || atoi(e) != g->rank) return false;
  for (const char* q = c + 1; *q;) {
    char* end = nullptr;
    const long long at = strtoll(q, &end, 10);
    if (end == q) break;
    if (at == k) return true;
    q = *end == ',' ? end + 1 : end;
  }
  return false;
}

// code of a failure inside a collective step (the step's exception is not
// rethrown: the caller must still reach the next agree()); the first message
// of the calling thread is kept for cbg_last_error()
std::string& step_error() {
  static thread_local std::string m;
  return m;
}
template <class F>
static int step(F&& f) {
  try {
    f();
    return CBG_OK;
  } catch (const HipError& e) {
    if (std::getenv("CBG_DEBUG_ERRORS")) std::fprintf(stderr, "[cbg] %s\n", e.what());
    if (step_error().empty()) step_error() = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    if (step_error().empty()) step_error() = "host allocation failed";
    return CBG_ERR_OOM;
  } catch (const std::exception& e) {  // anything else still reaches the next agree()
    if (step_error().empty()) step_error() = e.what();
    return CBG_ERR_HIP;
  }
}

// Broadcast a tile within a row/col communicator (BCastMatrix: the essentials
// {m,n,nnz,nzc} are known from the allgather; Create(ess) then 4 broadcasts).
// `t` is the root's tile on the root and an allocated receive tile elsewhere.
// RCCL: enqueued on g->comm (callers group the broadcasts of one step and
// order the consumer with g->ev_comm); host transport: synchronous.
static void bcast_tile(cbg_grid* g, int which, int root, const int64_t ess[4], cbg_tile& t, bool mine) {
  const int64_t nnz = ess[2], nzc = ess[3];
  if (g->host_mode) {
    if (comm_size(g, which) == 1) return;
    CBG_HIP(hipStreamSynchronize(g->comm));
    auto hb = [&](void* dptr, size_t bytes) {
      if (bytes == 0) return;
      std::vector<char> h(bytes);
      if (mine) CBG_HIP(hipMemcpy(h.data(), dptr, bytes, hipMemcpyDeviceToHost));
      host_check(g, g->hc.bcast(g->hc.user, which, h.data(), bytes, root), "bcast");
      if (!mine) CBG_HIP(hipMemcpy(dptr, h.data(), bytes, hipMemcpyHostToDevice));
    };
    hb(t.cp, sizeof(int64_t) * (nzc + 1));
    hb(t.jc, sizeof(int32_t) * nzc);
    hb(t.ir, sizeof(int32_t) * nnz);
    hb(t.val, sizeof(double) * nnz);
    return;
  }
  // RCCL, one-rank communicators included
  ncclComm_t c = pick(g, which);
  CBG_NCCL(ncclBroadcast(t.cp, t.cp, nzc + 1, ncclInt64, root, c, g->comm));
  if (nzc) CBG_NCCL(ncclBroadcast(t.jc, t.jc, nzc, ncclInt32, root, c, g->comm));
  if (nnz) {
    CBG_NCCL(ncclBroadcast(t.ir, t.ir, nnz, ncclInt32, root, c, g->comm));
    CBG_NCCL(ncclBroadcast(t.val, t.val, nnz, ncclFloat64, root, c, g->comm));
  }
}

// one step's broadcasts as one RCCL group
template <class F>
static void bcast_group(cbg_grid* g, F&& f) {
  if (!g->host_mode) CBG_NCCL(ncclGroupStart());
  try {
    f();
  } catch (...) {
    if (!g->host_mode) (void)ncclGroupEnd();
    throw;
  }
  if (!g->host_mode) CBG_NCCL(ncclGroupEnd());
}

static void tile_ess(const cbg_tile& t, int64_t e[4]) {
  e[0] = t.m;
  e[1] = t.n;
  e[2] = t.nnz;
  e[3] = t.nzc;
}

static void alloc_like(cbg_tile& t, const int64_t e[4]) { tile_alloc_device(t, e[0], e[1], e[2], e[3]); }

// ---------------------------------------------------------------------------
// PANEL (pipelined): Mult_AnXBn_DoubleBuff / _Synch as ONE local multiply of
// the A block row by the B block column (ParFriends.h:845-964 computes the
// same sum of stage products), the B block column arriving in column pieces
// cuts[0] = 0 < cuts[1] < ... < cuts[np] = B.n.  Comm stream, every rank in
// the same order: [A row broadcasts][piece 0][agree][piece 1][agree]...;
// the compute stream multiplies piece p while piece p+1 is broadcast.
// fn != NULL: each piece's C goes to fn and is freed (MemEfficientSpGEMM
// phases); else the pieces' entries go end to end into one EntryArena and C
// is their column concatenation (ColConcatenate without a copy).
// ---------------------------------------------------------------------------
static int64_t tile_bytes(const int64_t e[4]) { return 8 * (e[3] + 1) + 4 * e[3] + 12 * e[2]; }

SummaInfo& summa_info() {
  static thread_local SummaInfo s;
  return s;
}

// extra local multiply an additional pipeline piece costs (CBG_PIPELINE_MIN_MS):
// measured 2.5-3.0 ms on scale-22 rank tiles of 2x2 and 4x2 grids (68-132 ms)
static double pipeline_min_ms() {
  static const char* e = getenv("CBG_PIPELINE_MIN_MS");
  return e ? atof(e) : 3.0;
}
// ... and on larger tiles a share of the rank's multiply (CBG_PIPELINE_COST_FRAC,
// default 0.04: 1-7 % measured on the scale-22 2x1 rank tiles of 258 ms), taken
// from this thread's previous adaptive PANEL call (the same product repeated)
static thread_local double g_last_panel_ms = 0.0;
static double pipeline_cost_ms() {
  static const char* e = getenv("CBG_PIPELINE_COST_FRAC");
  static const double frac = e ? atof(e) : 0.04;
  return std::max(pipeline_min_ms(), frac * g_last_panel_ms);
}

// One phase's local multiply handed to fn (MemEfficientSpGEMM with a phase
// consumer).  A phase whose C does not fit the device -- the multiply learns
// nnz(C) from its symbolic pass and its allocation fails with CBG_ERR_OOM
// before any output is written -- is computed as two column halves of its B
// piece, each handed to fn with the same phase index and its own column
// offset, so an underestimated phase count costs a repeated symbolic pass, not
// the job.  The split is local: the piece's B columns are already on this rank.
static void multiply_to_fn(const cbg_tile& A, const cbg_tile& B, int sr, hipStream_t cs, int p, int64_t off,
                           cbg_phase_fn fn, void* user, int& cb_rc, double& ms, int depth) {
  TileGuard Cp;
  LocalStats ls;
  try {
    local_spgemm(A, B, sr, Cp.t, cs, &ls, nullptr);
  } catch (const HipError& e) {
    if (e.code != CBG_ERR_OOM || B.n < 2 || depth >= 12) throw;
    pool().trim();
    summa_info().oom_splits++;
    const int64_t h = B.n / 2;
    for (int k = 0; k < 2; ++k) {
      TileGuard half;
      tile_slice_cols(B, k ? h : 0, k ? B.n : h, half.t, cs);
      multiply_to_fn(A, half.t, sr, cs, p, off + (k ? h : 0), fn, user, cb_rc, ms, depth + 1);
    }
    return;
  }
  ms += ls.ms_symbolic + ls.ms_numeric;
  CBG_HIP(hipStreamSynchronize(cs));
  const int r = fn(user, p, off, &Cp.t);
  if (r && !cb_rc) cb_rc = r;
}

// CUs the persistent slab kernels leave free while a broadcast is in flight
static int comm_reserve_default() { return 8; }

// one_phase: the cuts are pipeline pieces of ONE phase (fn gets phase 0 for
// each of them, at its column offset), else piece p is phase p
static int summa_panel(cbg_grid* g, const cbg_tile& A, const cbg_tile& B, int64_t A_gncol, int64_t B_gnrow, int sr,
                       const std::vector<int64_t>& cuts_in, cbg_phase_fn fn, void* user, cbg_tile* C,
                       bool adaptive = false, bool one_phase = false) {
  std::vector<int64_t> cuts = cuts_in;
  int np = (int)cuts.size() - 1;
  const int pr = g->pr, pc = g->pc;
  hipStream_t cs = g->compute;
  // my B pieces (column slices; the whole tile when np == 1)
  std::vector<TileGuard> own(np);
  std::vector<cbg_tile> piece(np);
  int rc = step([&] {
    for (int p = 0; p < np; ++p) {
      if (np == 1) {
        piece[p] = B;
      } else {
        tile_slice_cols(B, cuts[p], cuts[p + 1], own[p].t, cs);
        piece[p] = own[p].t;
      }
    }
  });
  if ((rc = agree(g, rc))) return rc;
  // GetSetSizes: A tiles along my grid row, every piece of the B tiles along my grid column
  int64_t ea[4];
  tile_ess(A, ea);
  std::vector<int64_t> eb((size_t)4 * np);
  for (int p = 0; p < np; ++p) tile_ess(piece[p], &eb[4 * p]);
  std::vector<int64_t> EA((size_t)4 * pc), EB((size_t)4 * np * pr);
  allgather_i64(g, COMM_ROW, ea, EA.data(), 4);
  allgather_i64(g, COMM_COL, eb.data(), EB.data(), 4 * np);
  auto eB = [&](int s, int p) { return &EB[(size_t)4 * (s * np + p)]; };
  int64_t kA = 0, kB = 0;
  for (int s = 0; s < pc; ++s) kA += EA[4 * s + 1];
  for (int s = 0; s < pr; ++s) kB += eB(s, 0)[0];
  if ((rc = agree(g, (kA != A_gncol || kB != B_gnrow) ? CBG_ERR_DIMMISMATCH : CBG_OK))) return rc;
  std::vector<int64_t> aoff(pc + 1, 0), boff(pr + 1, 0);
  for (int s = 0; s < pc; ++s) aoff[s + 1] = aoff[s] + EA[4 * s + 1];
  for (int s = 0; s < pr; ++s) boff[s + 1] = boff[s] + eB(s, 0)[0];

  std::vector<TileGuard> Ar(pc);
  std::vector<std::vector<TileGuard>> Bc(np);
  for (auto& v : Bc) v.resize(pr);
  auto alloc_piece = [&](int p) {
    for (int s = 0; s < pr; ++s)
      if (s != g->prow) alloc_like(Bc[p][s].t, eB(s, p));
  };
  auto post_piece = [&](int p) {
    bcast_group(g, [&] {
      for (int s = 0; s < pr; ++s)
        bcast_tile(g, COMM_COL, s, eB(s, p), s == g->prow ? piece[p] : Bc[p][s].t, s == g->prow);
    });
    CBG_HIP(hipEventRecord(g->ev_comm, g->comm));
  };
  rc = step([&] {
    for (int s = 0; s < pc; ++s)
      if (s != g->pcol) alloc_like(Ar[s].t, &EA[4 * s]);
    alloc_piece(0);
  });
  if ((rc = agree(g, rc))) return rc;
  // from here on every rank has posted the same broadcasts: errors are
  // recorded, agreed on at the next step, and the comm stream is drained
  SummaInfo& info = summa_info();
  info = SummaInfo{};
  info.pieces = np;
  // bytes this rank receives: the remote A tiles of its grid row and the remote
  // B tiles (all pieces) of its grid column
  int64_t bytes_a = 0, bytes_b0 = 0, bytes_b1 = 0;
  for (int s = 0; s < pc; ++s)
    if (s != g->pcol) bytes_a += tile_bytes(&EA[4 * s]);
  for (int s = 0; s < pr; ++s)
    if (s != g->prow)
      for (int p = 0; p < np; ++p) (p == 0 ? bytes_b0 : bytes_b1) += tile_bytes(eB(s, p));
  info.bytes_recv = bytes_a + bytes_b0 + bytes_b1;
  double host_ms0 = 0.0;
  // the A block row's gather and B piece 0 in ONE broadcast group (their
  // transfers overlap on the row and column links); piece 0's multiply waits
  // for both
  int local = step([&] {
    CBG_HIP(hipEventRecord(g->ev_t0, g->comm));
    const auto h0 = std::chrono::steady_clock::now();
    bcast_group(g, [&] {
      for (int s = 0; s < pc; ++s) {
        cbg_tile& t = s == g->pcol ? const_cast<cbg_tile&>(A) : Ar[s].t;
        bcast_tile(g, COMM_ROW, s, &EA[4 * s], t, s == g->pcol);
      }
      for (int s = 0; s < pr; ++s)
        bcast_tile(g, COMM_COL, s, eB(s, 0), s == g->prow ? piece[0] : Bc[0][s].t, s == g->prow);
    });
    CBG_HIP(hipEventRecord(g->ev_comm, g->comm));
    CBG_HIP(hipEventRecord(g->ev_t1, g->comm));
    host_ms0 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
  });
  // Double buffering (PANEL with the default two pieces on a grid).  On RCCL
  // grids whose B block column has more than one remote tile (pr >= 3) piece 1
  // is always broadcast while piece 0 multiplies (rule 1).  Otherwise
  // (one remote B tile, or the host transport) adaptively: the first group's
  // measured time (A gather + piece 0, 1/8 of B's columns), scaled to the
  // rest's bytes, is the transfer that pipelining would hide behind piece 0's
  // multiply; an extra piece costs about pipeline_cost_ms() of compute, so the
  // ranks keep the two pieces only when the hidden transfer is larger (rule 2,
  // agreed over the grid: every rank cuts its B tile alike); otherwise the
  // rest is broadcast at once and the pieces are rejoined into one multiply
  // (rule 3).
  if (np == 2 && adaptive && !g->host_mode && pr >= 3) info.rule = 1;
  // several pieces without the adaptive decision (CBG_PIPELINE, or the phases
  // of MemEfficientSpGEMM given as pieces): a fixed pipeline (rule 4)
  if (np > 1 && !adaptive) info.rule = 4;
  if (adaptive && np == 2 && !local && info.rule == 0) {
    float ms0 = 0.f;
    local = step([&] {
      wait_comm(g);
      if (g->host_mode) ms0 = (float)host_ms0;
      else CBG_HIP(hipEventElapsedTime(&ms0, g->ev_t0, g->ev_t1));
    });
    const int64_t b0 = bytes_a + bytes_b0, b1 = bytes_b1;
    const double hidden = b0 > 0 ? ms0 * (double)b1 / (double)b0 : 0.0;
    info.bcast_ms_piece0 = ms0;
    info.est_hidden_ms = hidden;
    info.piece_cost_ms = pipeline_cost_ms();
    const int want = hidden > info.piece_cost_ms ? 1 : 0;
    const int dec = agree(g, local ? local : want);  // codes >= 3001 are failures
    info.rule = dec == 1 ? 2 : 3;
    if (dec > 1) {
      rc = dec;
    } else if (dec == 0) {
      local = step([&] { alloc_piece(1); });
      if (!(rc = agree(g, local))) {
        local = step([&] {
          post_piece(1);
          wait_comm(g);  // the rest arrives now (its transfer is cheaper than a piece)
          for (int s = 0; s < pr; ++s) {
            const bool me = s == g->prow;
            std::vector<cbg_tile> parts = {me ? piece[0] : Bc[0][s].t, me ? piece[1] : Bc[1][s].t};
            TileGuard joined;
            tile_concat_cols(parts, {0, cuts[1]}, eB(s, 0)[0], cuts[2], joined.t, cs);
            if (me) {
              own[0] = std::move(joined);
              piece[0] = own[0].t;
              tile_free_device(own[1].t);
            } else {
              Bc[0][s] = std::move(joined);
              tile_free_device(Bc[1][s].t);
            }
          }
          CBG_HIP(hipEventRecord(g->ev_comm, g->comm));
        });
        np = 1;
        cuts = {0, cuts[2]};
        info.pieces = 1;
      }
    }
  }
  APrepScope aprep_scope;  // every piece multiplies the same A panel: keep its column maps
  std::unique_ptr<EntryArena> arena;
  if (!fn && np > 1) arena.reset(new EntryArena());
  std::vector<TileGuard> outs;
  std::vector<cbg_tile> outv;
  TileGuard Apanel;
  const cbg_tile* Ause = &A;
  int cb_rc = 0;
  double panel_ms = 0.0;
  // exposed communication: the compute stream's wait for each piece's broadcast
  // (an event before and after the wait; ~0 when the broadcast finished first)
  std::vector<hipEvent_t> wev;
  struct EvFree {
    std::vector<hipEvent_t>& v;
    ~EvFree() {
      for (auto e : v) (void)hipEventDestroy(e);
    }
  } wev_free{wev};
  for (int p = 0; p < np && !rc; ++p) {
    local = std::max(local, step([&] {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      CBG_HIP(hipEventCreate(&e0));
      wev.push_back(e0);
      CBG_HIP(hipEventCreate(&e1));
      wev.push_back(e1);
      CBG_HIP(hipEventRecord(e0, cs));
      CBG_HIP(hipStreamWaitEvent(cs, g->ev_comm, 0));
      CBG_HIP(hipEventRecord(e1, cs));
    }));
    if (p + 1 < np) {
      // every rank holds piece p+1's receive buffers before anyone posts it
      local = std::max(local, step([&] { alloc_piece(p + 1); }));
      if ((rc = agree(g, local))) break;
      local = std::max(local, step([&] { post_piece(p + 1); }));
    }
    if (local) continue;  // agreed at the next step
    local = step([&] {
      maybe_inject_fault(g);
      // piece p+1's broadcast runs on the comm stream during this multiply:
      // the persistent kernels leave comm_reserve_default() (8) CUs to it
      CommReserve reserve(p + 1 < np && !g->host_mode ? comm_reserve_default() : 0);
      if (p == 0 && pc > 1) {
        std::vector<cbg_tile> parts(pc);
        for (int s = 0; s < pc; ++s) parts[s] = s == g->pcol ? A : Ar[s].t;
        tile_concat_cols(parts, std::vector<int64_t>(aoff.begin(), aoff.end() - 1), A.m, A_gncol, Apanel.t, cs);
        for (auto& t : Ar) tile_free_device(t.t);
        Ause = &Apanel.t;
      }
      TileGuard Bp;
      const cbg_tile* Buse = &piece[p];
      if (pr > 1) {
        std::vector<cbg_tile> parts(pr);
        for (int s = 0; s < pr; ++s) parts[s] = s == g->prow ? piece[p] : Bc[p][s].t;
        tile_concat_rows(parts, std::vector<int64_t>(boff.begin(), boff.end() - 1), B_gnrow, cuts[p + 1] - cuts[p],
                         Bp.t, cs);
        Buse = &Bp.t;
      }
      if (fn) {
        multiply_to_fn(*Ause, *Buse, sr, cs, one_phase ? 0 : p, cuts[p], fn, user, cb_rc, panel_ms, 0);
        for (auto& t : Bc[p]) tile_free_device(t.t);
        tile_free_device(own[p].t);
      } else {
        TileGuard Cp;
        LocalStats ls;
        local_spgemm(*Ause, *Buse, sr, Cp.t, cs, &ls, arena.get());
        panel_ms += ls.ms_symbolic + ls.ms_numeric;
        for (auto& t : Bc[p]) tile_free_device(t.t);
        tile_free_device(own[p].t);
        outv.push_back(Cp.t);
        outs.push_back(std::move(Cp));
      }
    });
  }
  if (!rc) rc = agree(g, local);
  if (!rc && adaptive) g_last_panel_ms = panel_ms;
  if (!rc) {
    double exposed = 0.0;
    for (size_t k = 0; k + 1 < wev.size(); k += 2) {
      float ms = 0.f;
      if (hipEventSynchronize(wev[k + 1]) == hipSuccess && hipEventElapsedTime(&ms, wev[k], wev[k + 1]) == hipSuccess)
        exposed += ms;
      else
        (void)hipGetLastError();
    }
    info.exposed_comm_ms = exposed;
  }
  if (rc) {
    if (!g->broken) wait_comm(g);  // posted broadcasts complete before their buffers are released
    return rc;
  }
  if (fn) return agree(g, cb_rc ? CBG_ERR_INVALIDPARAMS : CBG_OK);
  rc = step([&] {
    if (np == 1) {
      *C = outs[0].release();
    } else {
      std::vector<int64_t> off(cuts.begin(), cuts.end() - 1);
      tile_assemble_cols(outv, off, A.m, B.n, *arena, *C, cs);
    }
  });
  return agree(g, rc);
}

// ---------------------------------------------------------------------------
// STAGED: the reference's stages (ParFriends.h:845-964 DoubleBuff: A split by
// columns at n/2 and B by rows at m/2, 2 sqrt(P) stages; :1004-1108 Synch:
// sqrt(P) stages), generalized to pr x pc grids: the inner dimension is cut
// at the union of A's column-block and B's row-block boundaries (lcm(pr, pc)
// ranges for power-of-two grids), DoubleBuff halves every range and runs all
// first halves before all second halves.  Stage s+1's broadcasts are posted
// before stage s multiplies; the partials are merged on device (MergeAll /
// MultiwayMerge, 64-bit entry counts).  On square grids the stages, their
// roots and their pieces are exactly the reference's.
// ---------------------------------------------------------------------------
static int summa_staged(cbg_grid* g, const cbg_tile& A, const cbg_tile& B, int64_t A_gncol, int64_t B_gnrow, int sr,
                        int algo, cbg_tile& C) {
  const int pr = g->pr, pc = g->pc;
  hipStream_t cs = g->compute;
  const int64_t K = A_gncol;
  auto blk = [](int64_t ext, int np_, int i) {  // SpParMat::Owner block start
    return i >= np_ ? ext : (int64_t)i * (ext / np_);
  };
  std::vector<int64_t> bnd;
  for (int s = 0; s <= pc; ++s) bnd.push_back(blk(K, pc, s));
  for (int s = 0; s <= pr; ++s) bnd.push_back(blk(K, pr, s));
  std::sort(bnd.begin(), bnd.end());
  bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
  struct Stage {
    int64_t lo, hi;
    int sa, sb;
  };
  auto owner = [&](int64_t k, int np_) {  // block of inner index k
    int s = (int)std::min<int64_t>(np_ - 1, K / np_ ? k / (K / np_) : np_ - 1);
    while (s > 0 && blk(K, np_, s) > k) --s;
    while (s + 1 < np_ && blk(K, np_, s + 1) <= k) ++s;
    return s;
  };
  std::vector<Stage> st;
  for (int half = 0; half < (algo == CBG_DOUBLEBUFF ? 2 : 1); ++half)
    for (size_t j = 0; j + 1 < bnd.size(); ++j) {
      int64_t lo = bnd[j], hi = bnd[j + 1];
      if (hi <= lo) continue;
      const int sa = owner(lo, pc), sb = owner(lo, pr);
      if (algo == CBG_DOUBLEBUFF) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (half == 0) hi = mid; else lo = mid;
      }
      st.push_back({lo, hi, sa, sb});
    }
  const int S = (int)st.size();
  // the stage slices below assume the block layout (SpParMat::Owner): my A
  // tile holds inner columns blk(K, pc, pcol) .. blk(K, pc, pcol + 1) and my
  // B tile the same rows of B's row blocks; a tile of another width would be
  // cut past its end or lose columns, so it is a dimension mismatch (agreed)
  const bool layout_ok = A.n == blk(K, pc, g->pcol + 1) - blk(K, pc, g->pcol) &&
                         B.m == blk(K, pr, g->prow + 1) - blk(K, pr, g->prow);
  int rc = agree(g, layout_ok ? CBG_OK : CBG_ERR_DIMMISMATCH);
  if (rc) return rc;
  // my pieces: A columns of the stages rooted at my grid column, B rows of those rooted at my grid row
  std::vector<TileGuard> myA(S), myB(S);
  rc = step([&] {
    for (int s = 0; s < S; ++s) {
      if (st[s].sa == g->pcol) {
        const int64_t o = blk(K, pc, st[s].sa);
        tile_slice_cols(A, st[s].lo - o, st[s].hi - o, myA[s].t, cs);
      }
      if (st[s].sb == g->prow) {
        const int64_t o = blk(K, pr, st[s].sb);
        tile_slice_rows(B, st[s].lo - o, st[s].hi - o, myB[s].t, cs);
      }
    }
  });
  if ((rc = agree(g, rc))) return rc;
  std::vector<int64_t> ea((size_t)4 * S, 0), eb((size_t)4 * S, 0);
  for (int s = 0; s < S; ++s) {
    tile_ess(myA[s].t, &ea[4 * s]);
    tile_ess(myB[s].t, &eb[4 * s]);
  }
  std::vector<int64_t> EA((size_t)4 * S * pc), EB((size_t)4 * S * pr);
  allgather_i64(g, COMM_ROW, ea.data(), EA.data(), 4 * S);  // GetSetSizes (ParFriends.h:834-835 / :1025-1026)
  allgather_i64(g, COMM_COL, eb.data(), EB.data(), 4 * S);
  auto eA = [&](int s) { return &EA[(size_t)4 * (st[s].sa * S + s)]; };
  auto eB = [&](int s) { return &EB[(size_t)4 * (st[s].sb * S + s)]; };
  int64_t kA = 0, kB = 0;
  for (int s = 0; s < S; ++s) {
    kA += eA(s)[1];
    kB += eB(s)[0];
  }
  if ((rc = agree(g, (kA != A_gncol || kB != B_gnrow) ? CBG_ERR_DIMMISMATCH : CBG_OK))) return rc;
  std::vector<TileGuard> Ar(S), Bc(S);
  auto alloc_stage = [&](int s) {
    if (st[s].sa != g->pcol) alloc_like(Ar[s].t, eA(s));
    if (st[s].sb != g->prow) alloc_like(Bc[s].t, eB(s));
  };
  auto post = [&](int s) {
    bcast_group(g, [&] {
      bcast_tile(g, COMM_ROW, st[s].sa, eA(s), st[s].sa == g->pcol ? myA[s].t : Ar[s].t, st[s].sa == g->pcol);
      bcast_tile(g, COMM_COL, st[s].sb, eB(s), st[s].sb == g->prow ? myB[s].t : Bc[s].t, st[s].sb == g->prow);
    });
    CBG_HIP(hipEventRecord(g->ev_comm, g->comm));
  };
  rc = step([&] { alloc_stage(0); });
  if ((rc = agree(g, rc))) return rc;
  int local = step([&] { post(0); });
  std::vector<TileGuard> partials;
  std::vector<cbg_tile> pv;
  for (int s = 0; s < S && !rc; ++s) {
    local = std::max(local, step([&] { CBG_HIP(hipStreamWaitEvent(cs, g->ev_comm, 0)); }));
    if (s + 1 < S) {
      local = std::max(local, step([&] { alloc_stage(s + 1); }));
      if ((rc = agree(g, local))) break;
      local = std::max(local, step([&] { post(s + 1); }));
    }
    if (local) continue;
    local = step([&] {
      maybe_inject_fault(g);
      CommReserve reserve(s + 1 < S && !g->host_mode ? comm_reserve_default() : 0);
      const cbg_tile& a = st[s].sa == g->pcol ? myA[s].t : Ar[s].t;
      const cbg_tile& b = st[s].sb == g->prow ? myB[s].t : Bc[s].t;
      TileGuard P;
      local_spgemm(a, b, sr, P.t, cs, nullptr);  // LocalHybridSpGEMM (ParFriends.h:888-891)
      tile_free_device(Ar[s].t);
      tile_free_device(Bc[s].t);
      tile_free_device(myA[s].t);
      tile_free_device(myB[s].t);
      if (P.t.nnz > 0) {
        pv.push_back(P.t);
        partials.push_back(std::move(P));
      }
    });
  }
  if (!rc) rc = agree(g, local);
  if (rc) {
    if (!g->broken) wait_comm(g);
    return rc;
  }
  // MergeAll (DoubleBuff, Friends.h:657-741) / MultiwayMerge (Synch, MultiwayMerge.h:409-526)
  rc = step([&] {
    if (pv.size() == 1) {
      C = partials[0].release();
    } else {
      merge_tiles(pv, A.m, B.n, sr, C, cs);
    }
  });
  return agree(g, rc);
}

// pieces of the pipelined PANEL multiply when C stays resident: the first
// piece small (its broadcast is exposed), the rest behind its multiply.
// CBG_PIPELINE=k: k equal pieces (1 = no pipelining); CBG_PIPELINE=1/d: two
// pieces, the first 1/d of B's columns; default: 1 piece without
// communication (one grid cell), else 1/8.
// The piece COUNT is a collective property (one broadcast group and one
// agree() per piece), so it is chosen from n_min, the narrowest B tile of the
// world (agreed by the caller): every rank cuts its own B tile into the same
// number of nonempty pieces, whatever the widths of the grid's column blocks.
static std::vector<int64_t> pipeline_cuts(cbg_grid* g, int64_t n, int64_t n_min) {
  static const char* e = getenv("CBG_PIPELINE");
  const bool comm = g->pr > 1;  // B tiles are broadcast only along grid columns of >1 rank
  if (n_min < 16) return {0, n};
  if (!e) return comm ? std::vector<int64_t>{0, n / 8, n} : std::vector<int64_t>{0, n};
  if (!strncmp(e, "1/", 2)) {
    const int64_t d = std::min<int64_t>(std::max(2, atoi(e + 2)), n_min);
    return {0, n / d, n};
  }
  int k = atoi(e);
  if (k <= 1) return {0, n};
  k = (int)std::min<int64_t>(k, n_min);
  std::vector<int64_t> c;
  for (int i = 0; i <= k; ++i) c.push_back((int64_t)i * n / k);
  return c;
}

// ---------------------------------------------------------------------------
// Mult_AnXBn_{DoubleBuff,Synch}
// ---------------------------------------------------------------------------
int summa_spgemm(cbg_grid* g, const cbg_tile& A, const cbg_tile& B, int64_t A_gncol, int64_t B_gnrow, int sr, int algo,
                 int exec, cbg_tile& C) {
  check_usable(g);
  arm_fault(g);
  // CheckSpGEMMCompliance (ParFriends.h:160-183), agreed over the grid, with
  // the narrowest B tile of the world (the pipeline's piece count)
  int rc = A_gncol != B_gnrow ? CBG_ERR_DIMMISMATCH
           : (&A == &B || (A.ir == B.ir && A.nnz > 0)) ? CBG_ERR_MATRIXALIAS
           : CBG_OK;
  int64_t n_min = 0;
  if ((rc = agree_val(g, rc, B.n, &n_min, nullptr))) return rc;
  if (exec == CBG_EXEC_PANEL) {
    const bool adaptive = !getenv("CBG_PIPELINE") && g->pr * g->pc > 1;
    return summa_panel(g, A, B, A_gncol, B_gnrow, sr, pipeline_cuts(g, B.n, n_min), nullptr, nullptr, &C, adaptive);
  }
  return summa_staged(g, A, B, A_gncol, B_gnrow, sr, algo, C);
}

// ---------------------------------------------------------------------------
// MemEfficientSpGEMM's phase count from memory (ParFriends.h:482-535, with
// EstPerProcessNnzSUMMA :1243-1341).  The reference estimates this rank's
// unmerged nnz(C) by a symbolic SUMMA (every tile broadcast once more) and
// divides the memory left after the inputs.  Here:
//  * flops of this rank's product C(prow, pcol) = sum over the inner index k
//    of nnz(A(:,k) in my grid row) * nnz(B(k,:) in my grid column), from the
//    column counts of A's tiles (allgathered along the grid row) and the row
//    counts of B's tiles (along the grid column): count vectors, not tiles;
//  * nnz(C) <= flops; the compression nnz/flops is measured by an exact
//    symbolic of a sample of the product (one rank: every 256th column of B, ~1/256
//    of a symbolic pass; a grid: every 8th row of the A block row times every
//    16th column of the B block column, gathered like the SUMMA's tiles) and the
//    estimate is flops x ratio x 1.1 -- only where the flops bound alone asks for
//    more than one phase on some rank;
//  * the C bytes a phase may take: CBG_PHASE_MEM_FRAC (0.6) of the memory left
//    after the tiles the SUMMA gathers -- perProcessMemory (GB, like the
//    reference) when given, else the device's free memory plus libcbg's pool
//    cache -- which leaves room for the symbolic bitmaps (<= 1/4 of the free
//    memory) and the per-column arrays;
//  * phases = ceil(12 B x nnz_est / budget), the maximum over the world (the
//    pieces are broadcast collectively), at most the narrowest B tile's width.
// A phase that still does not fit is split in column halves by multiply_to_fn.
// ---------------------------------------------------------------------------
PhasePlan& phase_plan() {
  static thread_local PhasePlan p;
  return p;
}

static double phase_mem_frac() {
  static const char* e = getenv("CBG_PHASE_MEM_FRAC");
  const double f = e ? atof(e) : 0.6;
  return f > 0 && f <= 1 ? f : 0.6;
}

static int plan_phases(cbg_grid* g, const cbg_tile& A, const cbg_tile& B, int64_t K, int64_t mem_gb, int64_t n_min,
                       int fallback, int& phases) {
  hipStream_t cs = g->compute;
  static const bool dbg = getenv("CBG_DEBUG_PLAN") != nullptr;
  const auto t_start = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (dbg)
      std::fprintf(stderr, "[cbg plan] %s at %.2f ms\n", what,
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
  };
  const int pr = g->pr, pc = g->pc;
  // widths of A's tiles along my grid row and heights of B's along my grid column
  std::vector<int64_t> WA(pc), HB(pr);
  allgather_i64(g, COMM_ROW, &A.n, WA.data(), 1);
  allgather_i64(g, COMM_COL, &B.m, HB.data(), 1);
  int64_t wmax = 0, hmax = 0, sa = 0, sb = 0;
  for (auto w : WA) wmax = std::max(wmax, w), sa += w;
  for (auto h : HB) hmax = std::max(hmax, h), sb += h;
  int rc = agree(g, (sa != K || sb != K) ? CBG_ERR_DIMMISMATCH : CBG_OK);
  if (rc) return rc;
  int64_t flops = 0;
  if (g->nranks == 1) {
    // one rank: the flops straight from A's column counts and B's entries
    DBuf<int32_t> ca(std::max<int64_t>(A.n, 1));
    rc = agree(g, step([&] {
      tile_counts_device(A, 0, ca.p, A.n, cs);
      flops = entry_sum_device(B, ca.p, cs);
    }));
  } else {
    // the count vectors, padded to the widest tile, gathered on the device
    DBuf<int32_t> ca(std::max<int64_t>(wmax, 1)), rb(std::max<int64_t>(hmax, 1));
    DBuf<int32_t> CA(std::max<int64_t>(wmax * pc, 1)), RB(std::max<int64_t>(hmax * pr, 1));
    rc = agree(g, step([&] { tile_counts_device(A, 0, ca.p, wmax, cs), tile_counts_device(B, 1, rb.p, hmax, cs); }));
    if (rc) return rc;
    mark("counts");
    allgather_device(g, COMM_ROW, ca.p, CA.p, sizeof(int32_t) * wmax);
    allgather_device(g, COMM_COL, rb.p, RB.p, sizeof(int32_t) * hmax);
    mark("count allgathers");
    rc = agree(g, step([&] {
      std::vector<int64_t> aoff(pc + 1, 0), boff(pr + 1, 0);
      for (int s = 0; s < pc; ++s) aoff[s + 1] = aoff[s] + WA[s];
      for (int s = 0; s < pr; ++s) boff[s + 1] = boff[s] + HB[s];
      flops = blocked_dot_device(CA.p, wmax, aoff, RB.p, hmax, boff, K, cs);
    }));
  }
  if (rc) return rc;
  mark("flops");
  // compression nnz/flops of a sample of this rank's product: one rank: every
  // 256th column of B; a grid: every 8th row of the A block row
  // times every 16th column of the B block column, the samples broadcast like
  // the SUMMA's tiles (1/8 and 1/16 of their bytes); ids, not positions, so the
  // tiles of a grid row / column sample the same rows / columns
  // (skipped, agreed, where the flops bound alone leaves one phase on every rank)
  auto tbytes = [](const cbg_tile& t) { return (double)(8 * (t.nzc + 1) + 4 * t.nzc + 12 * t.nnz); };
  const double gathered = (pc - 1) * tbytes(A) + (pr - 1) * tbytes(B);
  double avail;
  if (mem_gb > 0) {
    avail = (double)mem_gb * 1e9 - tbytes(A) - tbytes(B) - gathered;
  } else {
    size_t fr = 0, tot = 0;
    CBG_HIP(hipMemGetInfo(&fr, &tot));
    avail = (double)fr + (double)pool().bytes_cached() - gathered;
  }
  const double budget = phase_mem_frac() * avail;
  int64_t need_sample = 0;
  if ((rc = agree_val(g, CBG_OK, flops > 0 && 12.0 * (double)flops > budget ? 1 : 0, nullptr, &need_sample)))
    return rc;
  double ratio = 1.0;
  if (need_sample) {
    const int cstride = g->nranks == 1 ? 256 : 16;
    const int rstride = g->nranks == 1 ? 1 : 8;
    TileGuard As, Bs;
    rc = agree(g, step([&] {
      if (rstride > 1) tile_sample_rows(A, rstride, As.t, cs);
      tile_sample_cols(B, cstride, Bs.t, cs);
    }));
    if (rc) return rc;
    const cbg_tile& Amine = rstride > 1 ? As.t : A;
    int64_t ea[4], eb[4];
    tile_ess(Amine, ea);
    tile_ess(Bs.t, eb);
    std::vector<int64_t> EA((size_t)4 * pc), EB((size_t)4 * pr);
    allgather_i64(g, COMM_ROW, ea, EA.data(), 4);
    allgather_i64(g, COMM_COL, eb, EB.data(), 4);
    std::vector<TileGuard> Ar(pc), Bc(pr);
    rc = agree(g, step([&] {
      for (int q = 0; q < pc; ++q)
        if (q != g->pcol) alloc_like(Ar[q].t, &EA[4 * q]);
      for (int q = 0; q < pr; ++q)
        if (q != g->prow) alloc_like(Bc[q].t, &EB[4 * q]);
    }));
    if (rc) return rc;
    int64_t fs = 0, zs = 0;
    rc = agree(g, step([&] {
      bcast_group(g, [&] {
        for (int q = 0; q < pc; ++q)
          bcast_tile(g, COMM_ROW, q, &EA[4 * q], q == g->pcol ? const_cast<cbg_tile&>(Amine) : Ar[q].t, q == g->pcol);
      });
      bcast_group(g, [&] {
        for (int q = 0; q < pr; ++q) bcast_tile(g, COMM_COL, q, &EB[4 * q], q == g->prow ? Bs.t : Bc[q].t, q == g->prow);
      });
      wait_comm(g);
      TileGuard Ap, Bp;
      const cbg_tile* Au = &Amine;
      const cbg_tile* Bu = &Bs.t;
      if (pc > 1) {
        std::vector<cbg_tile> parts(pc);
        std::vector<int64_t> off(pc, 0);
        for (int q = 0; q < pc; ++q) {
          parts[q] = q == g->pcol ? Amine : Ar[q].t;
          if (q) off[q] = off[q - 1] + WA[q - 1];
        }
        tile_concat_cols(parts, off, Amine.m, K, Ap.t, cs);
        Au = &Ap.t;
      }
      if (pr > 1) {
        std::vector<cbg_tile> parts(pr);
        std::vector<int64_t> off(pr, 0);
        for (int q = 0; q < pr; ++q) {
          parts[q] = q == g->prow ? Bs.t : Bc[q].t;
          if (q) off[q] = off[q - 1] + HB[q - 1];
        }
        tile_concat_rows(parts, off, K, B.n, Bp.t, cs);
        Bu = &Bp.t;
      }
      local_symbolic(*Au, *Bu, cs, &fs, &zs);
    }));
    if (rc) return rc;
    if (fs > 0) ratio = std::min(1.0, 1.1 * (double)zs / (double)fs);
    mark("sample symbolic");
  }
  const double need = 12.0 * ratio * (double)flops;
  int64_t want = budget > 0 ? (int64_t)std::ceil(need / budget) : fallback;  // the reference keeps the given phases
  want = std::max<int64_t>(1, std::min<int64_t>(want, std::max<int64_t>(1, n_min)));
  int64_t agreed = 0;
  if ((rc = agree_val(g, CBG_OK, want, nullptr, &agreed))) return rc;
  phases = (int)agreed;
  PhasePlan& pp = phase_plan();
  pp.automatic = 1;
  pp.flops = flops;
  pp.nnz_est = (int64_t)(ratio * (double)flops);
  pp.c_budget_bytes = budget;
  pp.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  mark("planned");
  return CBG_OK;
}

// ---------------------------------------------------------------------------
// MemEfficientSpGEMM (ParFriends.h:449-730) minus its Markov-clustering pruning:
// B's local tile is cut into `phases` column pieces like SpDCCols::ColSplit
// (SpDCCols.cpp:936-970), each piece goes through the SUMMA, and the phase
// results are streamed to `fn` or column-concatenated (ColConcatenate,
// ParFriends.h:724-725).  Column pieces keep every C column's products inside
// one phase, so the result is identical to the unphased product.  PANEL: the
// phases are the pipeline's pieces (A's row panel is gathered once, phase
// p+1's B pieces are broadcast while phase p multiplies); STAGED: one staged
// SUMMA per phase.  phases <= 0 or mem_gb > 0: the count comes from
// plan_phases (perProcessMemory, ParFriends.h:482-535).
// ---------------------------------------------------------------------------
int summa_spgemm_phased(cbg_grid* g, const cbg_tile& A, const cbg_tile& B, int64_t A_gncol, int64_t B_gnrow, int sr,
                        int algo, int exec, int phases, int64_t mem_gb, cbg_phase_fn fn, void* user, cbg_tile* C) {
  check_usable(g);
  arm_fault(g);
  phase_plan() = PhasePlan{};
  summa_info() = SummaInfo{};
  // PANEL: every local multiply of this call (the plan's sample included on
  // one rank) multiplies the same A, so its column maps are built once.  Not
  // for STAGED, whose stages multiply different A slices.
  std::unique_ptr<APrepScope> aprep_scope;
  if (exec == CBG_EXEC_PANEL) aprep_scope.reset(new APrepScope());
  // phases == CBG_PHASES_AUTO or a memory budget: the count comes from memory;
  // otherwise phases < 1 or >= A_gncol is "Resetting to 1" (ParFriends.h:468-473)
  const bool automatic = phases == CBG_PHASES_AUTO || mem_gb > 0;
  if (!automatic && (phases < 1 || phases >= A_gncol)) phases = 1;
  int rc = A_gncol != B_gnrow ? CBG_ERR_DIMMISMATCH : CBG_OK;
  int64_t n_min = 0;
  if ((rc = agree_val(g, rc, B.n, &n_min, nullptr))) return rc;
  if (automatic && (rc = plan_phases(g, A, B, A_gncol, mem_gb, n_min, std::max(1, phases), phases))) return rc;
  phase_plan().phases = phases;
  if ((rc = agree(g, B.n < phases ? CBG_ERR_INVALIDPARAMS : CBG_OK))) return rc;  // ColSplit: "Matrix is too small to be splitted"
  hipStream_t cs = g->compute;
  const int64_t w = B.n / phases;
  std::vector<int64_t> cuts;
  for (int p = 0; p < phases; ++p) cuts.push_back((int64_t)p * w);
  cuts.push_back(B.n);
  if (exec == CBG_EXEC_PANEL) {
    // the reference copies B first, so A and B may alias here (ParFriends.h:547-549);
    // the copy is a step of every rank (a no-op where they do not alias), so
    // an empty tile on one rank cannot skip an agree() its peers make
    const bool alias = (&A == &B) || (A.ir == B.ir && A.nnz > 0);
    TileGuard Bcopy;
    rc = step([&] {
      if (alias) tile_slice_cols(B, 0, B.n, Bcopy.t, cs);
    });
    if ((rc = agree(g, rc))) return rc;
    const cbg_tile& Bu = alias ? Bcopy.t : B;
    if (phases == 1) {
      // one phase is Mult_AnXBn_DoubleBuff: B's block column arrives in the
      // (adaptive) pipeline's pieces, each handed to fn as phase 0 at its column offset
      const bool adaptive = !getenv("CBG_PIPELINE") && g->pr * g->pc > 1;
      return summa_panel(g, A, Bu, A_gncol, B_gnrow, sr, pipeline_cuts(g, Bu.n, n_min), fn, user, C, adaptive,
                         true);
    }
    return summa_panel(g, A, Bu, A_gncol, B_gnrow, sr, cuts, fn, user, C);
  }
  std::vector<TileGuard> parts;
  std::vector<cbg_tile> pv;
  int cb_rc = 0;
  for (int p = 0; p < phases; ++p) {
    TileGuard piece, Cp;
    rc = step([&] { tile_slice_cols(B, cuts[p], cuts[p + 1], piece.t, cs); });
    if ((rc = agree(g, rc))) return rc;
    rc = summa_staged(g, A, piece.t, A_gncol, B_gnrow, sr, algo, Cp.t);
    if (rc) return rc;
    if (fn) {
      rc = step([&] {
        CBG_HIP(hipStreamSynchronize(cs));
        const int r = fn(user, p, cuts[p], &Cp.t);
        if (r && !cb_rc) cb_rc = r;
      });
      if ((rc = agree(g, rc))) return rc;
    } else {
      pv.push_back(Cp.t);
      parts.push_back(std::move(Cp));
    }
  }
  if (fn) return agree(g, cb_rc ? CBG_ERR_INVALIDPARAMS : CBG_OK);
  rc = step([&] {
    if (pv.size() == 1) {
      *C = parts[0].release();
    } else {
      std::vector<int64_t> off(cuts.begin(), cuts.end() - 1);
      tile_concat_cols(pv, off, A.m, B.n, *C, cs);
    }
  });
  return agree(g, rc);
}

// ---------------------------------------------------------------------------
// SpParMat::Transpose (SpParMat.cpp:3528-3590) on a square grid: a diagonal
// rank transposes its tile; rank (r,c) transposes the tile of its complement
// (c,r) (GetComplementRank), received over RCCL send/recv (host transport:
// world broadcasts, test only).  `out` is this rank's tile of the transpose.
// ---------------------------------------------------------------------------
int grid_transpose(cbg_grid* g, const cbg_tile& T, cbg_tile& out) {
  check_usable(g);
  if (g->pr != g->pc) return CBG_ERR_NOTSQUARE;  // the grid's shape: the same answer on every rank
  hipStream_t cs = g->compute;
  const bool inject = redist_fault(g);
  // essentials of every rank's tile (world allgather: collective, diagonal ranks too)
  int64_t e[4] = {T.m, T.n, T.nnz, T.nzc};
  std::vector<int64_t> E((size_t)4 * g->nranks);
  allgather_i64(g, COMM_WORLD, e, E.data(), 4);
  const bool diag = g->prow == g->pcol;
  const int peer = g->pcol * g->pc + g->prow;
  const int64_t* pe = &E[4 * (size_t)peer];
  // every rank holds its receive buffer before anyone sends (agreed)
  TileGuard R;
  int rc = step([&] {
    if (inject) throw HipError("injected fault (CBG_FAULT_INJECT_REDIST) in Transpose", CBG_ERR_OOM);
    if (!diag) tile_alloc_device(R.t, pe[0], pe[1], pe[2], pe[3]);
  });
  if ((rc = agree(g, rc))) return rc;
  int local = step([&] {
    if (g->host_mode && g->nranks > 1) {
      // every off-diagonal rank broadcasts its tile over the world communicator
      for (int q = 0; q < g->nranks; ++q) {
        const int qr = q / g->pc, qc = q % g->pc;
        if (qr == qc) continue;
        const int64_t* qe = &E[4 * (size_t)q];
        const bool mine = q == g->rank, keep = !diag && q == peer;
        auto hb = [&](void* dst, const void* src, size_t bytes) {
          if (bytes == 0) return;
          std::vector<char> h(bytes);
          if (mine) CBG_HIP(hipMemcpy(h.data(), src, bytes, hipMemcpyDeviceToHost));
          host_check(g, g->hc.bcast(g->hc.user, COMM_WORLD, h.data(), bytes, q), "transpose bcast");
          if (keep) CBG_HIP(hipMemcpy(dst, h.data(), bytes, hipMemcpyHostToDevice));
        };
        hb(R.t.cp, T.cp, sizeof(int64_t) * (qe[3] + 1));
        hb(R.t.jc, T.jc, sizeof(int32_t) * qe[3]);
        hb(R.t.ir, T.ir, sizeof(int32_t) * qe[2]);
        hb(R.t.val, T.val, sizeof(double) * qe[2]);
      }
    } else if (!diag) {
      ncclComm_t c = g->world;
      CBG_NCCL(ncclGroupStart());
      CBG_NCCL(ncclSend(T.cp, T.nzc + 1, ncclInt64, peer, c, g->comm));
      CBG_NCCL(ncclRecv(R.t.cp, pe[3] + 1, ncclInt64, peer, c, g->comm));
      if (T.nzc) CBG_NCCL(ncclSend(T.jc, T.nzc, ncclInt32, peer, c, g->comm));
      if (pe[3]) CBG_NCCL(ncclRecv(R.t.jc, pe[3], ncclInt32, peer, c, g->comm));
      if (T.nnz) {
        CBG_NCCL(ncclSend(T.ir, T.nnz, ncclInt32, peer, c, g->comm));
        CBG_NCCL(ncclSend(T.val, T.nnz, ncclFloat64, peer, c, g->comm));
      }
      if (pe[2]) {
        CBG_NCCL(ncclRecv(R.t.ir, pe[2], ncclInt32, peer, c, g->comm));
        CBG_NCCL(ncclRecv(R.t.val, pe[2], ncclFloat64, peer, c, g->comm));
      }
      CBG_NCCL(ncclGroupEnd());
      wait_comm(g);
    }
  });
  // the local transpose (SpDCCols::Transpose) only where the exchange worked
  TileGuard O;
  if (!local) local = step([&] { tile_transpose(diag ? T : R.t, O.t, cs); });
  if ((rc = agree(g, local))) return rc;
  out = O.release();
  return CBG_OK;
}

// ---------------------------------------------------------------------------
// SpParMat::BlockSplit (SpParMat.cpp:2974-3058) for the splits BlockSpGEMM
// uses (bi = 1, BlockSpGEMM.h:39-45): global rows [lo, hi) of a distributed
// matrix (dim 0) or columns [lo, hi) (dim 1) as a distributed matrix of its
// own on the same grid, in the standard block layout (Owner,
// SpParMat.cpp:5068-5097).  Rows only move inside a grid column (columns
// inside a grid row): every rank broadcasts its slice of the range to its
// column (row) communicator and keeps the part of each slice that falls in
// its new block.  Collective steps agree on a code like the SUMMA's: a rank
// that cannot allocate a receive buffer makes every rank return the code
// before any of them posts the broadcast it would have skipped.
// ---------------------------------------------------------------------------
int grid_block_extract(cbg_grid* g, const cbg_tile& T, int64_t gm, int64_t gn, int dim, int64_t lo, int64_t hi,
                       cbg_tile& out) {
  check_usable(g);
  if (dim != 0 && dim != 1) return CBG_ERR_INVALIDPARAMS;
  const int64_t gext = dim == 0 ? gm : gn;
  if (lo < 0 || hi < lo || hi > gext) return CBG_ERR_INVALIDPARAMS;
  hipStream_t cs = g->compute;
  const bool inject = redist_fault(g);
  const int which = dim == 0 ? COMM_COL : COMM_ROW;
  const int np = comm_size(g, which), me = comm_rank(g, which);
  // my old range [S0, S1) along dim and my new range [lo + T0, lo + T1)
  auto span = [](int64_t ext, int np_, int i, int64_t& a, int64_t& b) {
    const int64_t per = ext / np_;
    a = (int64_t)i * per;
    b = i == np_ - 1 ? ext : a + per;
  };
  int64_t S0, S1, T0, T1;
  span(gext, np, me, S0, S1);
  span(hi - lo, np, me, T0, T1);
  T0 += lo;
  T1 += lo;
  auto cut = [&](const cbg_tile& X, int64_t a, int64_t b, cbg_tile& piece) {  // local range [a, b) of X
    TileGuard head, rest, tail;
    if (dim == 0) {
      tile_split_rows(X, b, head.t, tail.t, cs);
      tail = TileGuard();
      tile_split_rows(head.t, a, rest.t, piece, cs);
    } else {
      tile_split_cols(X, b, head.t, tail.t, cs);
      tail = TileGuard();
      tile_split_cols(head.t, a, rest.t, piece, cs);
    }
  };
  // my slice of [lo, hi)
  const int64_t x0 = std::max(S0, lo), x1 = std::max(x0, std::min(S1, hi));
  TileGuard mine;
  int rc = step([&] { cut(T, x0 - S0, x1 - S0, mine.t); });
  int64_t e[4] = {mine.t.m, mine.t.n, mine.t.nnz, mine.t.nzc};
  if (rc) e[0] = e[1] = e[2] = e[3] = 0;
  if ((rc = agree(g, rc))) return rc;
  std::vector<int64_t> E((size_t)4 * np);
  allgather_i64(g, which, e, E.data(), 4);
  std::vector<TileGuard> parts;
  std::vector<int64_t> offs;
  int local = CBG_OK;
  for (int q = 0; q < np; ++q) {
    int64_t Q0, Q1;
    span(gext, np, q, Q0, Q1);
    const int64_t y0 = std::max(Q0, lo), y1 = std::max(y0, std::min(Q1, hi));  // slice of rank q
    TileGuard recv;
    rc = step([&] {
      if (inject && q == (me + 1) % np) throw HipError("injected fault (CBG_FAULT_INJECT_REDIST) in BlockSplit", CBG_ERR_OOM);
      if (q != me) alloc_like(recv.t, &E[4 * (size_t)q]);
    });
    if ((rc = agree(g, rc))) return rc;  // every receive buffer of this broadcast exists
    cbg_tile& sl = q == me ? mine.t : recv.t;
    local = std::max(local, step([&] {
      bcast_group(g, [&] { bcast_tile(g, which, q, &E[4 * (size_t)q], sl, q == me); });
      wait_comm(g);
    }));
    const int64_t z0 = std::max(y0, T0), z1 = std::min(y1, T1);  // the part of it in my new range
    if (!local && z1 > z0)
      local = step([&] {
        TileGuard piece;
        cut(sl, z0 - y0, z1 - y0, piece.t);
        parts.push_back(std::move(piece));
        offs.push_back(z0 - T0);
      });
  }
  mine = TileGuard();
  const int64_t om = dim == 0 ? T1 - T0 : T.m, on = dim == 0 ? T.n : T1 - T0;
  TileGuard O;
  if (!local)
    local = step([&] {
      std::vector<cbg_tile> pv;
      for (auto& t : parts) pv.push_back(t.t);
      if (pv.empty()) {
        tile_alloc_device(O.t, om, on, 0, 0);
      } else if (dim == 0) {
        tile_concat_rows(pv, offs, om, on, O.t, cs);
      } else {
        tile_concat_cols(pv, offs, om, on, O.t, cs);
      }
      CBG_HIP(hipStreamSynchronize(cs));
    });
  if ((rc = agree(g, local))) return rc;
  out = O.release();
  return CBG_OK;
}

}  // namespace cbg

extern "C" int cbg_get_unique_id(void* id) {
  if (!id) return CBG_ERR_INVALIDPARAMS;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return CBG_ERR_RCCL;
  std::memcpy(id, &u, sizeof(u));
  return CBG_OK;
}

extern "C" int cbg_grid_info(const cbg_grid* g, int* rank, int* nranks, int* rows, int* cols, int* prow, int* pcol) {
  if (!g) return CBG_ERR_INVALIDPARAMS;
  if (rank) *rank = g->rank;
  if (nranks) *nranks = g->nranks;
  if (rows) *rows = g->pr;
  if (cols) *cols = g->pc;
  if (prow) *prow = g->prow;
  if (pcol) *pcol = g->pcol;
  return CBG_OK;
}
